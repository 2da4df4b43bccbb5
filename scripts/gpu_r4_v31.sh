#!/bin/bash
# Round 4, iteration 31: chunk-local observed-first order (each 4096-pixel chunk
# partitioned in place, one pass) vs the global partition, interleaved: tip7 at
# T = 500 / 32, spatial, prosail10, multisensor; the order tests first.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r4v31
O=gpurun_out/r4v31
stop() { echo "!! $1 rc=$2"; exit ${2:-1}; }
run() { local n=$1 log=$2 to=$3; shift 3; timeout -k 10 $to "$@" > $log 2>&1; local rc=$?; \
        if [ $rc -ne 0 ]; then tail -40 $log; stop $n $rc; fi; }
run tests $O/tests.log 400 python -u -m pytest tests/test_gpu.py -k "obs_order or observed_first" -x -v --timeout 150 --timeout-method thread
tail -1 $O/tests.log
for rep in 1 2; do
  for l in true false; do
    run tip7_${l}_$rep $O/tip7_${l}_$rep.log 300 python -u bench.py --set observed_first_local=$l
    echo "tip7 local=$l rep=$rep $(grep -o '"ms_per_step": [0-9.]*' $O/tip7_${l}_$rep.log)"
  done
done
for l in true false; do
  run t32_$l $O/t32_$l.log 300 python -u bench.py --config tip7 --n-train 32 --set observed_first_local=$l
  echo "T32 local=$l $(grep -o '"ms_per_step": [0-9.]*' $O/t32_$l.log)"
done
for c in spatial prosail10 multisensor; do
  for l in true false; do
    run ${c}_$l $O/${c}_$l.log 400 python -u bench.py --config $c --set observed_first_local=$l
    echo "$c local=$l $(grep -o '"ms_per_step": [0-9.]*' $O/${c}_$l.log)"
  done
done
echo all-done
