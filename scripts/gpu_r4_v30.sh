#!/bin/bash
# Round 4, iteration 30: XCD-aware block numbering of the MFMA analysis kernels
# (default) vs the hardware numbering (variant 19), interleaved: tip7 (T = 500
# and 32), prosail10; GPU tests first.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r4v30
O=gpurun_out/r4v30
stop() { echo "!! $1 rc=$2"; exit ${2:-1}; }
run() { local n=$1 log=$2 to=$3; shift 3; timeout -k 10 $to "$@" > $log 2>&1; local rc=$?; \
        if [ $rc -ne 0 ]; then tail -40 $log; stop $n $rc; fi; }
run tests $O/gpu_tests.log 700 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread
tail -1 $O/gpu_tests.log
for rep in 1 2; do
  for v in 0 19; do
    run tip7_v${v}_$rep $O/tip7_v${v}_$rep.log 300 env KAFKA_ANALYSIS_VARIANT=$v python -u bench.py
    echo "tip7 v=$v rep=$rep $(grep -o '"ms_per_step": [0-9.]*' $O/tip7_v${v}_$rep.log)"
  done
done
for v in 0 19; do
  run t32_v$v $O/t32_v$v.log 300 env KAFKA_ANALYSIS_VARIANT=$v python -u bench.py --config tip7 --n-train 32
  echo "T32 v=$v $(grep -o '"ms_per_step": [0-9.]*' $O/t32_v$v.log)"
done
for v in 0 19; do
  run pro_v$v $O/pro_v$v.log 400 env KAFKA_ANALYSIS_VARIANT=$v python -u bench.py --config prosail10
  echo "prosail10 v=$v $(grep -o '"ms_per_step": [0-9.]*' $O/pro_v$v.log)"
done
echo all-done
