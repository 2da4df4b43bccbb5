#!/bin/bash
# Round 4, iteration 28: vectorised obs_order passes (16 px per thread, LDS-ranked
# coalesced scatter): device-vs-host partition tests, the T = 32 kernel trace, and
# the bench configs that use the order.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r4v28
O=gpurun_out/r4v28
stop() { echo "!! $1 rc=$2"; exit ${2:-1}; }
run() { local n=$1 log=$2 to=$3; shift 3; timeout -k 10 $to "$@" > $log 2>&1; local rc=$?; \
        if [ $rc -ne 0 ]; then tail -40 $log; stop $n $rc; fi; }
run tests $O/tests.log 400 python -u -m pytest tests/test_gpu.py -k "obs_order or observed_first" -x -v --timeout 150 --timeout-method thread
tail -1 $O/tests.log
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/tr_on" -o run --output-format csv -- \
    python "$R/bench.py" --config tip7 --steps 6 --warmup 2 --n-train 32 > "$R/$O/tr_on.log" 2>&1) || { tail -5 $O/tr_on.log; stop trace 1; }
echo "trace T32 $(grep metric $O/tr_on.log | cut -c1-150)"
for rep in 1 2; do
  run tip7_$rep $O/tip7_$rep.log 300 python -u bench.py
  echo "default rep=$rep $(tail -1 $O/tip7_$rep.log | cut -c1-170)"
done
for c in spatial prosail10 multisensor; do
  run cfg_$c $O/cfg_$c.log 400 python -u bench.py --config $c
  echo "$c $(tail -1 $O/cfg_$c.log | cut -c1-170)"
done
echo all-done
