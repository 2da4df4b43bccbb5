#!/bin/bash
# Round 4, iteration 33: obs_order decode for every source (DN16 fast path
# without an uncertainty floor; coalesced ballot fallback): order tests, then
# prosail10 kernel trace, tip7 and multisensor benches.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r4v33
O=gpurun_out/r4v33
stop() { echo "!! $1 rc=$2"; exit ${2:-1}; }
run() { local n=$1 log=$2 to=$3; shift 3; timeout -k 10 $to "$@" > $log 2>&1; local rc=$?; \
        if [ $rc -ne 0 ]; then tail -40 $log; stop $n $rc; fi; }
run tests $O/tests.log 400 python -u -m pytest tests/test_gpu.py -k "obs_order or observed_first" -x -v --timeout 150 --timeout-method thread
tail -1 $O/tests.log
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/tr_prosail10" -o run --output-format csv -- \
    python "$R/bench.py" --config prosail10 --steps 5 --warmup 2 > "$R/$O/tr_prosail10.log" 2>&1) || { tail -5 $O/tr_prosail10.log; stop trace 1; }
echo "prosail10 trace $(grep -o '"ms_per_step": [0-9.]*' $O/tr_prosail10.log)"
for c in tip7 prosail10 multisensor spatial; do
  run cfg_$c $O/cfg_$c.log 400 python -u bench.py --config $c
  echo "$c $(grep -o '"ms_per_step": [0-9.]*' $O/cfg_$c.log)"
done
echo all-done
