#!/bin/bash
# Round 4 final check (after the vectorised order passes) on one MI355X: GPU tests, smoke(), every bench config,
# a kernel-trace summary of the default bench (copied into profiles/).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r4final3
O=gpurun_out/r4final3
stop() { echo "!! $1 rc=$2"; exit ${2:-1}; }
run() { local n=$1 log=$2 to=$3; shift 3; timeout -k 10 $to "$@" > $log 2>&1; local rc=$?; \
        if [ $rc -ne 0 ]; then tail -40 $log; stop $n $rc; fi; }
run tests $O/gpu_tests.log 700 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread
tail -1 $O/gpu_tests.log
run smoke $O/smoke.log 200 python -c "import __graft_entry__ as g; g.smoke()"
tail -1 $O/smoke.log
run bench_default $O/bench_default.log 400 python -u bench.py
echo "default $(tail -1 $O/bench_default.log | cut -c1-220)"
for c in tip7 spatial prosail10 identity7 multisensor prosail10_hard; do
  run cfg_$c $O/cfg_$c.log 600 python -u bench.py --config $c
  echo "$c $(tail -1 $O/cfg_$c.log | cut -c1-200)"
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/trace_default" -o run \
    --output-format csv -- python "$R/bench.py" --steps 5 --warmup 2 > "$R/$O/trace_default.log" 2>&1) \
  || { tail -5 $O/trace_default.log; stop trace 1; }
echo all-done
