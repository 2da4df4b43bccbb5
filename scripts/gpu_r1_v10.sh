#!/bin/bash
# Round-1 re-check of the current tree: gpu tests, smoke, identity7 + default bench,
# rocprof kernel stats of a short default bench.  Stops at the first failing step.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
stop() { echo "!! $1 rc=$2"; exit $2; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; stop tests $?; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || stop smoke $?
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python -u bench.py --config identity7 --steps 30 --warmup 3 > gpurun_out/identity7.log 2>&1 || stop id7 $?
tail -1 gpurun_out/identity7.log | cut -c1-300
timeout -k 10 400 python -u bench.py > gpurun_out/bench_default.log 2>&1 || stop bench $?
tail -1 gpurun_out/bench_default.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- python "$R/bench.py" --steps 4 --warmup 1 > "$R/gpurun_out/prof.log" 2>&1 || stop prof $?
echo prof-done
