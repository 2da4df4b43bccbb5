#!/bin/bash
# tests + smoke + full bench (+ optional rocprof); stops on faults/timeouts
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
stop() { echo "!! $1 rc=$2"; exit $2; }
timeout -k 10 900 python -m pytest tests/test_gpu.py -q > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -le 1 ] || stop tests $rc
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || stop smoke $?
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python bench.py --steps 8 --warmup 2 --watchdog 120 > gpurun_out/bench_full.log 2>&1 || stop bfull $?
tail -1 gpurun_out/bench_full.log
if [ -n "$PROF" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- python "$R/bench.py" --steps 4 --warmup 1 > "$R/gpurun_out/prof.log" 2>&1 || stop prof $?
  echo prof-done
fi
