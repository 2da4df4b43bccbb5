#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
stop() { echo "!! $1 rc=$2"; exit $2; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; stop tests $?; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || stop smoke $?
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python -u bench.py --config identity7 --steps 30 --warmup 3 > gpurun_out/identity7.log 2>&1 || stop id7 $?
tail -1 gpurun_out/identity7.log | cut -c1-220
timeout -k 10 400 python -u bench.py --steps 8 --warmup 2 > gpurun_out/bench_default.log 2>&1 || stop bench $?
tail -1 gpurun_out/bench_default.log | cut -c1-220
