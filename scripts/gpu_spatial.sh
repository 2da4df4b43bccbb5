#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
stop() { echo "!! $1 rc=$2"; exit $2; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; stop tests $?; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 500 python -u bench.py --config spatial --steps 6 --warmup 2 > gpurun_out/spatial_full.log 2>&1 || stop spatial $?
tail -1 gpurun_out/spatial_full.log | cut -c1-260
