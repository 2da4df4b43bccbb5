#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r4v20
O=gpurun_out/r4v20
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
grep -E "async_copies|rccl" $O/gpu_tests.log | cut -c1-150
