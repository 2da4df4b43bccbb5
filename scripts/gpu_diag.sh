#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 120 python bench.py --size 256 --steps 2 --warmup 1 --verbose --watchdog 30 > gpurun_out/diag_256.log 2>&1; echo "rc256=$?"
tail -5 gpurun_out/diag_256.log
timeout -k 10 150 python bench.py --size 1024 --steps 2 --warmup 1 --verbose --watchdog 30 > gpurun_out/diag_1024.log 2>&1; echo "rc1024=$?"
tail -40 gpurun_out/diag_1024.log
