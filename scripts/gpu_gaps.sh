#!/bin/bash
# Kernel trace of the N=8 per-rank strip (3882^2) to measure inter-kernel gaps.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d "$R/gpurun_out/gaps" -o run --output-format csv -- python "$R/bench.py" --size 3882 --steps 12 --warmup 3 > "$R/gpurun_out/gaps.log" 2>&1 || { tail -5 "$R/gpurun_out/gaps.log"; exit 1; }
tail -1 "$R/gpurun_out/gaps.log" | cut -c1-200
