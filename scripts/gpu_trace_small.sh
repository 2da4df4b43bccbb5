#!/bin/bash
# Kernel + memory-copy trace of the per-rank (N=8) strip size: gaps between kernels.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d "$R/gpurun_out/trace_small" -o run --output-format csv -- \
  python "$R/bench.py" --size ${SIZE:-3882} --steps 6 --warmup 2 > "$R/gpurun_out/trace_small.log" 2>&1 || exit $?
tail -1 "$R/gpurun_out/trace_small.log" | cut -c1-200
