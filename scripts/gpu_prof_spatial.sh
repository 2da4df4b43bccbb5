#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_spatial" -o run --output-format csv -- \
  python "$R/bench.py" --config spatial --steps 3 --warmup 1 > "$R/gpurun_out/prof_spatial.log" 2>&1 || exit $?
echo done
