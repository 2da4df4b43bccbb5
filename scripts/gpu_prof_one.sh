#!/bin/bash
# rocprofv3 kernel statistics of one bench.py configuration:
#   bash scripts/gpu_prof_one.sh TAG [bench args...]  -> gpurun_out/prof_TAG/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
tag=$1; shift
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$tag" -o run --output-format csv \
  -- python "$R/bench.py" "$@" > "$R/gpurun_out/prof_$tag.log" 2>&1 || { echo "!! prof $tag rc=$?"; tail -5 "$R/gpurun_out/prof_$tag.log"; exit 1; }
tail -1 "$R/gpurun_out/prof_$tag.log" | cut -c1-300
