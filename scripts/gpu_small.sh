#!/bin/bash
# per-GPU share of an 8-GPU run (10980^2/8 ~ 3882^2 px) on one GPU: host overhead check
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
stop() { echo "!! $1 rc=$2"; exit $2; }
timeout -k 10 300 python bench.py --size 3882 --steps 20 --warmup 3 --metrics gpurun_out/small_metrics.jsonl > gpurun_out/small.log 2>&1 || stop small $?
tail -1 gpurun_out/small.log | cut -c1-220
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_small" -o run --output-format csv -- python "$R/bench.py" --size 3882 --steps 10 --warmup 2 > "$R/gpurun_out/prof_small.log" 2>&1 || stop prof $?
echo prof ok
