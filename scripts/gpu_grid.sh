#!/bin/bash
# Grid-cap A/B of the headline analysis kernel at the per-rank strip sizes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
for s in 3882 7764 10980; do
  timeout -k 10 300 python -u scripts/bench_kernels.py --size $s --rounds 5 \
     --variants "0@4096,0@1024,0@2048,0@3072,0@6144,0@8192,0@16384" > gpurun_out/grid_$s.json 2> gpurun_out/grid_$s.err || { echo "!! $s rc=$?"; tail -5 gpurun_out/grid_$s.err; exit 1; }
  cat gpurun_out/grid_$s.json
done
