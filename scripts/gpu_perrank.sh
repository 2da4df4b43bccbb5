#!/bin/bash
# Per-rank work of the strong-scaling run on one GPU: the 10980^2 tile split
# over N ranks gives ~120.6M/N px per rank; time that strip size alone.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
for s in 3882 5490 7764; do
  timeout -k 10 300 python -u bench.py --size $s --steps 16 --warmup 3 > gpurun_out/perrank_$s.log 2>&1 || { echo "!! $s rc=$?"; exit 1; }
  tail -1 gpurun_out/perrank_$s.log | cut -c1-200
done
