#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
for s in 3882 10980; do
  timeout -k 10 300 python -u scripts/bench_kernels.py --size $s --rounds 5 \
     --variants "0@16384,0@4096,0@32768,0@65536,0@131072,0@1000000" > gpurun_out/grid2_$s.json 2> gpurun_out/grid2_$s.err || { echo "!! $s rc=$?"; tail -5 gpurun_out/grid2_$s.err; exit 1; }
  cat gpurun_out/grid2_$s.json
done
for mb in 4096 16384 65536; do
  KAFKA_MAX_BLOCKS=$mb timeout -k 10 300 python -u bench.py --config prosail10 --size 5490 --steps 3 --warmup 1 > gpurun_out/grid2_p10_$mb.log 2>&1 || { echo "!! p10 $mb rc=$?"; exit 1; }
  echo "mb=$mb $(tail -1 gpurun_out/grid2_p10_$mb.log | cut -c1-200)"
done
