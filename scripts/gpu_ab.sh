#!/bin/bash
# A/B: analysis-kernel variants / grid caps (one process), then the full bench per grid cap
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
stop() { echo "!! $1 rc=$2"; exit $2; }
timeout -k 10 300 python scripts/bench_kernels.py --size 4096 --n-train 500 --rounds 7 \
    --variants "${VARIANTS:-0,0@16384,0@65536,0@1000000,1@1000000}" > gpurun_out/ab_kernels.json 2> gpurun_out/ab_kernels.err || stop ab $?
cat gpurun_out/ab_kernels.json
for cap in ${CAPS:-0 1000000}; do
  if [ "$cap" = 0 ]; then unset KAFKA_MAX_BLOCKS; else export KAFKA_MAX_BLOCKS=$cap; fi
  timeout -k 10 600 python bench.py --steps 8 --warmup 2 > gpurun_out/ab_bench_$cap.log 2>&1 || stop bench$cap $?
  echo "cap=$cap $(tail -1 gpurun_out/ab_bench_$cap.log | cut -c1-200)"
done
