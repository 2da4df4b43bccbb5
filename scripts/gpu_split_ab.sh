#!/bin/bash
# prosail10 / multisensor with the split-path GP unroll 4 vs 2, plus GPU tests
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
stop() { echo "!! $1 rc=$2"; exit $2; }
timeout -k 10 300 python -m pytest tests/test_gpu.py -q > gpurun_out/gpu_tests.log 2>&1; tail -1 gpurun_out/gpu_tests.log
for u in 4 2; do
  KAFKA_GP_UNROLL=$u timeout -k 10 600 python bench.py --config prosail10 --steps 3 --warmup 1 > gpurun_out/split_p10_u$u.log 2>&1 || stop p10u$u $?
  echo "prosail10 unroll=$u $(tail -1 gpurun_out/split_p10_u$u.log | cut -c1-160)"
done
timeout -k 10 900 python bench.py --config multisensor --steps 3 --warmup 1 > gpurun_out/split_ms.log 2>&1 || stop ms $?
echo "multisensor $(tail -1 gpurun_out/split_ms.log | cut -c1-160)"
