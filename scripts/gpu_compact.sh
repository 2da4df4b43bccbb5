#!/bin/bash
# compacted analysis kernel: GPU tests, kernel A/B, full bench default vs variant 4
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
stop() { echo "!! $1 rc=$2"; exit $2; }
timeout -k 10 300 python -m pytest tests/test_gpu.py -q > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -le 1 ] || stop tests $rc
timeout -k 10 300 python scripts/bench_kernels.py --size 4096 --n-train 500 --rounds 7 --variants 0,4,0,4 > gpurun_out/ab_compact.json 2>&1 || stop ab $?
cat gpurun_out/ab_compact.json
for v in 0 4; do
  KAFKA_ANALYSIS_VARIANT=$v timeout -k 10 600 python bench.py --steps 8 --warmup 2 > gpurun_out/bench_v$v.log 2>&1 || stop bench$v $?
  echo "variant=$v $(tail -1 gpurun_out/bench_v$v.log | cut -c1-200)"
done
