#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
stop() { echo "!! $1 rc=$2"; exit $2; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; stop tests $?; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u scripts/bench_kernels.py --size 4096 --rounds 5 --variants "0,1,2,3" > gpurun_out/ab_rec.json 2> gpurun_out/ab_rec.err || stop abk $?
cat gpurun_out/ab_rec.json
for u in 4 -2 -1; do
  KAFKA_GP_UNROLL=$u timeout -k 10 300 python -u bench.py --config prosail10 --size 4096 --steps 3 --warmup 1 > gpurun_out/x2_$u.log 2>&1 || stop p10$u $?
  echo "u=$u $(tail -1 gpurun_out/x2_$u.log | cut -c100-200)"
done
timeout -k 10 600 python -u bench.py > gpurun_out/bench_default.log 2>&1 || stop bench $?
tail -1 gpurun_out/bench_default.log | cut -c1-250
