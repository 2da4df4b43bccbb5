#!/bin/bash
# gpu tests + host overhead + per-rank strip benches + full bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
stop() { echo "!! $1 rc=$2"; exit $2; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; stop tests $?; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python scripts/host_overhead.py > gpurun_out/host_overhead.log 2>&1 || stop host $?
grep "ms/step" gpurun_out/host_overhead.log
for s in 3882 ${SIZES}; do
  timeout -k 10 300 python -u bench.py --size $s --steps 16 --warmup 3 > gpurun_out/perrank_$s.log 2>&1 || stop perrank$s $?
  tail -1 gpurun_out/perrank_$s.log | cut -c1-200
done
timeout -k 10 600 python -u bench.py > gpurun_out/bench_default.log 2>&1 || stop bench $?
tail -1 gpurun_out/bench_default.log | cut -c1-250
