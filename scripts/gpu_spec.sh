#!/bin/bash
# Speculative next-step iteration: gpu tests, A/B on the N=8 per-rank strip
# (3882^2) and the full tile, kernel trace of the strip.  Stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
stop() { echo "!! $1 rc=$2"; exit $2; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; stop tests $?; }
tail -1 gpurun_out/gpu_tests.log
for sp in false true false true; do
  timeout -k 10 300 python -u bench.py --size 3882 --steps 20 --warmup 3 --set speculate=$sp > gpurun_out/spec_3882_$sp.log 2>&1 || stop s3882 $?
  echo "3882 speculate=$sp $(tail -1 gpurun_out/spec_3882_$sp.log | cut -c1-190)"
done
for sp in false true; do
  timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --set speculate=$sp > gpurun_out/spec_full_$sp.log 2>&1 || stop full $?
  echo "full speculate=$sp $(tail -1 gpurun_out/spec_full_$sp.log | cut -c1-190)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/gaps_spec" -o run --output-format csv -- python "$R/bench.py" --size 3882 --steps 12 --warmup 3 > "$R/gpurun_out/gaps_spec.log" 2>&1 || stop trace $?
echo trace-done
