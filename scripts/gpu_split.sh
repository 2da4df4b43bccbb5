#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu.py -q > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -le 1 ] || exit $rc
: > gpurun_out/bench_split.jsonl
for c in prosail10 multisensor; do
  timeout -k 10 600 python bench.py --config $c --steps 3 --warmup 1 --watchdog 120 > gpurun_out/split_$c.out 2> gpurun_out/split_$c.err || { echo "$c failed"; tail -5 gpurun_out/split_$c.err; exit 1; }
  tail -1 gpurun_out/split_$c.out >> gpurun_out/bench_split.jsonl
done
cut -c1-400 gpurun_out/bench_split.jsonl
