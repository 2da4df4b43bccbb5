#!/bin/bash
# first GPU validation pass: tests, smoke, benches, rocprof kernel stats
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
echo "== gpu tests"; timeout -k 10 900 python -m pytest tests/test_gpu.py -x -q > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -5 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke"; timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
echo "== bench 2048"; timeout -k 10 300 python bench.py --size 2048 --steps 5 --warmup 2 > gpurun_out/bench_2048.log 2>&1 || { tail -20 gpurun_out/bench_2048.log; exit 1; }
tail -3 gpurun_out/bench_2048.log
echo "== bench full"; timeout -k 10 600 python bench.py --steps 6 --warmup 2 > gpurun_out/bench_full.log 2>&1 || { tail -20 gpurun_out/bench_full.log; exit 1; }
tail -4 gpurun_out/bench_full.log
echo "== rocprof"; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- python "$R/bench.py" --size 4096 --steps 3 --warmup 1 > "$R/gpurun_out/prof.log" 2>&1 || { tail -20 "$R/gpurun_out/prof.log"; exit 1; }
find "$R/gpurun_out/prof" -name "*stats*" | head
