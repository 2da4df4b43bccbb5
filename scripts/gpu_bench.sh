#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
stop() { echo "!! $1 rc=$2"; exit $2; }
timeout -k 10 200 python bench.py --size 2048 --steps 5 --warmup 2 --watchdog 60 > gpurun_out/bench_2048.log 2>&1 || stop b2048 $?
tail -2 gpurun_out/bench_2048.log
timeout -k 10 500 python bench.py --steps 6 --warmup 2 --watchdog 120 > gpurun_out/bench_full.log 2>&1 || stop bfull $?
tail -4 gpurun_out/bench_full.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- python "$R/bench.py" --size 4096 --steps 3 --warmup 1 > "$R/gpurun_out/prof.log" 2>&1 || stop prof $?
find "$R/gpurun_out/prof" -name "*stats*"
