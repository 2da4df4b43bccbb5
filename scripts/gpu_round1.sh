#!/bin/bash
# GPU validation pass: tests, smoke, benches, rocprof kernel stats.
# Assertion failures (rc 1) do not stop the later steps; any other non-zero
# exit (fault, abort, timeout) ends the script.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
step() { local name=$1; shift; echo "== $name"; "$@"; local rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "!! $name rc=$rc; stopping"; exit $rc; fi; return $rc; }
# (gpu tests passed in the previous call)

step bench2048 timeout -k 10 300 python bench.py --size 2048 --steps 5 --warmup 2 > gpurun_out/bench_2048.log 2>&1; tail -2 gpurun_out/bench_2048.log
step benchfull timeout -k 10 600 python bench.py --steps 6 --warmup 2 > gpurun_out/bench_full.log 2>&1; tail -3 gpurun_out/bench_full.log
cd /tmp && export TMPDIR=/tmp
step rocprof timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- python "$R/bench.py" --size 4096 --steps 3 --warmup 1 > "$R/gpurun_out/prof.log" 2>&1; tail -3 "$R/gpurun_out/prof.log"
find "$R/gpurun_out/prof" -name "*stats*"
