#!/bin/bash
# GP-loop throughput vs training-set size (scalar-cache footprint) + counter list
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
stop() { echo "!! $1 rc=$2"; exit $2; }
for T in 64 128 256 500 1000; do
  timeout -k 10 300 python scripts/bench_kernels.py --size 4096 --n-train $T --variants 0 >> gpurun_out/probe_T.jsonl 2> gpurun_out/probe_T.err || stop probe$T $?
done
cat gpurun_out/probe_T.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > "$R/gpurun_out/counters.txt" 2>&1 || echo "list rc=$?"
grep -c . "$R/gpurun_out/counters.txt"
