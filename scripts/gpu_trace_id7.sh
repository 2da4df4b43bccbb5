#!/bin/bash
# identity7 (1024^2) kernel + memory-copy trace: where a 0.3-0.5 ms step goes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/trace_id7"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$R/gpurun_out/trace_id7" -o run \
    --output-format csv -- python "$R/bench.py" --config identity7 --steps 60 --warmup 10 --no-telemetry \
    > "$R/gpurun_out/trace_id7.log" 2>&1 || { echo "!! trace rc=$?"; tail -5 "$R/gpurun_out/trace_id7.log"; exit 1; }
echo trace-done
