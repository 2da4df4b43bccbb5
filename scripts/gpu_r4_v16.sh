#!/bin/bash
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.} && mkdir -p gpurun_out/r4v16 && \
timeout -k 10 120 python -u scripts/probes/copy_stall_probe.py > gpurun_out/r4v16/warm.txt 2>&1 && cat gpurun_out/r4v16/warm.txt && \
timeout -k 10 120 python -u scripts/probes/copy_stall_probe.py --no-warm > gpurun_out/r4v16/nowarm.txt 2>&1 && cat gpurun_out/r4v16/nowarm.txt && \
timeout -k 10 120 python -u scripts/probes/copy_stall_probe.py --kernel-ms 2 > gpurun_out/r4v16/warm2.txt 2>&1 && cat gpurun_out/r4v16/warm2.txt
