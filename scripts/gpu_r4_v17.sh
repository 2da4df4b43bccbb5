#!/bin/bash
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.} && mkdir -p gpurun_out/r4v17 && \
AMD_LOG_LEVEL=4 timeout -k 10 120 python -u scripts/probes/copy_stall_probe.py --steps 12 > gpurun_out/r4v17/log4.txt 2>&1; echo rc=$?; \
grep prefetch_ms gpurun_out/r4v17/log4.txt | cut -c1-200; wc -l gpurun_out/r4v17/log4.txt
