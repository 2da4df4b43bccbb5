#!/bin/bash
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.} && mkdir -p gpurun_out/r4v13 && \
SIZE=1024 NSTEP=60 timeout -k 10 200 python -u scripts/host_breakdown.py > gpurun_out/r4v13/hb_id7.txt 2>&1 && cat gpurun_out/r4v13/hb_id7.txt && \
SIZE=1024 NSTEP=60 timeout -k 10 200 python -u scripts/host_breakdown.py > gpurun_out/r4v13/hb_id7b.txt 2>&1 && cat gpurun_out/r4v13/hb_id7b.txt
