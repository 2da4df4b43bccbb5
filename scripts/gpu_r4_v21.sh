#!/bin/bash
# SURVEY 7.3 MVP slice at its specified size, 1024^2 (10 dates, T = 500), on the
# device against the float64 block oracle (oracle progress printed per date).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.} && mkdir -p gpurun_out/r4v21 && \
timeout -k 10 1000 python -u scripts/mvp_precision.py --size 1024 --variants ${VARIANTS:-0} > gpurun_out/r4v21/mvp1024.jsonl 2>&1; rc=$?; \
tail -3 gpurun_out/r4v21/mvp1024.jsonl | cut -c1-400; exit $rc
