#!/bin/bash
# Multi-rank rehearsal on ONE GPU: 2 ranks of bench.py under torchrun, gloo backend
# (RCCL needs one GPU per rank; the 8-GPU RCCL run is the driver's)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export KAFKA_DIST_BACKEND=gloo
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 \
    --master-port=29611 bench.py --gpus 2 --device cuda:0 --size 4096 --steps 4 --warmup 1 \
    > gpurun_out/rehearse2.log 2>&1; rc=$?
tail -2 gpurun_out/rehearse2.log | cut -c1-300; exit $rc
