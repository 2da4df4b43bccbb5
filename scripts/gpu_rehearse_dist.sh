#!/bin/bash
# Multi-rank rehearsal on ONE GPU: 2 ranks of bench.py under torchrun, gloo backend
# (RCCL needs one GPU per rank; the 8-GPU RCCL run is the driver's)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out

port=29611
for c in ${REH_CONFIGS:-tip7 spatial}; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 \
      --master-port=$port bench.py --gpus 2 --device cuda:0 --rehearse-gloo --config $c --size 4096 --steps 4 --warmup 1 \
      > gpurun_out/rehearse2_$c.log 2>&1 || { echo "!! $c rc=$?"; tail -20 gpurun_out/rehearse2_$c.log; exit 1; }
  port=$((port+1))
  echo "$c: $(tail -1 gpurun_out/rehearse2_$c.log | cut -c1-220)"
done
