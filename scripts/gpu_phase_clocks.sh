#!/bin/bash
# Phase attribution of the fused JRC-TIP analysis kernel with the phase-clock
# build (_build.py --prof, KAFKA_PROF=1): bench.py at 4096^2 for T = 500 and 32.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/phase
for T in ${TS:-500 32}; do
  KAFKA_PROF=1 timeout -k 10 300 python -u bench.py --config ${CONFIG:-tip7} --size ${SIZE:-4096} --steps 4 --warmup 1 --n-train $T \
      > gpurun_out/phase/T$T.log 2>&1 || { echo "!! T=$T rc=$?"; tail -5 gpurun_out/phase/T$T.log; exit 1; }
  echo "T=$T $(grep phase_clocks gpurun_out/phase/T$T.log)"
  echo "T=$T $(tail -1 gpurun_out/phase/T$T.log | cut -c1-160)"
done
