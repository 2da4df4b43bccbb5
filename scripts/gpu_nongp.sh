#!/bin/bash
# Non-GP share of the fused headline step: bench.py tip7 at the full tile with
# T = 500 and T = 32 training points (the step time at T -> 0 is the per-pixel
# work outside the GP loop), then one PMC pass per T over the fused kernel at
# 4096^2 (VALU / transcendental / VMEM instruction counts per dispatch).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/nongp
for T in ${TS:-500 32}; do
  timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --n-train $T > gpurun_out/nongp/bench_T$T.log 2>&1 \
    || { echo "!! bench T=$T rc=$?"; tail -5 gpurun_out/nongp/bench_T$T.log; exit 1; }
  echo "T=$T $(tail -1 gpurun_out/nongp/bench_T$T.log | cut -c1-200)"
done
cd /tmp && export TMPDIR=/tmp
for T in ${TS:-500 32}; do
  timeout -k 10 -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU \
      SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
      --kernel-include-regex "analysis_mfma" -d "$R/gpurun_out/nongp/pmc_T$T" -o run --output-format csv -- \
      python "$R/bench.py" --size 4096 --steps 2 --warmup 1 --n-train $T > "$R/gpurun_out/nongp/pmc_T$T.log" 2>&1 \
    || { echo "!! pmc T=$T rc=$?"; tail -5 "$R/gpurun_out/nongp/pmc_T$T.log"; exit 1; }
  echo "pmc T=$T done"
done
