#!/bin/bash
# One PMC pass (kernel-trace + counters) over the headline analysis kernel
# (bench_kernels.py, JRC-TIP, 4096^2, T=500, variant 0).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/pmc_tip"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 -s KILL 180 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_VALU_MFMA_BUSY_CYCLES \
    SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
    --kernel-include-regex "analysis_mfma" -d "$R/gpurun_out/pmc_tip" -o run --output-format csv -- \
    python "$R/scripts/bench_kernels.py" --size 4096 --variants 0 --rounds 2 > "$R/gpurun_out/pmc_tip.log" 2>&1 \
  || { echo "!! pmc rc=$?"; tail -5 "$R/gpurun_out/pmc_tip.log"; exit 1; }
echo pmc-done
