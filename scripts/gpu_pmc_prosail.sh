#!/bin/bash
# One PMC pass (kernel-trace + counters, no sys/runtime trace) over the
# many-band matrix-core analysis kernel (prosail10 at 4096^2, one step).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/pmc_g"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 -s KILL 240 rocprofv3 --kernel-trace --pmc ${PMC:-SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_VALU_MFMA_BUSY_CYCLES \
    SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE} \
    --kernel-include-regex "analysis_mfma" -d "$R/gpurun_out/pmc_g${TAG:-}" -o run --output-format csv -- \
    python "$R/bench.py" --config prosail10 --size 4096 --steps 1 --warmup 0 > "$R/gpurun_out/pmc_g.log" 2>&1 \
  || { echo "!! pmc rc=$?"; tail -5 "$R/gpurun_out/pmc_g.log"; exit 1; }
echo pmc-done
