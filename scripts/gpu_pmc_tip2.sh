#!/bin/bash
# Second PMC pass over the headline analysis kernel: where the wave cycles go
# (issue-stalled vs parked vs active) and the LDS side.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/pmc_tip2"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 -s KILL 180 rocprofv3 --kernel-trace --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY \
    SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE \
    --kernel-include-regex "analysis_mfma" -d "$R/gpurun_out/pmc_tip2" -o run --output-format csv -- \
    python "$R/scripts/bench_kernels.py" --size 4096 --variants 0 --rounds 2 > "$R/gpurun_out/pmc_tip2.log" 2>&1 \
  || { echo "!! pmc rc=$?"; tail -5 "$R/gpurun_out/pmc_tip2.log"; exit 1; }
echo pmc2-done
