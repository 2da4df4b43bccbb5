#!/bin/bash
# One PMC pass (VALU / MFMA / wave counters) over the fused analysis kernels of
# the tip7 and prosail10 bench configs at 4096^2 (bench.py, 2 timed steps).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/pmc_final"
cd /tmp && export TMPDIR=/tmp
for c in ${CONFIGS:-tip7 prosail10}; do
  timeout -k 10 -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 \
      SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU \
      --kernel-include-regex "analysis_mfma" -d "$R/gpurun_out/pmc_final/$c" -o run --output-format csv -- \
      python "$R/bench.py" --config $c --size 4096 --steps 2 --warmup 1 > "$R/gpurun_out/pmc_final/$c.log" 2>&1 \
    || { echo "!! pmc $c rc=$?"; tail -5 "$R/gpurun_out/pmc_final/$c.log"; exit 1; }
  echo "pmc $c done"
done
