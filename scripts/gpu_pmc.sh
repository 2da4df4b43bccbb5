#!/bin/bash
# PMC counters of the headline analysis kernel (bench_kernels.py, 4096^2, T=500),
# one rocprofv3 pass per counter group, kernel-trace only (no sys/runtime trace).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/pmc"
cd /tmp && export TMPDIR=/tmp
stop() { echo "!! $1 rc=$2"; exit $2; }
i=0
for grp in "GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES" \
           "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_INSTS_SALU" \
           "SQC_DCACHE_HITS SQC_DCACHE_MISSES SQ_WAIT_INST_ANY SQ_INSTS_VALU_TRANS_F32" \
           "SQ_INST_CYCLES_SMEM SQ_THREAD_CYCLES_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_SCA" \
           "SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32" \
           "FETCH_SIZE TCP_TOTAL_CACHE_ACCESSES_sum" ${EXTRA_PMC}; do
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --kernel-include-regex "analysis_kernel" \
      -d "$R/gpurun_out/pmc/g$i" -o run --output-format csv -- \
      python "$R/scripts/bench_kernels.py" --size 4096 --n-train ${NTRAIN:-500} --variants ${VARIANTS:-0} --rounds 2 \
      > "$R/gpurun_out/pmc/g$i.log" 2>&1 || { echo "group $i ($grp) failed rc=$?"; tail -3 "$R/gpurun_out/pmc/g$i.log"; continue; }
  echo "group $i done"
done
