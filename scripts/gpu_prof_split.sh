#!/bin/bash
# Kernel stats of the split-path configs (prosail10, multisensor) + PMC of the
# headline analysis kernel and the split GP operator kernel.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/pmc"
cd /tmp && export TMPDIR=/tmp
stop() { echo "!! $1 rc=$2"; exit $2; }
for c in prosail10 multisensor; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$c" -o run --output-format csv -- \
    python "$R/bench.py" --config $c --steps 2 --warmup 1 > "$R/gpurun_out/prof_$c.log" 2>&1 || stop $c $?
  tail -1 "$R/gpurun_out/prof_$c.log" | cut -c1-300
done
i=0
for grp in "GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES" \
           "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_INSTS_SALU" \
           "SQC_DCACHE_HITS SQC_DCACHE_MISSES SQ_WAIT_INST_ANY SQ_INSTS_VALU_TRANS_F32" \
           "SQ_INST_CYCLES_SMEM SQ_THREAD_CYCLES_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_SCA"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp --kernel-include-regex "gp_operator_kernel|analysis_kernel" \
      -d "$R/gpurun_out/pmc/s$i" -o run --output-format csv -- \
      python "$R/bench.py" --config prosail10 --size 2048 --steps 1 --warmup 1 \
      > "$R/gpurun_out/pmc/s$i.log" 2>&1 || stop pmc$i $?
  echo "group $i done"
done
