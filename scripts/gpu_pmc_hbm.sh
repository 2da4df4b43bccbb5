#!/bin/bash
# HBM-traffic PMC of the fused analysis kernels (tip7, prosail10 at 4096^2,
# bench.py, 2 timed steps): pass A = FETCH_SIZE (3 TCC) + TCC_HIT_sum + kernel
# time, pass B = WRITE_SIZE (2 TCC) + TCC_MISS_sum.  One run per pass (the
# per-block counter limits of rocprofv3: <= 4 TCC, <= 2 GRBM).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/pmc_hbm"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
SIZE=${SIZE:-4096}
for c in ${CONFIGS:-tip7 prosail10}; do
  for pass in A B; do
    if [ $pass = A ]; then CTR="FETCH_SIZE TCC_HIT_sum GRBM_GUI_ACTIVE"; else CTR="WRITE_SIZE TCC_MISS_sum"; fi
    timeout -k 10 -s KILL 240 rocprofv3 --kernel-trace --pmc $CTR \
        --kernel-include-regex "${REGEX:-analysis_mfma}" -d "$O/${c}_$pass" -o run --output-format csv -- \
        python "$R/bench.py" --config $c --size $SIZE --steps 2 --warmup 1 > "$O/${c}_$pass.log" 2>&1 \
      || { echo "!! pmc $c $pass rc=$?"; tail -5 "$O/${c}_$pass.log"; exit 1; }
    echo "pmc $c $pass done"
  done
done
