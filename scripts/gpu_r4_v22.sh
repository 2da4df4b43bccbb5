#!/bin/bash
# Grid cap A/B for the fused analysis (KAFKA_MAX_BLOCKS): 16384 = 21.33 rounds
# of the 768 resident JRC-TIP workgroups (3 per CU) -- the last round runs a
# third full; multiples of 768 have no partial round.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r4v22
O=gpurun_out/r4v22
for rep in 1 2; do
  for mb in ${MBS:-16384 768 1536 16128 3072}; do
    timeout -k 10 300 env KAFKA_MAX_BLOCKS=$mb python -u bench.py --config tip7 --steps 8 --warmup 2 > $O/mb_${mb}_$rep.log 2>&1 || { tail -20 $O/mb_${mb}_$rep.log; exit 1; }
    echo "mb=$mb rep=$rep $(grep -o '"ms_per_step": [0-9.]*' $O/mb_${mb}_$rep.log)"
  done
done
