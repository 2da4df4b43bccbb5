#!/bin/bash
# Grid cap 65536 (new default) vs 16384 (round-3/4 default) across configs, and the GPU tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r4v23
O=gpurun_out/r4v23
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for rep in 1 2; do
  for mb in 65536 16384; do
    for c in tip7 spatial prosail10; do
      timeout -k 10 400 env KAFKA_MAX_BLOCKS=$mb python -u bench.py --config $c --steps 6 --warmup 2 > $O/${c}_${mb}_$rep.log 2>&1 || { tail -20 $O/${c}_${mb}_$rep.log; exit 1; }
      echo "$c mb=$mb rep=$rep $(grep -o '"ms_per_step": [0-9.]*' $O/${c}_${mb}_$rep.log)"
    done
  done
done
