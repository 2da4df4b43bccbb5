#!/bin/bash
# Observed-first pixel order (obs_order, EngineConfig.observed_first): GPU
# tests (bit-identity with the natural order, device order = host order),
# then A/B per config, 2 interleaved reps.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r4v24
O=gpurun_out/r4v24
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for rep in 1 2; do
  for on in 1 0; do
    for c in tip7 spatial prosail10; do
      timeout -k 10 400 python -u bench.py --config $c --steps 6 --warmup 2 --set observed_first=$on > $O/${c}_${on}_$rep.log 2>&1 || { tail -20 $O/${c}_${on}_$rep.log; exit 1; }
      echo "$c observed_first=$on rep=$rep $(grep -o '"ms_per_step": [0-9.]*' $O/${c}_${on}_$rep.log)"
    done
  done
done
timeout -k 10 400 python -u bench.py --config multisensor --steps 3 --warmup 1 > $O/ms_1.log 2>&1 && echo "multisensor on $(grep -o '"ms_per_step": [0-9.]*' $O/ms_1.log)"
timeout -k 10 400 python -u bench.py --config multisensor --steps 3 --warmup 1 --set observed_first=0 > $O/ms_0.log 2>&1 && echo "multisensor off $(grep -o '"ms_per_step": [0-9.]*' $O/ms_0.log)"
echo all-done
