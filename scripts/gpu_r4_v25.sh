#!/bin/bash
# Band-group observation classes: GPU tests, multisensor A/B, tip7/prosail10 sanity.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r4v25
O=gpurun_out/r4v25
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for rep in 1 2; do
  for on in 1 0; do
    timeout -k 10 500 python -u bench.py --config multisensor --steps 3 --warmup 1 --set observed_first=$on > $O/ms_${on}_$rep.log 2>&1 || { tail -20 $O/ms_${on}_$rep.log; exit 1; }
    echo "multisensor observed_first=$on rep=$rep $(grep -o '"ms_per_step": [0-9.]*' $O/ms_${on}_$rep.log)"
  done
done
for c in tip7 prosail10; do
  timeout -k 10 400 python -u bench.py --config $c --steps 6 --warmup 2 > $O/$c.log 2>&1 || { tail -20 $O/$c.log; exit 1; }
  echo "$c $(grep -o '"ms_per_step": [0-9.]*' $O/$c.log)"
done
echo all-done
