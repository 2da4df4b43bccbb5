#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r4v19
O=gpurun_out/r4v19
for i in 1 2 3 4; do
  timeout -k 10 200 python -u bench.py --config identity7 > $O/id_$i.log 2>&1 || { tail -20 $O/id_$i.log; exit 1; }
  echo "id rep $i $(grep -o '"ms_per_step": [0-9.]*' $O/id_$i.log) $(grep 'step [0-9]' $O/id_$i.log | awk '{print $4}' | tr '\n' ' ')"
done
timeout -k 10 200 python -u -m pytest tests/test_gpu.py -x -q -k "stream" --timeout 120 --timeout-method thread 2>&1 | tail -2
