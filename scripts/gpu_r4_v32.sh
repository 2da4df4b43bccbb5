#!/bin/bash
# Round 4, iteration 32: kernel-trace summaries of the final tree's spatial and
# prosail10 steps (profiles/).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r4v32
O=gpurun_out/r4v32
cd /tmp && export TMPDIR=/tmp
for c in spatial prosail10; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/tr_$c" -o run --output-format csv -- \
      python "$R/bench.py" --config $c --steps 5 --warmup 2 > "$R/$O/tr_$c.log" 2>&1 \
    || { echo "!! trace $c"; tail -5 "$R/$O/tr_$c.log"; exit 1; }
  echo "$c $(grep -o '"ms_per_step": [0-9.]*' $R/$O/tr_$c.log)"
done
echo all-done
