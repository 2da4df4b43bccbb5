#!/bin/bash
# Round 4, iteration 27: why the observed-first order costs at T = 32: kernel
# traces of tip7 T = 32 (10980^2) with the order off, on, and an identity order
# (the gather alone, KAFKA_ORDER_DEBUG=identity).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r4v27
O=gpurun_out/r4v27
cd /tmp && export TMPDIR=/tmp
for m in off on identity; do
  of=true; [ $m = off ] && of=false
  dbg=none; [ $m = identity ] && dbg=identity
  KAFKA_ORDER_DEBUG=$dbg timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/tr_$m" -o run --output-format csv -- \
      python "$R/bench.py" --config tip7 --steps 6 --warmup 2 --n-train 32 --set observed_first=$of > "$R/$O/tr_$m.log" 2>&1 \
    || { echo "!! trace $m"; tail -5 "$R/$O/tr_$m.log"; exit 1; }
  echo "$m $(tail -1 $R/$O/tr_$m.log | cut -c1-160)"
done
echo all-done
