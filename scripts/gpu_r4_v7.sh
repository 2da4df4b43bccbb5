#!/bin/bash
# Round 4, iteration 7: per-rank share of the strong-scaling run on one GPU
# (tile edges with the pixel count of a 1/2, 1/4, 1/8 strip of 10980^2) for
# tip7 and spatial, plus a kernel trace of the 1/8 share (fixed per-step costs).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r4v7
O=gpurun_out/r4v7
stop() { echo "!! $1 rc=$2"; exit ${2:-1}; }
run() { local n=$1 log=$2 to=$3; shift 3; timeout -k 10 $to "$@" > $log 2>&1; local rc=$?; \
        if [ $rc -ne 0 ]; then tail -40 $log; stop $n $rc; fi; }
for c in tip7 spatial; do
  for s in 10980 7764 5490 3882; do
    run share_${c}_$s $O/share_${c}_$s.log 400 python -u bench.py --config $c --size $s --steps 10 --warmup 2
    echo "$c size=$s $(tail -1 $O/share_${c}_$s.log | cut -c1-200)"
  done
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/trace_tip7_3882" -o run \
    --output-format csv -- python "$R/bench.py" --config tip7 --size 3882 --steps 6 --warmup 2 > "$R/$O/trace_tip7_3882.log" 2>&1) \
  || { tail -5 $O/trace_tip7_3882.log; stop trace 1; }
echo all-done
