#!/bin/bash
# Round 4, iteration 3: GPU tests (incl. the MVP pin with the interleaved GP
# table order), MVP precision per variant, tip7 / spatial benches (spatial with
# the fused plain first iteration), spatial kernel trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r4v3
O=gpurun_out/r4v3
stop() { echo "!! $1 rc=$2"; exit ${2:-1}; }
run() { local n=$1 log=$2 to=$3; shift 3; timeout -k 10 $to "$@" > $log 2>&1; local rc=$?; \
        if [ $rc -ne 0 ]; then tail -40 $log; stop $n $rc; fi; }
run tests $O/gpu_tests.log 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
tail -3 $O/gpu_tests.log; grep "^MVP" $O/gpu_tests.log | cut -c1-200
run mvp $O/mvp_precision.jsonl 400 python -u scripts/mvp_precision.py --size 256 --variants 0,4
cut -c1-220 $O/mvp_precision.jsonl
for c in tip7 spatial; do
  run bench_$c $O/bench_$c.log 400 python -u bench.py --config $c --steps 10 --warmup 2
  echo "$c $(tail -1 $O/bench_$c.log | cut -c1-200)"
done
run bench_spatial_coupled $O/bench_spatial_coupled.log 400 python -u bench.py --config spatial --steps 10 --warmup 2 --set spatial_first_plain=0
echo "spatial coupled-first $(tail -1 $O/bench_spatial_coupled.log | cut -c1-200)"
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/trace_spatial" -o run \
    --output-format csv -- python "$R/bench.py" --config spatial --steps 3 --warmup 1 > "$R/$O/trace_spatial.log" 2>&1) \
  || { tail -5 $O/trace_spatial.log; stop trace_spatial 1; }
echo all-done
