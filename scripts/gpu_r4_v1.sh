#!/bin/bash
# Round 4 check: GPU tests (the MVP precision test last, separately), smoke,
# deep-halo strip timing, tip7 / spatial benches, HBM PMC, MVP precision study.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r4
O=gpurun_out/r4
stop() { echo "!! $1 rc=$2"; exit ${2:-1}; }
# run STEP LOG TIMEOUT CMD...: one GPU step with its own time limit; stop on failure
run() { local n=$1 log=$2 to=$3; shift 3; timeout -k 10 $to "$@" > $log 2>&1; local rc=$?; \
        if [ $rc -ne 0 ]; then tail -30 $log; stop $n $rc; fi; }
run tests $O/gpu_tests.log 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    --deselect tests/test_mvp.py::test_mvp_slice_on_device
tail -2 $O/gpu_tests.log
run smoke $O/smoke.log 300 python -u __graft_entry__.py smoke
tail -1 $O/smoke.log
run reg_deep $O/reg_deep.jsonl 300 python -u scripts/bench_reg_deep.py
cat $O/reg_deep.jsonl
for c in tip7 spatial; do
  run bench_$c $O/bench_$c.log 400 python -u bench.py --config $c --steps 10 --warmup 2
  tail -1 $O/bench_$c.log | cut -c1-400
done
bash scripts/gpu_pmc_hbm.sh || stop pmc $?
run mvp $O/mvp_precision.jsonl 500 python -u scripts/mvp_precision.py --size 256 --variants 0,4
cut -c1-200 $O/mvp_precision.jsonl
