#!/bin/bash
# Round 4 first check: GPU tests, smoke, tip7 bench, spatial bench (device
# schedule + tiled passes), the deep-halo strip kernel timing, HBM PMC.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r4
O=gpurun_out/r4
stop() { echo "!! $1 rc=$2"; exit $2; }
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; stop tests $?; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -u __graft_entry__.py smoke > $O/smoke.log 2>&1 || stop smoke $?
tail -1 $O/smoke.log
timeout -k 10 300 python -u scripts/bench_reg_deep.py > $O/reg_deep.jsonl 2>&1 || { tail -5 $O/reg_deep.jsonl; stop reg_deep $?; }
cat $O/reg_deep.jsonl
for c in tip7 spatial; do
  timeout -k 10 400 python -u bench.py --config $c --steps 10 --warmup 2 > $O/bench_$c.log 2>&1 || { tail -5 $O/bench_$c.log; stop bench_$c $?; }
  tail -1 $O/bench_$c.log
done
bash scripts/gpu_pmc_hbm.sh || stop pmc $?
