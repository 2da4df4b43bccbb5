#!/bin/bash
# every BASELINE.json config on one GPU; JSON lines -> gpurun_out/bench_configs.jsonl
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
: > gpurun_out/bench_configs.jsonl
run() { local name=$1; local t=$2; shift 2
  timeout -k 10 $t python bench.py --config $name --watchdog 120 "$@" > gpurun_out/cfg_$name.out 2> gpurun_out/cfg_$name.err
  local rc=$?; tail -1 gpurun_out/cfg_$name.out >> gpurun_out/bench_configs.jsonl; echo "$name rc=$rc $(tail -1 gpurun_out/cfg_$name.out | grep -o '"ms_per_step": [0-9.]*')"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/cfg_$name.err; exit $rc; fi; }
run tip7 400 --steps 10 --warmup 2
run identity7 300 --steps 20 --warmup 3
run prosail10 600 --steps 4 --warmup 2
run spatial 600 --steps 30 --warmup 2
run multisensor 900 --steps 3 --warmup 2
