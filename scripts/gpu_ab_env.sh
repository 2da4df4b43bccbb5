#!/bin/bash
# Interleaved bench.py A/B of environment settings on one box:
#   AB="KAFKA_ANALYSIS_VARIANT=0|KAFKA_ANALYSIS_VARIANT=10" ROUNDS=2 BENCH_ARGS="--steps 8" bash scripts/gpu_ab_env.sh
# (optional TESTS=<pytest -k filter> runs those GPU tests first).  One JSON line
# per run in gpurun_out/ab_env.jsonl, tagged with its setting.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$TESTS" \
      > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; echo "!! tests rc=$?"; exit 1; }
  tail -1 gpurun_out/ab_tests.log
fi
IFS='|' read -ra SETS <<< "${AB:?set AB}"
OUT=${OUT:-gpurun_out/ab_env.jsonl}; : > $OUT
for r in $(seq 1 "${ROUNDS:-2}"); do
  for s in "${SETS[@]}"; do
    timeout -k 10 300 env $s python -u bench.py ${BENCH_ARGS} > gpurun_out/ab_run.log 2>&1 \
      || { tail -5 gpurun_out/ab_run.log; echo "!! bench ($s) rc=$?"; exit 1; }
    line=$(tail -1 gpurun_out/ab_run.log)
    echo "{\"setting\": \"$s\", \"round\": $r, \"result\": $line}" >> $OUT
    echo "$s r$r: $(echo "$line" | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
  done
done
