#!/bin/bash
# bench.py once per analysis-kernel variant (KAFKA_ANALYSIS_VARIANT), interleaved:
#   bash scripts/gpu_bench_variants.sh "4 0 8" [bench args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" && mkdir -p gpurun_out
vars=${1:-"4 0"}; shift
for v in $vars; do
  KAFKA_ANALYSIS_VARIANT=$v timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 "$@" > gpurun_out/bench_v$v.log 2>&1 || exit $?
  echo "v$v $(tail -1 gpurun_out/bench_v$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
done
