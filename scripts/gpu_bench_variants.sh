set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for v in 4 0 5 4 0; do
  KAFKA_ANALYSIS_VARIANT=$v timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 > gpurun_out/bench_v$v.log 2>&1 || exit $?
  echo "v$v $(tail -1 gpurun_out/bench_v$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
done
