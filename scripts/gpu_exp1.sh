set -o pipefail
mkdir -p gpurun_out
for T in 32 128 500; do timeout -k 10 120 python -u scripts/bench_kernels.py --size 4096 --n-train $T --variants 0,4 --rounds 5 >> gpurun_out/exp1_T.jsonl 2>gpurun_out/exp1_err.log || exit 1; done
timeout -k 10 200 python -u bench.py --config identity7 --steps 50 --warmup 5 > gpurun_out/exp1_id7.json 2>gpurun_out/exp1_id7.err || exit 1
timeout -k 10 200 python -u bench.py --config identity7 --steps 200 --warmup 20 > gpurun_out/exp1_id7_200.json 2>>gpurun_out/exp1_id7.err || exit 1
cat gpurun_out/exp1_T.jsonl; cut -c1-400 gpurun_out/exp1_id7.json gpurun_out/exp1_id7_200.json
