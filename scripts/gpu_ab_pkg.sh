set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu_step.sh tests_nox || exit $?
run() { timeout -k 10 300 python -u $1 --config $2 > gpurun_out/ab_$3_$2.log 2>&1 || { tail -5 gpurun_out/ab_$3_$2.log; exit 1; }; tail -1 gpurun_out/ab_$3_$2.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$3', d['config']['name'], d['ms_per_step'])"; }
run ab_old/bench.py tip7 old && run bench.py tip7 new && run ab_old/bench.py prosail10 old && run bench.py prosail10 new && run ab_old/bench.py tip7 old2 && run bench.py tip7 new2
