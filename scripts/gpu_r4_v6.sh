#!/bin/bash
# Round 4, iteration 6: GPU tests (incl. the forced one-rank RCCL bench test),
# the matrix-core precision prints, PROSAIL register prefetch A/B (variant 7 vs
# the same order without prefetch, variant 16).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r4v6
O=gpurun_out/r4v6
stop() { echo "!! $1 rc=$2"; exit ${2:-1}; }
run() { local n=$1 log=$2 to=$3; shift 3; timeout -k 10 $to "$@" > $log 2>&1; local rc=$?; \
        if [ $rc -ne 0 ]; then tail -40 $log; stop $n $rc; fi; }
run tests $O/gpu_tests.log 700 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread
tail -1 $O/gpu_tests.log
run prec $O/mfma_prec.log 300 python -u -m pytest tests/test_gpu_mfma.py -x -s -q --timeout 150 --timeout-method thread -k "analysis_vs_oracle or value_vs_float64 or cancelling"
grep -E "err|passed" $O/mfma_prec.log | head -20
for rep in 1 2; do
  for v in 16 7; do
    run pf_v${v}_$rep $O/pf_v${v}_$rep.log 400 env KAFKA_ANALYSIS_VARIANT=$v python -u bench.py --config prosail10 --steps 4 --warmup 1
    echo "prosail10 v=$v rep=$rep $(tail -1 $O/pf_v${v}_$rep.log | cut -c1-150)"
  done
done
echo all-done
