#!/bin/bash
# Round 4, iteration 10: GPU tests, PROSAIL SPEC_PROP kernel vs generic
# (variant 18) A/B, telemetry-trimmed tip7 at the 1/8 share.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r4v10
O=gpurun_out/r4v10
stop() { echo "!! $1 rc=$2"; exit ${2:-1}; }
run() { local n=$1 log=$2 to=$3; shift 3; timeout -k 10 $to "$@" > $log 2>&1; local rc=$?; \
        if [ $rc -ne 0 ]; then tail -40 $log; stop $n $rc; fi; }
run tests $O/gpu_tests.log 700 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread
tail -1 $O/gpu_tests.log
for rep in 1 2; do
  for v in 0 18; do
    run ps_v${v}_$rep $O/ps_v${v}_$rep.log 400 env KAFKA_ANALYSIS_VARIANT=$v python -u bench.py --config prosail10 --steps 4 --warmup 1
    echo "prosail10 v=$v rep=$rep $(tail -1 $O/ps_v${v}_$rep.log | cut -c1-150)"
  done
done
run ms $O/ms.log 400 python -u bench.py --config multisensor --steps 3 --warmup 1
echo "multisensor $(tail -1 $O/ms.log | cut -c1-150)"
for tel in on off; do
  X=""; [ $tel = off ] && X="--no-telemetry"
  run t_$tel $O/t_$tel.log 300 python -u bench.py --config tip7 --size 3882 --steps 30 --warmup 3 $X
  echo "3882 tel=$tel $(tail -1 $O/t_$tel.log | cut -c1-150)"
done
echo all-done
