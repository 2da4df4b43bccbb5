#!/bin/bash
# Round 4, iteration 9: per-step host overhead at the 1/8 strong-scaling share
# (3882^2 ~ a 1373-row strip of 10980^2): telemetry (phase hipEvents) on vs off.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r4v9
O=gpurun_out/r4v9
stop() { echo "!! $1 rc=$2"; exit ${2:-1}; }
run() { local n=$1 log=$2 to=$3; shift 3; timeout -k 10 $to "$@" > $log 2>&1; local rc=$?; \
        if [ $rc -ne 0 ]; then tail -40 $log; stop $n $rc; fi; }
for rep in 1 2; do
  for tel in on off; do
    X=""; [ $tel = off ] && X="--no-telemetry"
    run t_${tel}_$rep $O/t_${tel}_$rep.log 300 python -u bench.py --config tip7 --size 3882 --steps 30 --warmup 3 $X
    echo "tel=$tel rep=$rep $(tail -1 $O/t_${tel}_$rep.log | cut -c1-200)"
  done
done
echo all-done
