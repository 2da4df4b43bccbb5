#!/bin/bash
# Round 4, iteration 18: H2D copies issued from the HostRing submitter thread
# (h2d_async): the copy-stall probe, GPU tests, identity7 x4, tip7.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r4v18
O=gpurun_out/r4v18
stop() { echo "!! $1 rc=$2"; exit ${2:-1}; }
run() { local n=$1 log=$2 to=$3; shift 3; timeout -k 10 $to "$@" > $log 2>&1; local rc=$?; \
        if [ $rc -ne 0 ]; then tail -40 $log; stop $n $rc; fi; }
run probe $O/probe.txt 120 python -u scripts/probes/copy_stall_probe.py
cut -c1-300 $O/probe.txt
run tests $O/gpu_tests.log 700 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread
tail -1 $O/gpu_tests.log
for i in 1 2 3 4; do
  run id_$i $O/id_$i.log 200 python -u bench.py --config identity7
  echo "id rep $i $(grep -o '"ms_per_step": [0-9.]*' $O/id_$i.log) $(grep 'step [0-9]' $O/id_$i.log | awk '{print $4}' | tr '\n' ' ')"
done
run tip7 $O/tip7.log 300 python -u bench.py
echo "tip7 $(grep -o '"ms_per_step": [0-9.]*' $O/tip7.log)"
run sp $O/sp.log 300 python -u bench.py --config spatial
echo "spatial $(grep -o '"ms_per_step": [0-9.]*' $O/sp.log)"
echo all-done
