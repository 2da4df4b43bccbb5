#!/bin/bash
# identity7 step-time outliers: default bench twice, no telemetry, 50 steps.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r4v12
O=gpurun_out/r4v12
stop() { echo "!! $1 rc=$2"; exit ${2:-1}; }
run() { local n=$1 log=$2 to=$3; shift 3; timeout -k 10 $to "$@" > $log 2>&1; local rc=$?; \
        if [ $rc -ne 0 ]; then tail -40 $log; stop $n $rc; fi; }
for i in 1 2; do
  run id_$i $O/id_$i.log 200 python -u bench.py --config identity7
  echo "id rep=$i $(tail -1 $O/id_$i.log | cut -c180-300)"; grep "step" $O/id_$i.log | tr '\n' ' ' | cut -c1-600; echo
done
run id_notel $O/id_notel.log 200 python -u bench.py --config identity7 --no-telemetry
echo "id notel $(tail -1 $O/id_notel.log | cut -c180-300)"; grep "step" $O/id_notel.log | tr '\n' ' ' | cut -c1-600; echo
run id_50 $O/id_50.log 200 python -u bench.py --config identity7 --steps 50 --warmup 5
echo "id 50 $(tail -1 $O/id_50.log | cut -c180-300)"
grep "step" $O/id_50.log | awk '{print $4}' | sort -n | tail -5 | tr '\n' ' '; echo
run id_res $O/id_res.log 200 python -u bench.py --config identity7 --resident --steps 50 --warmup 5
echo "id resident $(tail -1 $O/id_res.log | cut -c180-300)"
echo all-done
