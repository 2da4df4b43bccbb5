#!/bin/bash
# Round 4, iteration 11: LDS transpose of the GP sums in the global-table
# kernel vs the round-4 HEAD build (experiment module _kafka_hip_old):
# bit-identity of the final state, prosail10 / multisensor A/B, GPU tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r4v11
O=gpurun_out/r4v11
stop() { echo "!! $1 rc=$2"; exit ${2:-1}; }
run() { local n=$1 log=$2 to=$3; shift 3; timeout -k 10 $to "$@" > $log 2>&1; local rc=$?; \
        if [ $rc -ne 0 ]; then tail -40 $log; stop $n $rc; fi; }
run tests $O/gpu_tests.log 700 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread
tail -1 $O/gpu_tests.log
for m in new old; do
  E=""; [ $m = old ] && E=old
  for c in prosail10 multisensor; do
    run id_${c}_$m $O/id_${c}_$m.log 300 env KAFKA_EXT=$E python -u bench.py --config $c --size 512 --steps 2 --warmup 1 --dump-state $O/state_${c}_$m
  done
done
python - <<PY
import numpy as np
for c in ("prosail10", "multisensor"):
    a = np.load("$O/state_" + c + "_new.strip0.npy"); b = np.load("$O/state_" + c + "_old.strip0.npy")
    print(c, "bit-identical" if np.array_equal(a, b) else "DIFFERENT max %g" % np.abs(a - b).max())
PY
for rep in 1 2; do
  for m in new old; do
    E=""; [ $m = old ] && E=old
    run ab_ps_${m}_$rep $O/ab_ps_${m}_$rep.log 400 env KAFKA_EXT=$E python -u bench.py --config prosail10 --steps 4 --warmup 1
    echo "prosail10 $m rep=$rep $(tail -1 $O/ab_ps_${m}_$rep.log | cut -c1-150)"
  done
done
for m in new old; do
  E=""; [ $m = old ] && E=old
  run ab_ms_$m $O/ab_ms_$m.log 400 env KAFKA_EXT=$E python -u bench.py --config multisensor --steps 3 --warmup 1
  echo "multisensor $m $(tail -1 $O/ab_ms_$m.log | cut -c1-150)"
done
echo all-done
