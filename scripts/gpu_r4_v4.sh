#!/bin/bash
# Round 4, iteration 4: A/B of compile-time specialised fused-analysis kernels
# (experiment modules _kafka_hip_pr: forecast-fused, no regulariser code;
# _kafka_hip_hot: hot path only) against the release module, tip7 at 10980^2
# (interleaved, 2 reps) and T = 32; PMC VALU counts at 4096^2.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r4v4
O=gpurun_out/r4v4
stop() { echo "!! $1 rc=$2"; exit ${2:-1}; }
run() { local n=$1 log=$2 to=$3; shift 3; timeout -k 10 $to "$@" > $log 2>&1; local rc=$?; \
        if [ $rc -ne 0 ]; then tail -40 $log; stop $n $rc; fi; }
for rep in 1 2; do
  for m in rel pr hot; do
    E=""; [ $m != rel ] && E=$m
    run ab_${m}_$rep $O/ab_${m}_$rep.log 400 env KAFKA_EXT=$E python -u bench.py --config tip7 --steps 6 --warmup 2
    echo "ab $m rep=$rep $(tail -1 $O/ab_${m}_$rep.log | cut -c1-150)"
  done
done
for m in rel pr hot; do
  E=""; [ $m != rel ] && E=$m
  run t32_$m $O/t32_$m.log 400 env KAFKA_EXT=$E python -u bench.py --config tip7 --steps 6 --warmup 2 --n-train 32
  echo "T32 $m $(tail -1 $O/t32_$m.log | cut -c1-150)"
done
cd /tmp && export TMPDIR=/tmp
for m in rel pr; do
  E=""; [ $m != rel ] && E=$m
  for T in 32 500; do
    KAFKA_EXT=$E timeout -k 10 -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU_TRANS_F32 \
        --kernel-include-regex analysis_mfma -d "$R/$O/pmc_${m}_T$T" -o run --output-format csv -- \
        python "$R/bench.py" --config tip7 --size 4096 --steps 2 --warmup 1 --n-train $T > "$R/$O/pmc_${m}_T$T.log" 2>&1 \
      || { echo "!! pmc $m $T"; tail -5 "$R/$O/pmc_${m}_T$T.log"; exit 1; }
    echo "pmc $m T=$T done"
  done
done
echo all-done
