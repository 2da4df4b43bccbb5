#!/bin/bash
# Round 4, iteration 5: GPU tests, then A/B of the JRC-TIP kernels specialised
# for the fused forecast (default) vs the generic kernel (variant 18), tip7 /
# spatial at 10980^2 interleaved, tip7 at T = 32, PMC VALU counts at 4096^2.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r4v5
O=gpurun_out/r4v5
stop() { echo "!! $1 rc=$2"; exit ${2:-1}; }
run() { local n=$1 log=$2 to=$3; shift 3; timeout -k 10 $to "$@" > $log 2>&1; local rc=$?; \
        if [ $rc -ne 0 ]; then tail -40 $log; stop $n $rc; fi; }
run tests $O/gpu_tests.log 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
tail -1 $O/gpu_tests.log
for rep in 1 2; do
  for v in 0 18; do
    for c in tip7 spatial; do
      run ab_${c}_v${v}_$rep $O/ab_${c}_v${v}_$rep.log 400 env KAFKA_ANALYSIS_VARIANT=$v python -u bench.py --config $c --steps 6 --warmup 2
      echo "ab $c v=$v rep=$rep $(tail -1 $O/ab_${c}_v${v}_$rep.log | cut -c1-150)"
    done
  done
done
for v in 0 18; do
  run t32_v$v $O/t32_v$v.log 400 env KAFKA_ANALYSIS_VARIANT=$v python -u bench.py --config tip7 --steps 6 --warmup 2 --n-train 32
  echo "T32 v=$v $(tail -1 $O/t32_v$v.log | cut -c1-150)"
done
cd /tmp && export TMPDIR=/tmp
for v in 0 18; do
  for T in 32 500; do
    KAFKA_ANALYSIS_VARIANT=$v timeout -k 10 -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU_TRANS_F32 \
        --kernel-include-regex analysis_mfma -d "$R/$O/pmc_v${v}_T$T" -o run --output-format csv -- \
        python "$R/bench.py" --config tip7 --size 4096 --steps 2 --warmup 1 --n-train $T > "$R/$O/pmc_v${v}_T$T.log" 2>&1 \
      || { echo "!! pmc $v $T"; tail -5 "$R/$O/pmc_v${v}_T$T.log"; exit 1; }
    echo "pmc v=$v T=$T done"
  done
done
echo all-done
