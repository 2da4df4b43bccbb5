#!/bin/bash
# Round 4, iteration 26: tip7 at T = 32 (VERDICT r3 #4 target) with and without
# the observed-first order, 10980^2; PMC VALU/MFMA/trans counts per wave at 4096^2,
# T = 500 and 32, observed-first on / off.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r4v26
O=gpurun_out/r4v26
stop() { echo "!! $1 rc=$2"; exit ${2:-1}; }
run() { local n=$1 log=$2 to=$3; shift 3; timeout -k 10 $to "$@" > $log 2>&1; local rc=$?; \
        if [ $rc -ne 0 ]; then tail -40 $log; stop $n $rc; fi; }
for rep in 1 2; do
  for of in true false; do
    run t32_${of}_$rep $O/t32_${of}_$rep.log 300 python -u bench.py --config tip7 --steps 10 --warmup 3 --n-train 32 --set observed_first=$of
    echo "T32 observed_first=$of rep=$rep $(tail -1 $O/t32_${of}_$rep.log | cut -c1-150)"
  done
done
cd /tmp && export TMPDIR=/tmp
for of in true false; do
  for T in 32 500; do
    timeout -k 10 -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_MFMA \
        --kernel-include-regex analysis_mfma -d "$R/$O/pmc_of${of}_T$T" -o run --output-format csv -- \
        python "$R/bench.py" --config tip7 --size 4096 --steps 2 --warmup 1 --n-train $T --set observed_first=$of > "$R/$O/pmc_of${of}_T$T.log" 2>&1 \
      || { echo "!! pmc $of $T"; tail -5 "$R/$O/pmc_of${of}_T$T.log"; exit 1; }
    echo "pmc of=$of T=$T done"
  done
done
echo all-done
