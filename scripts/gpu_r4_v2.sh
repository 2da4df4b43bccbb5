#!/bin/bash
# Round 4 measurements: (1) issue-overlap probe (VERDICT r3 #4a), (2) fixed
# vs per-point cost of the multi-band PROSAIL kernels (T = 32 vs 250 at
# 4096^2) and the phase clocks of multisensor (is the normal-
# equation share worth the matrix cores), (3) tip7 at T = 32 / 500 on the
# full tile (the non-GP floor, VERDICT r3 #4b).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r4v2
O=gpurun_out/r4v2
stop() { echo "!! $1 rc=$2"; exit ${2:-1}; }
run() { local n=$1 log=$2 to=$3; shift 3; timeout -k 10 $to "$@" > $log 2>&1; local rc=$?; \
        if [ $rc -ne 0 ]; then tail -30 $log; stop $n $rc; fi; }
# kernel trace of the spatial step (where its 1.34x over tip7 goes)
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/trace_spatial" -o run \
    --output-format csv -- python "$R/bench.py" --config spatial --steps 3 --warmup 1 > "$R/$O/trace_spatial.log" 2>&1) \
  || { tail -5 $O/trace_spatial.log; stop trace_spatial 1; }
echo trace-spatial-done
if [ -z "$SKIP_PROBE" ]; then
  (cd scripts/probes && hipcc --offload-arch=gfx950 -O3 -Wno-unused-value -o issue_overlap_probe issue_overlap_probe.hip) || stop build_probe 1
  run probe $O/issue_overlap_probe.jsonl 300 ./scripts/probes/issue_overlap_probe
  cat $O/issue_overlap_probe.jsonl
fi
for c in ${FIXED_CONFIGS:-multisensor prosail10}; do
  for T in 32 250; do
    run fixed_${c}_$T $O/fixed_${c}_T$T.log 400 python -u bench.py --config $c --size 4096 --steps 3 --warmup 1 --n-train $T
    echo "$c T=$T $(tail -1 $O/fixed_${c}_T$T.log | cut -c1-140)"
  done
done
run phase_multisensor $O/phase_multisensor.log 400 env KAFKA_PROF=1 python -u bench.py --config multisensor --size 4096 --steps 3 --warmup 1
grep phase_clocks $O/phase_multisensor.log
# A/B (interleaved, same box): variant 16 = both column blocks' exponent MFMAs first
for rep in 1 2; do
  for v in 0 16; do
    for c in ${AB_CONFIGS:-tip7 prosail10}; do
      run ab_${c}_v${v}_$rep $O/ab_${c}_v${v}_$rep.log 400 env KAFKA_ANALYSIS_VARIANT=$v python -u bench.py --config $c --steps 6 --warmup 2
      echo "ab $c v=$v rep=$rep $(tail -1 $O/ab_${c}_v${v}_$rep.log | cut -c1-120)"
    done
  done
done
for T in 32 500; do
  run tip7_T$T $O/tip7_T$T.log 400 python -u bench.py --config tip7 --steps 6 --warmup 2 --n-train $T
  echo "tip7 T=$T $(tail -1 $O/tip7_T$T.log | cut -c1-140)"
done
