#!/bin/bash
# Granule-scale file ingest on one MI355X: synthesize a 10980^2 Sentinel-2 archive
# (tiled-DEFLATE uint16 GeoTIFFs, written by the native writer) on local disk, then
# run the file-driven PROSAIL assimilation with per-phase timing.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" && mkdir -p gpurun_out
SZ=${SZ:-10980}; D=${D:-3}; OUT=${OUT:-/tmp/kafka_s2_archive}
# RUNARGS: extra run flags, e.g. "--out /tmp/kafka_out --out-level 1" or
# "--checkpoint-dir /tmp/kafka_ckpt --checkpoint-every 1 --checkpoint-keep 1";
# RUNS="flags A;flags B": several runs on one synthesised archive
RUNARGS=${RUNARGS:-}
df -h /tmp | tail -1; free -g | head -2
rm -rf "$OUT"
T0=$SECONDS
timeout -k 10 400 python -u -m kafka_inferenceengine_amd synth-s2 --out "$OUT" --size $SZ $SZ --dates $D \
  > gpurun_out/s2_synth.log 2> gpurun_out/s2_synth.err || { tail -20 gpurun_out/s2_synth.err; exit 1; }
tail -1 gpurun_out/s2_synth.log; echo "synth wall $((SECONDS - T0)) s"
du -sh "$OUT"
# one run per RUNARGS entry (RUNS="args1;args2;..." overrides RUNARGS): output off / on, checkpoints
IFS=';' read -ra runs <<< "${RUNS:-$RUNARGS}"
[ ${#runs[@]} -eq 0 ] && runs=("")
i=0
for ra in "${runs[@]}"; do
  T0=$SECONDS
  timeout -k 10 500 python -u -m kafka_inferenceengine_amd run --sensor s2 --s2-folder "$OUT/data" \
    --emulator-folder "$OUT/emus" --size $SZ $SZ --steps $D --phase-timing $ra > gpurun_out/s2_run$i.log \
    2> gpurun_out/s2_run$i.err || { tail -20 gpurun_out/s2_run$i.err; exit 1; }
  echo "run$i [$ra]: $(tail -1 gpurun_out/s2_run$i.log | cut -c1-400)"; echo "run$i wall $((SECONDS - T0)) s"
  du -sh /tmp/kafka_out /tmp/kafka_ckpt 2>/dev/null
  rm -rf /tmp/kafka_out /tmp/kafka_ckpt
  i=$((i + 1))
done
rm -rf "$OUT"
