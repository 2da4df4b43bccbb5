#!/bin/bash
# Granule-scale file ingest on one MI355X: synthesize a 10980^2 Sentinel-2 archive
# (tiled-DEFLATE uint16 GeoTIFFs, written by the native writer) on local disk, then
# run the file-driven PROSAIL assimilation with per-phase timing.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" && mkdir -p gpurun_out
SZ=${SZ:-10980}; D=${D:-3}; OUT=${OUT:-/tmp/kafka_s2_archive}
# RUNARGS: extra run flags, e.g. "--out /tmp/kafka_out --out-level 1" or
# "--checkpoint-dir /tmp/kafka_ckpt --checkpoint-every 1 --checkpoint-keep 1"
RUNARGS=${RUNARGS:-}
df -h /tmp | tail -1; free -g | head -2
rm -rf "$OUT"
T0=$SECONDS
timeout -k 10 400 python -u -m kafka_inferenceengine_amd synth-s2 --out "$OUT" --size $SZ $SZ --dates $D \
  > gpurun_out/s2_synth.log 2> gpurun_out/s2_synth.err || { tail -20 gpurun_out/s2_synth.err; exit 1; }
tail -1 gpurun_out/s2_synth.log; echo "synth wall $((SECONDS - T0)) s"
du -sh "$OUT"
T0=$SECONDS
timeout -k 10 400 python -u -m kafka_inferenceengine_amd run --sensor s2 --s2-folder "$OUT/data" \
  --emulator-folder "$OUT/emus" --size $SZ $SZ --steps $D --phase-timing $RUNARGS > gpurun_out/s2_run.log 2> gpurun_out/s2_run.err \
  || { tail -20 gpurun_out/s2_run.err; exit 1; }
tail -1 gpurun_out/s2_run.log; echo "run wall $((SECONDS - T0)) s"
du -sh /tmp/kafka_out /tmp/kafka_ckpt 2>/dev/null
rm -rf "$OUT" /tmp/kafka_out /tmp/kafka_ckpt
