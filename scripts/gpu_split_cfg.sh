#!/bin/bash
# EngineConfig A/B for the split-path configs (bench --set)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
stop() { echo "!! $1 rc=$2"; exit $2; }
run() { local tag=$1; shift; timeout -k 10 300 python -u bench.py --size 4096 --steps 3 --warmup 1 "$@" > gpurun_out/sc_$tag.log 2>&1 || stop $tag $?; echo "$tag $(tail -1 gpurun_out/sc_$tag.log | grep -o '"ms_per_step": [0-9.]*')"; }
run p10 --config prosail10
run p10_fused --config prosail10 --set gp_split=never
run ms --config multisensor
run ms_c17 --config multisensor --set band_chunk=17
run ms_c34 --config multisensor --set band_chunk=34
