#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
stop() { echo "!! $1 rc=$2"; exit $2; }
run() { local tag=$1; shift; timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 "$@" > gpurun_out/sc_$tag.log 2>&1 || stop $tag $?; echo "$tag $(tail -1 gpurun_out/sc_$tag.log | grep -o '"ms_per_step": [0-9.]*')"; }
run ms_fused --size 4096 --config multisensor --set gp_split=never
run p10_full --config prosail10
run p10_full_fused --config prosail10 --set gp_split=never
run ms_full_c34 --config multisensor --set band_chunk=34
