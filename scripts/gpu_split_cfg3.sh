#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
stop() { echo "!! $1 rc=$2"; exit $2; }
run() { local tag=$1; shift; timeout -k 10 500 python -u bench.py --steps 3 --warmup 1 "$@" > gpurun_out/sc_$tag.log 2>&1 || stop $tag $?; echo "$tag $(tail -1 gpurun_out/sc_$tag.log | cut -c1-240)"; }
run ms_full --config multisensor
run p10_full --config prosail10
