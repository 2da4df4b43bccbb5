#!/bin/bash
# rocprofv3 kernel stats of the non-headline configs (short runs)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
stop() { echo "!! $1 rc=$2"; exit $2; }
for cfg in ${CFGS:-prosail10 multisensor spatial}; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$cfg" -o run --output-format csv -- \
      python "$R/bench.py" --config $cfg --steps 2 --warmup 1 > "$R/gpurun_out/prof_$cfg.log" 2>&1 || stop $cfg $?
  echo "$cfg done"
done
