#!/bin/bash
# All BASELINE.json bench configs on one MI355X, one JSON line each into
# gpurun_out/configs.jsonl (each run under its own time limit; stop at the first failure).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" && mkdir -p gpurun_out
: > gpurun_out/configs.jsonl
run() {
  local tag=$1; shift
  timeout -k 10 300 python -u bench.py "$@" > gpurun_out/cfg_$tag.json 2> gpurun_out/cfg_$tag.err \
    || { echo "!! $tag rc=$?"; tail -5 gpurun_out/cfg_$tag.err; exit 1; }
  python -c "import json,sys; r=json.load(open('gpurun_out/cfg_$tag.json')); r['tag']='$tag'; print(json.dumps(r))" \
    >> gpurun_out/configs.jsonl
  python -c "import json; r=json.load(open('gpurun_out/cfg_$tag.json')); print('$tag', r['config']['tile'], r['ms_per_step'], '%.3g' % r['value'], r['config']['gn_iterations'][-1], r['config']['finite'])"
}
for c in ${CONFIGS:-tip7 tip7_gain spatial prosail10 prosail10_hard multisensor identity7 identity7_10980}; do
  case $c in
    tip7) run tip7 --config tip7 --steps 8 --warmup 2 ;;
    tip7_gain) run tip7_gain --config tip7 --steps 8 --warmup 2 --set analysis_form=gain ;;
    spatial) run spatial --config spatial --steps 6 --warmup 2 ;;
    prosail10) run prosail10 --config prosail10 --steps 4 --warmup 1 ;;
    prosail10_hard) run prosail10_hard --config prosail10_hard --steps 3 --warmup 1 ;;
    multisensor) run multisensor --config multisensor --steps 3 --warmup 1 ;;
    identity7) run identity7 --config identity7 --steps 50 --warmup 5 ;;
    identity7_10980) run identity7_10980 --config identity7 --size 10980 --steps 6 --warmup 2 ;;
  esac
done
