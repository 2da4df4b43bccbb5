#!/bin/bash
# Round 4 closing check of the final tree: every GPU test, smoke(), default bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r4final4
O=gpurun_out/r4final4
stop() { echo "!! $1 rc=$2"; exit ${2:-1}; }
run() { local n=$1 log=$2 to=$3; shift 3; timeout -k 10 $to "$@" > $log 2>&1; local rc=$?; \
        if [ $rc -ne 0 ]; then tail -40 $log; stop $n $rc; fi; }
run tests $O/gpu_tests.log 700 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread
tail -1 $O/gpu_tests.log
run smoke $O/smoke.log 200 python -c "import __graft_entry__ as g; g.smoke()"
tail -1 $O/smoke.log
run bench_default $O/bench_default.log 400 python -u bench.py
echo "default $(tail -1 $O/bench_default.log | cut -c1-220)"
echo all-done
