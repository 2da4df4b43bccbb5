#!/bin/bash
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.} && mkdir -p gpurun_out/r4v14 && \
timeout -k 10 200 python -u bench.py --config identity7 --profile gpurun_out/r4v14/id7_trace.json > gpurun_out/r4v14/id7.log 2>&1 && \
grep step gpurun_out/r4v14/id7.log | tr '\n' ' ' && python - <<'PY'
import json
d = json.load(open("gpurun_out/r4v14/id7_trace.json"))
ev = [e for e in d["traceEvents"] if e.get("ph") == "X" and e.get("dur", 0) > 500]
ev.sort(key=lambda e: -e["dur"])
for e in ev[:25]:
    print(round(e["dur"] / 1e3, 3), "ms", e.get("cat"), e.get("name")[:90])
PY
