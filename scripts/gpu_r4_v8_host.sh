set -o pipefail
cd ${GRAFT_REPO_ROOT:-.} && mkdir -p gpurun_out/r4v8 && \
SIZE=3882 NSTEP=60 timeout -k 10 300 python -u scripts/host_breakdown.py --tip7 > gpurun_out/r4v8/hb_tip7_3882.txt 2>&1 && cat gpurun_out/r4v8/hb_tip7_3882.txt && \
SIZE=10980 NSTEP=40 timeout -k 10 300 python -u scripts/host_breakdown.py --tip7 > gpurun_out/r4v8/hb_tip7_10980.txt 2>&1 && cat gpurun_out/r4v8/hb_tip7_10980.txt
