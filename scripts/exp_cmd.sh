set -o pipefail
run() { tag=$1; shift; timeout -k 10 300 env "$@" python -u -m pytest tests/test_mvp.py -k "1024 or on_device" -s -q --timeout 200 > gpurun_out/mvp_$tag.log 2>&1; rc=$?; echo "mvp_$tag rc=$rc"; grep -o '"in_domain": {[^}]*' gpurun_out/mvp_$tag.log | cut -c1-300; case $rc in 0|1) ;; *) exit $rc;; esac; }
run base KAFKA_X=1 && run s64 KAFKA_EXT=solve64 && bash scripts/gpu_step.sh 'cfg:tip7' 'cfg:tip7 --size 3882 --steps 30 --warmup 3' && KAFKA_EXT=solve64 LOGTAG=_s64 bash scripts/gpu_step.sh 'cfg:tip7' 'cfg:tip7 --size 3882 --steps 30 --warmup 3'
