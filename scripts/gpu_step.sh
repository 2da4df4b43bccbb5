#!/bin/bash
# One GPU call = a list of named steps, each under its own time limit, stopping at
# the first failure (gpurun rules: no retries, nothing after a fault/timeout).
#   bash scripts/gpu_step.sh tests[:FILTER] tests_nox[:FILTER] smoke ab[:ARGS] bench[:ARGS] \
#        cfg:CONFIG[ ARGS] py:SCRIPT[ ARGS] prof[:TAG/ARGS] trace[:TAG/ARGS] phase:ARGS \
#        pmc:V/COUNTERS pmcb:COUNTERS/BENCH_ARGS dist:N/BENCH_ARGS ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export PYTHONPATH="$R${PYTHONPATH:+:$PYTHONPATH}"
stop() { echo "!! step $1 rc=$2"; exit "$2"; }
declare -A seen
for step in "$@"; do
  name=${step%%:*}; arg=""; [ "$name" != "$step" ] && arg=${step#*:}
  case $name in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${arg:+-k "$arg"} \
        > gpurun_out/gpu_tests.log 2>&1 || { rc=$?; tail -40 gpurun_out/gpu_tests.log; stop tests $rc; }
      tail -3 gpurun_out/gpu_tests.log ;;
    tests_nox)
      # every GPU test, no stop at the first failure (tolerance surveys)
      timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread ${arg:+-k "$arg"} \
        > gpurun_out/gpu_tests.log 2>&1; rc=$?
      grep -E "PASSED|FAILED|ERROR|^E " gpurun_out/gpu_tests.log | grep -E "FAILED|ERROR|^E " | head -40; tail -3 gpurun_out/gpu_tests.log
      [ $rc -le 1 ] || stop tests_nox $rc ;;
    smoke)
      timeout -k 10 300 python -u __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { rc=$?; tail -20 gpurun_out/smoke.log; stop smoke $rc; }
      tail -1 gpurun_out/smoke.log ;;
    ab)
      timeout -k 10 400 python -u scripts/bench_kernels.py $arg > gpurun_out/ab.log 2>&1 || { rc=$?; tail -20 gpurun_out/ab.log; stop ab $rc; }
      tail -5 gpurun_out/ab.log ;;
    bench)
      timeout -k 10 600 python -u bench.py $arg > gpurun_out/bench.log 2>&1 || { rc=$?; tail -20 gpurun_out/bench.log; stop bench $rc; }
      tail -1 gpurun_out/bench.log ;;
    cfg)
      # cfg:CONFIG [bench args] -> gpurun_out/bench_CONFIG.log (one JSON line at its end)
      # (a repeated CONFIG logs to bench_CONFIG_2.log, _3, ...)
      c=${arg%% *}; rest=""; [ "$c" != "$arg" ] && rest=${arg#* }
      # LOGTAG=x: bench_CONFIGx.log (A/B of modules in one call: KAFKA_EXT=name LOGTAG=_name)
      seen[$c]=$(( ${seen[$c]:-0} + 1 )); lg=bench_$c${LOGTAG:-}; [ ${seen[$c]} -gt 1 ] && lg=${lg}_${seen[$c]}
      timeout -k 10 900 python -u bench.py --config $c $rest > gpurun_out/$lg.log 2>&1 \
        || { rc=$?; tail -20 gpurun_out/$lg.log; stop cfg_$c $rc; }
      echo "$lg $(tail -1 gpurun_out/$lg.log | cut -c1-300)" ;;
    py)
      # py:SCRIPT [args] -> gpurun_out/py_<script name>.log
      sc=${arg%% *}; rest=""; [ "$sc" != "$arg" ] && rest=${arg#* }; tag=$(basename $sc .py)
      timeout -k 10 900 python -u $sc $rest > gpurun_out/py_$tag.log 2>&1 \
        || { rc=$?; tail -20 gpurun_out/py_$tag.log; stop py_$tag $rc; }
      tail -5 gpurun_out/py_$tag.log ;;
    prof|trace)
      # prof[:TAG/BENCH ARGS]  kernel statistics of bench.py (default: tip7, 4 steps) -> gpurun_out/prof[_TAG]/
      # trace[:TAG/BENCH ARGS] the same plus the memory-copy trace (inter-kernel gaps, H2D overlap)
      tag=""; rest="--steps 4 --warmup 1"
      if [ -n "$arg" ]; then tag=_${arg%%/*}; rest=${arg#*/}; fi
      extra=""; [ "$name" = trace ] && extra="--memory-copy-trace"
      out="$R/gpurun_out/$name$tag"
      ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace $extra --stats -d "$out" -o run \
        --output-format csv -- python "$R/bench.py" $rest > "$out.log" 2>&1 ) \
        || { rc=$?; tail -20 "$out.log"; stop $name $rc; }
      echo "$name$tag $(tail -1 "$out.log" | cut -c1-200)" ;;
    phase)
      # phase:BENCH ARGS  phase clocks of the fused analysis kernel (_build.py --prof, KAFKA_PROF=1)
      KAFKA_PROF=1 timeout -k 10 300 python -u bench.py $arg > gpurun_out/phase.log 2>&1 \
        || { rc=$?; tail -20 gpurun_out/phase.log; stop phase $rc; }
      grep phase_clocks gpurun_out/phase.log; tail -1 gpurun_out/phase.log | cut -c1-200 ;;
    dist)
      # dist:N/BENCH ARGS  N ranks of bench.py on this box's one GPU over gloo (a logic /
      # contention rehearsal, not a scaling point: the ranks share the GPU and the CPUs)
      n=${arg%%/*}; rest=${arg#*/}; port=$((29700 + RANDOM % 200))
      timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node=$n \
        --master-addr=127.0.0.1 --master-port=$port bench.py --gpus $n --device cuda:0 --rehearse-gloo $rest \
        > gpurun_out/dist$n.log 2>&1 || { rc=$?; tail -20 gpurun_out/dist$n.log; stop dist $rc; }
      echo "dist$n $(tail -1 gpurun_out/dist$n.log | cut -c1-300)" ;;
    pmc)
      # pmc:V/C1,C2,...  (V = analysis variant, one counter pass per step)
      v=${arg%%/*}; ctrs=${arg#*/}; tag=${PMC_TAG:-pmc}_v${v}_$(echo "$ctrs" | md5sum | cut -c1-6)
      ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc ${ctrs//,/ } -d "$R/gpurun_out/pmc" -o "$tag" \
        --output-format csv -- python "$R/scripts/bench_kernels.py" --rounds 1 --variants $v > "$R/gpurun_out/pmc.log" 2>&1 ) \
        || { rc=$?; tail -20 gpurun_out/pmc.log; stop pmc $rc; }
      echo pmc-done ;;
    pmcb)
      # pmcb:C1,C2,.../BENCH ARGS  one counter pass over bench.py's fused analysis kernels
      # -> gpurun_out/pmcb/<md5 of the step>/ (+ .log)
      ctrs=${arg%%/*}; rest=${arg#*/}; tag=$(echo "$arg" | md5sum | cut -c1-8)
      mkdir -p "$R/gpurun_out/pmcb"; echo "$arg" > "$R/gpurun_out/pmcb/$tag.args"
      ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 -s KILL 300 rocprofv3 --kernel-trace --pmc ${ctrs//,/ } \
        --kernel-include-regex "analysis" -d "$R/gpurun_out/pmcb/$tag" -o run --output-format csv -- \
        python "$R/bench.py" $rest > "$R/gpurun_out/pmcb/$tag.log" 2>&1 ) \
        || { rc=$?; tail -20 "gpurun_out/pmcb/$tag.log"; stop pmcb $rc; }
      echo "pmcb $tag $arg" ;;
    *) echo "unknown step $name"; exit 2 ;;
  esac
done
