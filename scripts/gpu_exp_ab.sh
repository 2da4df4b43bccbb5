# kernel A/B (scripts/bench_kernels.py) against experiment builds exp_<V>/ and the main tree
cd $GRAFT_REPO_ROOT
for V in $1; do
  if [ "$V" = main ]; then dir=$GRAFT_REPO_ROOT; else dir=$GRAFT_REPO_ROOT/exp_$V; fi
  ( cd $dir && timeout -k 10 300 python -u -c "import kafka_inferenceengine_amd as k, runpy, sys; sys.argv=['x','--variants','${2:-4,0,5}','--rounds','5']; runpy.run_path('$GRAFT_REPO_ROOT/scripts/bench_kernels.py', run_name='__main__')" > $GRAFT_REPO_ROOT/gpurun_out/ab_$V.log 2>&1 ) || exit $?
  echo "$V: $(tail -1 gpurun_out/ab_$V.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k:(round(v['median_ms'],3), round(v['max_abs_diff_vs_first'],4)) for k,v in d['variants'].items()})")"
done
