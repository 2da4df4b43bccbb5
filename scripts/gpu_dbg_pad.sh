# run scripts/debug_mfma_tiles.py against experiment builds exp_<V>/ (kernel variants)
cd $GRAFT_REPO_ROOT
for V in $1; do
  for a in "--size 512" "--size 2048 --partials"; do
    ( cd exp_$V && timeout -k 10 300 python -u -c "import kafka_inferenceengine_amd as k, runpy, sys; sys.argv=['x'] + '$a'.split(); runpy.run_path('$GRAFT_REPO_ROOT/scripts/debug_mfma_tiles.py', run_name='__main__')" > $GRAFT_REPO_ROOT/gpurun_out/dbg_$V.log 2>&1 ) || exit $?
    echo "$V $a: $(tail -1 gpurun_out/dbg_$V.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k:(v['max'],v['n_bad']) for k,v in d.items()})")"
  done
done
