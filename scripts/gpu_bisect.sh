cd $GRAFT_REPO_ROOT
bash scripts/gpu_dbg_pad.sh "MIX_OLD ONEPHASE MIX_OLD" || exit 1
bash scripts/gpu_exp_ab.sh "MIX_OLD ONEPHASE main MIX_OLD ONEPHASE" "4,0,5"
