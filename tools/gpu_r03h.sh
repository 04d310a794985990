cd $GRAFT_REPO_ROOT
bash tools/probes/profile_r03.sh
