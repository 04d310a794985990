cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export VARIANTS="base||
l16x32|CASR_OPTS=REC_LAYOUT=2|
eager||--graphs 0"
export ROUNDS=2
bash tools/probes/ab_bench.sh || exit 1
bash tools/probes/profile_r03.sh
