cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export VARIANTS="base||
eager||--graphs 0
nocoop|CASR_OPTS=REC_COOP=0|"
export ROUNDS=2
bash tools/probes/ab_bench.sh || exit 1
timeout -k 10 240 python tools/probes/split_decode_probe.py > gpurun_out/split_probe.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/split_probe.txt; exit $rc
