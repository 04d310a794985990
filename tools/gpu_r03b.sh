# round 3: re-run the scale tests, the split-decode probe and the bench
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gputest_scale.log 2>&1
rc=$?; tail -3 gpurun_out/gputest_scale.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/probes/split_decode_probe.py > gpurun_out/split_probe.txt 2>&1
rc=$?; cat gpurun_out/split_probe.txt | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; tail -3 gpurun_out/bench.err; exit $rc
