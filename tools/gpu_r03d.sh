cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 ./tools/probes/gemm16_probe 256 > gpurun_out/gemm16_probe.txt 2>&1
rc=$?; cat gpurun_out/gemm16_probe.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 ./tools/probes/gemm16_probe 37 > gpurun_out/gemm16_probe37.txt 2>&1
rc=$?; grep -i "differ" gpurun_out/gemm16_probe37.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python tools/probes/decode_batch_probe.py > gpurun_out/decode_batch.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/decode_batch.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py -m gpu -x -v --timeout 300 --timeout-method thread -k "beam8_b256 or config3" > gpurun_out/gputest_scale.log 2>&1
rc=$?; tail -3 gpurun_out/gputest_scale.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline --no-f32-compare > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; tail -3 gpurun_out/bench.err; exit $rc
