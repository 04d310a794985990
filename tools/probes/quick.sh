# GPU parity tests, then one bench line with the per-class breakdown (speed iteration)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_gpu.log
grep -Eq 'illegal memory|HSA_STATUS_ERROR|Memory access fault|core dumped|Aborted' gpurun_out/pytest_gpu.log && exit 99
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/quick.json 2> gpurun_out/quick.err || { tail -5 gpurun_out/quick.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/quick.json')); print(round(d['ms_per_step'],3), d['kernel_breakdown_ms'], '| beam', round(d['beam']['ms_per_step'],3), d['beam']['kernel_breakdown_ms'])"
