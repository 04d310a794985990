#!/bin/bash
# Round-4 pass e: the whole -m gpu suite, the log-mel line + profile, the greedy decode phase trace,
# the default bench line, then a rocprofv3 kernel trace + stats of the shipped default (cooperative
# recurrence launch).  The profiled process ends in SIGSEGV after rocprofv3 has written its results
# (ROCm cooperative-launch teardown under the profiler, reproduced by tools/probes/coop_exit_probe
# without any casr code), so that step runs last and its status is recorded, not acted on.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04e
mkdir -p $O
timeout -k 10 1000 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  --durations=10 > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
bash tools/probes/logmel_profile.sh || exit 1
timeout -k 10 200 python tools/probes/dg_trace.py > $O/dg_trace_greedy.txt 2>&1 || { tail -5 $O/dg_trace_greedy.txt; exit 1; }
head -8 $O/dg_trace_greedy.txt
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print('bench', round(d['value']), round(d['ms_per_step'],3), d['device_ms_per_step']['median'], d['kernel_breakdown_ms'], d['beam']['ms_per_step'], d['config3_beam8_b128']['ms_per_step'], d['config2_greedy_b32']['ms_per_step'], d['config5_beam16_lm']['ms_per_step'], d['config1_single_wav']['latency_ms'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 bench.py --steps 20 --warmup 2 --no-beam --no-configs --no-f32-compare --no-cpu-baseline > $O/prof_bench.json 2> $O/prof.err
echo "rocprofv3 of the default (cooperative) launch: exit status $?" | tee $O/prof_rc.txt
python tools/prof_by_grid.py $O/prof/run_kernel_trace.csv 30 > $O/prof_by_grid.txt 2>&1
head -8 $O/prof_by_grid.txt
