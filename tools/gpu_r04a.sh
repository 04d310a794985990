#!/bin/bash
# Round-4 first GPU pass: the whole -m gpu suite (incl. the new config 4 / 5 shard-chain oracle
# tests), smoke, the default bench line, then one rocprofv3 kernel trace of the SHIPPED default
# (cooperative recurrence launch) with its stderr and exit status kept.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04a
mkdir -p $O
timeout -k 10 1000 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  --durations=25 > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -30 $O/pytest_gpu.log | grep -v "^$"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print('bench', round(d['value']), round(d['ms_per_step'],3), d['device_ms_per_step'], d['roofline']['avg_launch_us'], d['beam']['ms_per_step'], d['config3_beam8_b128']['ms_per_step'], d['config2_greedy_b32']['ms_per_step'], d['config5_beam16_lm']['ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 bench.py --steps 20 --warmup 2 --no-beam --no-configs --no-f32-compare --no-cpu-baseline > $O/prof_bench.json 2> $O/prof.err
rc=$?
echo "rocprofv3 (cooperative launch, default) exit status $rc" | tee $O/prof_rc.txt
tail -20 $O/prof.err
python tools/prof_by_grid.py $O/prof/run_kernel_trace.csv 30 > $O/prof_by_grid.txt 2>&1
head -12 $O/prof_by_grid.txt
exit $rc
