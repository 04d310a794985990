#!/bin/bash
# Round-4 pass d: the whole -m gpu suite, smoke, the log-mel front end's line + profile, the greedy
# decode phase trace, the default bench line, then the cooperative-launch exit probe under rocprofv3
# (a bare HIP program, no casr code: plain launch, then cooperative, last).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04d
mkdir -p $O
timeout -k 10 1000 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  --durations=10 > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash tools/probes/logmel_profile.sh || exit 1
timeout -k 10 200 python tools/probes/dg_trace.py > $O/dg_trace_greedy.txt 2>&1 || { tail -5 $O/dg_trace_greedy.txt; exit 1; }
cat $O/dg_trace_greedy.txt
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print('bench', round(d['value']), round(d['ms_per_step'],3), d['device_ms_per_step'], d['kernel_breakdown_ms'], d['beam']['ms_per_step'], d['config3_beam8_b128']['ms_per_step'], d['config2_greedy_b32'], d['config5_beam16_lm']['ms_per_step'], d['config1_single_wav']['latency_ms'])"
for mode in plain coop; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/coop_$mode -o run -- \
    ./tools/probes/coop_exit_probe $mode > $O/coop_$mode.log 2>&1
  echo "coop_exit_probe $mode under rocprofv3: exit status $?" | tee -a $O/coop_rc.txt
  grep -v "^    @" $O/coop_$mode.log | tail -4
done
