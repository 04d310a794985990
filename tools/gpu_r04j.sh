#!/bin/bash
# Round-4 pass j (branch-light beam epilogue): the whole -m gpu suite, the greedy decode phase trace (prologue sub-phases), the
# log-mel kernel variants probe and line, the default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04j
mkdir -p $O
timeout -k 10 1000 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  --durations=10 > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 200 python tools/probes/dg_trace.py > $O/dg_trace_greedy.txt 2>&1 || { tail -5 $O/dg_trace_greedy.txt; exit 1; }
head -12 $O/dg_trace_greedy.txt
BEAM=1 BB=256 K=8 timeout -k 10 200 python tools/probes/dg_trace.py > $O/dg_trace_beam.txt 2>&1 || { tail -5 $O/dg_trace_beam.txt; exit 1; }
head -30 $O/dg_trace_beam.txt
timeout -k 10 120 ./tools/probes/logmel_variants_ni > $O/logmel_variants.txt 2>&1 || { tail -5 $O/logmel_variants.txt; exit 1; }
cat $O/logmel_variants.txt
timeout -k 10 200 python tools/probes/logmel_probe.py > $O/logmel_line.json 2> $O/logmel_line.err || { tail -5 $O/logmel_line.err; exit 1; }
cat $O/logmel_line.json
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print('bench', round(d['value']), round(d['ms_per_step'],3), d['device_ms_per_step']['median'], d['kernel_breakdown_ms'], d['beam']['ms_per_step'], d['config3_beam8_b128']['ms_per_step'], d['config2_greedy_b32']['ms_per_step'], d['config5_beam16_lm']['ms_per_step'], d['config1_single_wav']['latency_ms'])"
