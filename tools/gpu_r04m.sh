#!/bin/bash
# Round-4 pass m: the -m gpu suite (the folded greedy step now also under f32), the default bench
# line, then the round-4 profiles (tools/gpu_r04_prof.sh: log-mel, PMC passes, kernel traces, the
# cooperative launch under rocprofv3 last).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04m
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  --durations=10 > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); f=d['f32_exact_path']; print('bench', round(d['value']), round(d['ms_per_step'],3), d['kernel_breakdown_ms'], '| f32', f.get('ms_per_step'), f.get('kernel_breakdown_ms'), '| beam', d['beam']['ms_per_step'])"
bash tools/gpu_r04_prof.sh
