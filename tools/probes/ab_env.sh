#!/bin/bash
# interleaved A/B of one environment switch (greedy + beam bench lines): ab_env.sh VAR [rounds]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
VAR=$1; N=${2:-2}
for i in $(seq $N); do for v in 0 1; do
  if [ $v = 1 ]; then export $VAR=1; else unset $VAR; fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-configs --no-cpu-baseline --no-f32-compare \
    > gpurun_out/ab$v.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
  python -c "
import json;d=json.load(open('gpurun_out/ab$v.json'));b=d['beam']
print('$VAR=$v greedy', round(d['ms_per_step'],3), d['kernel_breakdown_ms']['proj'], d['kernel_breakdown_ms']['attention'], '| beam', round(b['ms_per_step'],3), b['kernel_breakdown_ms']['proj'], b['kernel_breakdown_ms']['attention'], 'clean', d['device_flags_clean'])"
done; done
