# A/B of tuning-knob environments on one box: each line of $ENVS is one run ("base" = none)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
i=0
while IFS= read -r e; do
  [ -z "$e" ] && continue
  i=$((i+1))
  [ "$e" = base ] && e=""
  env $e timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-f32-compare ${BENCH_ARGS} > gpurun_out/env_$i.json 2> gpurun_out/env_$i.err || { echo "run $i ($e) failed"; tail -5 gpurun_out/env_$i.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/env_$i.json')); print('[$e]', round(d['ms_per_step'],3), d['kernel_breakdown_ms'], '| beam', round(d['beam']['ms_per_step'],3), d['beam']['kernel_breakdown_ms'])"
done <<< "$ENVS"
