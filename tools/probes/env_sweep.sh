# Interleaved sweep of environment knob settings on one box: $SWEEP is a list of
# space-separated "VAR=x,VAR2=y" settings; $ROUNDS rounds; one greedy bench per setting per round
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
i=0
for r in $(seq 1 ${ROUNDS:-2}); do
  for cfg in $SWEEP; do
    i=$((i+1))
    envs=$(echo $cfg | tr ',' ' ')
    env $envs timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-f32-compare --no-configs ${BENCH_ARGS} > gpurun_out/sw_$i.json 2> gpurun_out/sw_$i.err || { tail -5 gpurun_out/sw_$i.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/sw_$i.json')); b=d['kernel_breakdown_ms']; bb=d['beam']['kernel_breakdown_ms'] if d['beam'] else {}; print('$cfg', round(d['ms_per_step'],3), round(d['beam']['ms_per_step'],3) if d['beam'] else '-', 'rec', b['rec_step'], '| beam rec', bb.get('rec_step'))"
  done
done
