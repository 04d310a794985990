# env_sweep.sh for the beam line: prints beam ms and its GEMM/select breakdown per setting
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
i=0
for r in $(seq 1 ${ROUNDS:-2}); do
  for cfg in $SWEEP; do
    i=$((i+1))
    envs=$(echo $cfg | tr ',' ' ')
    env $envs timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-f32-compare --no-configs ${BENCH_ARGS} > gpurun_out/swb_$i.json 2> gpurun_out/swb_$i.err || { tail -5 gpurun_out/swb_$i.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/swb_$i.json')); bb=d['beam']['kernel_breakdown_ms']; print('$cfg', round(d['ms_per_step'],3), round(d['beam']['ms_per_step'],3), 'dec', bb.get('dec_lstm'), 'att', bb.get('attention'), 'proj', bb.get('proj'), 'sel', bb.get('select'))"
  done
done
