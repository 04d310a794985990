# Interleaved A/B/C on one box: library A (libcasr_hip.so) under each env setting of $SWEEP, and
# library $ALT (B) with no setting; $ROUNDS rounds; decode classes printed (as ab_dec.sh)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
cp chinese-asr_amd/casr/libcasr_hip.so /tmp/A.so
cp chinese-asr_amd/casr/$ALT /tmp/B.so
i=0
for r in $(seq 1 ${ROUNDS:-2}); do
  for cfg in $SWEEP ALT; do
    i=$((i+1))
    if [ $cfg = ALT ]; then cp /tmp/B.so chinese-asr_amd/casr/libcasr_hip.so; envs=""; else cp /tmp/A.so chinese-asr_amd/casr/libcasr_hip.so; envs=$(echo $cfg | tr ',' ' '); fi
    env $envs timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-f32-compare --no-configs ${BENCH_ARGS} > gpurun_out/ae_$i.json 2> gpurun_out/ae_$i.err || { tail -5 gpurun_out/ae_$i.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ae_$i.json')); b=d['kernel_breakdown_ms']; bb=d['beam']['kernel_breakdown_ms'] if d['beam'] else {}; print('$cfg', round(d['ms_per_step'],3), round(d['beam']['ms_per_step'],3) if d['beam'] else '-', 'lstm', b['dec_lstm'], 'att', b['attention'], 'proj', b['proj'], '| beam lstm', bb.get('dec_lstm'), 'att', bb.get('attention'), 'proj', bb.get('proj'), 'sel', bb.get('select'))"
  done
done
cp /tmp/A.so chinese-asr_amd/casr/libcasr_hip.so
