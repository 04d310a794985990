# A/B of two library builds on one box, interleaved: libcasr_hip.so (A) and $ALT (B), $ROUNDS
# rounds of one bench run each (greedy + beam ms per step, per-class breakdown)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
cp chinese-asr_amd/casr/libcasr_hip.so /tmp/A.so
cp chinese-asr_amd/casr/$ALT /tmp/B.so
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in A B; do
    cp /tmp/$v.so chinese-asr_amd/casr/libcasr_hip.so
    timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-f32-compare --no-configs ${BENCH_ARGS} > gpurun_out/ab_$v$r.json 2> gpurun_out/ab_$v$r.err || { tail -5 gpurun_out/ab_$v$r.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab_$v$r.json')); b=d['kernel_breakdown_ms']; bb=d['beam']['kernel_breakdown_ms'] if d['beam'] else {}; print('$v$r', round(d['ms_per_step'],3), round(d['beam']['ms_per_step'],3) if d['beam'] else '-', 'rec', b['rec_step'], 'in', b['input_proj'], '| beam rec', bb.get('rec_step'), 'proj', bb.get('proj'), 'sel', bb.get('select'))"
  done
done
cp /tmp/A.so chinese-asr_amd/casr/libcasr_hip.so
