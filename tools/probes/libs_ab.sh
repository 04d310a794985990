# A/B/C... of library builds on one box: each name in $LIBS (files in chinese-asr_amd/casr/) is
# copied over libcasr_hip.so in turn and timed with bench.py; "base" = the tree's own build
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
L=chinese-asr_amd/casr
cp $L/libcasr_hip.so /tmp/casr_base.so
for n in $LIBS; do
  if [ "$n" = base ]; then cp /tmp/casr_base.so $L/libcasr_hip.so; else cp $L/$n $L/libcasr_hip.so; fi
  touch $L/libcasr_hip.so
  timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-f32-compare ${BENCH_ARGS} > gpurun_out/ab_$n.json 2> gpurun_out/ab_$n.err || { echo "$n failed"; tail -5 gpurun_out/ab_$n.err; cp /tmp/casr_base.so $L/libcasr_hip.so; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab_$n.json')); print('$n', round(d['ms_per_step'],3), round(d['beam']['ms_per_step'],3), d['kernel_breakdown_ms'])"
done
cp /tmp/casr_base.so $L/libcasr_hip.so
touch $L/libcasr_hip.so
