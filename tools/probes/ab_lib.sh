# A/B of two builds of the library on one box: default, then $ALT (copied over the default)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {
  timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-f32-compare > gpurun_out/ab_$1.json 2> gpurun_out/ab_$1.err || { tail -5 gpurun_out/ab_$1.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab_$1.json')); print('$1', round(d['ms_per_step'],3), round(d['beam']['ms_per_step'],3), d['kernel_breakdown_ms'])"
}
run base
cp chinese-asr_amd/casr/libcasr_hip.so /tmp/base.so
cp chinese-asr_amd/casr/$ALT chinese-asr_amd/casr/libcasr_hip.so
run alt
cp /tmp/base.so chinese-asr_amd/casr/libcasr_hip.so
run base2
