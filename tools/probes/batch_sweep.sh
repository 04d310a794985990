cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for B in 64 128 256; do
  timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-f32-compare --no-beam --batch $B > gpurun_out/bs_$B.json 2> gpurun_out/bs_$B.err || { tail -5 gpurun_out/bs_$B.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bs_$B.json')); print($B, round(d['ms_per_step'],3), d['kernel_breakdown_ms'])"
done
