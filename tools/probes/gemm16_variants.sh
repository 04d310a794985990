cd $GRAFT_REPO_ROOT
for w in ${VARIANTS:-0 4 8}; do
  CASR_GEMM16_WAVES=$w timeout -k 10 120 python bench.py --steps 3 --warmup 1 --no-beam --no-cpu-baseline > gpurun_out/gv_$w.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/gv_$w.json'));print($w, d['ms_per_step'], d['kernel_breakdown_ms']['input_proj'])"
done
