# decode-GEMM ring variants (CASR_DG="lstm_stages,proj_variant"; speed only, same results)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for V in ${DG_VARIANTS:-"6,0" "2,3" "4,1" "6,2"}; do
  CASR_DG=$V timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-f32-compare \
    > gpurun_out/dg_$V.json 2> gpurun_out/dg_$V.err || { tail -5 gpurun_out/dg_$V.err; exit 1; }
  python - "$V" <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/dg_{sys.argv[1]}.json"))
print(sys.argv[1], round(d["ms_per_step"], 3), round(d["beam"]["ms_per_step"], 3), d["kernel_breakdown_ms"])
PY
done
