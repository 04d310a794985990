# Interleaved A/B of bench.py variants on one box: each line of $VARIANTS is "name|env|args";
# $ROUNDS rounds; prints greedy / beam ms per step and the per-class breakdowns.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
  while IFS='|' read -r name envs bargs; do
    [ -z "$name" ] && continue
    env $envs timeout -k 10 200 python bench.py --steps 10 --warmup 2 --beam-steps 5 --no-cpu-baseline --no-f32-compare --no-configs $bargs > gpurun_out/ab_${name}_$r.json 2> gpurun_out/ab_${name}_$r.err || { echo "$name failed"; tail -5 gpurun_out/ab_${name}_$r.err; exit 1; }
    python - "$name" "$r" <<'PY'
import json, sys
n, r = sys.argv[1], sys.argv[2]
d = json.load(open(f"gpurun_out/ab_{n}_{r}.json"))
b = d["kernel_breakdown_ms"]; bb = (d.get("beam") or {}).get("kernel_breakdown_ms", {})
print(f"{n:>14s} r{r} greedy {d['ms_per_step']:.3f} beam {d['beam']['ms_per_step'] if d.get('beam') else 0:.3f} | rec {b.get('rec_step')} in {b.get('input_proj')} lstm {b.get('dec_lstm')} att {b.get('attention')} proj {b.get('proj')} | beam rec {bb.get('rec_step')} lstm {bb.get('dec_lstm')} att {bb.get('attention')} proj {bb.get('proj')} sel {bb.get('select')} | flags {d['device_flags_clean']}", flush=True)
PY
  done <<< "$VARIANTS"
done
