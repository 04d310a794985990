#!/bin/bash
# folded greedy step: targeted parity tests, then an interleaved A/B bench (DEC_FOLD 0/1)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
K="${TESTS_K:-fold or greedy_matches or fused_select or batch_invariance or graph_replay or split_form}"
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "$K" \
  > $OUT/t_fold.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" $OUT/t_fold.log | tail -40; [ $rc -eq 0 ] || exit $rc
for v in ${AB_ORDER:-0 1 0 1}; do
  CASR_OPTS=DEC_FOLD=$v timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-configs --no-cpu-baseline \
    --no-f32-compare ${BENCH_EXTRA} > $OUT/b_fold$v.json 2> $OUT/b_fold.err || { tail -5 $OUT/b_fold.err; exit 1; }
  python - $v <<'PY'
import json, sys
v = sys.argv[1]
d = json.load(open(f"gpurun_out/b_fold{v}.json"))
b = d.get("beam", {})
print("fold", v, "greedy ms", round(d["ms_per_step"], 3), d.get("kernel_breakdown_ms"), "flags", d.get("device_flags_clean"),
      "| beam ms", b.get("ms_per_step"))
PY
done
