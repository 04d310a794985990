#!/bin/bash
# beam-path parity subset, two bench lines (beam, config 3, config 5 select times) and the beam phase trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_scale.py \
  -k "beam or batch_invariance or dropin or temperature or sharded" > gpurun_out/t_bm.log 2>&1 || { tail -20 gpurun_out/t_bm.log; exit 1; }
tail -1 gpurun_out/t_bm.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-f32-compare > gpurun_out/bm.json 2> gpurun_out/bm.err || { tail -5 gpurun_out/bm.err; exit 1; }
  python - <<'PY'
import json
d = json.load(open("gpurun_out/bm.json")); b = d["beam"]; c = d["config3_beam8_b128"]; c5 = d["config5_beam16_lm"]
print("greedy", round(d["ms_per_step"], 3), "beam", round(b["ms_per_step"], 3), b["kernel_breakdown_ms"]["select"],
      "cfg3", round(c["ms_per_step"], 3), c["kernel_breakdown_ms"]["select"], "cfg5", round(c5["ms_per_step"], 2))
PY
done
BEAM=1 BB=256 timeout -k 10 200 python tools/probes/dg_trace.py > gpurun_out/dgt_beam.txt 2>&1 || exit 1
grep -A8 beam_select gpurun_out/dgt_beam.txt
