# GPU session: parity suite, decode phase traces (greedy B=256, beam 8 B=256), short bench
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 120 python tools/probes/dg_trace.py > gpurun_out/trace_greedy.txt 2>&1 || { tail gpurun_out/trace_greedy.txt; exit 1; }
BEAM=1 BB=256 timeout -k 10 120 python tools/probes/dg_trace.py > gpurun_out/trace_beam256.txt 2>&1 || { tail gpurun_out/trace_beam256.txt; exit 1; }
grep -A6 "attention" gpurun_out/trace_greedy.txt gpurun_out/trace_beam256.txt
timeout -k 10 300 python bench.py --steps 10 --no-cpu-baseline --no-f32-compare > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err || { tail gpurun_out/bench_quick.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/bench_quick.json"))
print("greedy", round(d["value"]), round(d["ms_per_step"], 3), d["kernel_breakdown_ms"])
b = d["beam"]; print("beam", round(b["value"]), round(b["ms_per_step"], 3), b["kernel_breakdown_ms"], d["device_flags_clean"])
c = d.get("config3_beam8_b128")
if c: print("config3", round(c["value"]), round(c["ms_per_step"], 3), c["kernel_breakdown_ms"], "config2", round(d["config2_greedy_b32"]["ms_per_step"], 3), "config5", round(d["config5_beam16_lm"]["ms_per_step"], 2))
PY
