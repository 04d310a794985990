"""One-line summary of a bench.py JSON line (tools/gpu_session.sh): headline, beam line, the
per-class breakdowns and the guard flags.  usage: python tools/bench_line.py gpurun_out/x/bench.json"""
import json
import sys


def main(path):
    with open(path) as f:
        d = json.loads(f.read().strip().splitlines()[-1])
    parts = [f"greedy {d['value']:.0f} utt/s {d['ms_per_step']:.3f} ms",
             f"frac {d.get('roofline', {}).get('frac')}"]
    kb = d.get("kernel_breakdown_ms")
    if kb:
        parts.append("greedy classes " + " ".join(f"{k}={v:.3f}" for k, v in kb.items()))
    b = d.get("beam") or {}
    if b.get("ms_per_step"):
        parts.append(f"| beam {b['ms_per_step']:.3f} ms")
        if b.get("kernel_breakdown_ms"):
            parts.append("beam classes " + " ".join(f"{k}={v:.3f}" for k, v in b["kernel_breakdown_ms"].items()))
    f32 = d.get("f32_exact_path") or {}
    if f32.get("ms_per_step"):
        parts.append(f"| f32 {f32['ms_per_step']:.3f} ms")
    for c in ("config3_beam8_b128", "config2_greedy_b32", "config4_beam8_sharded", "config5_beam16_lm",
              "config1_single_wav"):
        x = d.get(c) or {}
        ms = x.get("ms_per_step") or x.get("ms_per_batch") or x.get("latency_ms")
        if ms:
            parts.append(f"| {c} {ms:.3f} ms" + (f" ({x['value']:.0f} utt/s)" if x.get("value") else ""))
    parts.append(f"| flags {d.get('device_flags_clean')}")
    print(" ".join(parts))


if __name__ == "__main__":
    main(sys.argv[1])
