"""Per-kernel PMC summary from rocprofv3 --pmc passes (tools/probes/pmc_passes.sh).

Groups dispatches by (kernel, grid size) and prints per-dispatch averages plus derived figures:
  clock   = GRBM_GUI_ACTIVE / 8 / duration (GRBM sums the 8 XCDs; MI355X_MICROARCH.md DVFS note)
  mfma%   = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 1024 SIMDs)
  wait%, stall%, active% = SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES
  fetch   = 2 x FETCH_SIZE (gfx950 tallies 128-B requests at 64 B: MICROARCH §HBM), write = WRITE_SIZE
With --json, writes {class: hbm_bytes_per_launch} for bench.py's roofline.traffic.

usage: python tools/pmc_summary.py gpurun_out/pmc [--json profiles/pmc_traffic.json]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

# bench.py kernel classes -> (kernel-name prefixes after short(), launches of the class per step
# as bench.py counts them: one "launch" of input_proj = one layer's projection, persistent kernel
# and half-tile tail together; None = one launch per dispatch, counted: the folded decode step
#  launches the LSTMCell GEMM once per decode and its fused GEMM is the proj class)
CLASS_OF = {
    "input_proj": (("gemm16_persist_kernel", "gemm16_bias_kernel", "gemm16_pp_kernel", "gemm16_tail_kernel"), 4),
    "rec_step": (("rec_layer_kernel",), 4),
    "keys": (("gemm_nt_kernel<KeysEpi", "keys16_kernel"), 1),
    "dec_lstm": (("dgemm_kernel<*DecLstmA",), None),
    "proj": (("dgemm_kernel<*ProjA",), None),
    "select": (("beam_select_kernel",), None),
    "attention": (("attention_kernel",), None),
    "features": (("features_stats_kernel", "features_rows_kernel"), 1),
}


def matches(name, pres):
    for p in pres:
        if "*" in p:
            a, b = p.split("*")
            if name.startswith(a) and b in name:
                return True
        elif name.startswith(p):
            return True
    return False


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    n = name[:name.index("(")] if "(" in name else name
    return n.replace("void ", "").replace("casr::", "")


def load(d):
    per = defaultdict(lambda: defaultdict(list))  # (kernel, grid) -> counter -> [values]
    dur = defaultdict(dict)
    for f in glob.glob(os.path.join(d, "*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            key = (short(r["Kernel_Name"]), int(r["Grid_Size"]))
            per[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
            dur[key][(f, r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    return per, dur


def main(d, json_out=None):
    per, dur = load(d)
    rows = []
    for key, cs in per.items():
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        us = sum(dur[key].values()) / max(1, len(dur[key]))
        rows.append((key, avg, us, max(len(v) for v in cs.values())))
    rows.sort(key=lambda r: -r[2] * r[3])
    print(f"{'kernel':52s} {'grid':>8s} {'n':>4s} {'us':>8s} {'clkGHz':>6s} {'mfma%':>6s} {'wait%':>6s} {'stall%':>6s} "
          f"{'lds%':>5s} {'fetchMB':>8s} {'writeMB':>8s}")
    traffic = {}
    for (name, grid), a, us, n in rows[:30]:
        g = a.get("GRBM_GUI_ACTIVE")
        cyc = g / 8 if g else None
        clk = cyc / (us * 1e3) if cyc and us else float("nan")
        mf = 100 * a["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * 1024) if cyc and "SQ_VALU_MFMA_BUSY_CYCLES" in a else float("nan")
        wc = a.get("SQ_WAVE_CYCLES")
        wait = 100 * a["SQ_WAIT_ANY"] / wc if wc else float("nan")
        stall = 100 * a["SQ_WAIT_INST_ANY"] / wc if wc else float("nan")
        lds = 100 * a["SQ_WAIT_INST_LDS"] / wc if wc and "SQ_WAIT_INST_LDS" in a else float("nan")
        fetch = 2 * a["FETCH_SIZE"] / 1024 if "FETCH_SIZE" in a else float("nan")  # KB -> MB
        write = a["WRITE_SIZE"] / 1024 if "WRITE_SIZE" in a else float("nan")
        print(f"{name[:52]:52s} {grid:8d} {n:4d} {us:8.1f} {clk:6.2f} {mf:6.1f} {wait:6.1f} {stall:6.1f} {lds:5.1f} "
              f"{fetch:8.2f} {write:8.2f}")
    # per class: every dispatch of its kernels summed over the run, then per bench launch
    steps = int(os.environ.get("STEPS", 2))
    for cls, (pres, per_step) in CLASS_OF.items():
        tot = defaultdict(float)
        ndisp = 0
        for (name, grid), cs in per.items():
            if matches(name, pres):
                for c, v in cs.items():
                    tot[c] += sum(v)
                ndisp += len(cs.get("FETCH_SIZE", []))
        if "FETCH_SIZE" not in tot:
            continue
        launches = steps * per_step if per_step else ndisp
        per_step = per_step or ndisp / steps
        fetch = 2 * tot["FETCH_SIZE"] * 1024 / launches  # KB -> B, gfx950 x2
        write = tot.get("WRITE_SIZE", 0.0) * 1024 / launches
        rec = {"fetch_bytes": fetch, "write_bytes": write, "hbm_bytes": fetch + write,
               "launches_per_step": per_step,
               "note": "per bench launch: all dispatches of the class summed, FETCH_SIZE x2 (gfx950) + WRITE_SIZE"}
        if "SQ_VALU_MFMA_BUSY_CYCLES" in tot and tot.get("GRBM_GUI_ACTIVE"):
            rec["mfma_busy"] = tot["SQ_VALU_MFMA_BUSY_CYCLES"] / (tot["GRBM_GUI_ACTIVE"] / 8 * 1024)
        traffic[cls] = rec
    if json_out:
        json.dump(traffic, open(json_out, "w"), indent=1)
        print("wrote", json_out)


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0], a[a.index("--json") + 1] if "--json" in a else None)
