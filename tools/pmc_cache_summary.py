"""Where a kernel's bytes come from: per-kernel L2 and fabric-side counters from rocprofv3 --pmc
passes (tools/gpu_session.sh stage pmc with the cache counter sets).

  l2_hit%   = TCC_HIT / (TCC_HIT + TCC_MISS)                      (MI355X_MICROARCH.md, L2)
  rdreq_MB  = TCC_EA0_RDREQ x 128 B (gfx950 tallies a 128-B request once: FETCH_SIZE = RDREQ x 64 B
              is half the bytes of a wide streaming read, MICROARCH §HBM)
  dram%     = TCC_EA0_RDREQ_DRAM / TCC_EA0_RDREQ (requests addressed to the memory controller; the
              Infinity Cache sits behind it, so this does not split Infinity-Cache hits from HBM)
  ea_lat    = TCC_EA0_RDREQ_LEVEL / TCC_EA0_RDREQ: average cycles a fabric read is in flight
              (an Infinity-Cache hit vs an HBM miss: ~365 vs ~720 cycles beyond the L2 on an idle chip,
              MICROARCH per-instruction constants; under load both grow)
  wrreq_MB  = TCC_EA0_WRREQ x 64 B, wr_dram% likewise
usage: python tools/pmc_cache_summary.py gpurun_out/x/pmc_greedy [kernel-prefix ...]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    n = name[:name.index("(")] if "(" in name else name
    return n.replace("void ", "").replace("casr::", "")


def main(d, prefixes):
    per = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    for f in glob.glob(os.path.join(d, "*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            key = (short(r["Kernel_Name"]), int(r["Grid_Size"]))
            per[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
            dur[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    rows = []
    for key, cs in per.items():
        if prefixes and not any(key[0].startswith(p) for p in prefixes):
            continue
        a = {c: sum(v) / len(v) for c, v in cs.items()}
        us = sum(dur[key]) / len(dur[key])
        rows.append((key, a, us, max(len(v) for v in cs.values())))
    rows.sort(key=lambda r: -r[2] * r[3])
    print(f"{'kernel':58s} {'grid':>8s} {'n':>4s} {'us':>8s} {'l2_hit%':>7s} {'rdreq_MB':>9s} {'dram%':>6s} "
          f"{'ea_lat':>7s} {'wrreq_MB':>9s} {'wr_dram%':>8s}")
    nan = float("nan")
    for (name, grid), a, us, n in rows[:40]:
        hit, miss = a.get("TCC_HIT_sum"), a.get("TCC_MISS_sum")
        l2 = 100 * hit / (hit + miss) if hit is not None and miss is not None and hit + miss > 0 else nan
        rq = a.get("TCC_EA0_RDREQ_sum")
        rmb = rq * 128 / 1e6 if rq is not None else nan
        dram = 100 * a["TCC_EA0_RDREQ_DRAM_sum"] / rq if rq and "TCC_EA0_RDREQ_DRAM_sum" in a else nan
        lat = a["TCC_EA0_RDREQ_LEVEL_sum"] / rq if rq and "TCC_EA0_RDREQ_LEVEL_sum" in a else nan
        wq = a.get("TCC_EA0_WRREQ_sum")
        wmb = wq * 64 / 1e6 if wq is not None else nan
        wd = 100 * a["TCC_EA0_WRREQ_DRAM_sum"] / wq if wq and "TCC_EA0_WRREQ_DRAM_sum" in a else nan
        print(f"{name[:58]:58s} {grid:8d} {n:4d} {us:8.1f} {l2:7.1f} {rmb:9.1f} {dram:6.1f} {lat:7.0f} {wmb:9.1f} {wd:8.1f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
