"""Per-(kernel, grid) durations from a rocprofv3 --kernel-trace CSV.

The --stats summary averages every dispatch of a kernel, mixing the greedy (B = 256) and beam
(B = 128) encodes of one bench.py run.  This splits dispatches by launch grid so the average
duration of the bench line's dominant kernel at the headline configuration can be compared
with bench.py's own HIP-event figure (roofline.avg_launch_us).

usage: python tools/prof_by_grid.py gpurun_out/prof/run_kernel_trace.csv [top_n]
"""
import csv
import sys
from collections import defaultdict


def main(path, top=25):
    acc = defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"].replace("(anonymous namespace)::", "")
            short = name[:name.index("(")] if "(" in name else name
            grid = tuple(int(r[f"Grid_Size_{a}"]) // max(1, int(r[f"Workgroup_Size_{a}"])) for a in "XYZ")
            wg = int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]) * int(r["Workgroup_Size_Z"])
            acc[(short, grid, wg)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    rows = sorted(acc.items(), key=lambda kv: -sum(kv[1]))
    print(f"{'kernel':58s} {'workgroups (x,y,z) x threads':30s} {'calls':>6s} {'avg_us':>10s} {'median_us':>10s} "
          f"{'total_ms':>9s}")
    for (name, grid, wg), d in rows[:top]:
        med = sorted(d)[len(d) // 2]
        print(f"{name[:58]:58s} {str(grid) + ' x ' + str(wg):30s} {len(d):6d} {sum(d) / len(d):10.2f} {med:10.2f} "
              f"{sum(d) / 1e3:9.2f}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 25)
