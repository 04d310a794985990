"""Per-class milliseconds per step from a rocprofv3 kernel trace (tools/gpu_session.sh profbeam:
tools/probes/one_step.py, STEPS steps of one workload) beside a bench.py line's HIP-event classes
for the same workload (one instrumented step), and their ratio.

usage: python tools/prof_vs_bench.py TRACE.csv STEPS BENCH.json LINE
  LINE: "greedy" (the headline), "beam" (the metric's beam line) or "config3_beam8_b128"
"""
import csv
import json
import sys
from collections import defaultdict

from pmc_summary import CLASS_OF, matches, short


def main(trace, steps, bench, line):
    steps = int(steps)
    tot = defaultdict(float)
    calls = defaultdict(int)
    with open(trace) as f:
        for r in csv.DictReader(f):
            name = short(r["Kernel_Name"])
            for cls, (pres, _) in CLASS_OF.items():
                if matches(name, pres):
                    tot[cls] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
                    calls[cls] += 1
    with open(bench) as f:
        d = json.loads(f.read().strip().splitlines()[-1])
    kb = d["kernel_breakdown_ms"] if line == "greedy" else d[line]["kernel_breakdown_ms"]
    print(f"{'class':12s} {'rocprof ms/step':>16s} {'launches/step':>14s} {'bench ms/step':>14s} {'rocprof/bench':>14s}")
    for cls in CLASS_OF:
        if cls not in tot and cls not in kb:
            continue
        r = tot.get(cls, 0.0) / steps
        b = kb.get(cls)
        ratio = f"{r / b:14.3f}" if b else f"{'-':>14s}"
        print(f"{cls:12s} {r:16.3f} {calls.get(cls, 0) / steps:14.1f} {b if b is not None else float('nan'):14.3f} {ratio}")


if __name__ == "__main__":
    main(*sys.argv[1:5])
