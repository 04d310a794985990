"""Overlap of kernels on one GPU from a rocprofv3 --kernel-trace CSV (batches in flight).

For the dispatches inside [t0, t1] (default: the last `--window` ms of the trace, the timed region
of a bench run): the time with no kernel running, with one, with two or more; and per kernel class
the fraction of its run time during which another class's kernel ran beside it (on any queue).
Kernel classes: the short kernel name without template arguments.

usage: python tools/pipeline_timeline.py run_kernel_trace.csv [--window MS]
"""
import argparse
import csv
from collections import defaultdict


def load(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"].replace("(anonymous namespace)::", "")
            name = name[:name.index("(")] if "(" in name else name
            name = name.replace("void ", "").split("<")[0]
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    return sorted(rows)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--window", type=float, default=100.0, help="ms at the end of the trace")
    a = ap.parse_args()
    rows = load(a.csv)
    t1 = max(e for _, e, _ in rows)
    t0 = t1 - int(a.window * 1e6)
    rows = [(max(s, t0), e, n) for s, e, n in rows if e > t0]
    ev = sorted([(s, 1, i) for i, (s, e, n) in enumerate(rows)] + [(e, -1, i) for i, (s, e, n) in enumerate(rows)])
    level = defaultdict(int)  # concurrency level -> ns
    beside = defaultdict(int)  # class -> ns with another class running beside it
    own = defaultdict(int)     # class -> ns it ran (union over its own dispatches)
    live = set()
    prev = t0
    for t, kind, i in ev:
        if t > prev:
            dt = t - prev
            level[min(len(live), 2)] += dt
            classes = {rows[j][2] for j in live}
            for c in classes:
                own[c] += dt
                if len(classes) > 1:
                    beside[c] += dt
            prev = t
        if kind > 0:
            live.add(i)
        else:
            live.discard(i)
    span = t1 - t0
    print(f"window {span / 1e6:.2f} ms, {len(rows)} dispatches")
    print(f"  idle {level[0] / 1e6:8.3f} ms ({level[0] / span:.1%})   one kernel {level[1] / 1e6:8.3f} ms "
          f"({level[1] / span:.1%})   two or more {level[2] / 1e6:8.3f} ms ({level[2] / span:.1%})")
    print(f"  {'class':34s} {'run ms':>8s} {'share':>7s} {'beside another class':>22s}")
    for c in sorted(own, key=lambda c: -own[c]):
        print(f"  {c[:34]:34s} {own[c] / 1e6:8.3f} {own[c] / span:7.1%} {beside[c] / max(own[c], 1):22.1%}")


if __name__ == "__main__":
    main()
