"""Every counter of rocprofv3 --pmc passes, averaged per dispatch, for the kernels whose short
name starts with a prefix (tools/pmc_summary.py prints only the derived columns).  Also the
per-dispatch cycle figures the input-GEMM diagnosis uses:
  clock    = GRBM_GUI_ACTIVE / 8 / duration     (GRBM sums the 8 XCDs)
  SQ_* counters in quad-cycles are left as reported (MI355X_MICROARCH.md: SQ_WAVE_CYCLES, SQ_WAIT_*,
  SQ_ACTIVE_INST_* count quad-cycles; SQ_VALU_MFMA_BUSY_CYCLES counts cycles)

usage: python tools/pmc_dump.py gpurun_out/x/pmc_greedy gemm16_pp_kernel [more prefixes]
"""
import sys

from pmc_summary import load


def main(d, prefixes):
    per, dur = load(d)
    for (name, grid), cs in sorted(per.items(), key=lambda kv: kv[0]):
        if not any(name.startswith(p) for p in prefixes):
            continue
        us = sum(dur[(name, grid)].values()) / max(1, len(dur[(name, grid)]))
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        n = max(len(v) for v in cs.values())
        print(f"== {name} grid {grid}: {n} dispatches, {us:.1f} us average")
        g = avg.get("GRBM_GUI_ACTIVE")
        if g:
            print(f"   clock {g / 8 / (us * 1e3):.3f} GHz ({g / 8:.0f} cycles per XCD)")
        for c in sorted(avg):
            print(f"   {c:32s} {avg[c]:18.1f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
