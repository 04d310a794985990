"""A/B of one tuning option (include/casr.h CASR_OPT_*, speed only) on the bench workload (B = 256,
T = 800, synthetic weights): greedy and / or beam 8, interleaved rounds over the values given, every
output compared bit for bit against the first value's, per-class times from the handle's profiler
(ms per batch) and the whole batch from HIP events.
usage: python tools/probes/option_ab.py OPTION v1,v2,... [rounds] [greedy,beam]
(round 5: DG_PREFETCH 0,1,2,4,8, a since-removed L2-touch option of the fused GEMM,
profiles/r05/dg_prefetch/; FUSE_SELECT 1,0 for the beam select in the attention prologue)"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "chinese-asr_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import fbank_batch  # noqa: E402
from casr.config import CasrConfig  # noqa: E402
from casr.engine import Engine  # noqa: E402
from casr.lib import pack_weights  # noqa: E402
from casr.weights import synthetic_state_dicts  # noqa: E402


def main():
    opt = sys.argv[1]
    dists = [int(x) for x in sys.argv[2].split(",")]
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    modes = sys.argv[4].split(",") if len(sys.argv) > 4 else ["greedy", "beam"]
    dev = torch.device("cuda", 0)
    cfg = CasrConfig()
    packed = torch.from_numpy(pack_weights(cfg, *synthetic_state_dicts(cfg, peaked=True, eos_bias=0.0))).to(dev)
    eng = Engine(cfg, packed=packed, device=dev)
    eng.set_precision("s16x3")
    B, T = 256, 800
    fb = torch.from_numpy(fbank_batch(0, B, T)).to(dev)
    frames = torch.full((B,), T, dtype=torch.int32, device=dev)
    eng.encode_fbank(fb, frames)
    torch.cuda.synchronize()

    def run(mode):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        eng.profile(["attention", "proj", "select", "dec_lstm"])
        ev[0].record()
        out = eng.greedy() if mode == "greedy" else eng.beam(8)
        ev[1].record()
        torch.cuda.synchronize()
        prof = eng.profile_read()
        eng.profile([])
        if mode == "beam":
            out = dict(out, **dict(zip(("rec_tokens", "rec_score", "rec_valid"), eng.beam_records())))
        res = {k: v.detach().cpu().numpy().copy() for k, v in out.items() if torch.is_tensor(v)}
        return ev[0].elapsed_time(ev[1]), {k: round(v[1], 4) for k, v in prof.items()}, res

    ref = {}
    log = {m: {d: [] for d in dists} for m in modes}
    for r in range(rounds):
        for d in dists:
            eng.set_option(opt, d)
            for mode in modes:
                run(mode)  # warm (and the graph / table state for this setting)
                ms, prof, res = run(mode)
                if mode not in ref:
                    ref[mode] = res
                else:
                    for k in ref[mode]:
                        if not np.array_equal(ref[mode][k], res[k], equal_nan=True):
                            raise SystemExit(f"MISMATCH {mode} {opt}={d} output {k}")
                log[mode][d].append({"batch": round(ms, 4), **prof})
                print(json.dumps({"round": r, "mode": mode, "dist": d, "batch_ms": round(ms, 4), **prof}), flush=True)
        flags = eng.device_flags()
        if flags:
            raise SystemExit(f"device flags {flags}")
    print("SUMMARY", json.dumps({m: {d: {c + "_ms_median": float(np.median([x.get(c, 0.0) for x in v]))
                                              for c in ("batch", "attention", "proj", "select")}
                                          for d, v in log[m].items()} for m in log}), flush=True)
    print(f"bitwise equal across {opt} values: yes")


if __name__ == "__main__":
    main()
