"""Per-block phase stamps of the decode GEMMs (CASR_DG_TRACE diagnostics; GPU box).

One greedy decode at B x T; the stamps of the last launch of each GEMM class (s_memrealtime,
100 MHz) are split into prologue (row binding + first ring stages issued), first tile landed,
k loop, epilogue."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "chinese-asr_amd"))
PATH = "/tmp/dg_trace.bin"
os.environ["CASR_DG_TRACE"] = PATH
from casr.config import CasrConfig  # noqa: E402
from casr.engine import Engine  # noqa: E402
from casr.weights import synthetic_state_dicts  # noqa: E402

B, T = int(os.environ.get("B", 256)), 800


def attn_report(r, title, sub=True):
    r = r[r[:, 0] > 0]
    t = (r[:, :6] - r[:, 0].min()) * 10 / 1000.0
    print(f"{title}: {len(r)} blocks, span {t[:, 5].max():.2f} us")
    for i, n in enumerate(["q partials", "scores", "softmax", "context", "reduce+store"]):
        v = t[:, i + 1] - t[:, i]
        print(f"  {n:14s} p10 {np.percentile(v, 10):6.2f}  p50 {np.percentile(v, 50):6.2f}  p90 {np.percentile(v, 90):6.2f}")
    v = t[:, 0]
    print(f"  {'start':14s} p10 {np.percentile(v, 10):6.2f}  p50 {np.percentile(v, 50):6.2f}  p90 {np.percentile(v, 90):6.2f}")
    if sub and (r[:, 6] > 0).all() and (r[:, 7] > 0).all():  # the folded greedy prologue (CELL 1 stamps 6, 7)
        t6 = (r[:, 6] - r[:, 0].min()) * 10 / 1000.0
        t7 = (r[:, 7] - r[:, 0].min()) * 10 / 1000.0
        for n, v in (("  select", t6 - t[:, 0]), ("  cell", t7 - t6), ("  query", t[:, 1] - t7)):
            print(f"  {n:14s} p10 {np.percentile(v, 10):6.2f}  p50 {np.percentile(v, 50):6.2f}  p90 {np.percentile(v, 90):6.2f}")
def gemm_report(raw, tag):
    for cls, name in ((0, "dec_lstm"), (1, "proj")):
        r = raw[cls]
        bid = np.nonzero(r[:, 0] > 0)[0]  # blockIdx.x of the stamped blocks
        r = r[bid]
        t = (r[:, :5] - r[:, 0].min()) * 10 / 1000.0  # us
        span = t[:, 4].max()
        ph = {"start": t[:, 0], "prologue": t[:, 1] - t[:, 0], "first tile": t[:, 2] - t[:, 1],
              "k loop": t[:, 3] - t[:, 2], "epilogue": t[:, 4] - t[:, 3], "block": t[:, 4] - t[:, 0]}
        print(f"{name} ({tag}): {len(r)} blocks, span {span:.2f} us")
        for k, v in ph.items():
            print(f"  {k:12s} p10 {np.percentile(v, 10):6.2f}  p50 {np.percentile(v, 50):6.2f}  "
                  f"p90 {np.percentile(v, 90):6.2f}  max {v.max():6.2f}")
        if os.environ.get("CASR_DG_TRACE_STEP") and cls == 1 and (r[:, 7] > 0).all():
            # one step's fused GEMM: blocks by column-block kind (words 5-7: nb, rb, NB) and by XCD
            nb, nt = r[:, 5], int(os.environ.get("NTN", 14))
            V = 5004
            kind = np.where((nb + 1) * nt * 16 <= V, 0, np.where(nb * nt * 16 < V, 1, 2))
            xcd = bid % 8
            for kk, kn in enumerate(("vocabulary", "boundary", "gates")):
                m = kind == kk
                if m.any():
                    print(f"    {kn:10s} {m.sum():3d} blocks: k loop p50 {np.median(ph['k loop'][m]):6.2f} max "
                          f"{ph['k loop'][m].max():6.2f}  epilogue p50 {np.median(ph['epilogue'][m]):6.2f} max "
                          f"{ph['epilogue'][m].max():6.2f}  end p50 {np.median(t[m, 4]):6.2f} max {t[m, 4].max():6.2f}")
            ends = " ".join(f"{t[xcd == x, 4].max():6.2f}" for x in range(8) if (xcd == x).any())
            print(f"    end max per blockIdx % 8: {ends}")


cfg = CasrConfig()
eng = Engine(cfg, *synthetic_state_dicts(cfg, peaked=True, eos_bias=0.0))
fb = torch.from_numpy(np.stack([np.random.RandomState(1234 + b).standard_normal((T, 80)).astype(np.float32)
                                for b in range(B)])).cuda()
feat, flen = eng.features(fb, torch.full((B,), T, dtype=torch.int32, device="cuda"))
eng.encode(feat, flen)
eng.greedy()["tokens"].cpu()
eng.greedy()["tokens"].cpu()
if os.environ.get("BEAM"):
    BB = int(os.environ.get("BB", 128))
    eng.encode(feat[:BB].contiguous(), flen[:BB].contiguous())
    kb = int(os.environ.get("K", 8))
    eng.beam(kb)["tokens"].cpu()
    eng.beam(kb)["tokens"].cpu()
    raw = np.fromfile(PATH, dtype=np.uint32).reshape(4, 4096, 8).astype(np.int64)
    r = raw[2]
    r = r[r[:, 0] > 0]
    t = (r[:, :7] - r[:, 0].min()) * 10 / 1000.0
    attn_report(raw[3], "attention (beam)", sub=False)
    gemm_report(raw, "beam")
    names = ["lse+partials", "tau+offer", "list insert", "row merge", "block merge", "bookkeeping"]
    print(f"beam_select: {len(r)} blocks, span {t[:, 6].max():.2f} us, candidates (wave 0) p50 {np.median(r[:, 7]):.0f} max {r[:, 7].max()}")
    for i, n in enumerate(names):
        v = t[:, i + 1] - t[:, i]
        print(f"  {n:14s} p10 {np.percentile(v, 10):6.2f}  p50 {np.percentile(v, 50):6.2f}  p90 {np.percentile(v, 90):6.2f}")
    sys.exit(0)
raw = np.fromfile(PATH, dtype=np.uint32).reshape(4, 4096, 8).astype(np.int64)
attn_report(raw[3], "attention (greedy)")
gemm_report(raw, "greedy")
