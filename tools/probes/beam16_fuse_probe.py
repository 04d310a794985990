"""Beam 16 at B = 256 (BASELINE config 5's device batch), T = 800: ms per batch (encode + beam +
records) with the select fused in the attention (CASR_OPT_FUSE_SELECT = 1) and as launches (0),
interleaved rounds; every output of the two forms compared bit for bit."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "chinese-asr_amd"))
sys.path.insert(0, REPO)
from bench import fbank_batch  # noqa: E402
from casr.config import CasrConfig  # noqa: E402
from casr.engine import Engine  # noqa: E402
from casr.weights import synthetic_state_dicts  # noqa: E402

cfg = CasrConfig()
e = Engine(cfg, *synthetic_state_dicts(cfg, peaked=True))
B, T = 256, 800
fb = torch.from_numpy(fbank_batch(0, B, T)).cuda()
fr = torch.full((B,), T, dtype=torch.int32, device="cuda")


def run():
    e.encode_fbank(fb, fr)
    r = e.beam(16, 1.5, 1.5)
    return [*r.values(), *e.beam_records()]


ref = {}
for rnd in range(4):
    for fuse in (1, 0):
        e.set_option("FUSE_SELECT", fuse)
        run()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(5):
            out = run()
        b.record()
        torch.cuda.synchronize()
        out = [t.cpu() for t in out]
        if "ref" not in ref:
            ref["ref"] = out
        assert all(torch.equal(x, y) for x, y in zip(ref["ref"], out)), "fused and launched selects differ"
        print(f"[{rnd}] FUSE_SELECT={fuse}: {a.elapsed_time(b) / 5:.3f} ms per batch", flush=True)
assert e.device_flags() == 0
print("bitwise equal across the two forms: yes")
