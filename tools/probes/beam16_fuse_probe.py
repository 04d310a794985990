"""Beam 16 at B = 256 (BASELINE config 5's device batch), T = 800: ms per batch (encode + beam +
records) over the values of one option, interleaved rounds (default: CASR_OPT_FUSE_SELECT 1 / 0;
env AB_OPT / AB_VALS for another, AB_BITWISE=0 when its values are numerics variants); outputs
compared bit for bit."""
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
OPT = os.environ.get("AB_OPT", "FUSE_SELECT")
VALS = [int(v) for v in os.environ.get("AB_VALS", "1,0").split(",")]
for rnd in range(4):
    for fuse in VALS:
        e.set_option(OPT, fuse)
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
        if os.environ.get("AB_BITWISE", "1") == "1":
            assert all(torch.equal(x, y) for x, y in zip(ref["ref"], out)), "the option's values differ in bits"
        print(f"[{rnd}] {OPT}={fuse}: {a.elapsed_time(b) / 5:.3f} ms per batch", flush=True)
assert e.device_flags() == 0
print("done")
