"""Probe: does a second handle on a second HIP stream overlap batch i+1's encoder with batch i's
decode?  Greedy B = 256, T = 800, STEPS batches back to back: one handle on one stream (as
bench.py) against two handles alternating over two streams.  Prints ms per batch of each and
whether the tokens are identical and the guard bits clean."""
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "chinese-asr_amd"))
from casr.config import CasrConfig  # noqa: E402
from casr.engine import Engine  # noqa: E402
from casr.lib import pack_weights  # noqa: E402
from casr.weights import synthetic_state_dicts  # noqa: E402

B, T, STEPS = int(os.environ.get("B", 256)), 800, int(os.environ.get("STEPS", 20))
cfg = CasrConfig()
blob = torch.from_numpy(pack_weights(cfg, *synthetic_state_dicts(cfg, peaked=True, eos_bias=0.0))).cuda()
engs = [Engine(cfg, packed=blob) for _ in range(2)]
streams = [torch.cuda.current_stream(), torch.cuda.Stream()]
fb = torch.from_numpy(np.stack([np.random.RandomState(1234 + b).standard_normal((T, 80)).astype(np.float32)
                                for b in range(B)])).cuda()
frames = torch.full((B,), T, dtype=torch.int32, device="cuda")
outs = [torch.empty(B, cfg.max_len, dtype=torch.int32, pin_memory=True) for _ in range(4)]


def run(n, two):
    res = []
    for i in range(n):
        j = (i & 1) if two else 0
        with torch.cuda.stream(streams[j]):
            engs[j].encode_fbank(fb, frames)
            t = engs[j].greedy()["tokens"]
            h = outs[i % 4]
            h.copy_(t, non_blocking=True)
            res.append(h)
    return res


for two in (False, True, False, True):
    run(3, two)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = run(STEPS, two)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    same = all(torch.equal(r[0], x) for x in r[-4:])
    flags = [e.device_flags() for e in engs]
    print(f"{'two' if two else 'one'} stream(s): {1000 * dt / STEPS:.3f} ms per batch, "
          f"{B * STEPS / dt:.0f} utt/s, tokens identical {same}, flags {flags}", flush=True)
for e in engs:
    e.close()
