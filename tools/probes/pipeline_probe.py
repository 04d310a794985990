"""Throughput of back-to-back batches: sequential vs two engines on two streams (batch i+1's
features/encoder overlapping batch i's decode).  Diagnostics only."""
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

B, T, K = 256, 800, int(os.environ.get("STEPS", 8))
cfg = CasrConfig()
packed = torch.from_numpy(pack_weights(cfg, *synthetic_state_dicts(cfg, peaked=True, eos_bias=0.0))).cuda()
engines = [Engine(cfg, packed=packed), Engine(cfg, packed=packed)]
fb = torch.from_numpy(np.stack([np.random.RandomState(1234 + b).standard_normal((T, 80)).astype(np.float32)
                                for b in range(B)])).cuda()
frames = torch.full((B,), T, dtype=torch.int32, device="cuda")
streams = [torch.cuda.Stream(), torch.cuda.Stream()]
host = [torch.empty(B, cfg.max_len, dtype=torch.int32).pin_memory() for _ in range(2)]


def step(i, pipelined):
    e = engines[i & 1] if pipelined else engines[0]
    s = streams[i & 1] if pipelined else torch.cuda.current_stream()
    with torch.cuda.stream(s):
        feat, flen = e.features(fb, frames)
        e.encode(feat, flen)
        out = e.greedy()
        host[i & 1].copy_(out["tokens"], non_blocking=True)


for mode in (False, True, False, True):
    for i in range(2):
        step(i, mode)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(K):
        step(i, mode)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    flags = [e.device_flags() for e in engines]
    print(f"{'pipelined ' if mode else 'sequential'}: {1000 * dt / K:7.2f} ms/batch  {B * K / dt:9.1f} utt/s  flags {flags}",
          flush=True)
same = torch.equal(host[0], host[1]) if K > 1 else True
print("tokens of both engines equal:", same)
