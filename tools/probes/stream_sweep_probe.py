"""Probe: batches in flight on one GPU (casr.pipeline.StreamPipeline) against the serial loop, per
workload: greedy B = 256 / 32, beam 8 B = 256 / 128.  Prints ms per batch per pipeline depth, and
checks each depth's tokens equal the serial loop's and the guard bits are clean."""
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "chinese-asr_amd"))
from casr.config import CasrConfig  # noqa: E402
from casr.lib import pack_weights  # noqa: E402
from casr.pipeline import StreamPipeline  # noqa: E402
from casr.weights import synthetic_state_dicts  # noqa: E402

T = 800
cfg = CasrConfig()
blob = torch.from_numpy(pack_weights(cfg, *synthetic_state_dicts(cfg, peaked=True, eos_bias=0.0))).cuda()
CASES = [("greedy", 256, 0, (1, 2, 3)), ("beam", 256, 8, (1, 2)), ("beam", 128, 8, (1, 2, 3)),
         ("greedy", 32, 0, (1, 2, 4, 8))]
STEPS = int(os.environ.get("STEPS", 12))
for mode, B, k, depths in CASES:
    fb = torch.from_numpy(np.stack([np.random.RandomState(1234 + b).standard_normal((T, 80)).astype(np.float32)
                                    for b in range(B)])).cuda()
    fr = torch.full((B,), T, dtype=torch.int32, device="cuda")
    ref = None
    for n in depths:
        pipe = StreamPipeline(cfg, blob, n=n)
        pins = [torch.empty(B, cfg.max_len, dtype=torch.int32, pin_memory=True) for _ in range(2 * n)]

        def step(e, i=[0]):
            e.encode_fbank(fb, fr)
            t = (e.beam(k) if k else e.greedy())["tokens"]
            h = pins[i[0] % len(pins)]
            i[0] += 1
            h.copy_(t, non_blocking=True)
            return h
        for _ in range(2 * n):
            pipe.submit(step)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        outs = [pipe.submit(step) for _ in range(STEPS)]
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / STEPS
        flags = pipe.device_flags()
        same = ref is None or all(torch.equal(ref, o) for o in outs[-2:])
        ref = outs[-1].clone() if ref is None else ref
        print(f"{mode} B={B} k={k} streams={n}: {1000 * dt:.3f} ms per batch, {B / dt:.0f} utt/s, "
              f"tokens equal to serial {same}, flags {flags}", flush=True)
        pipe.close()
