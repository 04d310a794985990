"""Dump the product's beam-16 finished-hypothesis records for BASELINE config 5's whole-shard test
(B = 64, T = 800, EOS-bias weights, lm_weight = length_weight = 1.5) in both arithmetics, for the
near-tie analysis of tools/probes/beam_tie_probe.py (run in the build container against the oracle).
usage (GPU box): python tools/probes/config5_records_dump.py gpurun_out/x/config5_records.npz"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "chinese-asr_amd"), os.path.join(REPO, "tests")]
from casr.config import CasrConfig  # noqa: E402
from casr.engine import Engine  # noqa: E402
from casr.weights import synthetic_state_dicts  # noqa: E402
from golden_util import fbank_for  # noqa: E402

B, K, T = 64, 16, 800
cfg = CasrConfig()
out = {}
fb = np.stack([fbank_for(b, T) for b in range(B)])
for prec in ("s16x3", "f32"):
    e = Engine(cfg, *synthetic_state_dicts(cfg, peaked=True))
    e.set_precision(prec)
    e.encode_fbank(torch.from_numpy(fb).to(e.device), torch.full((B,), T, dtype=torch.int32, device=e.device))
    r = e.beam(K, 1.5, 1.5)
    for n, v in r.items():
        out[f"{prec}_{n}"] = v.cpu().numpy()
    for n, v in zip(("rec_tokens", "rec_score", "rec_valid"), e.beam_records()):
        out[f"{prec}_{n}"] = v.cpu().numpy()
    assert e.device_flags() == 0
    e.close()
np.savez_compressed(sys.argv[1], **out)
print("ok", sys.argv[1])
