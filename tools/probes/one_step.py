"""STEPS (default 2) greedy steps at the headline config (B=256, T=800) for PMC collection
(rocprofv3 --pmc passes); runs the same launches as bench.py's step (casr_encode_fbank, greedy).  BEAM=k: a beam step instead (set B
too, e.g. B=128 BEAM=8 for the bench's beam line)."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "chinese-asr_amd"))
from casr.config import CasrConfig  # noqa: E402
from casr.engine import Engine  # noqa: E402
from casr.weights import synthetic_state_dicts  # noqa: E402

B, T = int(os.environ.get("B", 256)), 800
cfg = CasrConfig()
eng = Engine(cfg, *synthetic_state_dicts(cfg, peaked=True, eos_bias=0.0))
fb = torch.from_numpy(np.stack([np.random.RandomState(1234 + b).standard_normal((T, 80)).astype(np.float32)
                                for b in range(B)])).cuda()
frames = torch.full((B,), T, dtype=torch.int32, device="cuda")
for _ in range(int(os.environ.get("STEPS", 2))):
    eng.encode_fbank(fb, frames)  # as bench.py's step: features straight into the layer-0 image
    if int(os.environ.get("BEAM", 0)):
        eng.beam(int(os.environ["BEAM"]))
    else:
        eng.greedy()["tokens"].cpu()
torch.cuda.synchronize()
print("ok")
