"""Runs casr_encode_fbank's feature kernels a few times at B=256, T=800 (for rocprofv3 --stats)."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "chinese-asr_amd"))
from casr.config import CasrConfig  # noqa: E402
from casr.engine import Engine  # noqa: E402
from casr.weights import synthetic_state_dicts  # noqa: E402

B, T = 256, 800
eng = Engine(CasrConfig(), *synthetic_state_dicts(CasrConfig(), peaked=True, eos_bias=0.0))
fb = torch.from_numpy(np.random.RandomState(0).standard_normal((B, T, 80)).astype(np.float32)).cuda()
frames = torch.full((B,), T, dtype=torch.int32, device="cuda")
for _ in range(5):
    eng.features(fb, frames)
torch.cuda.synchronize()
print("ok")
