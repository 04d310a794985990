"""casr_log_mel at B = 256 x 8 s of 16 kHz audio (the wav -> log-mel front end, data.py:167-224):
HIP-event time per launch and the algorithmic bytes (wav read + fbank written), for rocprofv3
--kernel-trace --stats / --pmc runs (tools/probes/logmel_profile.sh)."""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "chinese-asr_amd"))
from casr.config import CasrConfig  # noqa: E402
from casr.engine import Engine  # noqa: E402
from casr.weights import synthetic_state_dicts  # noqa: E402

B, N = int(os.environ.get("B", "256")), 8 * 16000
iters = int(os.environ.get("ITERS", "20"))
eng = Engine(CasrConfig(), *synthetic_state_dicts(CasrConfig(), peaked=True, eos_bias=0.0))
wav = torch.from_numpy((np.random.RandomState(0).standard_normal((B, N)) * 0.1).astype(np.float32)).cuda()
ns = torch.full((B,), N, dtype=torch.int32, device="cuda")
fb, fr = eng.log_mel(wav, ns)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(iters):
    eng.log_mel(wav, ns)
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) * 1000 / iters
T = fb.shape[1]
nbytes = B * N * 4 + B * T * 80 * 4
print(json.dumps({"B": B, "samples": N, "frames": T, "us_per_call": round(us, 2),
                  "algorithmic_bytes": nbytes, "GBps": round(nbytes / us / 1e3, 1),
                  "note": "HIP events around casr_log_mel on torch's current stream (one kernel per call)"}))
