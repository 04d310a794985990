"""Features (f32, CMVN) and the layer-0 s16 image path (encode_fbank results) with the library at
argv[1], saved to argv[2] (.npz): compare two builds bit for bit (feat_bitwise.sh)."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "chinese-asr_amd"))
import casr.lib  # noqa: E402

casr.lib.load(sys.argv[1])
from casr.config import CasrConfig  # noqa: E402
from casr.engine import Engine  # noqa: E402
from casr.weights import synthetic_state_dicts  # noqa: E402

eng = Engine(CasrConfig(), *synthetic_state_dicts(CasrConfig(), peaked=True, eos_bias=0.0))
rs = np.random.RandomState(0)
out = {}
for name, frames in (("b256", [800] * 256), ("ragged", [800, 6, 7, 8, 9, 10, 11, 12, 101, 797, 798, 799, 1024, 640])):
    T = max(frames)
    fb = torch.from_numpy(rs.standard_normal((len(frames), T, 80)).astype(np.float32)).cuda()
    fr = torch.tensor(frames, dtype=torch.int32, device="cuda")
    feat, flen = eng.features(fb, fr)
    out[name + "_feat"] = feat.cpu().numpy()
    out[name + "_nocmvn"] = eng.features(fb, fr, eps=-1.0)[0].cpu().numpy()
    eng.encode_fbank(fb, fr)
    out[name + "_enc"] = eng.encoder_results()[0].cpu().numpy()
np.savez(sys.argv[2], **out)
print("saved", sys.argv[2])
