"""Diagnostic: per-step vs persistent encoder results (s16x3), where and how much they differ.
Run with CASR_FUSE_SPLIT=0/1 to separate the fused row-image store from the recurrence itself."""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "chinese-asr_amd"), os.path.join(ROOT, "tests")]
from golden_util import fbank_for
from casr.config import CasrConfig
from casr.lib import pack_weights
from casr.weights import synthetic_state_dicts
from casr.engine import Engine

CFG = CasrConfig()
B = int(sys.argv[1]) if len(sys.argv) > 1 else 37
e = Engine(CFG, *synthetic_state_dicts(CFG, peaked=True))
e.set_precision("s16x3")
rs = np.random.RandomState(11)
frames = rs.randint(9, 801, size=B)
frames[0], frames[-1] = 800, 9
x = np.zeros((B, 800, 80), np.float32)
for b in range(B):
    x[b, :frames[b]] = fbank_for(b, int(frames[b]))
feat, flen = e.features(torch.from_numpy(x).to(e.device), torch.from_numpy(frames.astype(np.int32)).to(e.device))
outs = []
for p in (False, True, True):
    e.set_persistent(p)
    e.encode(feat, flen)
    outs.append([t.cpu() for t in e.encoder_results()])
    print("flags", e.device_flags())
names = ["enc", "h", "c", "keys"]
for i, (a, b) in enumerate(zip(outs[0], outs[1])):
    d = (a - b).abs()
    nz = torch.nonzero(d > 0)
    print(names[i], tuple(a.shape), "maxdiff", float(d.max()), "n", len(nz), "first", nz[:5].tolist())
for i, (a, b) in enumerate(zip(outs[1], outs[2])):
    print("persistent rerun", names[i], "equal", torch.equal(a, b))
