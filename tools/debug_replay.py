"""GPU diagnostic: encoder / decoder graph replay vs eager on one weight set."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "chinese-asr_amd"), os.path.join(REPO, "tests")]
import numpy as np, torch
from golden_util import load_golden, fbank_for, golden_frames
from casr.config import CasrConfig
from casr.engine import Engine
from casr.weights import synthetic_state_dicts
G, META = load_golden(); CFG = CasrConfig(); FR = golden_frames(META)
x = np.zeros((len(FR), max(FR), 80), np.float32)
for b, t in enumerate(FR): x[b, :t] = fbank_for(b, t)
eng = Engine(CFG, *synthetic_state_dicts(CFG, peaked=True))
fb = torch.from_numpy(x).cuda(); fr = torch.tensor(FR, dtype=torch.int32).cuda()
feat, flen = eng.features(fb, fr)

def run(graphs, tag):
    eng.set_graphs(graphs)
    eng.encode(feat, flen)
    enc, h, c, keys = (t.clone() for t in eng.encoder_results())
    out = eng.greedy(alignment=False)
    torch.cuda.synchronize()
    return tag, enc, h, c, keys, out["tokens"].clone(), out["out_len"].clone(), eng.device_flags()

ref = run(False, "eager")
for tag in ("graph1", "graph2", "graph3"):
    r = run(True, tag)
    print(tag, "enc", torch.equal(r[1], ref[1]), "h", torch.equal(r[2], ref[2]), "c", torch.equal(r[3], ref[3]),
          "keys", torch.equal(r[4], ref[4]), "tok", torch.equal(r[5], ref[5]), "len", torch.equal(r[6], ref[6]),
          "flags", r[7], flush=True)
# decoder-only replay: encode eagerly, decode with graphs twice
eng.set_graphs(False); eng.encode(feat, flen); eng.set_graphs(True)
for i in range(3):
    o = eng.greedy(alignment=False); torch.cuda.synchronize()
    print("dec-only graph", i, "tok", torch.equal(o["tokens"], ref[5]), "len", torch.equal(o["out_len"], ref[6]),
          "flags", eng.device_flags(), flush=True)
# encoder-only replay: encode with graphs, decode eagerly
for i in range(3):
    eng.set_graphs(True); eng.encode(feat, flen); eng.set_graphs(False)
    o = eng.greedy(alignment=False); torch.cuda.synchronize()
    enc = eng.encoder_results()[0]
    print("enc-only graph", i, "enc", torch.equal(enc, ref[1]), "tok", torch.equal(o["tokens"], ref[5]), flush=True)
