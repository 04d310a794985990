"""GPU diagnostic: decode flags / parity for graph vs eager on the golden suites."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "chinese-asr_amd"), os.path.join(REPO, "tests")]
import numpy as np, torch
from golden_util import load_golden, fbank_for, golden_frames
from casr.config import CasrConfig
from casr.engine import Engine
from casr.lib import pack_weights
from casr.results import greedy_outputs
from casr.weights import synthetic_state_dicts
G, META = load_golden(); CFG = CasrConfig(); FR = golden_frames(META)
x = np.zeros((len(FR), max(FR), 80), np.float32)
for b, t in enumerate(FR): x[b, :t] = fbank_for(b, t)
eng = Engine(CFG, *synthetic_state_dicts(CFG, peaked=False))
fb = torch.from_numpy(x).cuda(); fr = torch.tensor(FR, dtype=torch.int32).cuda()
for name in ("plain", "peaked", "plain", "peaked"):
    eng.bind(pack_weights(CFG, *synthetic_state_dicts(CFG, peaked=(name == "peaked"))))
    for graphs in (False, True):
        eng.set_graphs(graphs)
        feat, flen = eng.features(fb, fr)
        eng.encode(feat, flen)
        out = eng.greedy(alignment=True)
        f = eng.device_flags()
        toks, _ = greedy_outputs(out["tokens"].cpu().numpy(), out["out_len"].cpu().numpy(),
                                 out["finished"].cpu().numpy().astype(bool), out["accum"].cpu().numpy())
        ok = toks == META[name]["greedy"]["tokens"]
        al = out["alignment"].cpu().numpy()
        print(f"{name} graphs={graphs} flags={f} tokens_ok={ok} align_nan={np.isnan(al).sum()} "
              f"lens={out['out_len'].cpu().tolist()} first_tok={out['tokens'][:, :3].cpu().tolist()}", flush=True)
