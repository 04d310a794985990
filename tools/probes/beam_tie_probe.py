"""Near-tie analysis of beam parity (build container, CPU): the product's config-5 whole-shard records
(tools/probes/config5_records_dump.py, run on the GPU box) against the oracle's, and for every
utterance whose records diverge, the oracle's candidate score gaps at the pruning boundaries of each
step up to the divergence (model.py:834-901: the top-2k candidate list, the first k of it whose EOS
candidates are recorded, the first k non-EOS that stay active).  A divergence is a near tie when some
boundary gap before it is at the f32 rounding level of scores of magnitude ~40 (ulp 3.8e-6).
usage: python tools/probes/beam_tie_probe.py gpurun_out/r05b/config5_records.npz"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "chinese-asr_amd"), os.path.join(REPO, "tests"),
                os.path.join(REPO, "tests", "golden")]
from casr.config import CasrConfig  # noqa: E402
from casr.results import records_by_utterance  # noqa: E402
from casr.weights import synthetic_state_dicts  # noqa: E402
from golden_util import fbank_for  # noqa: E402
from oracle import casr_oracle as O  # noqa: E402
from stub_lm import StubLM, pua_int2word  # noqa: E402

F32 = np.float32
CFG = CasrConfig()
B, K, T = 64, 16, 800


def boundary_gaps(feat, enc_sd, dec_sd, k, steps):
    """One utterance's beam search as O.beam_decode (no early stop), returning per step the gaps
    (top-2k list rank 2k-1 vs 2k, record rank k-1 vs k, active k-th vs (k+1)-th non-EOS) and the
    record list."""
    V = dec_sd["proj_linear.weight"].shape[0]
    enc, (h, c) = O.encoder_forward([feat], [feat.shape[0]], enc_sd)
    mask = O.mask_for_softmax(np.array([feat.shape[0]]))
    keys = O.compute_keys(enc, dec_sd)
    rep = np.zeros(k, np.int64)
    enc_t, mask_t, keys_t = enc[:, rep], mask[:, rep], keys[:, rep]
    h, c = h[rep], c[rep]
    ctx = np.zeros((k, enc.shape[2]), F32)
    hist = np.zeros((steps + 1, k), np.int64)
    hist[0] = CFG.sos
    score = np.zeros(k, F32)
    out, recs = [], []
    for l in range(steps):
        logit, h, c, ctx, _ = O.decoder_step(enc_t, mask_t, keys_t, hist[l], h, c, ctx, dec_sd)
        logp = (O._log_softmax(logit) + score[:, None]).astype(F32)
        s = logp.reshape(-1)
        if l == 0:
            s = s[:V]
        order = np.argsort(-s, kind="stable")[:4 * k]
        cs = s[order]
        tok = order % V
        ne = np.nonzero(tok != CFG.eos)[0]
        g_list = float(cs[2 * k - 1] - cs[2 * k])
        g_rec = float(cs[k - 1] - cs[k])
        g_act = float(cs[ne[k - 1]] - cs[ne[k]]) if len(ne) > k and ne[k] < 2 * k else float("inf")
        out.append((l, g_list, g_rec, g_act))
        for j in range(k):
            if tok[j] == CFG.eos:
                recs.append((hist[1:l + 1, order[j] // V].tolist(), float(cs[j])))
        top = np.argsort(np.arange(2 * k) + (tok[:2 * k] == CFG.eos) * 2 * k, kind="stable")[:k]
        bsel = order[top] // V
        h, c, ctx = h[bsel], c[bsel], ctx[bsel]
        hist = hist[:, bsel]
        hist[l + 1] = tok[top]
        score = cs[top].astype(F32)
    return out, recs


def main(path):
    z = np.load(path)
    enc_sd, dec_sd = synthetic_state_dicts(CFG, peaked=True)
    feats = [O.features_from_fbank(fbank_for(b, T)) for b in range(B)]
    ref = O.beam_decode(feats, [f.shape[0] for f in feats], enc_sd, dec_sd, K, second_pass=True, lm_model=StubLM(),
                        lm_weight=1.5, length_weight=1.5, int2word=pua_int2word(CFG.vocab))
    for prec in ("s16x3", "f32"):
        recs = records_by_utterance(z[f"{prec}_rec_tokens"], z[f"{prec}_rec_score"], z[f"{prec}_rec_valid"])
        flips = []
        worst = 0.0
        for b in range(B):
            mine, gold = recs.get(b, []), ref["records"][b]
            n = min(len(mine), len(gold))
            d = next((i for i in range(n) if mine[i][0] != gold[i][0]), None)
            if d is None and len(mine) == len(gold):
                worst = max([worst] + [abs(x[1] - y[1]) for x, y in zip(mine, gold)])
                continue
            d = n if d is None else d
            flips.append((b, d))
        print(f"{prec}: {len(flips)} of {B} utterances diverge; max record score diff elsewhere {worst:.2e}")
        for b, d in flips:
            mine, gold = recs.get(b, []), ref["records"][b]
            step = min(len(mine[d][0]) if d < len(mine) else 99, len(gold[d][0]) if d < len(gold) else 99)
            gaps, _ = boundary_gaps(feats[b], enc_sd, dec_sd, K, min(step + 1, CFG.max_len))
            tight = sorted(((min(g[1], g[2], g[3]), g[0]) for g in gaps))[:3]
            print(f"  utt {b}: records identical up to #{d} (step {step}); "
                  f"ours {mine[d][1] if d < len(mine) else None}, oracle {gold[d][1] if d < len(gold) else None}; "
                  f"tightest boundary gaps up to that step (gap, step): {[(f'{g:.2e}', s) for g, s in tight]}")


if __name__ == "__main__":
    main(sys.argv[1])
