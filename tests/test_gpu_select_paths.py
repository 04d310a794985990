"""The fused beam select's remaining paths, and beam 8 at B = 1024 on one GPU.

The folded beam step (R = B k >= 1024 decode rows, s16x3) runs the select of step l - 1 in step
l's attention prologue (attention.hip CELL 3: one block per utterance; CELL 4: two blocks, 4 rows
each).  test_gpu_parity.py compares that with the select launches at temperature 1, where the
select reads the projection's tile maxima.  Two more paths of the same code (beam_select.h):

  * temperature != 1 (model.py:834 divides the logits first): the select reads the full logit
    rows (beam_select_block<K2, false>: threshold candidates gathered with LDS atomics);
  * more candidates at the threshold than BS_CAP (256) -- a heavy tie: every element of the row
    through per-lane sorted lists (TopList + wave_merge).

Each is run with the select fused (CASR_OPT_FUSE_SELECT = 1, default) and as launches of its own
(0): tokens, lengths, scores, step counts and finished-hypothesis records equal bit for bit, and
the tokens equal to the CPU oracle's beam search (model.py:604-987; a tie is resolved to the lower
flat index there too: stable argsort).
"""
import numpy as np
import pytest
import torch

from golden_util import fbank_for
from oracle import casr_oracle as O
from casr.config import CasrConfig
from casr.weights import synthetic_state_dicts

pytestmark = pytest.mark.gpu


def _frames(B, seed, lo=30, hi=150):
    return np.random.RandomState(seed).randint(lo, hi, size=B).astype(np.int32)


def _run_fused_vs_launches(cfg, enc_sd, dec_sd, B, k, kpb, frames):
    from casr.engine import Engine
    e = Engine(cfg, enc_sd, dec_sd)
    e.set_precision("s16x3")
    outs = []
    try:
        T = int(frames.max())
        x = np.zeros((B, T, 80), np.float32)
        for b in range(B):
            x[b, :frames[b]] = fbank_for(b, int(frames[b]))
        e.encode_fbank(torch.from_numpy(x).to(e.device), torch.from_numpy(frames).to(e.device))
        e.set_option("ATTN_KPB", kpb)
        for fuse in (0, 1):
            e.set_option("FUSE_SELECT", fuse)
            e.profile(["select", "dec_lstm"])
            r = e.beam(k)
            rt, rs, rv = e.beam_records()
            prof = e.profile_read()
            e.profile([])
            assert e.device_flags() == 0
            assert prof["dec_lstm"][0] == 1, "the folded beam step"
            o = {n: v.cpu() for n, v in r.items()}
            o.update(rec_tokens=rt.cpu(), rec_score=rs.cpu(), rec_valid=rv.cpu())
            outs.append((o, prof["select"][0]))
    finally:
        e.set_option("FUSE_SELECT", 1)
        e.set_option("ATTN_KPB", 0)
        e.close()
    (a, na), (b, nb) = outs
    steps = int(a["steps"][0])
    assert na == steps and nb == 1, (na, nb)  # every select a launch / only the last step's
    for n in a:
        assert torch.equal(a[n], b[n]), n
    return b


@pytest.mark.parametrize("k,B,kpb", [(4, 256, 0), (8, 128, 0), (8, 256, 0), (8, 256, 4)])
def test_fused_select_temperature_07(k, B, kpb):
    """gpd['temperature'] = 0.7 at the folded beam shapes (k = 4, B = 256 and k = 8, B = 256: one
    attention block per utterance; k = 8 at B = 128, and at B = 256 with ATTN_KPB = 4: two blocks
    per utterance, both running the select).  Fused and launched selects bitwise equal; 8
    utterances against the oracle at the same temperature (tokens identical, scores 2e-3)."""
    cfg = CasrConfig(temperature=0.7)
    enc_sd, dec_sd = synthetic_state_dicts(cfg, peaked=True, eos_bias=0.0)
    frames = _frames(B, 31)
    r = _run_fused_vs_launches(cfg, enc_sd, dec_sd, B, k, kpb, frames)
    toks, blen, sc = (r[n].numpy() for n in ("tokens", "length", "score"))
    rows = list(range(0, B, B // 8))
    feats = [O.features_from_fbank(fbank_for(b, int(frames[b]))) for b in rows]
    ref = O.beam_decode(feats, [f.shape[0] for f in feats], enc_sd, dec_sd, k, temperature=0.7)
    assert [toks[b, :blen[b]].tolist() for b in rows] == ref["tokens"]
    np.testing.assert_allclose(sc[rows], ref["score"], rtol=0, atol=2e-3)


def _tied_weights(cfg, n_tied=400, first=700, lift=1000.0):
    """The bench recipe with n_tied vocabulary rows of the projection made identical (row `first`
    copied, the same bias lifted by `lift`): those tokens' logits are equal bit for bit in every
    row (the same products in the same order), and they are the top candidates of every beam row,
    so more than BS_CAP = 256 candidates sit exactly at the threshold.  (The lift must exceed the
    spread of the other logits, tens at the x40 peaking: a +30 lift left other tokens on top.)"""
    enc_sd, dec_sd = synthetic_state_dicts(cfg, peaked=True, eos_bias=0.0)
    W = dec_sd["proj_linear.weight"].copy()
    bias = dec_sd["proj_linear.bias"].copy()
    W[first:first + n_tied] = W[first]
    bias[first:first + n_tied] = bias[first] + lift
    dec_sd = dict(dec_sd)
    dec_sd["proj_linear.weight"], dec_sd["proj_linear.bias"] = W, bias
    return enc_sd, dec_sd


@pytest.mark.parametrize("k,B,kpb", [(8, 256, 0), (8, 128, 0)])
def test_fused_select_heavy_tie_past_bs_cap(k, B, kpb):
    """400 vocabulary entries tied exactly at the top of every row: the threshold candidates
    overflow BS_CAP and the select takes the sorted-list path over the whole row.  Fused and
    launched bitwise equal; every decoded token is from the tied block, the hypotheses run all 40
    steps, and 4 utterances equal the oracle's (its stable order resolves the ties to the lower
    flat index, as the select's better() does)."""
    cfg = CasrConfig()
    enc_sd, dec_sd = _tied_weights(cfg)
    frames = _frames(B, 33, 20, 60)
    r = _run_fused_vs_launches(cfg, enc_sd, dec_sd, B, k, kpb, frames)
    toks, blen = r["tokens"].numpy(), r["length"].numpy()
    assert (blen == cfg.max_len).all()  # no EOS can outrank the lifted block
    assert ((toks >= 700) & (toks < 1100)).all()
    rows = [0, B // 3, 2 * B // 3, B - 1]
    feats = [O.features_from_fbank(fbank_for(b, int(frames[b]))) for b in rows]
    ref = O.beam_decode(feats, [f.shape[0] for f in feats], enc_sd, dec_sd, k)
    assert [toks[b, :blen[b]].tolist() for b in rows] == ref["tokens"]


def test_beam8_b1024_one_gpu_equals_b256_batches():
    """bench.py's config-4 line at --gpus 1 decodes the whole 1,024-utterance global batch on one
    GPU (R = 8192 decode rows).  The same utterances as four B = 256 batches (R = 2048: the same
    decode-GEMM tile class) give the same tokens and lengths, and scores within 2e-4 (bit for bit
    expected; the tolerance covers another summation split)."""
    from casr.engine import Engine
    cfg = CasrConfig()
    T = 300
    e = Engine(cfg, *synthetic_state_dicts(cfg, peaked=True, eos_bias=0.0))
    try:
        fb = torch.from_numpy(np.stack([fbank_for(b, T) for b in range(1024)])).to(e.device)
        fr = torch.full((1024,), T, dtype=torch.int32, device=e.device)
        e.encode_fbank(fb, fr)
        full = {n: v.cpu() for n, v in e.beam(8).items()}
        assert e.device_flags() == 0
        for q in range(4):
            e.encode_fbank(fb[256 * q:256 * (q + 1)].contiguous(), fr[:256].contiguous())
            part = e.beam(8)
            assert e.device_flags() == 0
            assert torch.equal(full["tokens"][256 * q:256 * (q + 1)], part["tokens"].cpu())
            assert torch.equal(full["length"][256 * q:256 * (q + 1)], part["length"].cpu())
            np.testing.assert_allclose(full["score"][256 * q:256 * (q + 1)].numpy(), part["score"].cpu().numpy(),
                                       rtol=0, atol=2e-4)
    finally:
        e.close()
