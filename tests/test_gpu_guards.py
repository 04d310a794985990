"""The guards that send a decode back to the three-launch step (casr_capi.hip prepare_decode), and
the select paths of vocabularies past the projection's partial blocks, against the CPU oracle.

Each guard is a shape the folded step cannot take; a regression in one of them would not fail
loudly but give wrong tokens (a counter read past the prologue's 64 lanes, an LDS area past
160 KiB, a one-accumulator GEMM on weights it cannot carry).  So every test asserts which step ran
(the LSTMCell GEMM's launch count: max_len = three-launch step, 1 = folded) and checks the tokens
against the oracle.  Tolerances as in test_gpu_parity.py: token ids identical, scores 2e-3 abs.
"""
import numpy as np
import pytest
import torch

from golden_util import fbank_for
from oracle import casr_oracle as O
from casr.config import CasrConfig
from casr.lib import pack_weights
from casr.results import greedy_outputs
from casr.weights import synthetic_state_dicts

pytestmark = pytest.mark.gpu

PRECS = ["s16x3", "f32"]


def _engine(cfg, enc_sd, dec_sd, prec):
    from casr.engine import Engine
    e = Engine(cfg, enc_sd, dec_sd)
    e.set_precision(prec)
    assert e.precision() == prec
    return e


def _fbank_batch(frames, dev):
    x = np.zeros((len(frames), max(frames), 80), np.float32)
    for b, t in enumerate(frames):
        x[b, :t] = fbank_for(b, t)
    return torch.from_numpy(x).to(dev), torch.tensor(frames, dtype=torch.int32, device=dev)


def _counted(e, fn):
    """fn() with the LSTMCell GEMM launches counted: (result, launches)."""
    e.profile(["dec_lstm"])
    try:
        r = fn()
        n = e.profile_read().get("dec_lstm", (0, 0.0))[0]
    finally:
        e.profile([])
    assert e.device_flags() == 0
    return r, n


def _greedy_vs_oracle(cfg, frames, prec, want_lstm):
    enc_sd, dec_sd = synthetic_state_dicts(cfg, peaked=True, eos_bias=0.0)  # no EOS: every step runs
    e = _engine(cfg, enc_sd, dec_sd, prec)
    try:
        fb, fr = _fbank_batch(frames, e.device)
        e.encode_fbank(fb, fr)
        g, n = _counted(e, e.greedy)
        toks, score = greedy_outputs(g["tokens"].cpu().numpy(), g["out_len"].cpu().numpy(),
                                     g["finished"].cpu().numpy().astype(bool), g["accum"].cpu().numpy())
    finally:
        e.close()
    assert n == want_lstm, (n, want_lstm)
    feats = [O.features_from_fbank(fbank_for(b, t)) for b, t in enumerate(frames)]
    ref = O.greedy_decode(feats, [f.shape[0] for f in feats], enc_sd, dec_sd, max_len=cfg.max_len)
    assert toks == ref["tokens"]
    np.testing.assert_allclose(score, ref["score"], rtol=0, atol=2e-3)


@pytest.mark.parametrize("prec", PRECS)
def test_greedy_max_len_past_64_takes_three_launch_step(prec):
    """max_len = 70 (gpd['max_len'], model.py:539): the folded greedy prologue reads one early-exit
    counter per lane of one wave (lm <= 64), so prepare_decode's fold_len guard sends this decode to
    the three-launch step: the LSTMCell GEMM runs at every one of the 70 steps, and all 70 tokens
    of every row equal the oracle's (no EOS bias: no row finishes early)."""
    _greedy_vs_oracle(CasrConfig(max_len=70), [120, 96, 150], prec, want_lstm=70)


@pytest.mark.parametrize("prec", PRECS)
def test_greedy_max_len_64_still_folds(prec):
    """The guard's other side: max_len = 64, the most the folded prologue's counter read covers,
    still folds (one LSTMCell launch, at step 0) and matches the oracle over all 64 steps."""
    _greedy_vs_oracle(CasrConfig(max_len=64), [120, 96, 150], prec, want_lstm=1)


# The folded greedy attention (attention_kernel<1, 1>) holds its cell area (AT_CELL_FLOATS = 2560
# floats) on top of the three-launch attention's LDS, 560 + 9 Tq floats at KPB = 1 (attention.hip
# attn_smem_floats), plus 320-336 B of static __shared__ words: the folded form fits 160 KiB up to
# Tq = 4195, the three-launch form up to 4488.  T = 12900 frames (Tp = 4300, 129 s of audio) lies
# between the two.  (Round 5: the guard first counted the dynamic area only, so Tp = 4200 passed it
# and the launch was refused with 164,016 B; attention_smem_bytes now adds the static words.)
@pytest.mark.parametrize("prec", PRECS)
def test_greedy_long_utterance_past_fold_lds_takes_three_launch_step(prec):
    """An utterance of Tp = 4300 encoder frames: the folded attention's LDS would exceed 160 KiB,
    so prepare_decode's fold_lds guard keeps the three-launch step (LSTMCell GEMM at all 40 steps);
    tokens equal the oracle's (the T > 1024 two-pass feature kernels and a 4300-step recurrence on
    the way)."""
    _greedy_vs_oracle(CasrConfig(), [12900, 12000], prec, want_lstm=40)


@pytest.mark.parametrize("prec", PRECS)
def test_greedy_long_utterance_below_fold_lds_still_folds(prec):
    """Tp = 4180 (T = 12540): the folded attention still fits (163,296 B), one LSTMCell launch;
    oracle tokens."""
    _greedy_vs_oracle(CasrConfig(), [12540, 11000], prec, want_lstm=1)


@pytest.mark.parametrize("prec", PRECS)
def test_greedy_long_utterance_at_fold_lds_edge_takes_three_launch_step(prec):
    """Tp = 4200 (T = 12600): 163,680 B of dynamic LDS fit 160 KiB, but not with the kernel's 336 B
    of static LDS; the guard counts both and keeps the three-launch step (the launch itself would
    be refused)."""
    _greedy_vs_oracle(CasrConfig(), [12600, 11000], prec, want_lstm=40)


@pytest.mark.parametrize("prec", PRECS)
@pytest.mark.parametrize("k", [4, 8])
def test_vocab_past_partial_blocks_beam_and_greedy_match_oracle(prec, k):
    """max_num_words = 5200 (V = 5204 > 16 * GP_NT = 5120, decoder.py:11-12): the vocabulary is
    past the beam tile-maxima table, so the beam select at temperature 1 derives its lane bound and
    logsumexp from the full logit row (beam_select_kernel, decoder.hip), and the folded greedy
    step's select reduces 47 partial blocks of the wider fused image.  Beam k and greedy on a
    ragged batch with EOS-bias weights (finished and unfinished hypotheses) against the oracle."""
    cfg = CasrConfig(max_num_words=5200)
    enc_sd, dec_sd = synthetic_state_dicts(cfg, peaked=True)
    frames = [101, 150, 77, 131]
    e = _engine(cfg, enc_sd, dec_sd, prec)
    try:
        fb, fr = _fbank_batch(frames, e.device)
        e.encode_fbank(fb, fr)
        r = e.beam(k)
        assert e.device_flags() == 0
        toks, blen, sc = (x.cpu().numpy() for x in (r["tokens"], r["length"], r["score"]))
        g = e.greedy()
        assert e.device_flags() == 0
        gt, gs = greedy_outputs(g["tokens"].cpu().numpy(), g["out_len"].cpu().numpy(),
                                g["finished"].cpu().numpy().astype(bool), g["accum"].cpu().numpy())
    finally:
        e.close()
    feats = [O.features_from_fbank(fbank_for(b, t)) for b, t in enumerate(frames)]
    lens = [f.shape[0] for f in feats]
    ref = O.beam_decode(feats, lens, enc_sd, dec_sd, k)
    assert [toks[b, :blen[b]].tolist() for b in range(len(frames))] == ref["tokens"]
    np.testing.assert_allclose(sc, ref["score"], rtol=0, atol=2e-3)
    rg = O.greedy_decode(feats, lens, enc_sd, dec_sd)
    assert gt == rg["tokens"]
    np.testing.assert_allclose(gs, rg["score"], rtol=0, atol=2e-3)


def _large_proj_weights(cfg):
    """EOS-bias weights with one projection entry |W_p| = 20 >= 16: the blob's info word 4
    (every |W_p| < 16, casr_pack_weights) is 0, so no one-accumulator projection shape may run;
    the s16 images stay valid (|w| < 2^14), so s16x3 stays the arithmetic."""
    enc_sd, dec_sd = synthetic_state_dicts(cfg, peaked=True)
    dec_sd = dict(dec_sd)
    w = dec_sd["proj_linear.weight"].copy()
    w[7, 3] = 20.0
    dec_sd["proj_linear.weight"] = w
    return enc_sd, dec_sd


@pytest.mark.parametrize("prec", PRECS)
@pytest.mark.parametrize("B,k", [(1024, 1), (128, 8)])
def test_large_projection_weight_beam_takes_three_launch_step(prec, B, k):
    """Round-3 advice: casr_beam at k = 1 is a beam caller and must take the beam fold's guards,
    never the greedy clause (prepare_decode(..., greedy = false)).  With one |W_p| >= 16 the beam
    fold is refused at any R: beam 1 at B = 1024 and beam 8 at B = 128 (R = 1024 each, the folded
    beam's row count) run the three-launch step (LSTMCell GEMM at every step), equal the
    DEC_FOLD = 0 run bit for bit, and match the oracle on 4 utterances spread over the batch."""
    cfg = CasrConfig()
    enc_sd, dec_sd = _large_proj_weights(cfg)
    e = _engine(cfg, enc_sd, dec_sd, prec)
    T = 60
    try:
        fb, fr = _fbank_batch([T] * B, e.device)
        e.encode_fbank(fb, fr)
        outs = []
        for fold in (1, 0):
            e.set_option("DEC_FOLD", fold)
            try:
                r, n = _counted(e, lambda: {x: v.cpu() for x, v in e.beam(k).items()})
            finally:
                e.set_option("DEC_FOLD", 1)
            assert n == cfg.max_len, (fold, n)
            outs.append(r)
    finally:
        e.close()
    for name in outs[0]:
        assert torch.equal(outs[0][name], outs[1][name]), name
    rows = (0, B // 3, (2 * B) // 3, B - 1)
    feats = [O.features_from_fbank(fbank_for(b, T)) for b in rows]
    ref = O.beam_decode(feats, [f.shape[0] for f in feats], enc_sd, dec_sd, k)
    toks, blen, sc = (outs[0][x].numpy() for x in ("tokens", "length", "score"))
    assert [toks[b, :blen[b]].tolist() for b in rows] == ref["tokens"]
    np.testing.assert_allclose(sc[list(rows)], ref["score"], rtol=0, atol=2e-3)
