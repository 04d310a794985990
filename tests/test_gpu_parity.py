"""HIP path vs the reference (golden vectors) and vs the CPU oracle, through the C ABI.

Every test runs twice, once per MFMA arithmetic (s16x3 split-f16 and exact f32; the eng
fixture).  Tolerances (f32 data and accumulators everywhere; differences come only from
summation order, operand splitting (s16x3: 22-bit operands, measured error below the f32
chain's) and libm ulps):
  features 2e-5 abs, encoder outputs 1e-4 abs, beam / greedy scores 2e-3 abs (sums of up to
  40 log-probs of magnitude <= ~40), attention weights 1e-5 abs; token ids must be identical.
"""
import os

import numpy as np
import pytest
import torch

from golden_util import load_golden, fbank_for, golden_frames, near_tie_beam_check, teacher_forced_score
from oracle import casr_oracle as O
from stub_lm import StubLM, pua_int2word
from casr.config import CasrConfig
from casr.lib import pack_weights
from casr.results import greedy_outputs, greedy_steps, records_by_utterance, second_pass_select
from casr.weights import synthetic_state_dicts

pytestmark = pytest.mark.gpu

G, META = load_golden()
CFG = CasrConfig()
FRAMES = golden_frames(META)


@pytest.fixture(scope="module", params=["s16x3", "f32"])
def eng(request):
    """One handle per MFMA arithmetic (include/casr.h casr_set_precision): every parity test
    runs on both the split-f16 path (default) and the exact-f32 path."""
    from casr.engine import Engine
    e = Engine(CFG, *synthetic_state_dicts(CFG, peaked=False))
    e.set_precision(request.param)
    e.requested = request.param
    assert e.precision() == request.param
    yield e
    e.close()


def bind(eng, name):
    eng.bind(pack_weights(CFG, *synthetic_state_dicts(CFG, peaked=(name == "peaked"))))


def batch_fbank(frames, dev):
    T = max(frames)
    x = np.zeros((len(frames), T, 80), np.float32)
    for b, t in enumerate(frames):
        x[b, :t] = fbank_for(b, t)
    return torch.from_numpy(x).to(dev), torch.tensor(frames, dtype=torch.int32, device=dev)


def golden_features(eng):
    fb, fr = batch_fbank(FRAMES, eng.device)
    return eng.features(fb, fr, eps=1e-6)


def test_features_match_oracle(eng):
    feat, flen = golden_features(eng)
    feat = feat.cpu().numpy()
    assert flen.cpu().tolist() == [t // 3 for t in FRAMES]
    for b, t in enumerate(FRAMES):
        ref = O.features_from_fbank(fbank_for(b, t))
        np.testing.assert_allclose(feat[b, :t // 3], ref, atol=2e-5, rtol=0)
        assert not feat[b, t // 3:].any()
    # the reference's own captured features (T=101 utterance 0)
    fb = torch.from_numpy(fbank_for(0, 101))[None].to(eng.device)
    f1, _ = eng.features(fb, torch.tensor([101], dtype=torch.int32, device=eng.device))
    np.testing.assert_allclose(f1[0].cpu().numpy(), G["feat_cmvn_T101"], atol=2e-5, rtol=0)
    # T > 1024 frames (the block's fbank columns no longer fit 64 KB of LDS): two-pass kernels;
    # eps < 0: stacked features without CMVN, both paths
    for T in (1100, 640):
        fr = [T, T - 7]
        fb, frt = batch_fbank(fr, eng.device)
        f2, _ = eng.features(fb, frt)
        f3, _ = eng.features(fb, frt, eps=-1.0)
        for b, t in enumerate(fr):
            np.testing.assert_allclose(f2[b, :t // 3].cpu().numpy(), O.features_from_fbank(fbank_for(b, t)),
                                       atol=2e-5, rtol=0)
            np.testing.assert_allclose(f3[b, :t // 3].cpu().numpy(), O.stack_frames(O.add_delta_deltas(fbank_for(b, t))),
                                       atol=1e-5, rtol=0)


@pytest.mark.parametrize("name", ["plain", "peaked"])
def test_encoder_matches_reference_and_oracle(eng, name):
    bind(eng, name)
    feat, flen = golden_features(eng)
    eng.encode(feat, flen)
    enc, h, c, keys = (x.cpu().numpy() for x in eng.encoder_results())
    np.testing.assert_allclose(h, G[f"{name}_enc_h"], atol=1e-4, rtol=0)
    np.testing.assert_allclose(c, G[f"{name}_enc_c"], atol=1e-4, rtol=0)
    enc_tm = enc.transpose(1, 0, 2)  # [Tp, B, C] like EncoderOutput.out
    np.testing.assert_allclose(enc_tm[::7, :, ::64], G[f"{name}_enc_slice"], atol=1e-4, rtol=0)
    np.testing.assert_allclose(enc.astype(np.float64).sum(axis=(1, 2)), G[f"{name}_enc_sum_per_utt"],
                               rtol=1e-5, atol=2e-2)
    # keys over all Tp positions (padding rows hold b_attn), as the reference computes them
    np.testing.assert_allclose(keys.astype(np.float64).sum(axis=(1, 2)), G[f"{name}_keys_sum_per_utt"],
                               rtol=1e-5, atol=2e-2)


@pytest.mark.parametrize("name", ["plain", "peaked"])
def test_greedy_matches_reference(eng, name):
    bind(eng, name)
    feat, flen = golden_features(eng)
    eng.encode(feat, flen)
    out = eng.greedy(alignment=True)
    assert eng.device_flags() == 0
    tokens = out["tokens"].cpu().numpy()
    out_len = out["out_len"].cpu().numpy()
    fin = out["finished"].cpu().numpy().astype(bool)
    toks, score = greedy_outputs(tokens, out_len, fin, out["accum"].cpu().numpy())
    gold = META[name]["greedy"]
    assert toks == gold["tokens"]
    assert out_len.tolist() == gold["text_len"]
    assert greedy_steps(out_len, fin, CFG.max_len) == gold["steps"]
    np.testing.assert_allclose(score, gold["score"], atol=2e-3, rtol=0)
    align = out["alignment"].cpu().numpy()
    np.testing.assert_allclose(align[0], G[f"{name}_greedy_align_step0"], atol=1e-5)
    np.testing.assert_allclose(align[:gold["steps"]].astype(np.float64).sum(1), G[f"{name}_greedy_align_sum"],
                               atol=1e-4)


@pytest.mark.parametrize("name", ["plain", "peaked"])
@pytest.mark.parametrize("k", [1, 4, 8, 16])
def test_beam_matches_reference(eng, name, k):
    bind(eng, name)
    feat, flen = golden_features(eng)
    eng.encode(feat, flen)
    r = eng.beam(k)
    assert eng.device_flags() == 0
    toks = r["tokens"].cpu().numpy()
    blen = r["length"].cpu().numpy()
    gold = META[name][f"beam{k}"]
    if name == "plain" and k == 16:  # near-tied f32 candidates: test_oracle_golden.py, same check
        _, dec_sd = synthetic_state_dicts(CFG, peaked=False)
        enc_sd = synthetic_state_dicts(CFG, peaked=False)[0]
        feats = [O.features_from_fbank(fbank_for(b, t)) for b, t in enumerate(FRAMES)]
        near_tie_beam_check([toks[b, :blen[b]].tolist() for b in range(len(FRAMES))],
                            r["score"].cpu().numpy(), gold, atol=2e-3,
                            rescore=lambda b, t: teacher_forced_score(feats[b], t, enc_sd, dec_sd))
        return
    assert [toks[b, :blen[b]].tolist() for b in range(len(FRAMES))] == gold["tokens"]
    np.testing.assert_allclose(r["score"].cpu().numpy(), gold["score"], atol=2e-3, rtol=0)


@pytest.mark.parametrize("name", ["plain", "peaked"])
def test_beam_second_pass_and_length_weight(eng, name):
    bind(eng, name)
    feat, flen = golden_features(eng)
    eng.encode(feat, flen)
    r = eng.beam(4, 1.5, 1.5)
    toks, blen, sc = (x.cpu().numpy() for x in (r["tokens"], r["length"], r["score"]))
    best = {b: (toks[b, :blen[b]].tolist(), float(sc[b])) for b in range(len(FRAMES))}
    gold = META[name]["beam4_lw"]
    assert [best[b][0] for b in range(len(FRAMES))] == gold["tokens"]
    np.testing.assert_allclose([best[b][1] for b in range(len(FRAMES))], gold["score"], atol=2e-3)
    recs = records_by_utterance(*(x.cpu().numpy() for x in eng.beam_records()))
    best.update(second_pass_select(recs, pua_int2word(CFG.vocab), StubLM(), 1.5, 1.5))
    gold = META[name]["beam4_lm"]
    assert [best[b][0] for b in range(len(FRAMES))] == gold["tokens"]
    np.testing.assert_allclose([best[b][1] for b in range(len(FRAMES))], gold["score"], atol=2e-3)
    # BASELINE config 5: beam 16 + second pass
    r = eng.beam(16, 1.5, 1.5)
    assert eng.device_flags() == 0
    toks, blen, sc = (x.cpu().numpy() for x in (r["tokens"], r["length"], r["score"]))
    best = {b: (toks[b, :blen[b]].tolist(), float(sc[b])) for b in range(len(FRAMES))}
    recs = records_by_utterance(*(x.cpu().numpy() for x in eng.beam_records()))
    best.update(second_pass_select(recs, pua_int2word(CFG.vocab), StubLM(), 1.5, 1.5))
    gold = META[name]["beam16_lm"]
    if name == "plain":  # near-tied f32 candidates at beam 16 (test_beam_matches_reference)
        near_tie_beam_check([best[b][0] for b in range(len(FRAMES))], [best[b][1] for b in range(len(FRAMES))],
                            gold, atol=2e-3)
        return
    assert [best[b][0] for b in range(len(FRAMES))] == gold["tokens"]
    np.testing.assert_allclose([best[b][1] for b in range(len(FRAMES))], gold["score"], atol=2e-3)


def test_model_dropin_api_matches_reference():
    import model as M
    m = M.Model()
    m.load_state_dicts(*synthetic_state_dicts(CFG, peaked=True))
    m.model.eval()
    dev = m.device
    feats = [torch.from_numpy(O.features_from_fbank(fbank_for(b, t))).to(dev) for b, t in enumerate(FRAMES)]
    lens = torch.tensor([f.shape[0] for f in feats])
    from casr.vocab import load_vocab
    i2w = load_vocab()[1]
    g = m.eval_one_batch_with_greedy(dev, feats, lens, i2w, None)
    assert g.pred_text == META["peaked"]["greedy"]["text"]
    assert len(g.alignment) == META["peaked"]["greedy"]["steps"]
    assert g.n == len(FRAMES)
    r = m.eval_one_batch_with_beam(dev, 8, feats, lens, None, i2w, second_pass=False)
    assert r.pred_text == META["peaked"]["beam8"]["text"]
    assert r.alignment is None and r.text_len is None
    with pytest.raises(AttributeError):  # reference: second_pass with lm_model None crashes
        m.eval_one_batch_with_beam(dev, 4, feats, lens, None, i2w, second_pass=True, lm_model=None)
    r = m.eval_one_batch_with_beam(dev, 4, feats, lens, None, pua_int2word(CFG.vocab), second_pass=True,
                                   lm_model=StubLM(), lm_weight=1.5, length_weight=1.5)
    assert [[ord(ch) - 0xE000 for ch in t] for t in r.pred_text] == META["peaked"]["beam4_lm"]["tokens"]


def test_graph_replay_equals_eager(eng):
    """hipGraph replay (default) and eager launches give bitwise-identical results."""
    bind(eng, "peaked")
    feat, flen = golden_features(eng)
    outs = []
    for graphs in (False, True, True):  # second graph run replays the cached graph
        eng.set_graphs(graphs)
        eng.encode(feat, flen)
        enc = eng.encoder_results()[0].cpu()
        g = eng.greedy(alignment=True)
        bm = eng.beam(4, 1.5, 1.5)
        assert eng.device_flags() == 0
        outs.append((enc, g["tokens"].cpu(), g["accum"].cpu(), g["alignment"].cpu(), bm["tokens"].cpu(),
                     bm["score"].cpu(), bm["steps"].cpu()))
    eng.set_graphs(2)  # the default: decode eager, recurrence fallback replayed
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a, b)
    for a, b in zip(outs[1], outs[2]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("graphs", [False, True])
@pytest.mark.parametrize("eos_bias", [0.0, 12.0])
def test_fused_select_equals_select_launches(eng, eos_bias, graphs):
    """Greedy decoding with each step's select fused into the next LSTMCell (default) and with
    every select a launch of its own (CASR_OPT_FUSE_SELECT = 0) give the same tokens, lengths,
    scores and finished flags bit for bit: ragged lengths, B = 200 (a partial row block), without
    and with early finishers (eos_bias: rows end at different steps, the early exit counts them).
    With graphs on, the option is part of the captured graph's key: switching it between calls
    must replay the other variant, not the first one captured."""
    enc_sd, dec_sd = synthetic_state_dicts(CFG, peaked=True, eos_bias=eos_bias)
    eng.bind(pack_weights(CFG, enc_sd, dec_sd))
    B = 200
    rs = np.random.RandomState(5)
    frames = rs.randint(30, 400, size=B)
    x = np.zeros((B, 400, 80), np.float32)
    for b in range(B):
        x[b, :frames[b]] = fbank_for(b, int(frames[b]))
    feat, flen = eng.features(torch.from_numpy(x).to(eng.device),
                              torch.from_numpy(frames.astype(np.int32)).to(eng.device))
    eng.encode(feat, flen)
    outs = []
    try:
        eng.set_graphs(graphs)
        for fuse in (0, 1, 0):
            eng.set_option("FUSE_SELECT", fuse)
            if not graphs:  # select launches: one per step, or only the last step's when fused
                eng.profile(["select"])
            g = eng.greedy()
            assert eng.device_flags() == 0
            outs.append({k: v.cpu() for k, v in g.items() if torch.is_tensor(v)})
            if not graphs:
                assert eng.profile_read()["select"][0] == (1 if fuse else CFG.max_len)
                eng.profile([])
    finally:
        eng.set_option("FUSE_SELECT", 1)
        eng.set_graphs(2)
    assert outs[0].keys() == outs[1].keys() and "tokens" in outs[0]
    for o in outs[1:]:
        for k in outs[0]:
            assert torch.equal(outs[0][k], o[k]), k
    if eos_bias:
        assert bool(outs[1]["finished"].any()), "with the EOS bias some rows must finish early"


@pytest.mark.parametrize("k,eos_bias,graphs,B", [(8, 0.0, False, 256), (8, 12.0, True, 256), (8, 40.0, False, 256),
                                                 (4, 40.0, True, 256), (8, 0.0, False, 128), (8, 40.0, True, 128)])
def test_beam_select_in_attention_equals_select_launches(eng, k, eos_bias, graphs, B):
    """The folded beam step with one attention block per utterance (k = 4 or 8 at B = 256, R >= 1024
    rows): the select of step l - 1 run in step l's attention prologue (default, attention.hip CELL 3)
    and every select a launch of its own (CASR_OPT_FUSE_SELECT = 0) give the same tokens, lengths,
    scores, step counts and finished-hypothesis records bit for bit, without EOS bias, with finished
    hypotheses (eos_bias 12: the search still runs all 40 steps at B = 256) and with an early stop
    (eos_bias 40: every utterance's top candidate ends early, so the fused attention of the step after
    the last select runs on counters it cannot know complete).  Without graphs: the folded step is in
    effect (one LSTMCell launch, step 0's) and the fused decode launches one select (the last step's)
    instead of one per step.  B = 128, k = 8 (4 rows per attention block, CELL 4): both blocks of an
    utterance run its select, the first one writes the bookkeeping."""
    if eng.requested != "s16x3":
        pytest.skip("the beam fold, and with it the fused select, runs on the s16x3 images")
    enc_sd, dec_sd = synthetic_state_dicts(CFG, peaked=True, eos_bias=eos_bias)
    eng.bind(pack_weights(CFG, enc_sd, dec_sd))
    rs = np.random.RandomState(9)
    frames = rs.randint(30, 300, size=B)
    x = np.zeros((B, 300, 80), np.float32)
    for b in range(B):
        x[b, :frames[b]] = fbank_for(b, int(frames[b]))
    feat, flen = eng.features(torch.from_numpy(x).to(eng.device),
                              torch.from_numpy(frames.astype(np.int32)).to(eng.device))
    eng.encode(feat, flen)
    outs = []
    try:
        eng.set_graphs(graphs)
        for fuse in (0, 1, 0):
            eng.set_option("FUSE_SELECT", fuse)
            if not graphs:
                eng.profile(["select", "dec_lstm"])
            bm = eng.beam(k)
            rt, rsc, rv = eng.beam_records()
            assert eng.device_flags() == 0
            o = {n: v.cpu() for n, v in bm.items()}
            o.update(rec_tokens=rt.cpu(), rec_score=rsc.cpu(), rec_valid=rv.cpu())
            outs.append(o)
            if not graphs:
                prof = eng.profile_read()
                assert prof["dec_lstm"][0] == 1, "the folded beam step"
                assert prof["select"][0] == (1 if fuse else CFG.max_len)
                eng.profile([])
    finally:
        eng.set_option("FUSE_SELECT", 1)
        eng.set_graphs(2)
    for o in outs[1:]:
        for n in outs[0]:
            assert torch.equal(outs[0][n], o[n]), n
    if eos_bias >= 40:
        assert int(outs[1]["steps"][0]) < CFG.max_len, "with the EOS bias the search must stop early"
    elif eos_bias:
        assert bool(outs[1]["rec_valid"].any()), "with the EOS bias hypotheses finish"


@pytest.mark.parametrize("B,layout", [(37, 0), (37, 1), (37, 2), (256, 0)])
def test_persistent_recurrence_equals_per_step(eng, B, layout):
    """The persistent per-layer recurrence (granule hand-offs, either store flavour; chained
    ordinary, cooperative or unordered launch) and the per-step launches give bitwise-identical encoder outputs and
    final states, on ragged lengths (B = 37: a partial row group and padding rows, in the 16x16
    layout the batch selects and in the forced 32x16 and 16x32 ones; B = 256: the full
    256-workgroup grid of 32x16)."""
    eng.set_option("REC_LAYOUT", layout)
    enc_sd, dec_sd = synthetic_state_dicts(CFG, peaked=True)
    eng.bind(pack_weights(CFG, enc_sd, dec_sd))
    rs = np.random.RandomState(11)
    frames = rs.randint(9, 801, size=B)
    frames[0], frames[-1] = 800, 9  # longest and shortest (T' = 3)
    x = np.zeros((B, 800, 80), np.float32)
    for b in range(B):
        x[b, :frames[b]] = fbank_for(b, int(frames[b]))
    feat, flen = eng.features(torch.from_numpy(x).to(eng.device),
                              torch.from_numpy(frames.astype(np.int32)).to(eng.device))
    assert eng.recurrence_mode(B) == 1, "B <= 256 must take the persistent path on MI355X"
    outs = []
    # the persistent path four times: hand-off words stored plain (L2-kept, the default when each
    # group shares an XCD) and write-through (CASR_OPT_REC_STORE_PLAIN = 0), the chained ordinary
    # launch (default, CASR_OPT_REC_COOP = 2), the cooperative launch (1) and the unordered one (0)
    try:
        for persistent, plain, coop in ((False, 1, 2), (True, 1, 2), (True, 0, 2), (True, 1, 1), (True, 1, 0)):
            eng.set_option("REC_STORE_PLAIN", plain)
            eng.set_option("REC_COOP", coop)
            eng.set_persistent(persistent)
            eng.encode(feat, flen)
            assert eng.device_flags() == 0
            outs.append([t.cpu() for t in eng.encoder_results()])
    finally:
        for k, v in (("REC_STORE_PLAIN", 1), ("REC_COOP", 2), ("REC_LAYOUT", 0)):
            eng.set_option(k, v)
        eng.set_persistent(True)
    for got in outs[1:]:
        for a, b in zip(outs[0], got):
            assert torch.equal(a, b)


def test_cooperative_refusal_mid_encode_falls_back_bitwise(eng):
    """A refused cooperative launch (hipErrorCooperativeLaunchTooLarge: the grid cannot be
    co-resident) switches that layer and every later one to the per-step recurrence, and zeroes
    their outputs first (casr_capi.hip encode_impl).  Forced through CASR_OPT_REC_COOP_REFUSE at
    layer 0, 1 and 3 (the last: the keys then come from the fallback's split image): encoder
    outputs, final states, keys and greedy / beam tokens bitwise equal to an all-persistent and to
    an all-per-step encode, ragged lengths (B = 48)."""
    B = 48
    enc_sd, dec_sd = synthetic_state_dicts(CFG, peaked=True)
    eng.bind(pack_weights(CFG, enc_sd, dec_sd))
    rs = np.random.RandomState(23)
    frames = rs.randint(9, 601, size=B)
    frames[0] = 600
    x = np.zeros((B, 600, 80), np.float32)
    for b in range(B):
        x[b, :frames[b]] = fbank_for(b, int(frames[b]))
    feat, flen = eng.features(torch.from_numpy(x).to(eng.device),
                              torch.from_numpy(frames.astype(np.int32)).to(eng.device))

    def run():
        eng.encode(feat, flen)
        res = [t.cpu() for t in eng.encoder_results()]
        res.append(eng.greedy()["tokens"].cpu())
        res.append(eng.beam(4)["tokens"].cpu())
        assert eng.device_flags() == 0
        return res

    outs = {}
    try:
        outs["persistent"] = run()
        eng.set_persistent(False)
        outs["per_step"] = run()
        eng.set_persistent(True)
        for layer in (0, 1, 3):
            eng.set_option("REC_COOP_REFUSE", layer + 1)
            outs[f"refused_{layer}"] = run()
    finally:
        eng.set_option("REC_COOP_REFUSE", 0)
        eng.set_persistent(True)
    for name, got in outs.items():
        for i, (a, b) in enumerate(zip(outs["persistent"], got)):
            assert torch.equal(a, b), (name, i)


def test_recurrence_pacing_options_bitwise(eng):
    """The recurrence's pacing options (first-poll sleep, second-poll gap) change only when a
    workgroup looks at its producers' words, never what it computes: encoder results bitwise equal
    over the extremes of both (B = 256, T' = 266)."""
    bind(eng, "peaked")
    feat, flen = _bench_batch(eng, 256)
    outs = []
    try:
        for sleep, gap in ((-1, 2), (1, 2), (0, 1), (16, 8), (4, 1)):
            eng.set_option("REC_SLEEP", sleep)
            eng.set_option("REC_POLL_GAP", gap)
            eng.encode(feat, flen)
            assert eng.device_flags() == 0
            outs.append([t.cpu() for t in eng.encoder_results()])
    finally:
        eng.set_option("REC_SLEEP", -1)
        eng.set_option("REC_POLL_GAP", 2)
    for got in outs[1:]:
        for a, b in zip(outs[0], got):
            assert torch.equal(a, b)


def test_persistent_recurrence_nan_row_isolated(eng):
    """A T' = 1 utterance has NaN features (unbiased std of one frame, main.py:37, as in the
    reference).  Its NaN h must travel through the tagged hand-off (non-finite code) without
    stalling the other workgroups, and every other row must be bitwise unaffected."""
    enc_sd, dec_sd = synthetic_state_dicts(CFG, peaked=True)
    eng.bind(pack_weights(CFG, enc_sd, dec_sd))
    B, T = 40, 240
    frames = np.full(B, T, np.int32)
    x = np.stack([fbank_for(b, T) for b in range(B)])
    fb = torch.from_numpy(x).to(eng.device)
    eng.set_persistent(True)
    feat, flen = eng.features(fb, torch.from_numpy(frames).to(eng.device))
    eng.encode(feat, flen)
    assert eng.device_flags() == 0
    clean = [t.cpu() for t in eng.encoder_results()]
    frames[5] = 3  # T' = 1
    feat, flen = eng.features(fb, torch.from_numpy(frames).to(eng.device))
    assert torch.isnan(feat[5, 0]).all()
    eng.encode(feat, flen)
    assert eng.device_flags() == 0, "a NaN row must not stall the persistent recurrence"
    enc, h, c, keys = [t.cpu() for t in eng.encoder_results()]
    keep = [b for b in range(B) if b != 5]
    for a, b_ in zip(clean, (enc, h, c, keys)):
        assert torch.equal(a[keep], b_[keep])
    assert torch.isnan(enc[5, 0]).all() and (enc[5, 1:] == 0).all()


def _bench_batch(eng, B, T=800):
    x = np.stack([fbank_for(b, T) for b in range(B)])
    fb = torch.from_numpy(x).to(eng.device)
    return eng.features(fb, torch.full((B,), T, dtype=torch.int32, device=eng.device))


def test_encode_fbank_equals_features_then_encode(eng):
    """casr_encode_fbank (features kept inside the handle; s16x3: written straight as the
    layer-0 split-f16 image) gives the two-call sequence's encoder results bit for bit, ragged
    lengths included, and the same feature lengths."""
    bind(eng, "peaked")
    fb, fr = batch_fbank(FRAMES, eng.device)
    feat, flen = eng.features(fb, fr)
    eng.encode(feat, flen)
    a = [x.cpu() for x in eng.encoder_results()]
    ga = eng.greedy()["tokens"].cpu()
    flen2 = eng.encode_fbank(fb, fr)
    assert eng.device_flags() == 0
    b = [x.cpu() for x in eng.encoder_results()]
    gb = eng.greedy()["tokens"].cpu()
    assert torch.equal(flen.cpu(), flen2.cpu())
    for x, y in zip(a, b):
        assert torch.equal(x, y)
    assert torch.equal(ga, gb)


def test_batch_invariance_and_determinism(eng):
    """Size-independent properties at the benchmark size B = 256: two runs are bitwise equal,
    and a 16-utterance sub-batch decodes to the same tokens as inside the full batch
    (utterances are independent; the reference is batch-invariant too: SURVEY §8e)."""
    eng.bind(pack_weights(CFG, *synthetic_state_dicts(CFG, peaked=True, eos_bias=0.0)))
    feat, flen = _bench_batch(eng, 256)
    eng.encode(feat, flen)
    a = eng.greedy()["tokens"].cpu()
    eng.encode(feat, flen)
    b = eng.greedy()["tokens"].cpu()
    assert torch.equal(a, b)
    eng.encode(feat[100:116].contiguous(), flen[100:116].contiguous())
    c = eng.greedy()["tokens"].cpu()
    assert torch.equal(a[100:116], c)
    # 128 x 8 = 1024 beam rows (the 128-row decode GEMM tiles) against 16 x 8 = 128 (32 / 64 rows)
    eng.encode(feat[:128].contiguous(), flen[:128].contiguous())
    r1 = eng.beam(8)
    t1 = r1["tokens"].cpu()
    eng.encode(feat[:16].contiguous(), flen[:16].contiguous())
    t2 = eng.beam(8)["tokens"].cpu()
    assert torch.equal(t1[:16], t2)
    # k = 16: 64 x 16 = 1024 rows (the 128 x 160 projection blocks) against 8 x 16 = 128 rows (the
    # 64 x 80 ones); both take the tile-maxima threshold at temperature 1 (the select path over
    # full logit rows, T != 1, is covered by test_beam_temperature_matches_reference)
    eng.encode(feat[:64].contiguous(), flen[:64].contiguous())
    t3 = eng.beam(16)["tokens"].cpu()
    assert eng.device_flags() == 0
    eng.encode(feat[:8].contiguous(), flen[:8].contiguous())
    t4 = eng.beam(16)["tokens"].cpu()
    assert torch.equal(t3[:8], t4)


def test_out_of_range_weights_run_f32(eng):
    """A blob whose weights the f16 split cannot carry (an encoder W_ih entry >= 16) is marked
    invalid at pack time; a handle bound to it reports and runs exact f32 whatever is requested,
    and still decodes like the CPU oracle on the same weights."""
    enc_sd, dec_sd = synthetic_state_dicts(CFG, peaked=True)
    enc_sd = dict(enc_sd)
    w = enc_sd["rnn.rnn.0.weight_ih_l0"].copy()
    w[7, 11] = 20.0
    enc_sd["rnn.rnn.0.weight_ih_l0"] = w
    eng.bind(pack_weights(CFG, enc_sd, dec_sd))
    assert eng.precision() == "f32"
    frames = [150, 96]
    fbs = [fbank_for(b, t) for b, t in enumerate(frames)]
    x = np.zeros((2, max(frames), 80), np.float32)
    for b, f in enumerate(fbs):
        x[b, :len(f)] = f
    feat, flen = eng.features(torch.from_numpy(x).to(eng.device), torch.tensor(frames, dtype=torch.int32,
                                                                               device=eng.device))
    eng.encode(feat, flen)
    out = eng.greedy()
    assert eng.device_flags() == 0
    toks, _ = greedy_outputs(out["tokens"].cpu().numpy(), out["out_len"].cpu().numpy(),
                             out["finished"].cpu().numpy().astype(bool), out["accum"].cpu().numpy())
    feats = [O.features_from_fbank(f) for f in fbs]
    ref = O.greedy_decode(feats, [f.shape[0] for f in feats], enc_sd, dec_sd)
    assert toks == ref["tokens"]
    # a valid blob restores the requested arithmetic
    eng.bind(pack_weights(CFG, *synthetic_state_dicts(CFG, peaked=True)))
    assert eng.precision() == eng.requested


@pytest.mark.parametrize("name", ["plain", "peaked"])
def test_keys_elementwise_match_oracle(eng, name):
    """The keys GEMM alone, elementwise: keys = enc . W_enc + b_attn (attention.py:67-78) from the
    oracle on the GPU's own encoder output, so the check isolates the keys contraction (s16x3 or
    f32) from the encoder's.  Tolerance 2e-5 abs on |keys| <~ 3."""
    bind(eng, name)
    feat, flen = golden_features(eng)
    eng.encode(feat, flen)
    enc, _, _, keys = (x.cpu().numpy() for x in eng.encoder_results())
    _, dec_sd = synthetic_state_dicts(CFG, peaked=(name == "peaked"))
    for b, t in enumerate(FRAMES):
        ref = O.compute_keys(enc[b][:, None, :], dec_sd)[:, 0, :]   # [Tp, A]
        np.testing.assert_allclose(keys[b].T, ref, atol=2e-5, rtol=0)


@pytest.mark.parametrize("name", ["plain", "peaked"])
def test_attention_split_form_vs_direct(eng, name):
    """The attention's split exponential score form (default: sum_a v_a - 2 v_a / (1 + e^{2k}
    e^{2q}), attention.hip) against the direct tanh(k + q) form (CASR_OPT_ATTN_DIRECT), greedy and
    beam 8: same tokens, greedy alignments within 1e-5 and scores within 2e-4.  Then a blob whose
    attention bias puts every key above 43 (outside the split form's range, where e^{2k} is stored
    as NaN): every block falls back to the direct form, so the two options agree bit for bit."""
    def run():
        g = eng.greedy(alignment=True)
        bm = eng.beam(8)
        assert eng.device_flags() == 0
        return [x.cpu() for x in (g["tokens"], g["out_len"], g["accum"], g["alignment"], bm["tokens"],
                                  bm["length"], bm["score"])]

    def both():
        split = run()
        try:
            eng.set_option("ATTN_DIRECT", 1)
            direct = run()
        finally:
            eng.set_option("ATTN_DIRECT", 0)
        return split, direct

    bind(eng, name)
    feat, flen = golden_features(eng)
    eng.encode(feat, flen)
    split, direct = both()
    for i in (0, 1, 4, 5):
        assert torch.equal(split[i], direct[i])
    for i, tol in ((2, 2e-4), (3, 1e-5), (6, 2e-4)):
        np.testing.assert_allclose(split[i].numpy(), direct[i].numpy(), atol=tol, rtol=0)
    enc_sd, dec_sd = synthetic_state_dicts(CFG, peaked=(name == "peaked"))
    dec_sd = dict(dec_sd)
    dec_sd["attn_mechanism.b_attn"] = dec_sd["attn_mechanism.b_attn"] + 50.0
    eng.bind(pack_weights(CFG, enc_sd, dec_sd))
    eng.encode(feat, flen)
    split, direct = both()
    for a, b in zip(split, direct):
        assert torch.equal(a, b)


@pytest.mark.parametrize("B,T", [(37, 400), (256, 800)])
def test_keys_row_streaming_equals_tiles(eng, B, T):
    """The s16x3 keys GEMM in its two forms (CASR_OPT_KEYS_ROWS: W_enc in registers and 16-row items
    streamed through LDS, the default; or 128 x 128 tiles) gives the same keys and e^{2 keys} bit for
    bit (same MFMAs, same k order): the keys over every Tp slot, and greedy tokens, scores and
    alignments (which read e^{2 keys} through the split score form).  Ragged lengths at B = 37
    (Tp = 133: a partial last item per utterance), and the metric's B = 256, T = 800."""
    if eng.requested != "s16x3":
        pytest.skip("the f32 arithmetic keeps the f32 keys GEMM")
    bind(eng, "peaked")
    rs = np.random.RandomState(11)
    frames = rs.randint(max(30, T // 2), T + 1, size=B) if B < 256 else np.full(B, T)
    x = np.zeros((B, T, 80), np.float32)
    for b in range(B):
        x[b, :frames[b]] = fbank_for(b, int(frames[b]))
    feat, flen = eng.features(torch.from_numpy(x).to(eng.device),
                              torch.from_numpy(frames.astype(np.int32)).to(eng.device))
    outs = []
    try:
        for rows in (1, 0, 1):
            eng.set_option("KEYS_ROWS", rows)
            eng.encode(feat, flen)
            keys = eng.encoder_results()[3].cpu()
            g = eng.greedy(alignment=True)
            assert eng.device_flags() == 0
            outs.append([keys] + [g[n].cpu() for n in ("tokens", "accum", "alignment")])
    finally:
        eng.set_option("KEYS_ROWS", 1)
    for o in outs[1:]:
        for a, b in zip(outs[0], o):
            assert torch.equal(a, b)


@pytest.mark.parametrize("name", ["plain", "peaked"])
def test_decode_fold_vs_three_launches(eng, name):
    """The folded greedy step (CASR_OPT_DEC_FOLD, default under s16x3: the projection GEMM also
    computes the next step's LSTM gates from the same [ctx | h] rows, the embedding part of the gates
    comes from the per-token table, the cell and q = h . W_hidden run inside the attention kernel)
    against the three-launch step (LSTMCell GEMM, attention, projection): the same arithmetic
    regrouped (decoder.py:104-114, attention.py:92, decoder.py:129-135), so identical tokens,
    lengths and finished flags, scores within 2e-3 and alignments within 1e-5; on the golden batch
    (ragged) and at the headline size (B = 256, T = 800, all 40 steps).  In both arithmetics: under
    f32 the fused GEMM runs the exact-f32 MFMAs on the f32 fused image (round 4)."""
    def run(fold, **kw):
        eng.set_option("DEC_FOLD", fold)
        eng.profile(["dec_lstm"])
        try:
            g = eng.greedy(**kw)
            n_lstm = eng.profile_read()["dec_lstm"][0]
        finally:
            eng.profile([])
            eng.set_option("DEC_FOLD", 1)
        assert eng.device_flags() == 0
        return g, n_lstm

    bind(eng, name)
    for feat, flen in (golden_features(eng), _bench_batch(eng, 256)):
        eng.encode(feat, flen)
        align = feat.shape[0] < 64
        f, n_f = run(1, alignment=align)
        u, n_u = run(0, alignment=align)
        # the fold runs the LSTMCell GEMM at step 0 only; the three-launch step at every step
        assert n_u == CFG.max_len
        assert n_f == 1
        for k in ("tokens", "out_len", "finished"):
            assert torch.equal(f[k].cpu(), u[k].cpu()), k
        np.testing.assert_allclose(f["accum"].cpu().numpy(), u["accum"].cpu().numpy(), atol=2e-3, rtol=0)
        if align:
            np.testing.assert_allclose(f["alignment"].cpu().numpy(), u["alignment"].cpu().numpy(), atol=1e-5, rtol=0)


@pytest.mark.parametrize("eos_bias", [0.0, None])
@pytest.mark.parametrize("B,k", [(128, 8), (256, 8), (128, 16)])
def test_beam_fold_vs_three_launches(eng, B, k, eos_bias):
    """The folded beam step (CASR_OPT_DEC_FOLD at R >= 1024 rows: the fused projection | LSTM-gate
    GEMM in its one-accumulator 128 x 224 / 256 x 224 shapes, logits, tile maxima and row partials
    for the beam select; the cell at each row's predecessor inside the attention kernel) against the
    three-launch step: beam 8 at B = 128 (R = 1024, BASELINE config 3) and B = 256 (R = 2048, the
    metric's beam line), beam 16 at B = 128 (R = 2048 with 4 of an utterance's 16 rows per attention
    block, BASELINE config 5's shape); T = 800, with and without early finishers: identical tokens
    and lengths, scores within 2e-3 (decoder.py:104-135, model.py:604-987)."""
    kw = {} if eos_bias is None else {"eos_bias": eos_bias}
    eng.bind(pack_weights(CFG, *synthetic_state_dicts(CFG, peaked=True, **kw)))
    feat, flen = _bench_batch(eng, B)
    eng.encode(feat, flen)
    outs = []
    for fold in (1, 0):
        eng.set_option("DEC_FOLD", fold)
        eng.profile(["dec_lstm"])
        try:
            r = {n: v.cpu() for n, v in eng.beam(k).items()}
            n_lstm = eng.profile_read()["dec_lstm"][0]
        finally:
            eng.profile([])
            eng.set_option("DEC_FOLD", 1)
        assert eng.device_flags() == 0
        outs.append((r, n_lstm))
    (f, n_f), (u, n_u) = outs
    assert n_u == CFG.max_len
    assert n_f == (1 if eng.requested == "s16x3" else CFG.max_len)
    assert torch.equal(f["length"], u["length"])
    assert torch.equal(f["steps"], u["steps"])
    for b in range(B):
        n = int(u["length"][b])
        assert torch.equal(f["tokens"][b, :n], u["tokens"][b, :n]), b
    np.testing.assert_allclose(f["score"].numpy(), u["score"].numpy(), atol=2e-3, rtol=0)


def test_fold_graph_replay_equals_eager(eng):
    """The folded decode step captured and replayed as a hipGraph (casr_set_graphs mode 1) equals
    its eager launches bit for bit: greedy at B = 128 and beam 8 at B = 128 (R = 1024 rows, the
    folded beam shape), the second replay from the cached graph."""
    eng.bind(pack_weights(CFG, *synthetic_state_dicts(CFG, peaked=True)))
    feat, flen = _bench_batch(eng, 128)
    eng.encode(feat, flen)
    outs = []
    try:
        for graphs in (False, True, True):
            eng.set_graphs(3 if graphs else 0)
            g = eng.greedy()
            bm = eng.beam(8)
            assert eng.device_flags() == 0
            outs.append([x.cpu() for x in (g["tokens"], g["accum"], g["out_len"], bm["tokens"], bm["score"],
                                           bm["length"], bm["steps"])])
    finally:
        eng.set_graphs(2)
    for other in outs[1:]:
        for a, b in zip(outs[0], other):
            assert torch.equal(a, b)


def test_bind_refuses_foreign_blob(eng):
    """A blob of another layout (size or stamp) is refused on bind, not read past its end."""
    from casr import lib as L
    good = pack_weights(CFG, *synthetic_state_dicts(CFG, peaked=True))
    with pytest.raises(ValueError):
        eng.bind(torch.zeros(good.size + 64, dtype=torch.float32, device=eng.device))
    at = np.nonzero(good.view(np.uint32) == 0xCA5B0003)[0]
    assert len(at) == 1  # the layout stamp's magic word
    bad = torch.from_numpy(good.copy()).to(eng.device)
    bad.view(torch.int32)[int(at[0])] = 0
    with pytest.raises(L.CasrError):
        eng.bind(bad)
    eng.bind(good)
    assert eng.precision() == eng.requested


def test_model_reruns_f32_on_f16_range_overflow():
    """An s16x3 activation beyond the f16 range (device flag 128) would make every result after
    it wrong: the drop-in Model re-runs such a batch on the exact-f32 path (Engine.run_checked).
    A feature value of 1e5 forces it; the result must equal an f32-only run."""
    import model as M
    m = M.Model()
    m.load_state_dicts(*synthetic_state_dicts(CFG, peaked=True))
    dev = m.device
    feats = [torch.from_numpy(O.features_from_fbank(fbank_for(b, t))).to(dev) for b, t in enumerate(FRAMES)]
    feats[1] = feats[1].clone()
    feats[1][3, 17] = 1.0e5
    lens = torch.tensor([f.shape[0] for f in feats])
    assert m.engine.precision() == "s16x3"
    g = m.eval_one_batch_with_greedy(dev, feats, lens, None, None)
    assert m.engine.precision() == "s16x3"  # restored after the f32 re-run
    m.engine.set_precision("f32")
    g32 = m.eval_one_batch_with_greedy(dev, feats, lens, None, None)
    m.engine.set_precision("s16x3")
    assert g.pred_text == g32.pred_text
    np.testing.assert_array_equal(np.asarray(g.score), np.asarray(g32.score))


@pytest.mark.parametrize("B", [256, 128, 37])
def test_input_gemm_tail_split_bitwise(eng, B):
    """s16x3 input projection: the persistent kernel over whole rounds plus the 128 x 256 half-tile
    launch for the rows after them (default), the persistent kernel alone (CASR_OPT_GEMM16_TAIL = 0)
    and the per-tile kernel (CASR_OPT_GEMM16_PERSIST = 0) give bitwise-identical encoder outputs
    (B = 256 and 128: 80 / 40 tiles past the last whole round; B = 37: 48 tiles in one partial round).
    Round 5: the ping-pong persistent kernel (CASR_OPT_GEMM16_PERSIST = 2, the default: 16-deep
    stages, two staggered wave groups, buffer stores that drop rows past M) with and without the
    tail split, against the round-2 persistent kernel and the per-tile kernel; and the balanced tail
    (CASR_OPT_GEMM16_TAIL = 2, the default: one round of 160 x 128 tiles at B = 256, 96 x 128 at
    B = 128) against the half tiles; and the layer-input / W_ih images 16-k-block major
    (CASR_OPT_X16_KM = 1, the default with those forms: written by the feature kernel, the recurrence
    and split_rows, read by the ping-pong kernel, the balanced tail and the keys form) against row
    images."""
    if eng.precision() != "s16x3":
        pytest.skip("the split-f16 input GEMM only")
    bind(eng, "peaked")
    rs = np.random.RandomState(5)
    frames = [800] * (B - 2) + [int(rs.randint(9, 800)), 9]
    fb, fr = batch_fbank(frames, eng.device)
    outs = []
    try:
        for tail, persist, km in ((2, 2, 1), (2, 2, 0), (0, 2, 1), (1, 2, 0), (0, 2, 0), (2, 1, 0), (1, 1, 0),
                                  (0, 1, 0), (1, 0, 0)):
            eng.set_option("GEMM16_TAIL", tail)
            eng.set_option("GEMM16_PERSIST", persist)
            eng.set_option("X16_KM", km)
            eng.encode_fbank(fb, fr)
            assert eng.device_flags() == 0
            outs.append([t.cpu() for t in eng.encoder_results()])
    finally:
        eng.set_option("GEMM16_TAIL", 2)
        eng.set_option("GEMM16_PERSIST", 2)
        eng.set_option("X16_KM", 1)
    for got in outs[1:]:
        for a, b in zip(outs[0], got):
            assert torch.equal(a, b)


@pytest.mark.parametrize("T", [809, 803, 47, 50])
def test_features_km_row_pairs_any_tail(eng, T):
    """The feature kernel's 16-k-major image stores go out a row pair at a time (a wave-private
    transpose into whole 128-B lines); a block whose last row has no partner (T' = T // 3 with an
    odd number of rows in the last 16-row block: T' = 269, 267, 15) stores that row alone.  The
    encoder outputs through casr_encode_fbank with the 16-k-major images equal those with row
    images bit for bit, ragged lengths included."""
    if eng.precision() != "s16x3":
        pytest.skip("the split-f16 images only")
    bind(eng, "peaked")
    frames = [T, T - 4, max(3, T // 2), 7]
    fb, fr = batch_fbank(frames, eng.device)
    outs = []
    try:
        for km in (1, 0):
            eng.set_option("X16_KM", km)
            eng.encode_fbank(fb, fr)
            assert eng.device_flags() == 0
            outs.append([t.cpu() for t in eng.encoder_results()])
    finally:
        eng.set_option("X16_KM", 1)
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("B", [1, 33, 129])
def test_odd_batches_greedy_match_oracle(eng, B):
    """Batch sizes at the layout boundaries, through casr_encode_fbank (T = 60, T' = 20, ragged
    last utterance): B = 1 (one 16-row recurrence group, 32-row projection blocks, one attention
    block), B = 33 (the 64-row projection blocks again, a partial 16-row group), B = 129 (the
    recurrence back on 32 x 16 workgroups with a partial 32-row group).  Tokens identical to
    the CPU oracle, scores within 2e-3."""
    enc_sd, dec_sd = synthetic_state_dicts(CFG, peaked=True)
    eng.bind(pack_weights(CFG, enc_sd, dec_sd))
    frames = [60] * (B - 1) + [33]
    fb, fr = batch_fbank(frames, eng.device)
    flen = eng.encode_fbank(fb, fr)
    out = eng.greedy()
    assert eng.device_flags() == 0
    toks, score = greedy_outputs(out["tokens"].cpu().numpy(), out["out_len"].cpu().numpy(),
                                 out["finished"].cpu().numpy().astype(bool), out["accum"].cpu().numpy())
    feats = [O.features_from_fbank(fbank_for(b, t)) for b, t in enumerate(frames)]
    assert flen.cpu().tolist() == [f.shape[0] for f in feats]
    r = O.greedy_decode(feats, [f.shape[0] for f in feats], enc_sd, dec_sd)
    assert toks == r["tokens"]
    np.testing.assert_allclose(score, r["score"], atol=2e-3, rtol=0)


@pytest.mark.parametrize("B,graphs", [(1, False), (19, True), (32, False), (32, True)])
def test_greedy_ksplit_small_batch(eng, B, graphs):
    """BASELINE config 2's decode rows (R <= 32): the folded GEMM with its k range split over four
    workgroups per output block (CASR_OPT_DEC_KSPLIT = 1, default; the last to arrive adds the four
    sums in a fixed order) against one workgroup per output block: tokens identical, scores within
    1e-4 (the same products summed in another order: 1.5e-5 measured on sums near -45), both equal to the CPU oracle's tokens, the
    split path bitwise stable over repeated runs (graph replays included), and its arrival counters
    left at zero (a second decode matches the first)."""
    enc_sd, dec_sd = synthetic_state_dicts(CFG, peaked=True)
    eng.bind(pack_weights(CFG, enc_sd, dec_sd))
    frames = [120] * (B - 1) + [57]
    fb, fr = batch_fbank(frames, eng.device)
    eng.encode_fbank(fb, fr)
    eng.set_graphs(3 if graphs else 2)
    res = {}
    try:
        for ks in (0, 1):
            eng.set_option("DEC_KSPLIT", ks)
            runs = []
            for _ in range(3):
                out = eng.greedy()
                assert eng.device_flags() == 0
                runs.append({k: v.cpu().clone() for k, v in out.items() if torch.is_tensor(v)})
            for r2 in runs[1:]:
                for k in runs[0]:
                    assert torch.equal(runs[0][k], r2[k]), k
            res[ks] = runs[0]
    finally:
        eng.set_option("DEC_KSPLIT", 1)
        eng.set_graphs(2)
    a, b = res[0], res[1]
    assert torch.equal(a["tokens"], b["tokens"])
    assert torch.equal(a["out_len"], b["out_len"])
    np.testing.assert_allclose(b["accum"].numpy(), a["accum"].numpy(), atol=1e-4, rtol=0)
    toks, score = greedy_outputs(b["tokens"].numpy(), b["out_len"].numpy(), b["finished"].numpy().astype(bool),
                                 b["accum"].numpy())
    feats = [O.features_from_fbank(fbank_for(i, t)) for i, t in enumerate(frames)]
    r = O.greedy_decode(feats, [f.shape[0] for f in feats], enc_sd, dec_sd)
    assert toks == r["tokens"]
    np.testing.assert_allclose(score, r["score"], atol=2e-3, rtol=0)


@pytest.mark.parametrize("B,graphs", [(1, False), (19, True), (32, False), (32, True), (64, True)])
def test_greedy_split_attention_small_batch(eng, B, graphs):
    """BASELINE config 2's decode rows (R <= 64): the folded greedy attention with each utterance's
    time steps split over 8 (R <= 32) or 4 workgroups (CASR_OPT_ATTN_SPLIT = 1; off by default,
    DESIGN 9d item 5; the last to arrive merges the ranges' softmax maxima, sums and unnormalised contexts in split order)
    against one workgroup per utterance.  Ragged lengths from 60 to 800 frames, so the later ranges
    of the short utterances hold no step at all.  Tokens identical, scores within 1e-4, both equal
    to the CPU oracle's tokens, the split path bitwise stable over repeated runs (graph replays
    included) and its arrival counters left at zero (a second decode matches the first)."""
    enc_sd, dec_sd = synthetic_state_dicts(CFG, peaked=True)
    eng.bind(pack_weights(CFG, enc_sd, dec_sd))
    rs = np.random.RandomState(100 + B)
    frames = [800] if B == 1 else [800, 60] + rs.randint(60, 801, size=B - 2).tolist()
    fb, fr = batch_fbank(frames, eng.device)
    eng.encode_fbank(fb, fr)
    eng.set_graphs(3 if graphs else 2)
    res = {}
    try:
        for sp in (0, 1):
            eng.set_option("ATTN_SPLIT", sp)
            runs = []
            for _ in range(3):
                out = eng.greedy()
                assert eng.device_flags() == 0
                runs.append({k: v.cpu().clone() for k, v in out.items() if torch.is_tensor(v)})
            for r2 in runs[1:]:
                for k in runs[0]:
                    assert torch.equal(runs[0][k], r2[k]), k
            res[sp] = runs[0]
    finally:
        eng.set_option("ATTN_SPLIT", 0)
        eng.set_graphs(2)
    a, b = res[0], res[1]
    assert torch.equal(a["tokens"], b["tokens"])
    assert torch.equal(a["out_len"], b["out_len"])
    np.testing.assert_allclose(b["accum"].numpy(), a["accum"].numpy(), atol=1e-4, rtol=0)
    toks, score = greedy_outputs(b["tokens"].numpy(), b["out_len"].numpy(), b["finished"].numpy().astype(bool),
                                 b["accum"].numpy())
    feats = [O.features_from_fbank(fbank_for(i, t)) for i, t in enumerate(frames)]
    r = O.greedy_decode(feats, [f.shape[0] for f in feats], enc_sd, dec_sd)
    assert toks == r["tokens"]
    np.testing.assert_allclose(score, r["score"], atol=2e-3, rtol=0)
