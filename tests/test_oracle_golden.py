"""Pin the CPU oracle (oracle/casr_oracle.py) against vectors captured from the reference
implementation itself (tests/golden/make_golden.py) and the reference's own encoder
known-answer test (encoder.py:636-652)."""
import numpy as np
import pytest

from golden_util import load_golden, fbank_for, golden_frames, near_tie_beam_check, teacher_forced_score
from oracle import casr_oracle as O
from casr.config import CasrConfig
from casr.weights import synthetic_state_dicts, encoder_keys, decoder_keys
from stub_lm import StubLM, pua_int2word

G, META = load_golden()
CFG = CasrConfig()


def test_state_dict_key_order_matches_reference():
    assert [k for k, _ in encoder_keys(CFG)] == META["encoder_key_order"]
    assert [k for k, _ in decoder_keys(CFG)] == META["decoder_key_order"]


def test_encoder_kat_reference_numbers():
    # encoder.py:652 comment: 110345.5000, 2048, 28160 (all params = 1, lens [10, 8, 23, 14])
    kat = META["encoder_kat"]
    assert kat["out_sum"] == pytest.approx(110345.5, rel=1e-5)
    enc_sd = {k: np.ones(s, np.float32) for k, s in encoder_keys(CFG)}
    lens = [10, 8, 23, 14]
    out, (h, c) = O.encoder_forward([np.ones((l, 720), np.float32) for l in lens], lens, enc_sd)
    assert out.shape == (23, 4, 512)
    assert float(out.sum()) == pytest.approx(kat["out_sum"], rel=1e-5)
    assert float(h.sum()) == pytest.approx(2048.0, rel=1e-6)
    assert float(c.sum()) == pytest.approx(28160.0, rel=1e-6)


@pytest.mark.parametrize("T", [101, 800])
def test_features_match_reference(T):
    fb = fbank_for(0 if T == 101 else 1, T)
    raw = O.stack_frames(O.add_delta_deltas(fb))
    f = O.cmvn(raw, 1e-6)
    if T <= 128:
        np.testing.assert_allclose(raw, G[f"feat_raw_T{T}"], atol=2e-6, rtol=0)
        np.testing.assert_allclose(f, G[f"feat_cmvn_T{T}"], atol=5e-6, rtol=0)
    else:
        for nm, x in (("raw", raw), ("cmvn", f)):
            np.testing.assert_allclose(x[:6], G[f"feat_{nm}_T{T}_head"], atol=5e-6, rtol=0)
            np.testing.assert_allclose(x[-3:], G[f"feat_{nm}_T{T}_tail"], atol=5e-6, rtol=0)
            np.testing.assert_allclose(x.astype(np.float64).sum(0), G[f"feat_{nm}_T{T}_colsum"], atol=1e-3)


def test_log_mel_matches_reference():
    np.testing.assert_allclose(O.create_fb_matrix(), G["fb_matrix"], atol=2e-5, rtol=0)
    lm = O.log_mel(G["wav0"])
    assert lm.shape == G["wav0_logmel"].shape
    # float32 STFT rounding vs torch's FFT: log-domain differences stay tiny
    np.testing.assert_allclose(lm, G["wav0_logmel"], atol=5e-4, rtol=0)
    feats = O.stack_frames(O.add_delta_deltas(lm))
    np.testing.assert_allclose(feats, G["wav0_features"], atol=2e-3, rtol=0)


def _suite(name):
    frames = golden_frames(META)
    feats = [O.features_from_fbank(fbank_for(b, T)) for b, T in enumerate(frames)]
    lens = [f.shape[0] for f in feats]
    enc_sd, dec_sd = synthetic_state_dicts(CFG, peaked=(name == "peaked"))
    return feats, lens, enc_sd, dec_sd


@pytest.mark.parametrize("name", ["plain", "peaked"])
def test_encoder_matches_reference(name):
    feats, lens, enc_sd, dec_sd = _suite(name)
    enc, (h, c) = O.encoder_forward(feats, lens, enc_sd)
    np.testing.assert_allclose(enc[::7, :, ::64], G[f"{name}_enc_slice"], atol=1e-5, rtol=0)
    np.testing.assert_allclose(h, G[f"{name}_enc_h"], atol=1e-5, rtol=0)
    np.testing.assert_allclose(c, G[f"{name}_enc_c"], atol=1e-5, rtol=0)
    np.testing.assert_allclose(enc.astype(np.float64).sum(axis=(0, 2)), G[f"{name}_enc_sum_per_utt"],
                               rtol=1e-5, atol=1e-2)
    keys = O.compute_keys(enc, dec_sd)
    np.testing.assert_allclose(keys.astype(np.float64).sum(axis=(0, 2)), G[f"{name}_keys_sum_per_utt"],
                               rtol=1e-5, atol=1e-2)


@pytest.mark.parametrize("name", ["plain", "peaked"])
def test_greedy_matches_reference(name):
    feats, lens, enc_sd, dec_sd = _suite(name)
    r = O.greedy_decode(feats, lens, enc_sd, dec_sd, return_alignment=True)
    gold = META[name]["greedy"]
    assert r["tokens"] == gold["tokens"]
    assert list(map(int, r["text_len"])) == gold["text_len"]
    assert r["steps"] == gold["steps"]
    np.testing.assert_allclose(r["score"], gold["score"], rtol=0, atol=1e-4)
    np.testing.assert_allclose(r["alignment"][0], G[f"{name}_greedy_align_step0"], atol=1e-6)
    np.testing.assert_allclose(np.stack([a.astype(np.float64).sum(0) for a in r["alignment"]]),
                               G[f"{name}_greedy_align_sum"], atol=1e-5)


@pytest.mark.parametrize("name", ["plain", "peaked"])
@pytest.mark.parametrize("k", [1, 4, 8, 16])
def test_beam_matches_reference(name, k):
    feats, lens, enc_sd, dec_sd = _suite(name)
    r = O.beam_decode(feats, lens, enc_sd, dec_sd, k)
    gold = META[name][f"beam{k}"]
    if name == "plain" and k == 16:
        # unpeaked weights at beam 16: candidates near-tie in f32 (utterance 3 takes another path at
        # an earlier tie and ends 1.2e-3 from the reference's hypothesis); the beam bar is scores
        # within tolerance, so a token difference is accepted only with the scores that close
        near_tie_beam_check(r["tokens"], r["score"], gold, atol=2e-3, atol_same=2e-4,
                            rescore=lambda b, t: teacher_forced_score(feats[b], t, enc_sd, dec_sd))
        return
    assert r["tokens"] == gold["tokens"]
    np.testing.assert_allclose(r["score"], gold["score"], rtol=1e-6, atol=2e-4)


@pytest.mark.parametrize("name", ["plain", "peaked"])
@pytest.mark.parametrize("k", [4, 8])
def test_beam_temperature_matches_reference(name, k):
    """gpd['temperature'] = 0.7: logits / T before the log-softmax (model.py:834), captured from
    the reference by make_golden.py."""
    feats, lens, enc_sd, dec_sd = _suite(name)
    r = O.beam_decode(feats, lens, enc_sd, dec_sd, k, temperature=0.7)
    gold = META[name][f"beam{k}_t07"]
    assert r["tokens"] == gold["tokens"]
    np.testing.assert_allclose(r["score"], gold["score"], rtol=1e-6, atol=2e-4)


@pytest.mark.parametrize("name", ["plain", "peaked"])
def test_beam_second_pass_and_length_weight_match_reference(name):
    feats, lens, enc_sd, dec_sd = _suite(name)
    pua = pua_int2word(CFG.vocab)
    r = O.beam_decode(feats, lens, enc_sd, dec_sd, 4, second_pass=True, lm_model=StubLM(),
                      lm_weight=1.5, length_weight=1.5, int2word=pua)
    gold = META[name]["beam4_lm"]
    assert r["tokens"] == gold["tokens"]
    np.testing.assert_allclose(r["score"], gold["score"], rtol=1e-6, atol=2e-4)
    r = O.beam_decode(feats, lens, enc_sd, dec_sd, 4, lm_weight=1.5, length_weight=1.5)
    gold = META[name]["beam4_lw"]
    assert r["tokens"] == gold["tokens"]
    np.testing.assert_allclose(r["score"], gold["score"], rtol=1e-6, atol=2e-4)
    # BASELINE config 5: beam 16 + second pass
    r = O.beam_decode(feats, lens, enc_sd, dec_sd, 16, second_pass=True, lm_model=StubLM(),
                      lm_weight=1.5, length_weight=1.5, int2word=pua)
    gold = META[name]["beam16_lm"]
    if name == "plain":  # near-tied f32 candidates at beam 16 (test_beam_matches_reference)
        near_tie_beam_check(r["tokens"], r["score"], gold, atol=2e-3, atol_same=2e-4)
        return
    assert r["tokens"] == gold["tokens"]
    np.testing.assert_allclose(r["score"], gold["score"], rtol=1e-6, atol=2e-4)
