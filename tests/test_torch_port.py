"""The torch-CPU port that bench.py times as its CPU baseline (oracle/torch_port.py) decodes like
the reference: tokens identical to the reference-captured goldens, scores within 2e-4 (greedy and
beam), on both weight suites."""
import numpy as np
import pytest

from golden_util import load_golden, fbank_for, golden_frames
from oracle import torch_port as TP
from casr.config import CasrConfig
from casr.weights import synthetic_state_dicts

G, META = load_golden()
CFG = CasrConfig()
FRAMES = golden_frames(META)


def _port(name):
    enc_sd, dec_sd = synthetic_state_dicts(CFG, peaked=(name == "peaked"))
    feats = [TP.features_from_fbank(fbank_for(b, t)) for b, t in enumerate(FRAMES)]
    return TP.TorchPort(enc_sd, dec_sd), feats


def test_features_match_reference():
    f = TP.features_from_fbank(fbank_for(0, 101)).numpy()
    np.testing.assert_allclose(f, G["feat_cmvn_T101"], rtol=0, atol=2e-5)


@pytest.mark.parametrize("name", ["plain", "peaked"])
def test_greedy_matches_reference(name):
    m, feats = _port(name)
    toks, score = m.greedy(feats)
    gold = META[name]["greedy"]
    assert toks == gold["tokens"]
    np.testing.assert_allclose(score, gold["score"], rtol=0, atol=2e-4)


@pytest.mark.parametrize("name", ["plain", "peaked"])
@pytest.mark.parametrize("k", [4, 8])
def test_beam_matches_reference(name, k):
    m, feats = _port(name)
    toks, score = m.beam(feats, k)
    gold = META[name][f"beam{k}"]
    assert toks == gold["tokens"]
    np.testing.assert_allclose(score, gold["score"], rtol=0, atol=2e-4)
