"""Every row of the metric's shapes against the CPU oracle, in both MFMA arithmetics.

The north star promises identical token ids for the headline batch, so no row is sampled here:

  * greedy, B = 256, T = 800 (model.py:503-602): all 256 rows, on the bench weights (proj x40,
    no EOS bias: every row runs all 40 steps) AND on the EOS-bias weights (rows finish at
    different steps, so the early-finish bookkeeping of model.py:567-578 -- accum through the
    first EOS inclusive, final_lens, finished, the all-finished early exit -- is pinned at full
    size).  Tokens, lengths, finished flags and the loop's step count identical; accum and score
    within 2e-3.
  * beam 8 at B = 256 (the metric's beam line) and at B = 128 (BASELINE config 3), T = 800, bench
    weights (model.py:604-987): all 256 / 128 utterances.  Tokens identical and scores within
    2e-3, except that at most ONE utterance per arithmetic and shape may split at a near-tied
    pruning step (near_tie_beam_check: both hypotheses rescored by the oracle to their own scores).

Cost: the oracle runs once per weight set and is shared by both arithmetics (lru_cache): greedy
B = 256 twice (~20 s each on 8 container cores) and beam 8 over utterances 0..255 in 32-utterance
chunks (~15 s per chunk).  The beam oracle is batch-invariant on these weights (with
no EOS bias no chunk stops early, and an early stop could not change a first-max answer anyway),
so the B = 128 batch is checked against the first four chunks of the same oracle run.  Each test
covers one chunk, so no single test runs for more than about half a minute.  Added runtime of
the file on the GPU box: about 3-4 minutes, almost all of it oracle time.
"""
import functools

import numpy as np
import pytest
import torch

from golden_util import fbank_for, near_tie_beam_check, teacher_forced_score
from oracle import casr_oracle as O
from casr.config import CasrConfig
from casr.results import greedy_outputs, greedy_steps
from casr.weights import synthetic_state_dicts

pytestmark = pytest.mark.gpu

CFG = CasrConfig()
T = 800
TP = T // 3
CHUNK = 32
PRECS = ["s16x3", "f32"]


@functools.lru_cache(maxsize=None)
def weights(name):
    if name == "bench":
        return synthetic_state_dicts(CFG, peaked=True, eos_bias=0.0)
    return synthetic_state_dicts(CFG, peaked=True)  # the EOS-bias recipe (eos_bias 12)


@functools.lru_cache(maxsize=None)
def oracle_feats(b):
    return O.features_from_fbank(fbank_for(b, T))


def _fbank(B):
    return torch.from_numpy(np.stack([fbank_for(b, T) for b in range(B)]))


def _engine(name, prec):
    from casr.engine import Engine
    e = Engine(CFG, *weights(name))
    e.set_precision(prec)
    assert e.precision() == prec
    return e


@functools.lru_cache(maxsize=None)
def gpu_greedy(name, prec, B=256):
    e = _engine(name, prec)
    try:
        e.encode_fbank(_fbank(B).to(e.device), torch.full((B,), T, dtype=torch.int32, device=e.device))
        out = e.greedy()
        assert e.device_flags() == 0
        return {k: v.cpu().numpy() for k, v in out.items() if torch.is_tensor(v)}
    finally:
        e.close()


@functools.lru_cache(maxsize=None)
def oracle_greedy(name, B=256):
    feats = [oracle_feats(b) for b in range(B)]
    return O.greedy_decode(feats, [TP] * B, *weights(name))


@pytest.mark.parametrize("name", ["bench", "eos"])
@pytest.mark.parametrize("prec", PRECS)
def test_headline_greedy_b256_every_row(prec, name):
    """All 256 rows of the headline greedy batch against one oracle batch of the same 256
    utterances (model.py:503-602), through casr_encode_fbank as bench.py runs it."""
    g = gpu_greedy(name, prec)
    r = oracle_greedy(name)
    fin = g["finished"].astype(bool)
    toks, score = greedy_outputs(g["tokens"], g["out_len"], fin, g["accum"])
    assert toks == r["tokens"]
    np.testing.assert_array_equal(g["out_len"], r["text_len"])
    np.testing.assert_array_equal(fin, r["finished"])
    assert greedy_steps(g["out_len"], fin, CFG.max_len) == r["steps"]
    np.testing.assert_allclose(g["accum"], r["accum"], rtol=0, atol=2e-3)
    np.testing.assert_allclose(score, r["score"], rtol=0, atol=2e-3)
    if name == "eos":  # the early-finish bookkeeping is exercised: rows end at different steps
        assert fin.sum() > 0 and len(set(g["out_len"][fin].tolist())) > 5
    else:
        assert not fin.any() and r["steps"] == CFG.max_len
    # every step's token of the rows still running agrees too (not only the kept prefix)
    for b in range(256):
        n = min(int(g["out_len"][b]) + int(fin[b]), r["steps"])
        np.testing.assert_array_equal(g["tokens"][b, :n], r["all_tokens"][b, :n])


@functools.lru_cache(maxsize=None)
def gpu_beam(prec, B, k=8):
    e = _engine("bench", prec)
    try:
        e.encode_fbank(_fbank(B).to(e.device), torch.full((B,), T, dtype=torch.int32, device=e.device))
        r = e.beam(k)
        assert e.device_flags() == 0
        toks, blen, sc, st = (x.cpu().numpy() for x in (r["tokens"], r["length"], r["score"], r["steps"]))
        return [toks[b, :blen[b]].tolist() for b in range(B)], sc, int(st[0])
    finally:
        e.close()


@functools.lru_cache(maxsize=None)
def oracle_beam_chunk(c, k=8):
    rows = range(c * CHUNK, (c + 1) * CHUNK)
    r = O.beam_decode([oracle_feats(b) for b in rows], [TP] * CHUNK, *weights("bench"), k)
    return r


def _rescore(b, tokens):
    """Oracle log-probability of a hypothesis: unfinished (the sum over its tokens) or finished
    (+ the EOS token); the caller compares it with the reported score, so the reading that
    reproduces that score is the hypothesis's own."""
    feat = oracle_feats(b)
    return teacher_forced_score(feat, list(tokens), *weights("bench")), \
        teacher_forced_score(feat, list(tokens) + [CFG.eos], *weights("bench"))


FLIPS = {}  # (prec, B) -> utterances that split at a near tie, over all chunks of that batch


def _beam_chunk_vs_oracle(prec, B, c):
    toks, sc, steps = gpu_beam(prec, B)
    assert steps == CFG.max_len  # bench weights: no EOS bias, every step runs (as the oracle's)
    ref = oracle_beam_chunk(c)
    assert ref["steps"] == CFG.max_len
    lo = c * CHUNK
    mine = toks[lo:lo + CHUNK]

    def rescore(j, t):
        a, f = _rescore(lo + j, t)
        want = sc[lo + j] if list(t) == mine[j] else ref["score"][j]
        return a if abs(a - want) <= abs(f - want) else f

    near_tie_beam_check(mine, sc[lo:lo + CHUNK], ref, atol=2e-3, rescore=rescore)
    flips = [lo + j for j in range(CHUNK) if mine[j] != ref["tokens"][j]]
    FLIPS.setdefault((prec, B), set()).update(flips)
    assert len(FLIPS[(prec, B)]) <= 1, sorted(FLIPS[(prec, B)])


@pytest.mark.parametrize("chunk", range(256 // CHUNK))
@pytest.mark.parametrize("prec", PRECS)
def test_metric_beam8_b256_every_utterance(prec, chunk):
    """The metric's beam line, beam 8 at B = 256 (R = 2048 rows, the folded step with the fused
    select under s16x3): utterances [32 chunk, 32 chunk + 32) of the batch against the oracle."""
    _beam_chunk_vs_oracle(prec, 256, chunk)


@pytest.mark.parametrize("chunk", range(128 // CHUNK))
@pytest.mark.parametrize("prec", PRECS)
def test_config3_beam8_b128_every_utterance(prec, chunk):
    """BASELINE config 3, beam 8 at B = 128 (R = 1024 rows, 4 rows per attention block):
    utterances [32 chunk, 32 chunk + 32) of the batch against the oracle."""
    _beam_chunk_vs_oracle(prec, 128, chunk)
