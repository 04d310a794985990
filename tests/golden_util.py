"""Shared fixture helpers: regenerate the seeded inputs the golden vectors were captured on
(tests/golden/make_golden.py) and load the stored reference outputs."""
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")


def load_golden():
    g = np.load(os.path.join(GOLD, "golden.npz"))
    with open(os.path.join(GOLD, "golden.json"), encoding="utf-8") as f:
        meta = json.load(f)
    return g, meta


def fbank_for(b, T, n_mels=80):
    return np.random.RandomState(1234 + b).standard_normal((T, n_mels)).astype(np.float32)


def golden_frames(meta):
    return [int(x) for x in meta["frames"]]


def teacher_forced_score(feat, tokens, enc_sd, dec_sd, sos=1):
    """Oracle log-probability of one hypothesis (the sum of its tokens' log-softmax values fed
    back one by one, model.py:829-836 on a single beam): what beam search reports as its score
    when the hypothesis survives every pruning step unfinished."""
    from oracle import casr_oracle as O
    enc, (h, c) = O.encoder_forward([feat], [feat.shape[0]], enc_sd)
    mask = O.mask_for_softmax(np.array([feat.shape[0]]))
    keys = O.compute_keys(enc, dec_sd)
    ctx = np.zeros((1, enc.shape[2]), np.float32)
    tok = np.array([sos])
    tot = np.float32(0.0)
    for t in tokens:
        logit, h, c, ctx, _ = O.decoder_step(enc, mask, keys, tok, h, c, ctx, dec_sd)
        tot = np.float32(tot + O._log_softmax(logit)[0][t])
        tok = np.array([t])
    return float(tot)


def near_tie_beam_check(tokens, score, gold, atol, rescore=None, atol_same=None, max_flips=1):
    """Beam parity where f32 summation order can flip near-tied candidates at the pruning
    boundary (rank k vs k + 1 of some step): token sequences identical except for at most
    ``max_flips`` utterances.  Utterances that do not flip keep the plain tolerance
    (``atol_same``, default ``atol``).  A flipped utterance is accepted only when
      * its score is within ``atol`` of the reference's, and
      * with ``rescore(b, tokens) -> teacher-forced oracle score`` (unfinished hypotheses): both
        hypotheses are genuine, i.e. the oracle re-scores the reference's hypothesis to the
        reference's score and ours to our score, each within ``atol_same``.
    So the two searches kept different, correctly scored hypotheses whose scores differ by less
    than ``atol``; the token gap at the first diverging position need not be small (measured on
    plain beam 16, utterance 3: 0.024 at position 32), because the flip happens earlier, at a rank
    boundary, between prefixes of other hypotheses."""
    atol_same = atol if atol_same is None else atol_same
    score = np.asarray(score, np.float64)
    gs = np.asarray(gold["score"], np.float64)
    flips = [b for b, t in enumerate(tokens) if list(t) != gold["tokens"][b]]
    assert len(flips) <= max_flips, flips
    same = [b for b in range(len(tokens)) if b not in flips]
    np.testing.assert_allclose(score[same], gs[same], rtol=0, atol=atol_same)
    for b in flips:
        assert abs(score[b] - gs[b]) <= atol, (b, score[b], gs[b])
        if rescore is not None:
            assert abs(rescore(b, gold["tokens"][b]) - gs[b]) <= atol_same, b
            assert abs(rescore(b, list(tokens[b])) - score[b]) <= atol_same, b


TIE_ATOL = 1e-4  # the largest rank tie measured was 2.3e-5; 4x margin


def records_match_up_to_rank_ties(mine, gold, atol, tie_atol=TIE_ATOL):
    """Finished-hypothesis records (step, then rank order: parse_finished_tensors, model.py:708-733)
    equal up to the order of equal-scored records within one step.  Each step must record the same
    hypotheses (token lists) with scores within ``atol``; two records of one step may appear in the
    other order only when their scores differ by at most ``tie_atol`` (1e-4, not the score
    tolerance), since which of two candidates torch.topk ranks first (model.py:855) is then a matter
    of f32 summation order (measured: two EOS candidates of one step 4e-6 apart swapped between the
    product's s16x3 and the oracle, and 2.3e-5 in another case, tools/probes/beam_tie_probe.py).
    Returns True, or False when the lists differ otherwise."""
    def by_step(recs):
        out = {}
        for t, s in recs:
            out.setdefault(len(t), []).append((tuple(t), float(s)))
        return out
    a, b = by_step(mine), by_step(gold)
    if sorted(a) != sorted(b):
        return False
    for l in a:
        ra, rb = a[l], b[l]
        if sorted(t for t, _ in ra) != sorted(t for t, _ in rb) or len(set(t for t, _ in ra)) != len(ra):
            return False
        sb = dict(rb)
        if any(abs(s - sb[t]) > atol for t, s in ra):
            return False
        pos = {t: i for i, (t, _) in enumerate(rb)}
        for i in range(len(ra)):
            for j in range(i + 1, len(ra)):
                if pos[ra[i][0]] > pos[ra[j][0]] and abs(ra[i][1] - ra[j][1]) > tie_atol:
                    return False
    return True


def near_tie_records_check(mine, gold, atol, rescore=None):
    """Finished-hypothesis records of one utterance (parse_finished_tensors order: step, then
    rank; each (tokens, score)) against the oracle's.  Returns True when the lists are identical
    (tokens equal, scores within ``atol``), False when they diverge at a near-tied pruning
    decision, which is accepted only when:
      * every record before the first differing one is identical (tokens, scores within atol);
      * the two diverging records are genuine hypotheses: with ``rescore(tokens) -> oracle
        log-probability of tokens + EOS`` (teacher-forced), ours re-scores to our score and the
        oracle's to the oracle's, each within ``atol``.
    So both searches kept correctly scored hypotheses and split only where f32 summation order
    can reorder candidates of (near-)equal score (the same rule as near_tie_beam_check)."""
    n = min(len(mine), len(gold))
    d = next((i for i in range(n) if list(mine[i][0]) != list(gold[i][0])), None)
    if d is None and len(mine) == len(gold):
        np.testing.assert_allclose([x[1] for x in mine], [x[1] for x in gold], rtol=0, atol=atol)
        return True
    d = n if d is None else d
    np.testing.assert_allclose([x[1] for x in mine[:d]], [x[1] for x in gold[:d]], rtol=0, atol=atol)
    assert rescore is not None, "records diverge and no rescoring was given"
    for rec in (mine[d:d + 1] + gold[d:d + 1]):
        assert abs(rescore(list(rec[0])) - rec[1]) <= atol, (d, rec)
    return False
