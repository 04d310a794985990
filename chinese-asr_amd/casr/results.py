"""Host-side result assembly with the reference's exact finalize rules.

The device returns integer token arrays and float32 scores; this module turns them into the
reference's Python results: greedy (model.py:582-602), beam first-max / second-pass
selection (parse_finished_tensors, model.py:708-765) and the unfinished fallback
(model.py:961-972).  Also the reference's record types (util.py:2403-2406)."""
from collections import namedtuple

import numpy as np

EvalOutput = namedtuple('EvalOutput', ('pred_text', 'score', 'text', 'wer', 'n', 'alignment',
                                       'audio_feat_len', 'text_len'))
EncoderOutput = namedtuple('EncoderOutput', ('out', 'out_lens', 'state'))
DecoderOutput = namedtuple('DecoderOutput', ('logit', 'attn_hidden_state', 'alignment', 'cell_state'))


def edit_distance(a, b):
    """Levenshtein distance (the reference calls python-Levenshtein, util.py:237-262)."""
    m, n = len(a), len(b)
    if m == 0:
        return n
    if n == 0:
        return m
    prev = list(range(n + 1))
    for i in range(1, m + 1):
        cur = [i] + [0] * n
        ai = a[i - 1]
        for j in range(1, n + 1):
            cur[j] = prev[j - 1] if ai == b[j - 1] else 1 + min(prev[j - 1], prev[j], cur[j - 1])
        prev = cur
    return prev[n]


def edit_ops(pred, ref):
    """(insert, delete, replace) counts of one minimal edit script turning ``pred`` into ``ref``
    (python-Levenshtein ``editops(pred, ref)`` semantics, util.py:250-256).  The total always equals
    the distance; how it splits into the three kinds depends on the backtrace's tie order, which
    here prefers replace, then delete, then insert.  python-Levenshtein is absent (no fixture):
    the split is parity-unpinned, the total is exact."""
    m, n = len(pred), len(ref)
    d = np.zeros((m + 1, n + 1), np.int64)
    d[:, 0] = np.arange(m + 1)
    d[0, :] = np.arange(n + 1)
    for i in range(1, m + 1):
        for j in range(1, n + 1):
            d[i, j] = d[i - 1, j - 1] if pred[i - 1] == ref[j - 1] else \
                1 + min(d[i - 1, j - 1], d[i - 1, j], d[i, j - 1])
    i, j, ins, dele, rep = m, n, 0, 0, 0
    while i > 0 or j > 0:
        if i > 0 and j > 0 and pred[i - 1] == ref[j - 1] and d[i, j] == d[i - 1, j - 1]:
            i, j = i - 1, j - 1
        elif i > 0 and j > 0 and d[i, j] == d[i - 1, j - 1] + 1:
            rep += 1
            i, j = i - 1, j - 1
        elif i > 0 and d[i, j] == d[i - 1, j] + 1:
            dele += 1
            i -= 1
        else:
            ins += 1
            j -= 1
    return ins, dele, rep


def get_wer(pred, ref, normalize=True, return_tuple=False):
    """util.py:237-262: distance(pred, ref) [/ len(ref)]; return_tuple: (all, insert, delete,
    replace) [/ len(ref)] from the edit script (edit_ops)."""
    n = len(ref) * 1.
    if not return_tuple:
        r = edit_distance(pred, ref)
        return r / n if normalize else r
    ins, dele, rep = edit_ops(pred, ref)
    r = (ins + dele + rep, ins, dele, rep)
    return tuple(e / n for e in r) if normalize else r


def greedy_outputs(tokens, out_len, finished, accum):
    """model.py:582-593.  Host numpy inputs.  Returns (token lists, scores)."""
    toks = [tokens[b, :out_len[b]].tolist() for b in range(tokens.shape[0])]
    score = []
    for b, t in enumerate(toks):
        if len(t) == 0:
            score.append(0.0)
        else:
            score.append(float(accum[b]) / (int(out_len[b]) + int(finished[b])))
    return toks, score


def greedy_steps(out_len, finished, max_len):
    """Iterations the reference loop runs (model.py:578 breaks once all are finished)."""
    if len(finished) and bool(np.all(finished)):
        return int(np.max(out_len)) + 1
    return max_len


def records_by_utterance(rec_tokens, rec_score, rec_valid):
    """Finished hypotheses per utterance in the reference's list order (step, then rank):
    b -> [(tokens, score)] (model.py:715-733)."""
    bs, ls, cs = np.nonzero(rec_valid)  # row-major: already in (utterance, step, rank) order
    scores = rec_score[bs, ls, cs].tolist()
    # token lists converted per step, only the l tokens a step-l record holds
    toks = [None] * len(bs)
    for l in np.unique(ls).tolist():
        sel = np.nonzero(ls == l)[0]
        rows = rec_tokens[bs[sel], l, cs[sel], :l].tolist()
        for i, t in zip(sel.tolist(), rows):
            toks[i] = t
    res = {}
    for b, t, s in zip(bs.tolist(), toks, scores):
        res.setdefault(b, []).append((t, s))
    return res


def second_pass_select(records, int2word, lm_model, lm_weight, length_weight):
    """parse_finished_tensors with second_pass (model.py:749-763): for > 1 finished
    hypotheses pick argmax(logp + lm_w * LM(' '.join(words), bos=True) + len_w * len);
    returns the original (tokens, logp)."""
    out = {}
    for b, v in records.items():
        if len(v) == 1:
            out[b] = v[0]
            continue
        word = int2word.__getitem__
        lm = [lm_model.score(' '.join(map(word, t)), bos=True) for t, _ in v]
        comb = [s + lm_weight * q + length_weight * len(t) for (t, s), q in zip(v, lm)]
        out[b] = v[int(np.argmax(comb))]
    return out


def _word_array(int2word, n):
    """int2word as an object array over ids 0 .. n - 1 (the word strings themselves, not copies),
    or None when the mapping does not cover that range."""
    try:
        return np.array([int2word[i] for i in range(n)] + [None], dtype=object)[:n]
    except (KeyError, IndexError, TypeError):
        return None


def second_pass_arrays(rec_tokens, rec_score, rec_valid, int2word, lm_model, lm_weight, length_weight):
    """second_pass_select(records_by_utterance(rec_tokens, rec_score, rec_valid), ...) from the record
    arrays directly: the same choice per utterance with records (model.py:749-763) and the same
    returned (tokens, logp), the LM called with the same sentences in the same order, but without
    a Python token list per record (the words come from one object-array gather, and only the
    chosen records become lists).  Falls back to the list form when int2word does not cover the
    token ids."""
    bs, ls, cs = np.nonzero(rec_valid)
    if len(bs) == 0:
        return {}
    full = rec_tokens[bs, ls, cs]  # [n][L]: the records' token rows, in (utterance, step, rank) order
    used = full[np.arange(full.shape[1])[None, :] < ls[:, None]]  # the l tokens of each step-l record
    warr = _word_array(int2word, int(used.max()) + 1) if used.size else np.array([], dtype=object)
    if warr is None or (used.size and int(used.min()) < 0):
        return second_pass_select(records_by_utterance(rec_tokens, rec_score, rec_valid), int2word, lm_model,
                                  lm_weight, length_weight)
    full = np.where(np.arange(full.shape[1])[None, :] < ls[:, None], full, 0)  # (slots past l unused)
    scores = rec_score[bs, ls, cs].tolist()
    lens = ls.tolist()
    starts = np.flatnonzero(np.r_[True, bs[1:] != bs[:-1]]).tolist() + [len(bs)]
    words = None
    out = {}
    for a, z in zip(starts[:-1], starts[1:]):
        b = int(bs[a])
        if z - a == 1:
            out[b] = (full[a, :lens[a]].tolist(), scores[a])
            continue
        if words is None:
            words = warr[full] if len(warr) else np.empty(full.shape, dtype=object)
        rows = words[a:z].tolist()
        lm = [lm_model.score(' '.join(row[:l]), bos=True) for row, l in zip(rows, lens[a:z])]
        comb = [sc + lm_weight * q + length_weight * l for sc, q, l in zip(scores[a:z], lm, lens[a:z])]
        i = a + int(np.argmax(comb))
        out[b] = (full[i, :lens[i]].tolist(), scores[i])
    return out

