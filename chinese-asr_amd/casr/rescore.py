"""Second-pass LM rescoring spread over host worker processes.

The reference rescores on the host, one `lm_model.score(' '.join(words), bos=True)` call per
finished hypothesis of every utterance with more than one (model.py:749-763).  Those calls are
independent, so a serving process can make them in parallel: `ParallelRescorer` keeps a pool of
worker processes, each holding its own LM (built once by a picklable factory, e.g.
`functools.partial(kenlm.Model, path)`), sends each worker a share of the hypotheses as token-id
rows, and combines the returned scores in this process exactly as `second_pass_arrays` does --
the same sentences, the same float operations, the same first-maximum choice -- so the selected
(tokens, logp) per utterance are identical (tests/test_host_logic.py).

The pool must be started before this process initialises the GPU (a worker is a fresh interpreter,
started by fork + exec; bench.py starts it first thing).  The workers never touch the GPU.
"""
import multiprocessing as mp

import numpy as np

from .results import _word_array, second_pass_arrays

_W = {}  # worker-process state: the LM and the word array


def _init(lm_factory, words):
    _W["lm"] = lm_factory()
    _W["words"] = np.asarray(words, dtype=object)


def _score(task):
    toks, lens = task  # int16 [n, L] token ids, int32 [n] lengths
    words, lm = _W["words"], _W["lm"]
    rows = words[toks.astype(np.int64)].tolist()
    return [lm.score(' '.join(r[:l]), bos=True) for r, l in zip(rows, lens.tolist())]


class ParallelRescorer:
    """select(rec_tokens, rec_score, rec_valid, lm_weight, length_weight) -> {b: (tokens, logp)},
    the second_pass_arrays result, with the LM calls made by `workers` processes."""

    def __init__(self, lm_factory, int2word, n_words, workers=4, chunk=4096):
        self.words = _word_array(int2word, n_words)
        if self.words is None:
            raise ValueError("int2word must cover ids 0 .. n_words - 1")
        self.lm_factory = lm_factory
        self.workers = int(workers)
        self.chunk = int(chunk)
        ctx = mp.get_context("spawn")
        self.pool = ctx.Pool(self.workers, initializer=_init, initargs=(lm_factory, list(self.words)))

    def close(self):
        if self.pool is not None:
            self.pool.terminate()
            self.pool.join()
            self.pool = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def select(self, rec_tokens, rec_score, rec_valid, lm_weight, length_weight):
        bs, ls, cs = np.nonzero(rec_valid)
        if len(bs) == 0:
            return {}
        full = rec_tokens[bs, ls, cs]  # [n][L] in (utterance, step, rank) order
        full = np.where(np.arange(full.shape[1])[None, :] < ls[:, None], full, 0)
        if full.size and (int(full.min()) < 0 or int(full.max()) >= len(self.words)):
            # ids outside int2word: the in-process form (its own fallback) decides
            return second_pass_arrays(rec_tokens, rec_score, rec_valid, dict(enumerate(self.words)),
                                      self.lm_factory(), lm_weight, length_weight)
        n = len(bs)
        sc32 = rec_score[bs, ls, cs]
        starts = np.flatnonzero(np.r_[True, bs[1:] != bs[:-1]])
        size = np.diff(np.r_[starts, n])
        # the records whose sentences the LM scores (every record of a multi-record utterance), in order
        multi = np.repeat(size > 1, size)
        idx = np.flatnonzero(multi)
        lm = np.zeros(n, np.float64)
        if len(idx):
            t16 = full[idx].astype(np.int16)
            l32 = ls[idx].astype(np.int32)
            # about two tasks per worker (every worker busy, the last ones short), at most self.chunk rows
            step = max(64, min(self.chunk, -(-len(idx) // (2 * self.workers))))
            tasks = [(t16[i:i + step], l32[i:i + step]) for i in range(0, len(idx), step)]
            out = self.pool.map(_score, tasks)
            lm[idx] = [q for part in out for q in part]
        # comb = logp + lm_w * LM + len_w * len per record, as second_pass_arrays evaluates it on Python
        # floats: (logp + (lm_w * q)) + (len_w * l), each an IEEE double operation, so the vector form
        # gives the same bits; then the first maximum per utterance (np.argmax's choice)
        comb = (sc32.astype(np.float64) + lm_weight * lm) + length_weight * ls.astype(np.float64)
        seg_max = np.maximum.reduceat(comb, starts)
        pos = np.where(comb == np.repeat(seg_max, size), np.arange(n), n)
        first = np.minimum.reduceat(pos, starts)
        for j in np.flatnonzero(first >= n):  # a NaN in the utterance: np.argmax's first-NaN rule
            first[j] = starts[j] + int(np.argmax(comb[starts[j]:starts[j] + size[j]]))
        first = np.where(size == 1, starts, first)  # one record: it (no LM call, model.py:749-763)
        scores = sc32[first].tolist()
        lens = ls[first].tolist()
        rows = full[first]
        return {int(bs[i]): (rows[j, :lens[j]].tolist(), scores[j]) for j, i in enumerate(first.tolist())}
