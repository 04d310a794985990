"""Deterministic stand-in for ``kenlm.LanguageModel`` (model.py:13, main.py:82).

KenLM (third-party C++, version unpinned) and its LM file are absent, so LM scores have
no parity fixture; only the second-pass combination rule (model.py:749-763) is pinned,
using this stub on both the reference side (make_golden.py) and the tests.
Tokens are rendered with the private-use map ``PUA_INT2WORD`` (id -> chr(0xE000 + id)) so
the captured texts decode back to token ids exactly.
"""

PUA_BASE = 0xE000


def pua_int2word(vocab_size=5004):
    return {i: chr(PUA_BASE + i) for i in range(vocab_size)}


def pua_to_ids(text):
    return [ord(ch) - PUA_BASE for ch in text]


class StubLM:
    def score(self, s, bos=True):
        ids = [ord(w) - PUA_BASE for w in s.split(" ") if w]
        return -0.37 * len(ids) - 0.011 * sum(i % 97 for i in ids) - (0.5 if bos else 0.0)
