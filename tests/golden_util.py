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


def near_tie_beam_check(tokens, score, gold, atol, max_flips=1):
    """Beam parity where f32 summation order can flip near-tied candidates: every score within
    ``atol`` of the reference's, token sequences identical except for at most ``max_flips``
    utterances (whose scores are then within ``atol`` too)."""
    import numpy as np
    np.testing.assert_allclose(score, gold["score"], rtol=0, atol=atol)
    flips = [b for b, t in enumerate(tokens) if list(t) != gold["tokens"][b]]
    assert len(flips) <= max_flips, flips
