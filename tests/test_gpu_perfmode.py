"""BASELINE config 2's opt-in perf arithmetic, s16x1 (include/casr.h CASR_PREC_S16X1, SURVEY §7(ii);
the libcasr_hip_s16x1.so build, one f16 MFMA per split product): it runs through the same C ABI,
refuses the other s16 mode, leaves the exact-f32 path bit for bit as the shipped library has it,
and its token agreement with the oracle on config 2's batch (greedy, B = 32, T = 800, bench
weights) is measured and printed.  Tokens are NOT claimed identical: the floor asserted here is
far below the measured rate and only catches a broken build (DESIGN §9d item 8 records the rate)."""
import functools

import numpy as np
import pytest
import torch

from golden_util import fbank_for
from oracle import casr_oracle as O
from casr.config import CasrConfig
from casr.lib import CasrError, pack_weights
from casr.results import greedy_outputs
from casr.weights import synthetic_state_dicts

pytestmark = pytest.mark.gpu

CFG = CasrConfig()
T = 800
B = 32


@functools.lru_cache(maxsize=None)
def bench_weights():
    return synthetic_state_dicts(CFG, peaked=True, eos_bias=0.0)


@functools.lru_cache(maxsize=None)
def oracle_b32():
    feats = [O.features_from_fbank(fbank_for(b, T)) for b in range(B)]
    return O.greedy_decode(feats, [f.shape[0] for f in feats], *bench_weights())


def _run(e, precision=None):
    if precision:
        e.set_precision(precision)
    fb = torch.from_numpy(np.stack([fbank_for(b, T) for b in range(B)])).to(e.device)
    e.encode_fbank(fb, torch.full((B,), T, dtype=torch.int32, device=e.device))
    out = e.greedy()
    assert e.device_flags() == 0
    return {k: v.cpu().numpy() for k, v in out.items() if torch.is_tensor(v)}


def test_s16x1_refuses_other_mode_and_keeps_f32_bits():
    from casr.engine import Engine
    blob = torch.from_numpy(pack_weights(CFG, *bench_weights())).cuda()
    e0 = Engine(CFG, packed=blob)
    e1 = Engine(CFG, packed=blob, arithmetic="s16x1")
    try:
        assert e0.precision() == "s16x3" and e1.precision() == "s16x1"
        with pytest.raises(CasrError, match="UNSUPPORTED"):
            e1.set_precision("s16x3")
        with pytest.raises(CasrError, match="UNSUPPORTED"):
            e0.set_precision("s16x1")
        assert e1.precision() == "s16x1"
        a, b = _run(e0, "f32"), _run(e1, "f32")
        for k in a:
            np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    finally:
        e0.close()
        e1.close()


def test_s16x1_token_agreement_config2():
    from casr.engine import Engine
    e1 = Engine(CFG, *bench_weights(), arithmetic="s16x1")
    try:
        g = _run(e1)
        g2 = _run(e1)
    finally:
        e1.close()
    for k in g:  # deterministic run to run
        np.testing.assert_array_equal(g[k], g2[k], err_msg=k)
    r = oracle_b32()
    toks, _ = greedy_outputs(g["tokens"], g["out_len"], g["finished"].astype(bool), g["accum"])
    same = sum(a == b for a, b in zip(toks, r["tokens"]))
    pos = sum(max(len(a), len(b)) for a, b in zip(toks, r["tokens"]))
    hit = sum(sum(x == y for x, y in zip(a, b)) for a, b in zip(toks, r["tokens"]))
    d = np.abs(g["accum"] - r["accum"])
    print(f"s16x1 vs oracle, config 2 (B = {B}, T = {T}): utterances identical {same}/{B}, "
          f"token positions equal {hit}/{pos} ({hit / pos:.4f}); |accum - oracle| max {d.max():.3g} "
          f"median {np.median(d):.3g}")
    assert hit / pos >= 0.25 and same >= 1
