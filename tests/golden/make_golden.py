#!/usr/bin/env python
"""Capture golden vectors from the REFERENCE implementation (shawnthu/chinese-asr).

Runs only in the build container, where /root/reference exists (read-only).  It is never
imported by the tests; its outputs (small .npz/.json fixtures in this directory) are.

How the reference is run:
  * sys.dont_write_bytecode so nothing is written under /root/reference;
  * stub modules for the absent third-party deps: kenlm, Levenshtein, soundfile;
  * legacy-torch shims: integer ``torch.div(..., out=long)`` and ``int_tensor / int``
    (model.py:866, :886) use truncating division as torch<=1.4 did; ``torch.stft``
    without return_complex returns the legacy real [..., 2] layout (data.py:205);
  * dict.pkl is NOT unpickled: int2word comes from the package's safe opcode parser;
  * weights: the deterministic synthetic recipe (casr.weights), loaded through the
    reference's own ``load_state_dict``.

Inputs are regenerated from seeds (fbank[b] = RandomState(1234+b).standard_normal((T_b, 80)))
so only seeds and outputs are stored.
"""
import json
import os
import sys
import types

sys.dont_write_bytecode = True
os.environ["PYTHONDONTWRITEBYTECODE"] = "1"

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "chinese-asr_amd"))

import numpy as np
import torch

from casr.config import CasrConfig
from casr.vocab import load_dict_pkl
from casr.weights import synthetic_state_dicts

torch.set_num_threads(8)

# ---------------------------------------------------------------- stubs for absent deps
_WAV = {}


def _sf_read(path, dtype="float32"):
    return _WAV[path].astype(dtype), 16000


sys.modules["soundfile"] = types.SimpleNamespace(read=_sf_read)
sys.modules["kenlm"] = types.SimpleNamespace(LanguageModel=None)
sys.modules["Levenshtein"] = types.SimpleNamespace(distance=lambda a, b: 0, editops=lambda a, b: [])

# ---------------------------------------------------------------- legacy torch semantics
_div = torch.div


def _legacy_div(a, b, *args, **kw):
    if isinstance(a, torch.Tensor) and not a.is_floating_point() and \
            (not isinstance(b, torch.Tensor) or not b.is_floating_point()) and "rounding_mode" not in kw:
        kw["rounding_mode"] = "trunc"
    return _div(a, b, *args, **kw)


torch.div = _legacy_div
_truediv = torch.Tensor.__truediv__


def _legacy_truediv(a, b):
    if not a.is_floating_point() and isinstance(b, int):
        return _div(a, b, rounding_mode="trunc")
    return _truediv(a, b)


torch.Tensor.__truediv__ = _legacy_truediv
_stft = torch.stft


def _legacy_stft(*args, **kw):
    if "return_complex" not in kw:
        kw["return_complex"] = True
        return torch.view_as_real(_stft(*args, **kw))
    return _stft(*args, **kw)


torch.stft = _legacy_stft

sys.path.insert(0, REF)
import gpd as ref_gpd  # noqa: E402

ref_gpd.gpd["verbose"] = False
ref_gpd.gpd["use_cuda"] = False
ref_gpd.gpd["temperature"] = 1
import model as ref_model  # noqa: E402
import data as ref_data  # noqa: E402
import encoder as ref_encoder  # noqa: E402
import util as ref_util  # noqa: E402

assert not os.path.exists(os.path.join(REF, "__pycache__")), "bytecode written into the reference"

CFG = CasrConfig()
_, INT2WORD = load_dict_pkl(os.path.join(REF, "dict.pkl"))


sys.path.insert(0, HERE)
from stub_lm import StubLM, pua_int2word, pua_to_ids  # noqa: E402

PUA = pua_int2word(CFG.vocab)


def fbank_for(b, T):
    return np.random.RandomState(1234 + b).standard_normal((T, CFG.n_mels)).astype(np.float32)


def ref_features(fbank, eps=1e-6):
    """data.py:226-249 on a log-mel input, then main.py:37 CMVN."""
    f = ref_data.add_delta_deltas(torch.from_numpy(fbank)[None, None])   # [1, 3, L, 80]
    f = f.squeeze(0)
    f = f[:, :(3 * (f.size(1) // 3))]
    f = f.view(f.size(0), f.size(1) // 3, -1).transpose(0, 1).contiguous().view(f.size(1) // 3, -1)
    raw = f.clone()
    f = (f - f.mean(dim=0)) / (f.std(dim=0) + eps)
    return raw, f


def build_ref_model(enc_sd, dec_sd):
    m = ref_model.Model()
    m.encoder.load_state_dict({k: torch.from_numpy(v) for k, v in enc_sd.items()})
    m.decoder.load_state_dict({k: torch.from_numpy(v) for k, v in dec_sd.items()})
    m.model.eval()
    return m


def check_key_order():
    m = ref_model.Model()
    from casr.weights import encoder_keys, decoder_keys
    ek = list(m.encoder.state_dict().keys())
    dk = list(m.decoder.state_dict().keys())
    assert ek == [k for k, _ in encoder_keys(CFG)], ek
    assert dk == [k for k, _ in decoder_keys(CFG)], dk
    return ek, dk


def encoder_kat():
    """encoder.py:636-652 with input_size = 720 (the test's m.input_size does not exist)."""
    m = ref_encoder.RNNEncoder()
    for p in m.parameters():
        torch.nn.init.ones_(p)
    lens = [10, 8, 23, 14]
    x = [torch.ones(l, 720) for l in lens]
    with torch.no_grad():
        y = m(x, torch.tensor(lens))
    return dict(out_sum=float(y[0].sum()), h_sum=float(y[2][0].sum()), c_sum=float(y[2][1].sum()),
                out_shape=list(y[0].shape))


def decode_suite(name, peaked, frames, out):
    enc_sd, dec_sd = synthetic_state_dicts(CFG, peaked=peaked)
    m = build_ref_model(enc_sd, dec_sd)
    feats = [ref_features(fbank_for(b, T))[1] for b, T in enumerate(frames)]
    lens = torch.tensor([f.shape[0] for f in feats])
    dev = torch.device("cpu")
    with torch.no_grad():
        enc = m.encoder(feats, lens)
        keys, _ = m.attn_mechanism.compute_key_value(enc.out)
    out[f"{name}_enc_sum_per_utt"] = enc.out.double().sum(dim=(0, 2)).numpy()
    out[f"{name}_enc_abs_sum_per_utt"] = enc.out.double().abs().sum(dim=(0, 2)).numpy()
    out[f"{name}_enc_slice"] = enc.out[::7, :, ::64].numpy().astype(np.float32)
    out[f"{name}_enc_h"] = enc.state[0].numpy()
    out[f"{name}_enc_c"] = enc.state[1].numpy()
    out[f"{name}_keys_sum_per_utt"] = keys.double().sum(dim=(0, 2)).numpy()

    def rec(r):
        ids = [pua_to_ids(t) for t in r.pred_text]
        return {"tokens": ids, "score": [float(x) for x in r.score],
                "text": ["".join(INT2WORD[i] for i in t) for t in ids]}

    g = m.eval_one_batch_with_greedy(dev, feats, lens, PUA, None)
    meta = {"greedy": dict(rec(g), text_len=g.text_len.tolist(), steps=len(g.alignment))}
    out[f"{name}_greedy_align_sum"] = np.stack([a.double().sum(0).numpy() for a in g.alignment])
    out[f"{name}_greedy_align_step0"] = g.alignment[0].numpy()
    for k in (1, 4, 8, 16):
        r = m.eval_one_batch_with_beam(dev, k, feats, lens, None, PUA, second_pass=False,
                                       lm_model=None, lm_weight=0.0, length_weight=0.0)
        meta[f"beam{k}"] = rec(r)
    # main.py:45-51 passes lm_weight=1.5, length_weight=1.5; second pass with the stub LM
    r = m.eval_one_batch_with_beam(dev, 4, feats, lens, None, PUA, second_pass=True,
                                   lm_model=StubLM(), lm_weight=1.5, length_weight=1.5)
    meta["beam4_lm"] = rec(r)
    # BASELINE config 5: beam 16 + second pass
    r = m.eval_one_batch_with_beam(dev, 16, feats, lens, None, PUA, second_pass=True,
                                   lm_model=StubLM(), lm_weight=1.5, length_weight=1.5)
    meta["beam16_lm"] = rec(r)
    r = m.eval_one_batch_with_beam(dev, 4, feats, lens, None, PUA, second_pass=False,
                                   lm_model=None, lm_weight=1.5, length_weight=1.5)
    meta["beam4_lw"] = rec(r)
    # softmax temperature (model.py:834 reads gpd['temperature'] at every step; main.py:125 sets
    # it): round 3 capture, beam 4 and 8 at T = 0.7
    ref_gpd.gpd["temperature"] = 0.7
    try:
        for k in (4, 8):
            r = m.eval_one_batch_with_beam(dev, k, feats, lens, None, PUA, second_pass=False,
                                           lm_model=None, lm_weight=0.0, length_weight=0.0)
            meta[f"beam{k}_t07"] = rec(r)
    finally:
        ref_gpd.gpd["temperature"] = 1
    return meta


def main():
    ek, dk = check_key_order()
    out, meta = {}, {"encoder_key_order": ek, "decoder_key_order": dk}
    meta["encoder_kat"] = encoder_kat()

    # ---- features from fbank (two lengths incl. a ragged tail) and raw stacking
    for b, T in ((0, 101), (1, 800)):
        raw, f = ref_features(fbank_for(b, T))
        if T <= 128:
            out[f"feat_raw_T{T}"] = raw.numpy()
            out[f"feat_cmvn_T{T}"] = f.numpy()
        else:  # keep the fixture small: head/tail rows + per-dimension sums
            for nm, x in (("raw", raw), ("cmvn", f)):
                out[f"feat_{nm}_T{T}_head"] = x[:6].numpy()
                out[f"feat_{nm}_T{T}_tail"] = x[-3:].numpy()
                out[f"feat_{nm}_T{T}_colsum"] = x.double().sum(0).numpy()

    # ---- wav -> log-mel (data.py:167-224) on a synthetic 1.5 s waveform
    rs = np.random.RandomState(77)
    n = 24000
    t = np.arange(n) / 16000.0
    wav = (0.3 * np.sin(2 * np.pi * 440 * t) + 0.2 * np.sin(2 * np.pi * 1330 * t * (1 + 0.1 * t))
           + 0.05 * rs.standard_normal(n)).astype(np.float32)
    wav[5000:5400] = 0.0  # exact zeros: exercises the eps floor
    _WAV["wav0"] = wav
    ms = ref_data.MelScale(n_mels=80, sr=16000, f_max=7600, f_min=80, n_stft=257)
    window = torch.hann_window(400)
    ref_gpd.gpd["delta_delta"], ref_gpd.gpd["downsample"] = False, False
    lm = ref_data.get_log_mel(False, "wav0", ms, window, False)
    ref_gpd.gpd["delta_delta"], ref_gpd.gpd["downsample"] = True, True
    out["wav0"] = wav
    out["wav0_logmel"] = lm.numpy()
    out["wav0_features"] = ref_data.get_log_mel(False, "wav0", ms, window, False).numpy()
    out["fb_matrix"] = ms.fb.numpy()

    # ---- decode suites: 8 ragged utterances (T ~ U{450..800}) + 2 short (T'=2, 3)
    frames = list(np.random.RandomState(7).randint(450, 801, size=8)) + [6, 9]
    frames = [int(x) for x in frames]
    meta["frames"] = frames
    for name, peaked in (("plain", False), ("peaked", True)):
        meta[name] = decode_suite(name, peaked, frames, out)

    np.savez_compressed(os.path.join(HERE, "golden.npz"), **out)
    with open(os.path.join(HERE, "golden.json"), "w", encoding="utf-8") as f:
        json.dump(meta, f, ensure_ascii=False, indent=1)
    print("encoder KAT:", meta["encoder_kat"])
    for name in ("plain", "peaked"):
        g = meta[name]["greedy"]
        print(name, "greedy lens", g["text_len"], "steps", g["steps"])
        print(name, "beam8 lens", [len(t) for t in meta[name]["beam8"]["tokens"]])
        print(name, "beam4_lm lens", [len(t) for t in meta[name]["beam4_lm"]["tokens"]])


if __name__ == "__main__":
    main()
