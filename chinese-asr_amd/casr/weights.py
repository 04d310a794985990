"""Weights: the reference state-dict layout, the build's deterministic synthetic recipe,
and checkpoint IO.

State-dict keys follow the reference checkpoint format written by ``Model.save``
(model.py:347-355): ``encoder_state_dict`` (``rnn.rnn.{i}.{weight,bias}_{ih,hh}_l0[_reverse]``,
RNN_RES util.py:1150-1163) and ``decoder_state_dict`` (embedding, ``cell.cell.0.*``,
``proj_linear.*``, ``attn_mechanism.*``; decoder.py:30-52, attention.py:28-31).

There is no trained checkpoint in the reference, so benchmarks and parity
fixtures use the build-owned recipe of SURVEY §8d: tensor *i* (in key order) is
``RandomState(1000+i).standard_normal(shape) * s_i`` in float32.
"""
import numpy as np

from .config import CasrConfig


def encoder_keys(cfg: CasrConfig):
    H, D = cfg.enc_hidden, cfg.feat_dim
    out = []
    for i in range(cfg.enc_layers):
        din = D if i == 0 else 2 * H
        for suf in ("", "_reverse"):
            out += [
                (f"rnn.rnn.{i}.weight_ih_l0{suf}", (4 * H, din)),
                (f"rnn.rnn.{i}.weight_hh_l0{suf}", (4 * H, H)),
                (f"rnn.rnn.{i}.bias_ih_l0{suf}", (4 * H,)),
                (f"rnn.rnn.{i}.bias_hh_l0{suf}", (4 * H,)),
            ]
    return out


def decoder_keys(cfg: CasrConfig):
    Hd, E, A, V = cfg.dec_hidden, cfg.embed_dim, cfg.attn_size, cfg.vocab
    C = cfg.enc_size  # context size (map_enc False: attention.py:39)
    return [
        ("embedding.weight", (V, E)),
        ("cell.cell.0.weight_ih", (4 * Hd, E + C)),
        ("cell.cell.0.weight_hh", (4 * Hd, Hd)),
        ("cell.cell.0.bias_ih", (4 * Hd,)),
        ("cell.cell.0.bias_hh", (4 * Hd,)),
        ("proj_linear.weight", (V, Hd + C)),
        ("proj_linear.bias", (V,)),
        ("attn_mechanism.W_enc", (C, A)),
        ("attn_mechanism.b_attn", (A,)),
        ("attn_mechanism.W_hidden", (Hd, A)),
        ("attn_mechanism.v", (A,)),
    ]


def _scale_for(key, shape):
    if key.endswith("embedding.weight") or key.endswith(".v"):
        return 0.1                        # decoder.py:77, attention.py:57
    if "bias" in key or key.endswith("b_attn"):
        return 0.0
    if key.endswith("W_enc") or key.endswith("W_hidden"):
        return 1.0 / np.sqrt(shape[0])    # [in, out] matrices used as x @ W
    return 1.0 / np.sqrt(shape[1])        # [out, in] nn.Linear / LSTM matrices


def synthetic_state_dicts(cfg: CasrConfig = CasrConfig(), peaked=True, seed_base=1000,
                          eos_bias=12.0, proj_gain=40.0):
    """Deterministic synthetic weights.  Returns ``(enc_sd, dec_sd)`` of
    float32 numpy arrays.  LSTM forget-gate slices of both biases are 0.5, mirroring
    ``init_rnn`` (util.py:100-104).  ``peaked`` multiplies the output projection by
    ``proj_gain`` and sets ``proj_linear.bias[eos] = eos_bias`` so that decodes show
    early EOS, finished and unfinished beams."""
    enc, dec = {}, {}
    keys = [("enc", k, s) for k, s in encoder_keys(cfg)] + [("dec", k, s) for k, s in decoder_keys(cfg)]
    for i, (sec, key, shape) in enumerate(keys):
        s = _scale_for(key, shape)
        if s == 0.0:
            arr = np.zeros(shape, np.float32)
        else:
            arr = (np.random.RandomState(seed_base + i).standard_normal(shape) * s).astype(np.float32)
        if "bias" in key and ("rnn.rnn" in key or "cell.cell" in key):
            n = shape[0]
            arr[n // 4: n // 2] = 0.5
        (enc if sec == "enc" else dec)[key] = arr
    if peaked:
        dec["proj_linear.weight"] = (dec["proj_linear.weight"] * np.float32(proj_gain)).astype(np.float32)
        dec["proj_linear.bias"][cfg.eos] = np.float32(eos_bias)
    return enc, dec


def check_state_dicts(cfg: CasrConfig, enc_sd, dec_sd):
    """Validate key set and shapes; raise ``KeyError``/``ValueError`` like
    ``load_state_dict(strict=True)`` would."""
    for sd, spec, name in ((enc_sd, encoder_keys(cfg), "encoder_state_dict"),
                           (dec_sd, decoder_keys(cfg), "decoder_state_dict")):
        want = dict(spec)
        missing = [k for k in want if k not in sd]
        unexpected = [k for k in sd if k not in want]
        if missing or unexpected:
            raise KeyError(f"{name}: missing keys {missing}, unexpected keys {unexpected}")
        for k, shp in want.items():
            if tuple(np.shape(sd[k])) != tuple(shp):
                raise ValueError(f"{name}[{k}]: shape {tuple(np.shape(sd[k]))} != {shp}")


def to_numpy_sd(sd):
    out = {}
    for k, v in sd.items():
        if hasattr(v, "detach"):
            v = v.detach().to("cpu").float().numpy()
        out[k] = np.ascontiguousarray(np.asarray(v, dtype=np.float32))
    return out


class TrainVar(object):
    """Behaviour-free stand-in for the reference's training record ``util.TrainVar``
    (util.py:2356-2363), which ``Model.save`` stores as ``args`` (model.py:347-355).  Registered
    with torch's weights-only unpickler under the reference's module/name, so the safe loader
    rebuilds it by plain attribute assignment: nothing from the file is executed."""

    def __init__(self, step=None, loss=None, best_wer=None, lr=None, duration=None, num_no_imprv=None):
        self.step, self.loss, self.best_wer = step, loss, best_wer
        self.lr, self.duration, self.num_no_imprv = lr, duration, num_no_imprv

    def __repr__(self):
        return f"TrainVar({self.__dict__})"


TrainVar.__module__ = "util"


def load_checkpoint(path):
    """Read a reference ``.ckpt`` (model.py:357-370) without executing pickled code:
    ``torch.load(weights_only=True)`` with the reference's ``util.TrainVar`` record allow-listed
    as the plain stand-in above.  Any other non-tensor object is refused with a RuntimeError.
    Returns ``(enc_sd, dec_sd, args)``."""
    import torch
    try:
        with torch.serialization.safe_globals([TrainVar]):
            ck = torch.load(path, map_location="cpu", weights_only=True)
    except Exception as e:  # an object the safe loader will not build
        raise RuntimeError(
            f"{path}: refused by the weights_only loader ({e}). Re-save the checkpoint "
            f"with only tensors (encoder_state_dict/decoder_state_dict)") from None
    return to_numpy_sd(ck["encoder_state_dict"]), to_numpy_sd(ck["decoder_state_dict"]), ck.get("args")


def save_checkpoint(path, enc_sd, dec_sd, args=None):
    """Write the reference checkpoint format (model.py:347-355)."""
    import torch
    torch.save({
        "encoder_state_dict": {k: torch.from_numpy(np.asarray(v)) for k, v in enc_sd.items()},
        "decoder_state_dict": {k: torch.from_numpy(np.asarray(v)) for k, v in dec_sd.items()},
        "optimizer_state_dict": None,
        "args": args,
    }, path)
