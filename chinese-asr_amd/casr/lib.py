"""ctypes binding of the casr C ABI (include/casr.h).

There is no fallback: if ``libcasr_hip.so`` is missing or fails to load, every entry point
raises.  ``torch`` is imported first so the HIP runtime it ships (soname
libamdhip64.so.7) is the one the library binds to."""
import ctypes
import os

import numpy as np

from . import build as _build

CASR_MAX_LAYERS = 8
STATUS = {0: "CASR_OK", 1: "CASR_ERR_ARG", 2: "CASR_ERR_HIP", 3: "CASR_ERR_STATE",
          4: "CASR_ERR_UNSUPPORTED"}

# every symbol include/casr.h declares (tests check the library exports all of them)
EXPORTS = [
    "casr_api_version", "casr_packed_weights_floats", "casr_pack_weights", "casr_create",
    "casr_bind_weights", "casr_destroy", "casr_last_error", "casr_features",
    "casr_gather_utterances", "casr_encode", "casr_encode_fbank", "casr_encoder_results", "casr_greedy", "casr_beam",
    "casr_beam_records", "casr_profile_enable", "casr_profile_read", "casr_set_graphs",
    "casr_device_flags", "casr_set_persistent", "casr_recurrence_mode", "casr_log_mel",
    "casr_log_mel_frames", "casr_mel_filterbank", "casr_set_precision", "casr_get_precision",
    "casr_set_option", "casr_get_option",
]

# arithmetic of the MFMA contractions (casr_set_precision); s16x1 is the opt-in perf arithmetic of
# the libcasr_hip_s16x1.so build (build.py variant "s16x1"), which Engine(arithmetic="s16x1") loads
PRECISIONS = {"f32": 0, "s16x3": 1, "s16x1": 2}
VARIANT_OF = {"s16x3": None, "s16x1": "s16x1"}

# tuning options (include/casr.h CASR_OPT_*): speed only, every value gives the same bits, except
# ATTN_DIRECT (the direct tanh(k + q) attention scores) and DEC_FOLD (the folded decode step: two
# launches per step, greedy always, beam at R >= 1024 rows with the one-accumulator fused GEMM; the
# same arithmetic regrouped): numerics variants within tolerance, the same token ids.
# REC_COOP_REFUSE is for tests: layer n - 1's cooperative launch is treated as refused
OPTIONS = {"FUSE_SELECT": 0, "REC_LAYOUT": 1, "REC_STORE_PLAIN": 2, "REC_SLEEP": 3, "REC_POLL_GAP": 4,
           "REC_COOP": 5, "GEMM16_PERSIST": 6, "GEMM16_TAIL": 7, "ATTN_KPB": 8, "ATTN_DIRECT": 9,
           "DEC_FOLD": 10, "REC_COOP_REFUSE": 11, "DIAG_COLD": 12,
           "LOGMEL_Q16": 13, "KEYS_ROWS": 14, "X16_KM": 15, "DEC_KSPLIT": 16, "GEMM16_LEAN": 17,
           "ATTN_SPLIT": 18}

# kernel classes of casr_profile_enable / casr_profile_read (include/casr.h)
KERNEL_CLASSES = ["features", "input_proj", "rec_step", "keys", "dec_lstm", "attention", "proj", "select"]


class CasrConfigC(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in (
        "n_mels", "feat_dim", "enc_hidden", "enc_layers", "residual", "dec_hidden", "embed_dim",
        "attn_size", "vocab", "max_len", "sos", "eos")] + [("temperature", ctypes.c_float)]


_FP = ctypes.POINTER(ctypes.c_float)


class CasrWeightsHostC(ctypes.Structure):
    _fields_ = [
        ("enc_w_ih", (_FP * 2) * CASR_MAX_LAYERS),
        ("enc_w_hh", (_FP * 2) * CASR_MAX_LAYERS),
        ("enc_b_ih", (_FP * 2) * CASR_MAX_LAYERS),
        ("enc_b_hh", (_FP * 2) * CASR_MAX_LAYERS),
        ("embedding", _FP), ("dec_w_ih", _FP), ("dec_w_hh", _FP), ("dec_b_ih", _FP),
        ("dec_b_hh", _FP), ("proj_w", _FP), ("proj_b", _FP), ("attn_w_enc", _FP),
        ("attn_b", _FP), ("attn_w_hidden", _FP), ("attn_v", _FP),
    ]


class CasrError(RuntimeError):
    pass


_LIBS = {}     # variant -> loaded library
_HANDLES = {}  # casr handle address -> the library that created it (check() reads its error text)


def load(path=None, variant=None):
    """Load (building first if stale and a compiler is present) the HIP library: the shipped
    build, or variant "s16x1" (the opt-in perf arithmetic)."""
    key = path or variant
    if key in _LIBS:
        return _LIBS[key]
    import torch  # noqa: F401  (HIP runtime first)
    path = path or _build.lib_path(variant)
    if not os.path.exists(path) or _build.is_stale(variant):
        if os.path.exists(_build.HIPCC):
            _build.build(variant=variant)
        if not os.path.exists(path):
            raise CasrError(f"casr HIP library not found at {path}; run __graft_entry__.build()")
    lib = ctypes.CDLL(path)
    vp, i32, f32, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_size_t
    sig = {
        "casr_api_version": (i32, []),
        "casr_packed_weights_floats": (sz, [ctypes.POINTER(CasrConfigC)]),
        "casr_pack_weights": (i32, [ctypes.POINTER(CasrConfigC), ctypes.POINTER(CasrWeightsHostC), vp]),
        "casr_create": (i32, [ctypes.POINTER(CasrConfigC), i32, ctypes.POINTER(vp)]),
        "casr_bind_weights": (i32, [vp, vp]),
        "casr_destroy": (None, [vp]),
        "casr_last_error": (ctypes.c_char_p, [vp]),
        "casr_features": (i32, [vp, vp, vp, i32, i32, f32, vp, vp, vp]),
        "casr_gather_utterances": (i32, [vp, vp, vp, i32, i32, vp, vp]),
        "casr_encode": (i32, [vp, vp, vp, i32, i32, vp]),
        "casr_encode_fbank": (i32, [vp, vp, vp, i32, i32, f32, vp, vp]),
        "casr_encoder_results": (i32, [vp, vp, vp, vp, vp, vp]),
        "casr_greedy": (i32, [vp, vp, vp, vp, vp, vp, vp]),
        "casr_beam": (i32, [vp, i32, f32, f32, vp, vp, vp, vp, vp]),
        "casr_beam_records": (i32, [vp, vp, vp, vp, vp]),
        "casr_profile_enable": (i32, [vp, ctypes.c_uint32]),
        "casr_set_graphs": (i32, [vp, i32]),
        "casr_device_flags": (i32, [vp, ctypes.POINTER(ctypes.c_int32), vp]),
        "casr_set_persistent": (i32, [vp, i32]),
        "casr_recurrence_mode": (i32, [vp, i32]),
        "casr_set_precision": (i32, [vp, i32]),
        "casr_get_precision": (i32, [vp]),
        "casr_log_mel": (i32, [vp, vp, vp, i32, i32, i32, f32, vp, vp, vp]),
        "casr_log_mel_frames": (i32, [i32]),
        "casr_mel_filterbank": (i32, [i32, f32, f32, i32, vp]),
        "casr_profile_read": (i32, [vp, i32, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_double)]),
        "casr_set_option": (i32, [vp, i32, i32]),
        "casr_get_option": (i32, [vp, i32, ctypes.POINTER(ctypes.c_int32)]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.casr_api_version() != 3:
        raise CasrError("casr library API version mismatch")
    _LIBS[key] = lib
    return lib


def register_handle(handle, lib):
    _HANDLES[handle.value] = lib


def unregister_handle(handle):
    _HANDLES.pop(handle.value, None)


def check(rc, handle=None, lib=None):
    if rc != 0:
        lib = lib or (_HANDLES.get(handle.value) if handle is not None and handle.value else None) or load()
        msg = lib.casr_last_error(handle)
        raise CasrError(f"{STATUS.get(rc, rc)}: {msg.decode(errors='replace') if msg else ''}")


def mel_filterbank(n_stft=257, f_min=80.0, f_max=7600.0, n_mels=80):
    """The filterbank casr_log_mel uses (create_fb_matrix, data.py:21-57), computed by the
    library on the host: float32 [n_stft, n_mels]."""
    lib = load()
    out = np.empty((n_stft, n_mels), np.float32)
    check(lib.casr_mel_filterbank(n_stft, ctypes.c_float(f_min), ctypes.c_float(f_max), n_mels,
                                  out.ctypes.data_as(ctypes.c_void_p)))
    return out


def log_mel_frames(n_samples):
    """Frames of log-mel an utterance of n_samples produces (0 below 513 samples)."""
    return int(load().casr_log_mel_frames(int(n_samples)))


def config_struct(cfg):
    return CasrConfigC(cfg.n_mels, cfg.feat_dim, cfg.enc_hidden, cfg.enc_layers, int(cfg.residual),
                       cfg.dec_hidden, cfg.embed_dim, cfg.attn_size, cfg.vocab, cfg.max_len,
                       cfg.sos, cfg.eos, float(cfg.temperature))


def packed_floats(cfg):
    """Floats in this build's packed weight layout (casr_packed_weights_floats)."""
    c = config_struct(cfg)
    n = int(load().casr_packed_weights_floats(ctypes.byref(c)))
    if n == 0:
        check(4)
    return n


def pack_weights(cfg, enc_sd, dec_sd):
    """Pack reference state dicts (numpy float32) into the kernel blob (host numpy array)."""
    lib = load()
    c = config_struct(cfg)
    n = lib.casr_packed_weights_floats(ctypes.byref(c))
    if n == 0:
        check(4)
    keep = []

    def ptr(a):
        a = np.ascontiguousarray(a, dtype=np.float32)
        keep.append(a)
        return a.ctypes.data_as(_FP)

    w = CasrWeightsHostC()
    for l in range(cfg.enc_layers):
        for d, suf in enumerate(("", "_reverse")):
            p = f"rnn.rnn.{l}."
            w.enc_w_ih[l][d] = ptr(enc_sd[p + "weight_ih_l0" + suf])
            w.enc_w_hh[l][d] = ptr(enc_sd[p + "weight_hh_l0" + suf])
            w.enc_b_ih[l][d] = ptr(enc_sd[p + "bias_ih_l0" + suf])
            w.enc_b_hh[l][d] = ptr(enc_sd[p + "bias_hh_l0" + suf])
    w.embedding = ptr(dec_sd["embedding.weight"])
    w.dec_w_ih = ptr(dec_sd["cell.cell.0.weight_ih"])
    w.dec_w_hh = ptr(dec_sd["cell.cell.0.weight_hh"])
    w.dec_b_ih = ptr(dec_sd["cell.cell.0.bias_ih"])
    w.dec_b_hh = ptr(dec_sd["cell.cell.0.bias_hh"])
    w.proj_w = ptr(dec_sd["proj_linear.weight"])
    w.proj_b = ptr(dec_sd["proj_linear.bias"])
    w.attn_w_enc = ptr(dec_sd["attn_mechanism.W_enc"])
    w.attn_b = ptr(dec_sd["attn_mechanism.b_attn"])
    w.attn_w_hidden = ptr(dec_sd["attn_mechanism.W_hidden"])
    w.attn_v = ptr(dec_sd["attn_mechanism.v"])
    out = np.empty(n, np.float32)
    check(lib.casr_pack_weights(ctypes.byref(c), ctypes.byref(w), out.ctypes.data_as(ctypes.c_void_p)))
    return out
