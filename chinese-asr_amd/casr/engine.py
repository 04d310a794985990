"""Device-side engine: one casr handle per GPU, torch tensors as caller-owned buffers.

PyTorch supplies device memory, the current HIP stream and (for multi-GPU) RCCL; every
compute step is a call into the HIP C-ABI library.  There is no CPU or torch-op fallback:
without a GPU or the library, construction raises.
"""
import atexit
import ctypes
import os
import weakref

import numpy as np
import torch

from . import lib as _lib
from .config import CasrConfig

# casr_device_flags guard bits (include/casr.h) that invalidate results
FLAG_REC_TIMEOUT = 32   # a persistent-recurrence hand-off wait expired: that encode is invalid
FLAG_F16_RANGE = 128    # s16x3 / s16x1: an activation beyond the f16 range, the split images are wrong


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


# Every live Engine, closed at interpreter exit before module teardown: a handle's device work is
# drained and its buffers freed while the HIP runtime (and a profiler attached to it) is still
# fully up, not from __del__ during finalisation in whatever order the garbage collector picks.
_LIVE = weakref.WeakSet()


@atexit.register
def _close_all():
    for e in list(_LIVE):
        try:
            e.close()
        except Exception:
            pass


class Engine:
    """casr handle bound to packed weights on one device.

    arithmetic: "s16x3" (default, the shipped library) or "s16x1", the opt-in perf arithmetic of
    the libcasr_hip_s16x1.so build (include/casr.h CASR_PREC_S16X1: one f16 MFMA per split
    product; token ids not identical to the reference's).  Either can run "f32" by set_precision."""

    def __init__(self, cfg: CasrConfig, enc_sd=None, dec_sd=None, device=None, packed=None, arithmetic="s16x3"):
        if not torch.cuda.is_available():
            raise _lib.CasrError("casr Engine needs an MI355X GPU (torch.cuda.is_available() is False)")
        self.cfg = cfg
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else
                                   torch.device(device).index or 0)
        self.lib = _lib.load(variant=_lib.VARIANT_OF[arithmetic])
        self.handle = ctypes.c_void_p()
        c = _lib.config_struct(cfg)
        _lib.check(self.lib.casr_create(ctypes.byref(c), self.device.index, ctypes.byref(self.handle)), lib=self.lib)
        _lib.register_handle(self.handle, self.lib)
        _LIVE.add(self)
        self.packed = None
        if packed is None and enc_sd is not None:
            packed = _lib.pack_weights(cfg, enc_sd, dec_sd)
        if packed is not None:  # no weights: front-end only (log_mel / features)
            self.bind(packed)
        self._B = self._Tp = None
        self.requested = arithmetic
        # A/B tooling hook (tools/probes): CASR_OPTS="REC_SLEEP=2,REC_POLL_GAP=3" sets tuning
        # options on every new handle; the library itself reads no environment
        for item in filter(None, os.environ.get("CASR_OPTS", "").split(",")):
            name, val = item.split("=")
            self.set_option(name.strip(), int(val))

    def bind(self, packed):
        """packed: host numpy blob or a device tensor (e.g. received by RCCL broadcast)."""
        if isinstance(packed, np.ndarray):
            packed = torch.from_numpy(packed).to(self.device)
        if packed.device != self.device or packed.dtype != torch.float32:
            raise ValueError("packed weights must be a float32 tensor on the engine device")
        want = _lib.packed_floats(self.cfg)
        if packed.numel() != want:
            # a blob packed by another build (e.g. broadcast from a rank running a different
            # library version) would be read past its end by the kernels
            raise ValueError(f"packed weights hold {packed.numel()} floats; this build's layout has {want}")
        self.packed = packed.contiguous()
        _lib.check(self.lib.casr_bind_weights(self.handle, _ptr(self.packed)), self.handle)

    def close(self):
        """Destroy the handle (casr_destroy drains the device first).  Idempotent."""
        if self.handle:
            _lib.unregister_handle(self.handle)
            self.lib.casr_destroy(self.handle)
            self.handle = ctypes.c_void_p()
        _LIVE.discard(self)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------ features
    def log_mel(self, wav, n_samples, t_max=None, preemphasis=0.97):
        """wav [B, n_max] float32 (device), n_samples [B] int (device or host) ->
        (fbank [B, t_max, 80] log-mel, frames [B] int32).  get_log_mel data.py:167-224."""
        wav = wav.to(self.device, torch.float32).contiguous()
        B, n_max = wav.shape
        ns = torch.as_tensor(n_samples).to(self.device, torch.int32).contiguous()
        t_max = _lib.log_mel_frames(n_max) if t_max is None else int(t_max)
        fbank = torch.empty(B, max(t_max, 1), self.cfg.n_mels, device=self.device, dtype=torch.float32)
        frames = torch.empty(B, device=self.device, dtype=torch.int32)
        _lib.check(self.lib.casr_log_mel(self.handle, _ptr(wav), _ptr(ns), B, n_max, max(t_max, 1),
                                         ctypes.c_float(preemphasis), _ptr(fbank), _ptr(frames), _stream()),
                   self.handle)
        return fbank, frames

    def features(self, fbank, frames, eps=1e-6):
        """fbank [B, T, n_mels] float32 (device), frames [B] int32 (device) ->
        (feat [B, T//3, feat_dim], feat_len [B] int32).  eps < 0: no CMVN."""
        fbank = fbank.contiguous()
        B, T, _ = fbank.shape
        feat = torch.empty(B, T // 3, self.cfg.feat_dim, device=self.device, dtype=torch.float32)
        flen = torch.empty(B, device=self.device, dtype=torch.int32)
        _lib.check(self.lib.casr_features(self.handle, _ptr(fbank), _ptr(frames.to(torch.int32).contiguous()),
                                          B, T, ctypes.c_float(eps), _ptr(feat), _ptr(flen), _stream()),
                   self.handle)
        return feat, flen

    def gather(self, utts, lens, Tp=None):
        """list of B device tensors [T_b, feat_dim] -> padded [B, Tp, feat_dim]."""
        B = len(utts)
        utts = [u.contiguous().to(self.device, torch.float32) for u in utts]
        Tp = int(max(int(u.shape[0]) for u in utts)) if Tp is None else Tp
        ptrs = torch.tensor([u.data_ptr() for u in utts], dtype=torch.int64, device=self.device)
        lens_d = lens.to(self.device, torch.int32).contiguous()
        feat = torch.empty(B, Tp, self.cfg.feat_dim, device=self.device, dtype=torch.float32)
        _lib.check(self.lib.casr_gather_utterances(self.handle, _ptr(ptrs), _ptr(lens_d), B, Tp, _ptr(feat),
                                                   _stream()), self.handle)
        self._keep = (utts, ptrs)
        return feat, lens_d

    # ------------------------------------------------------------------ encoder
    def encode(self, feat, lens):
        feat = feat.contiguous()
        B, Tp, _ = feat.shape
        lens = lens.to(self.device, torch.int32).contiguous()
        _lib.check(self.lib.casr_encode(self.handle, _ptr(feat), _ptr(lens), B, Tp, _stream()), self.handle)
        self._B, self._Tp = B, Tp
        self._lens = lens

    def encode_fbank(self, fbank, frames, eps=1e-6):
        """features + encode in one call (casr_encode_fbank): fbank [B, T, n_mels] float32 and
        frames [B] int32 on the device; the features stay inside the handle (s16x3: written
        straight as the layer-0 split-f16 image).  Returns feat_len [B] int32 (= frames // 3)."""
        fbank = fbank.contiguous()
        B, T, _ = fbank.shape
        flen = torch.empty(B, device=self.device, dtype=torch.int32)
        _lib.check(self.lib.casr_encode_fbank(self.handle, _ptr(fbank), _ptr(frames.to(torch.int32).contiguous()),
                                              B, T, ctypes.c_float(eps), _ptr(flen), _stream()), self.handle)
        self._B, self._Tp = B, T // 3
        self._lens = flen
        return flen

    def encoder_results(self):
        B, Tp, Cz = self._B, self._Tp, 2 * self.cfg.enc_hidden
        enc = torch.empty(B, Tp, Cz, device=self.device)
        h = torch.empty(B, Cz, device=self.device)
        c = torch.empty(B, Cz, device=self.device)
        keys = torch.empty(B, self.cfg.attn_size, Tp, device=self.device)
        _lib.check(self.lib.casr_encoder_results(self.handle, _ptr(enc), _ptr(h), _ptr(c), _ptr(keys),
                                                 _stream()), self.handle)
        return enc, h, c, keys

    # ------------------------------------------------------------------ decode
    def greedy(self, alignment=False):
        B, L = self._B, self.cfg.max_len
        dev = self.device
        tokens = torch.empty(B, L, dtype=torch.int32, device=dev)
        out_len = torch.empty(B, dtype=torch.int32, device=dev)
        fin = torch.empty(B, dtype=torch.uint8, device=dev)
        accum = torch.empty(B, dtype=torch.float32, device=dev)
        align = torch.zeros(L, self._Tp, B, device=dev) if alignment else None
        _lib.check(self.lib.casr_greedy(self.handle, _ptr(tokens), _ptr(out_len), _ptr(fin), _ptr(accum),
                                        _ptr(align), _stream()), self.handle)
        return dict(tokens=tokens, out_len=out_len, finished=fin, accum=accum, alignment=align)

    def beam(self, k, lm_weight=0.0, length_weight=0.0):
        B, L = self._B, self.cfg.max_len
        dev = self.device
        toks = torch.empty(B, L, dtype=torch.int32, device=dev)
        blen = torch.empty(B, dtype=torch.int32, device=dev)
        score = torch.empty(B, dtype=torch.float32, device=dev)
        steps = torch.empty(1, dtype=torch.int32, device=dev)
        _lib.check(self.lib.casr_beam(self.handle, int(k), ctypes.c_float(lm_weight), ctypes.c_float(length_weight),
                                      _ptr(toks), _ptr(blen), _ptr(score), _ptr(steps), _stream()), self.handle)
        self._k = k
        return dict(tokens=toks, length=blen, score=score, steps=steps)

    def beam_records(self):
        B, L, k = self._B, self.cfg.max_len, self._k
        dev = self.device
        rt = torch.empty(B, L, k, L, dtype=torch.int32, device=dev)
        rs = torch.empty(B, L, k, dtype=torch.float32, device=dev)
        rv = torch.empty(B, L, k, dtype=torch.uint8, device=dev)
        _lib.check(self.lib.casr_beam_records(self.handle, _ptr(rt), _ptr(rs), _ptr(rv), _stream()), self.handle)
        return rt, rs, rv

    def device_flags(self):
        """Guard bits raised since the previous read (read and clear: every encode / decode in
        between is covered; 0 = clean); synchronises the stream."""
        f = ctypes.c_int32()
        _lib.check(self.lib.casr_device_flags(self.handle, ctypes.byref(f), _stream()), self.handle)
        return f.value

    def set_graphs(self, enable):
        """hipGraph replay of the launch-bound loops: True = decode loop and per-step recurrence
        fallback, False = both eager, or an int mode (include/casr.h CASR_GRAPHS_*; default 2:
        decode eager, recurrence fallback replayed)."""
        mode = (3 if enable else 0) if isinstance(enable, bool) else int(enable)
        _lib.check(self.lib.casr_set_graphs(self.handle, mode), self.handle)

    def set_persistent(self, enable):
        """Persistent per-layer recurrence (default on where its grid fits); off = per-step."""
        _lib.check(self.lib.casr_set_persistent(self.handle, int(bool(enable))), self.handle)

    def set_precision(self, precision):
        """'s16x3' (default: split-f16 MFMA, f32 accumulate) or 'f32' (exact-f32 MFMA); an
        Engine(arithmetic='s16x1') takes 's16x1' or 'f32'."""
        _lib.check(self.lib.casr_set_precision(self.handle, _lib.PRECISIONS[precision]), self.handle)
        self.requested = precision

    def check_flags(self):
        """Guard bits raised since the previous read (read and clear, casr_device_flags: every
        encode / decode since then is covered; synchronises).  Raises CasrError when a recurrence
        hand-off timed out (bit 32: those encoder results are invalid); returns the bits
        otherwise, so a caller can re-run at f32 on bit 128 (FLAG_F16_RANGE)."""
        f = self.device_flags()
        if f & FLAG_REC_TIMEOUT:
            raise _lib.CasrError("persistent recurrence hand-off wait expired (device flag 32): "
                                 "the encoder results of this batch are invalid")
        return f

    def run_checked(self, encode, decode):
        """encode(); out = decode(); then the guard bits.  Bit 32 raises; bit 128 (an s16x3
        operand beyond the f16 range) re-runs encode + decode on the exact-f32 path, so no
        result rests on a wrong split image.  Bits left by earlier unchecked calls are read and
        discarded first, so only this batch's bits decide."""
        self.device_flags()
        encode()
        out = decode()
        f = self.check_flags()
        if f & FLAG_F16_RANGE and self.precision() in ("s16x3", "s16x1"):
            req = self.requested
            self.set_precision("f32")
            try:
                encode()
                out = decode()
                f = self.check_flags()
            finally:
                self.set_precision(req)
        return out, f

    def set_option(self, name, value):
        """Tuning option (include/casr.h CASR_OPT_*, lib.OPTIONS): speed only, same bits, except the
        numerics variants ATTN_DIRECT, DEC_FOLD and DEC_KSPLIT (same tokens, results within tolerance)."""
        _lib.check(self.lib.casr_set_option(self.handle, _lib.OPTIONS[name], int(value)), self.handle)

    def get_option(self, name):
        v = ctypes.c_int32()
        _lib.check(self.lib.casr_get_option(self.handle, _lib.OPTIONS[name], ctypes.byref(v)), self.handle)
        return v.value

    def precision(self):
        """Effective arithmetic of the MFMA contractions ('s16x3', 's16x1' or 'f32')."""
        p = int(self.lib.casr_get_precision(self.handle))
        return {v: k for k, v in _lib.PRECISIONS.items()}[p]

    def recurrence_mode(self, B):
        """1 if casr_encode would run the persistent recurrence for batch B, else 0."""
        return int(self.lib.casr_recurrence_mode(self.handle, int(B)))

    # ------------------------------------------------------------------ launch timing
    def profile(self, classes):
        """Enable HIP-event timing for the named kernel classes (lib.KERNEL_CLASSES)."""
        mask = 0
        for c in classes:
            mask |= 1 << _lib.KERNEL_CLASSES.index(c)
        _lib.check(self.lib.casr_profile_enable(self.handle, mask), self.handle)

    def profile_read(self):
        """{class: (launches, total_ms)} for the enabled classes since profile()."""
        out = {}
        for i, name in enumerate(_lib.KERNEL_CLASSES):
            n = ctypes.c_int32()
            ms = ctypes.c_double()
            _lib.check(self.lib.casr_profile_read(self.handle, i, ctypes.byref(n), ctypes.byref(ms)), self.handle)
            if n.value:
                out[name] = (n.value, ms.value)
        return out
