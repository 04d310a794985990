"""Drop-in for the inference part of the reference's ``data.py`` on the MI355X path.

``get_log_mel`` (data.py:167-253): wav -> log-mel -> delta / delta-delta -> 3-frame stacking,
all HIP kernels (casr_log_mel + casr_features, include/casr.h).  ``AudioBase`` (data.py:371-382),
``MelScale`` / ``create_fb_matrix`` (data.py:21-106) and ``fast_read`` (data.py:109-121) keep their
reference names and meaning.  Training-time paths (dither, augmentation, the dataset / loader
classes, data.py:283-540) are out of scope.
"""
import os
import struct

import numpy as np
import torch

from gpd import gpd
from casr import lib as _lib
from casr.config import config_from_gpd
from casr.vocab import load_vocab

_ENGINE = None


def _engine():
    """Front-end-only casr handle on the current device (no weights bound)."""
    global _ENGINE
    if _ENGINE is None:
        from casr.engine import Engine
        _ENGINE = Engine(config_from_gpd(gpd))
    return _ENGINE


def create_fb_matrix(n_stft, f_min, f_max, n_mels):
    """data.py:21-57 (float32, incl. the linspace(f_min, f_max, n_stft) bin quirk): [n_stft, n_mels]."""
    return torch.from_numpy(_lib.mel_filterbank(n_stft, f_min, f_max, n_mels))


class MelScale(object):
    """data.py:84-106.  ``fb`` is the same matrix casr_log_mel applies on the device."""

    def __init__(self, n_mels=128, sr=16000, f_max=None, f_min=0., n_stft=None):
        self.n_mels, self.sr = n_mels, sr
        self.f_max = f_max if f_max is not None else sr // 2
        self.f_min = f_min
        self.fb = create_fb_matrix(n_stft, self.f_min, self.f_max, n_mels) if n_stft is not None else None

    def __call__(self, spec_f):
        return torch.matmul(spec_f, self.fb.to(spec_f.device))


class AudioBase(object):
    """data.py:371-382: vocabulary (dict.pkl is not unpickled: casr/vocab.py), mel scale, window."""

    def __init__(self):
        self.word2int, self.int2word = load_vocab()
        self.ms = MelScale(n_mels=gpd['n_mels'], sr=gpd['sample_rate'], f_max=7600, f_min=80, n_stft=257)
        self.window = torch.hann_window(int(gpd['window_len'] * gpd['sample_rate']))


def fast_read(path):
    """data.py:109-121 (soundfile ``read(path, dtype='float32')``): mono RIFF/WAVE, integer PCM
    scaled to [-1, 1) like libsndfile (x / 2^(bits-1); 8-bit unsigned centred) or IEEE float32."""
    with open(path, "rb") as f:
        riff = f.read()
    if riff[:4] != b"RIFF" or riff[8:12] != b"WAVE":
        raise ValueError(f"{path}: not a RIFF/WAVE file (convert it first, main.py:19-24)")
    pos, fmt, data = 12, None, None
    while pos + 8 <= len(riff):
        cid, size = riff[pos:pos + 4], struct.unpack("<I", riff[pos + 4:pos + 8])[0]
        body = riff[pos + 8:pos + 8 + size]
        if cid == b"fmt ":
            tag, ch, rate, _, _, bits = struct.unpack("<HHIIHH", body[:16])
            if tag == 0xFFFE and len(body) >= 26:  # WAVE_FORMAT_EXTENSIBLE: sub-format GUID
                tag = struct.unpack("<H", body[24:26])[0]
            fmt = (tag, ch, rate, bits)
        elif cid == b"data":
            data = body
        pos += 8 + size + (size & 1)
    if fmt is None or data is None:
        raise ValueError(f"{path}: missing fmt/data chunk")
    tag, ch, rate, bits = fmt
    if tag == 3 and bits == 32:
        x = np.frombuffer(data, "<f4").astype(np.float32)
    elif tag == 1 and bits == 16:
        x = np.frombuffer(data, "<i2").astype(np.float32) / 32768.0
    elif tag == 1 and bits == 32:
        x = (np.frombuffer(data, "<i4").astype(np.float64) / 2147483648.0).astype(np.float32)
    elif tag == 1 and bits == 24:
        b = np.frombuffer(data, np.uint8).reshape(-1, 3).astype(np.int32)
        v = b[:, 0] | (b[:, 1] << 8) | (b[:, 2] << 16)
        x = (np.where(v >= 1 << 23, v - (1 << 24), v) / 8388608.0).astype(np.float32)
    elif tag == 1 and bits == 8:
        x = (np.frombuffer(data, np.uint8).astype(np.float32) - 128.0) / 128.0
    else:
        raise ValueError(f"{path}: unsupported WAVE format tag {tag}, {bits} bits")
    if ch != 1:
        raise ValueError(f"{path}: {ch} channels; the path expects mono 16 kHz (main.py:22)")
    if rate != gpd['sample_rate'] and gpd['verbose']:
        print(f'[WARN] rate={rate}, dtype={x.dtype}, path={path}')  # data.py:118-119
    return x


def log_mel_batch(wavs, cmvn_eps=None):
    """Batched front-end: list of B float32 sample arrays -> device features [B, T', 720] and
    lengths [B] (int32).  cmvn_eps=None: no CMVN (get_log_mel's output); 1e-6: main.py:37."""
    eng = _engine()
    n = [int(len(w)) for w in wavs]
    if min(n) < 513:  # torch.stft raises on a signal shorter than n_fft (data.py:204)
        raise RuntimeError(f"audio of {min(n)} samples is shorter than n_fft + 1 = 513")
    wav = np.zeros((len(wavs), max(n)), np.float32)
    for b, w in enumerate(wavs):
        wav[b, :n[b]] = w
    fb, frames = eng.log_mel(torch.from_numpy(wav).to(eng.device), torch.tensor(n, dtype=torch.int32),
                             preemphasis=float(gpd['preemphasis']))
    return eng.features(fb, frames, eps=-1.0 if cmvn_eps is None else float(cmvn_eps))


def get_log_mel(training, file_path, ms, window, data_aug=False):
    """data.py:167-253 for inference: [T // 3, 720] features (delta + delta-delta, 3-frame stack),
    on the GPU.  ``file_path`` may also be an array of float32 samples."""
    if training or data_aug:
        raise NotImplementedError("dither / augmentation are training paths (out of scope)")
    if not (gpd['delta_delta'] and gpd['downsample']) or gpd['encoder_type'] == 'CNN2D':
        raise NotImplementedError("the deployed LSTM config uses delta_delta + downsample")
    audio = fast_read(file_path) if isinstance(file_path, (str, os.PathLike)) else np.asarray(file_path, np.float32)
    feat, flen = log_mel_batch([audio])
    return feat[0, :int(flen[0])]
