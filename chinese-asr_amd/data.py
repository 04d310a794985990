"""Drop-in for the inference part of the reference's ``data.py`` on the MI355X path.

``get_log_mel`` (data.py:167-253): wav -> log-mel -> delta / delta-delta -> 3-frame stacking,
all HIP kernels (casr_log_mel + casr_features, include/casr.h).  ``AudioBase`` (data.py:371-382),
``MelScale`` / ``create_fb_matrix`` (data.py:21-106) and ``fast_read`` (data.py:109-121) keep their
reference names and meaning.

Batch I/O for dataset-level evaluation: ``get_wav_path_text_list_from_manifest``
(data.py:402-405), ``AudioDst`` in its eval / infer modes (data.py:409-466) and ``AudioLoader``
(data.py:469-540) with the eval collate: per-utterance CMVN with eps 1e-7 (data.py:515-518), a
list of [T'_b, 720] tensors for the LSTM encoder, int lengths, and the texts as id lists.  The
loader runs the whole batch through the HIP front-end at once (one casr_log_mel + one
casr_features).  ``evaluate`` is the eval loop of model.py:240-261 (WER weighted by batch size).
Training-time paths (dither, augmentation, TrainSampler, train collate) are out of scope.
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
    """data.py:371-382: vocabulary (dict.pkl is not unpickled: casr/vocab.py), mel scale, window.

    The reference's AudioDst reads ``{train,dev,test}_wav_path_list`` / ``_text_list`` and
    ``infer_wav_path_list`` from its AudioBase, which never sets them; here they come from optional
    manifests (``manifests={'dev': path, ...}``, data.py:402-405 format) or stay None."""

    def __init__(self, manifests=None, infer_paths=None):
        self.word2int, self.int2word = load_vocab()
        self.ms = MelScale(n_mels=gpd['n_mels'], sr=gpd['sample_rate'], f_max=7600, f_min=80, n_stft=257)
        self.window = torch.hann_window(int(gpd['window_len'] * gpd['sample_rate']))
        for split in ('train', 'dev', 'test'):
            paths, texts = (None, None)
            if manifests and manifests.get(split):
                paths, texts = get_wav_path_text_list_from_manifest(manifests[split])
            setattr(self, f'{split}_wav_path_list', paths)
            setattr(self, f'{split}_text_list', texts)
        self.infer_wav_path_list = list(infer_paths) if infer_paths is not None else None


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


def get_wav_path_text_list_from_manifest(loc):
    """data.py:402-405: ``path,text`` lines.  As in the reference the text is everything after the
    first comma up to the next one, trailing newline included (it maps to <unk> in AudioDst)."""
    with open(loc, 'r') as f:
        lines = [line.split(',') for line in f.readlines()]
    return [line[0] for line in lines], [line[1] for line in lines]


class AudioDst(object):
    """data.py:409-466 in eval / infer mode: item idx -> (feature [T'/3, 720] on the device,
    text ids) or (feature,).  Train mode (augmentation, dither) is out of scope."""

    def __init__(self, audio_base, mode='train', dev_or_test='dev', path_list=None, text_list=None):
        assert mode in ('train', 'eval', 'infer'), "mode must be train, eval or infer"
        if dev_or_test is not None:
            assert dev_or_test in ('dev', 'test'), "dev_or_test must be dev or test"
        if mode == 'train':
            raise NotImplementedError("training data path (augmentation, dither) is out of scope")
        if path_list is not None:
            self.path_list = path_list
        elif mode == 'eval':
            self.path_list = getattr(audio_base, f'{dev_or_test}_wav_path_list')
        else:
            assert audio_base.infer_wav_path_list is not None, \
                "you must provide wav path list in infer mode in AudioBase"
            self.path_list = audio_base.infer_wav_path_list
        if text_list is not None:
            assert path_list is not None
            self.text_list = text_list
        elif path_list is not None:
            assert mode == 'infer'
            self.text_list = None
        else:
            self.text_list = getattr(audio_base, f'{dev_or_test}_text_list') if mode == 'eval' else None
        if self.path_list is None:
            raise ValueError(f"no {dev_or_test} manifest was given to AudioBase")
        self.word2int = audio_base.word2int
        self.data_aug = False
        self.audio_base = audio_base
        self.mode = mode

    def __len__(self):
        return len(self.path_list)

    def text_ids(self, idx):
        unk = self.word2int['<unk>']
        return [self.word2int.get(ele, unk) for ele in self.text_list[idx]]

    def __getitem__(self, idx):
        feature = get_log_mel(False, self.path_list[idx], self.audio_base.ms, self.audio_base.window)
        if self.text_list is not None:
            return feature, self.text_ids(idx)
        return (feature,)


class AudioLoader(object):
    """data.py:469-540, eval / infer mode: iterates ``(t, lens, text)`` batches of
    gpd['eval_batch_size'] utterances in dataset order, where t is a list of B device tensors
    [T'_b, 720] normalised per utterance and dimension with eps 1e-7 (batch_audio, data.py:515-518;
    LSTM encoders keep the list), lens an IntTensor and text a list of id lists (None in infer
    mode).  Each batch is one HIP front-end call (log_mel_batch)."""

    def __init__(self, dst, batch_size=None):
        if dst.mode == 'train':
            raise NotImplementedError("train collate is out of scope")
        self.dst = dst
        self.mode = dst.mode
        self.batch_size = int(batch_size or gpd['eval_batch_size'])
        self.loader = self  # the reference iterates ``loader.loader``

    def __len__(self):
        return (len(self.dst) + self.batch_size - 1) // self.batch_size

    def __iter__(self):
        for s in range(0, len(self.dst), self.batch_size):
            idx = list(range(s, min(s + self.batch_size, len(self.dst))))
            audios = [fast_read(self.dst.path_list[i]) for i in idx]
            eps = 1e-7 if gpd['normalize'] else None
            feat, flen = log_mel_batch(audios, cmvn_eps=eps)
            lens = flen.cpu()
            t = [feat[b, :int(lens[b])] for b in range(len(idx))]
            text = [self.dst.text_ids(i) for i in idx] if self.dst.text_list is not None else None
            yield t, lens.to(torch.int32), text


def evaluate(model, loader, int2word, bw=None, **beam_kwargs):
    """The eval loop of model.py:240-261: greedy (or beam bw) over every batch, WER weighted by
    batch size.  Returns (eval_wer, pred_texts, ref_texts)."""
    eval_nb, eval_wer, preds, refs = 0, 0.0, [], []
    dev = model.device
    for data, lens, text in loader.loader:
        if bw is None:
            res = model.eval_one_batch_with_greedy(dev, data, lens, int2word, text)
        else:
            res = model.eval_one_batch_with_beam(dev, bw, data, lens, text, int2word, **beam_kwargs)
        eval_wer += res.wer * lens.size(0)
        eval_nb += lens.size(0)
        preds.extend(res.pred_text)
        refs.extend(res.text)
    return eval_wer / max(eval_nb, 1), preds, refs
