#!/usr/bin/env python
"""Drop-in for the reference's ``main.py`` (main.py:19-102) on the MI355X path.

``parse(path, model, audio_base, lm_model, bw)`` and ``ASR(lm_path=None, bw=None)(path)`` keep
the reference signatures and results.  The chain wav -> log-mel -> delta/stack -> CMVN
(eps 1e-6, main.py:37) -> encoder -> greedy / beam (+ second pass with a KenLM-like
``lm_model.score(s, bos=True)``) runs on the GPU through the casr C ABI.  Format conversion
(``convert_audio``: ffmpeg + sox, main.py:19-24) stays an external tool: it is used when present,
otherwise the input must already be 16 kHz mono WAV.
"""
import os
import shutil
import subprocess
import sys
import tempfile
from time import time

HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)

from gpd import gpd  # noqa: E402
from data import AudioBase, fast_read, log_mel_batch  # noqa: E402
from model import Model  # noqa: E402


def convert_audio(path):
    """main.py:19-24: ffmpeg -> 16 kHz mono s16, sox --norm=-1.  Without the tools, a WAV input is
    used as is."""
    if shutil.which("ffmpeg") and shutil.which("sox"):
        td = tempfile.mkdtemp()
        tmp, norm = os.path.join(td, "tmp.wav"), os.path.join(td, "a.wav")
        subprocess.run(["ffmpeg", "-loglevel", "quiet", "-i", path, "-sample_fmt", "s16", "-ar", "16000",
                        "-ac", "1", tmp], check=True)
        subprocess.run(["sox", "--norm=-1", tmp, norm], check=True)
        return norm
    if not path.lower().endswith(".wav"):
        raise RuntimeError(f"{path}: ffmpeg/sox are not available to convert it; pass a 16 kHz mono WAV")
    return path


def features_for(audios):
    """Samples -> CMVN'd encoder inputs (data.py:167-253 + main.py:37), batched on the GPU.
    Returns the list-of-tensors form Model.eval_one_batch_* takes, plus lengths."""
    feat, flen = log_mel_batch(audios, cmvn_eps=1e-6)
    lens = flen.cpu()
    return [feat[b, :int(lens[b])] for b in range(len(audios))], lens


def parse(path, model, audio_base, lm_model, bw):
    """main.py:27-65: one file -> predicted text."""
    audio = path if not isinstance(path, (str, os.PathLike)) else fast_read(convert_audio(path))
    data, lens = features_for([audio])
    text = None
    if bw is not None:
        if gpd['verbose']:
            print(f"[INFO] Beam Decode [bw={bw}]...")
        res = model.eval_one_batch_with_beam(model.device, bw, data, lens, text, audio_base.int2word,
                                             second_pass=True if lm_model is not None else False,
                                             lm_model=lm_model, lm_weight=1.5, length_weight=1.5)
    else:
        res = model.eval_one_batch_with_greedy(model.device, data, lens, audio_base.int2word, text)
    return res.pred_text[0]


def parse_batch(paths, model, audio_base, lm_model=None, bw=None):
    """Batched form of parse (the reference's __init__.py names it but never defines it): all
    files go through the GPU path as one batch."""
    audios = [p if not isinstance(p, (str, os.PathLike)) else fast_read(convert_audio(p)) for p in paths]
    data, lens = features_for(audios)
    if bw is not None:
        res = model.eval_one_batch_with_beam(model.device, bw, data, lens, None, audio_base.int2word,
                                             second_pass=lm_model is not None, lm_model=lm_model,
                                             lm_weight=1.5, length_weight=1.5)
    else:
        res = model.eval_one_batch_with_greedy(model.device, data, lens, audio_base.int2word, None)
    return list(res.pred_text)


class ASR:
    """main.py:68-102."""

    def __init__(self, lm_path=None, bw=None, ckpt='./pretrain-0.06328.ckpt'):
        if lm_path is not None and bw is not None and bw > 1:
            import kenlm  # third-party (model.py:13); absent here -> ImportError like the reference
            print('loading language model...')
            ts = time()
            lm_model = kenlm.LanguageModel(lm_path)
            print('loading cost %.3fs' % (time() - ts))
        else:
            lm_model = None
        model = Model()
        model.load(ckpt)
        model.model.eval()
        self.audio_base = AudioBase()
        self.lm_model = lm_model
        self.model = model
        self.bw = bw

    def __call__(self, path):
        return parse(path, self.model, self.audio_base, self.lm_model, self.bw)


if __name__ == '__main__':
    gpd['verbose'] = False
    gpd['temperature'] = 1
    asr = ASR(bw=int(sys.argv[2]) if len(sys.argv) > 2 else None,
              ckpt=os.environ.get('CASR_CKPT', './pretrain-0.06328.ckpt'))
    print(asr(sys.argv[1]))
