"""CPU checks of the data.py / main.py drop-ins: WAV decoding with soundfile's float32 scaling
(fast_read, data.py:109-121) for every encoding the reader accepts, and the reference's
failure modes (non-WAV input, multi-channel, unsupported formats)."""
import struct
import wave

import numpy as np
import pytest

import data as D


def write_pcm(path, samples_int, width, rate=16000, ch=1):
    with wave.open(str(path), "wb") as w:
        w.setnchannels(ch)
        w.setsampwidth(width)
        w.setframerate(rate)
        w.writeframes(samples_int.tobytes())


def write_float(path, x, rate=16000):
    data = np.asarray(x, "<f4").tobytes()
    fmt = struct.pack("<HHIIHH", 3, 1, rate, rate * 4, 4, 32)
    body = b"WAVE" + b"fmt " + struct.pack("<I", len(fmt)) + fmt + b"data" + struct.pack("<I", len(data)) + data
    with open(path, "wb") as f:
        f.write(b"RIFF" + struct.pack("<I", len(body)) + body)


def test_fast_read_pcm16(tmp_path):
    x = np.array([0, 1, -1, 32767, -32768, 1234], np.int16)
    write_pcm(tmp_path / "a.wav", x, 2)
    np.testing.assert_array_equal(D.fast_read(str(tmp_path / "a.wav")), x.astype(np.float32) / 32768.0)


def test_fast_read_pcm24_pcm32_u8_float(tmp_path):
    v = np.array([0, 1, -1, 8388607, -8388608], np.int32)
    raw = np.stack([(v >> s) & 0xFF for s in (0, 8, 16)], 1).astype(np.uint8)
    write_pcm(tmp_path / "b.wav", raw, 3)
    np.testing.assert_array_equal(D.fast_read(str(tmp_path / "b.wav")), (v / 8388608.0).astype(np.float32))
    v32 = np.array([0, 1 << 30, -(1 << 31)], np.int32)
    write_pcm(tmp_path / "c.wav", v32, 4)
    np.testing.assert_array_equal(D.fast_read(str(tmp_path / "c.wav")), (v32 / 2147483648.0).astype(np.float32))
    u8 = np.array([128, 0, 255], np.uint8)
    write_pcm(tmp_path / "d.wav", u8, 1)
    np.testing.assert_array_equal(D.fast_read(str(tmp_path / "d.wav")), (u8.astype(np.float32) - 128) / 128)
    f = np.array([0.25, -0.5, 1e-3], np.float32)
    write_float(tmp_path / "e.wav", f)
    np.testing.assert_array_equal(D.fast_read(str(tmp_path / "e.wav")), f)


def test_fast_read_rejects_non_wav_and_stereo(tmp_path):
    (tmp_path / "x.mp3").write_bytes(b"ID3\x00\x00")
    with pytest.raises(ValueError):
        D.fast_read(str(tmp_path / "x.mp3"))
    write_pcm(tmp_path / "s.wav", np.zeros(8, np.int16), 2, ch=2)
    with pytest.raises(ValueError):
        D.fast_read(str(tmp_path / "s.wav"))


def test_create_fb_matrix_is_the_library_filterbank():
    from casr import lib as L
    fb = D.create_fb_matrix(257, 80.0, 7600.0, 80)
    np.testing.assert_array_equal(fb.numpy(), L.mel_filterbank())
