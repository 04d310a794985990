"""Host half of the C-ABI library under AddressSanitizer + UndefinedBehaviorSanitizer (CPU only).

casr_capi.hip (weight packing, argument and config checks, the mel filterbank, error
reporting) is compiled with the sanitizers on its host code only; the device code and the
other objects come from the product build.  ``tests/host_asan/host_check.cpp`` packs the
full-size synthetic weights with every tensor in its own exact-size heap buffer and checks the
error paths; the packed blob and the filterbank must equal the product library's bit for bit.
(GPU sanitizers are not available on the GPU pool; this covers the host code only.)"""
import os
import subprocess

import numpy as np
import pytest

from casr import build as B
from casr import lib as L
from casr.config import CasrConfig
from casr.weights import decoder_keys, encoder_keys, synthetic_state_dicts

HERE = os.path.dirname(os.path.abspath(__file__))
CLANG = "/opt/rocm/lib/llvm/bin/clang++"


def _sanitized_driver(tmp):
    B.build()  # the product objects (no-op when current)
    objdir = os.path.join(B.HERE, "_obj")
    capi = os.path.join(B.CSRC, "casr_capi.hip")
    capi_o = os.path.join(tmp, "casr_capi_asan.o")
    inc = [f"-I{B.INCLUDE}", f"-I{B.CSRC}"]
    san = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
           "-Xarch_host", "-fno-omit-frame-pointer", "-Xarch_host", "-fno-sanitize-recover=all"]
    subprocess.run([B.HIPCC, "-O1", "-g", "-std=c++17", f"--offload-arch={B.ARCH}", "-fPIC"] + inc + san
                   + ["-c", capi, "-o", capi_o], check=True, capture_output=True)
    drv_o = os.path.join(tmp, "host_check.o")
    subprocess.run([CLANG, "-O1", "-g", "-std=c++17", "-fsanitize=address,undefined",
                    "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", f"-I{B.INCLUDE}", "-c",
                    os.path.join(HERE, "host_asan", "host_check.cpp"), "-o", drv_o],
                   check=True, capture_output=True)
    others = [os.path.join(objdir, f) for f in sorted(os.listdir(objdir))
              if f.endswith(".o") and f != "casr_capi.o"]
    exe = os.path.join(tmp, "host_check")
    subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-fsanitize=address,undefined", "-fno-gpu-sanitize",
                    drv_o, capi_o] + others + ["-o", exe], check=True, capture_output=True)
    return exe


def _write_tensors(path, cfg, enc_sd, dec_sd, short=None):
    """short: a key whose tensor is written one float short (the sanitizer must see the read)."""
    c = L.config_struct(cfg)
    with open(path, "wb") as f:
        f.write(bytes(c))
        names = [k for k, _ in encoder_keys(cfg)]
        tensors = [enc_sd[k] for k in names] + [dec_sd[k] for k, _ in decoder_keys(cfg)]
        f.write(np.int64(len(tensors)).tobytes())
        keys = names + [k for k, _ in decoder_keys(cfg)]
        for k, t in zip(keys, tensors):
            a = np.ascontiguousarray(t, np.float32).ravel()
            if k == short:
                a = a[:-1]
            f.write(np.int64(a.size).tobytes())
            f.write(a.tobytes())


@pytest.mark.timeout(600)
def test_host_code_under_asan_ubsan(tmp_path):
    if not os.path.exists(B.HIPCC) or not os.path.exists(CLANG):
        pytest.skip("hipcc / clang++ not available")
    cfg = CasrConfig()
    names = [k for k, _ in decoder_keys(cfg)]
    assert names[:2] == ["embedding.weight", "cell.cell.0.weight_ih"] and names[-1] == "attn_mechanism.v", \
        "decoder_keys order must match casr_weights_host (host_check.cpp)"
    tmp = str(tmp_path)
    exe = _sanitized_driver(tmp)
    enc_sd, dec_sd = synthetic_state_dicts(cfg, peaked=True)
    tens, packed, fb = (os.path.join(tmp, n) for n in ("tensors.bin", "packed.bin", "fbank.bin"))
    _write_tensors(tens, cfg, enc_sd, dec_sd)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([exe, tens, packed, fb], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "host_check ok" in r.stdout
    assert "runtime error" not in r.stderr, r.stderr[-4000:]
    want = L.pack_weights(cfg, enc_sd, dec_sd)
    got = np.fromfile(packed, np.float32)
    assert got.size == want.size
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    np.testing.assert_array_equal(np.fromfile(fb, np.float32).reshape(257, 80), L.mel_filterbank())
    # the sanitizer is live: proj_linear.bias one float short is a heap-buffer-overflow read
    _write_tensors(tens, cfg, enc_sd, dec_sd, short="proj_linear.bias")
    r = subprocess.run([exe, tens, packed, fb], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode != 0 and "heap-buffer-overflow" in r.stderr, r.stderr[-2000:]
