"""CPU-side checks of the C-ABI library: it loads, exports every symbol include/casr.h declares,
rejects bad configurations, fails loudly without a GPU, and packs weights into the documented
kernel layouts (checked against a numpy restatement of the layout contract)."""
import ctypes
import os
import re

import numpy as np
import pytest

from casr import lib as L
from casr.config import CasrConfig
from casr.weights import synthetic_state_dicts

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CFG = CasrConfig()


def header_functions():
    src = open(os.path.join(REPO, "include", "casr.h")).read()
    return sorted(set(re.findall(r"\b(casr_[a-z_]+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    lib = L.load()
    declared = header_functions()
    assert declared == sorted(L.EXPORTS)
    for name in declared:
        assert hasattr(lib, name), name
    assert lib.casr_api_version() == 3


def test_s16x1_build_exports_the_same_symbols_and_layout():
    """The opt-in s16x1 perf arithmetic is a second build of the same sources (casr/build.py
    variant "s16x1", include/casr.h CASR_PREC_S16X1): the same exports, API version and packed
    blob (a blob packed by either library binds to both)."""
    base, var = L.load(), L.load(variant="s16x1")
    assert base is not var
    for name in header_functions():
        assert hasattr(var, name), name
    assert var.casr_api_version() == 3
    c = L.config_struct(CFG)
    assert var.casr_packed_weights_floats(ctypes.byref(c)) == base.casr_packed_weights_floats(ctypes.byref(c))
    hdr = open(os.path.join(REPO, "include", "casr.h")).read()
    precs = dict((m.group(1).lower(), int(m.group(2))) for m in re.finditer(r"CASR_PREC_([A-Z0-9]+) = (\d+)", hdr))
    assert precs == L.PRECISIONS


def test_check_reads_the_error_text_of_the_handle_s_library():
    """casr.lib.check on a handle asks the library that created it (an s16x1 Engine's handle is
    not the shipped library's); without a handle, the given library or the shipped one."""
    var = L.load(variant="s16x1")
    bad = L.config_struct(CFG)
    bad.enc_hidden = 128
    h = ctypes.c_void_p()
    rc = var.casr_create(ctypes.byref(bad), 0, ctypes.byref(h))
    with pytest.raises(L.CasrError, match="enc_hidden"):
        L.check(rc, lib=var)
    fake = ctypes.c_void_p(0x1000)
    L.register_handle(fake, var)
    try:
        assert L._HANDLES[fake.value] is var
    finally:
        L.unregister_handle(fake)
    assert fake.value not in L._HANDLES


def test_create_without_gpu_or_bad_config_fails_loudly():
    import torch
    lib = L.load()
    h = ctypes.c_void_p()
    bad = L.config_struct(CFG)
    bad.enc_hidden = 128
    assert lib.casr_create(ctypes.byref(bad), 0, ctypes.byref(h)) == 4
    assert b"enc_hidden" in lib.casr_last_error(None)
    if not torch.cuda.is_available():
        c = L.config_struct(CFG)
        assert lib.casr_create(ctypes.byref(c), 0, ctypes.byref(h)) == 2
        assert lib.casr_last_error(None)
    with pytest.raises(L.CasrError):
        L.check(3)
    # tuning options need a handle: a NULL one is refused, not dereferenced
    v = ctypes.c_int32(-7)
    assert lib.casr_get_option(None, 0, ctypes.byref(v)) == 1 and v.value == -7
    assert lib.casr_set_option(None, 0, 1) == 1
    # the option table of include/casr.h and the binding agree
    hdr = open(os.path.join(REPO, "include", "casr.h")).read()
    opts = dict((m.group(1), int(m.group(2))) for m in re.finditer(r"CASR_OPT_([A-Z0-9_]+) = (\d+)", hdr))
    assert opts.pop("COUNT") == len(L.OPTIONS)
    assert opts == L.OPTIONS


def _layout(cfg):
    off = 0
    lay = {}

    def take(name, n):
        nonlocal off
        lay[name] = off
        off += (n + 63) & ~63

    H, C, HD, E, A, D = 256, 512, 512, 256, 128, 720
    VP = (cfg.vocab + 63) // 64 * 64
    for l in range(cfg.enc_layers):
        din = D if l == 0 else C
        take(f"wih{l}", 8 * H * din)
        take(f"bias{l}", 8 * H)
        take(f"whh{l}", 8 * H * H)
    take("emb", cfg.vocab * E)
    take("dec_w", 4 * HD * (E + C + HD))
    take("dec_b", 4 * HD)
    take("proj_w", VP * (C + HD))
    take("proj_b", VP)
    take("wencT", A * C)
    take("b_attn", A)
    take("w_hidden", HD * A)
    take("v", A)
    take("info", 64)
    for l in range(cfg.enc_layers):
        din = D if l == 0 else C
        take(f"wih16_{l}", 8 * H * ((din + 63) // 64 * 64))
        take(f"whh16_{l}", 8 * H * H)
    take("emb16", cfg.vocab * E)
    take("dec_w16", 4 * HD * (E + C + HD))
    take("proj_w16", VP * (C + HD))
    take("wenc16", A * C)
    lay["total"] = off
    return lay, VP


def _frag(blob, base, nt, kc, nkc, n_local, k_local):
    """element (row n_local of n-tile nt, k = kc*64 + k_local) of a fragment-major matrix"""
    g, rem = divmod(k_local, 16)
    q, e = divmod(rem, 4)
    lane = n_local + 16 * g
    return blob[base + (nt * nkc + kc) * 1024 + (q * 64 + lane) * 4 + e]


def test_packed_layout_contract():
    enc, dec = synthetic_state_dicts(CFG)
    blob = L.pack_weights(CFG, enc, dec)
    lay, VP = _layout(CFG)
    assert blob.size == lay["total"]
    rs = np.random.RandomState(0)
    H = 256
    # encoder input projection rows: d*1024 + (u//16)*64 + (u%16)*4 + g <- W_ih_d[g*H + u]
    for l in (0, 2):
        din = 720 if l == 0 else 512
        for _ in range(20):
            d, g, u, k = rs.randint(2), rs.randint(4), rs.randint(H), rs.randint(din)
            pr = d * 1024 + (u // 16) * 64 + (u % 16) * 4 + g
            suf = "_reverse" if d else ""
            W = enc[f"rnn.rnn.{l}.weight_ih_l0{suf}"]
            assert blob[lay[f"wih{l}"] + pr * din + k] == W[g * H + u, k]
            bsum = np.float32(enc[f"rnn.rnn.{l}.bias_ih_l0{suf}"][g * H + u] + enc[f"rnn.rnn.{l}.bias_hh_l0{suf}"][g * H + u])
            assert blob[lay[f"bias{l}"] + pr] == bsum
        # recurrent fragments: n-tile jb*4 + g
        for _ in range(20):
            d, g, u, k = rs.randint(2), rs.randint(4), rs.randint(H), rs.randint(H)
            suf = "_reverse" if d else ""
            W = enc[f"rnn.rnn.{l}.weight_hh_l0{suf}"]
            jb = u // 16
            v = _frag(blob, lay[f"whh{l}"] + d * 4 * H * H, jb * 4 + g, k // 64, H // 64, u % 16, k % 64)
            assert v == W[g * H + u, k]
    # decoder LSTM fragments, k order [emb | ctx | h]
    Wih, Whh = dec["cell.cell.0.weight_ih"], dec["cell.cell.0.weight_hh"]
    for _ in range(40):
        g, u, k = rs.randint(4), rs.randint(512), rs.randint(1280)
        want = Wih[g * 512 + u, k] if k < 768 else Whh[g * 512 + u, k - 768]
        assert _frag(blob, lay["dec_w"], (u // 16) * 4 + g, k // 64, 20, u % 16, k % 64) == want
    # projection fragments, k order [ctx | h]; rows past V are zero
    Wp = dec["proj_linear.weight"]
    for _ in range(40):
        n, k = rs.randint(VP), rs.randint(1024)
        want = 0.0 if n >= CFG.vocab else (Wp[n, 512 + k] if k < 512 else Wp[n, k - 512])
        assert _frag(blob, lay["proj_w"], n // 16, k // 64, 16, n % 16, k % 64) == want
    np.testing.assert_array_equal(blob[lay["wencT"]:lay["wencT"] + 128 * 512].reshape(128, 512),
                                  dec["attn_mechanism.W_enc"].T)
    np.testing.assert_array_equal(blob[lay["emb"]:lay["emb"] + CFG.vocab * 256].reshape(CFG.vocab, 256),
                                  dec["embedding.weight"])
    # s16x3 images: hi = f16_rn(w), lo = f16_rn((w - hi) 2^11); hi + lo 2^-11 within 2^-22 |w|
    assert blob[lay["info"]] == 1.0
    h16 = blob.view(np.float16)

    def close(got, want):
        assert abs(got - float(want)) <= 2.0 ** -21 * abs(float(want)) + 1e-12, (got, want)

    for l in (0, 1):
        din = 720 if l == 0 else 512
        kp = (din + 63) // 64 * 64
        for _ in range(20):
            n, k = rs.randint(2048), rs.randint(kp)
            base = 2 * (lay[f"wih16_{l}"] + n * kp) + (k // 32) * 64 + k % 32
            got = float(h16[base]) + float(h16[base + 32]) / 2048.0
            want = blob[lay[f"wih{l}"] + n * din + k] if k < din else 0.0
            close(got, want)
            if k < din:
                assert h16[base] == np.float16(want)
        if l == 0:  # attention key weights: s16 row image of wencT [A][C] (keys GEMM)
            for _ in range(20):
                n, k = rs.randint(128), rs.randint(512)
                base = 2 * (lay["wenc16"] + n * 512) + (k // 32) * 64 + k % 32
                want = blob[lay["wencT"] + n * 512 + k]
                close(float(h16[base]) + float(h16[base + 32]) / 2048.0, want)
                assert h16[base] == np.float16(want)
        # recurrent s16 fragments: block (nt, kc) = [j][hi|lo][lane][8], k = 16(lane>>4) + 8j + e
        for _ in range(20):
            nt, kc, lane, j, e = rs.randint(64), rs.randint(4), rs.randint(64), rs.randint(2), rs.randint(8)
            blk = 2 * (lay[f"whh16_{l}"] + (nt * 4 + kc) * 1024)
            hi = h16[blk + ((j * 2) * 64 + lane) * 8 + e]
            lo = h16[blk + ((j * 2 + 1) * 64 + lane) * 8 + e]
            k_local = 16 * (lane >> 4) + 8 * j + e
            want = _frag(blob, lay[f"whh{l}"], nt, kc, 4, lane & 15, k_local)
            close(float(hi) + float(lo) / 2048.0, want)
    e16 = blob[lay["emb16"]:lay["emb16"] + 1000].view(np.float16).astype(np.float64)
    np.testing.assert_allclose(e16[0::2] + e16[1::2] / 2048.0, blob[lay["emb"]:lay["emb"] + 1000],
                               rtol=2.0 ** -21, atol=1e-12)


def test_out_of_range_weights_fall_back_to_f32_images():
    """A weight the f16 split cannot carry (|w| >= 16 for the input projection's 2^11-scaled hi)
    marks the s16 images invalid (blob info word 0): handles then run exact f32 MFMA."""
    enc, dec = synthetic_state_dicts(CFG)
    enc = dict(enc)
    w = enc["rnn.rnn.1.weight_ih_l0"].copy()
    w[3, 5] = 100.0
    enc["rnn.rnn.1.weight_ih_l0"] = w
    blob = L.pack_weights(CFG, enc, dec)
    lay, _ = _layout(CFG)
    assert blob[lay["info"]] == 0.0


def test_keys_weight_range_uses_f16_limit_and_layout_stamp():
    """The keys GEMM's s16 images (two accumulators, no 2^11 scaling) only need the f16 range:
    |W_enc| = 100 keeps the s16 path (the input projection's < 16 limit does not apply to it).
    The blob carries a layout stamp (magic, total floats) after the info word, which
    casr_bind_weights checks."""
    enc, dec = synthetic_state_dicts(CFG)
    dec = dict(dec)
    w = dec["attn_mechanism.W_enc"].copy()
    w[7, 3] = 100.0
    dec["attn_mechanism.W_enc"] = w
    blob = L.pack_weights(CFG, enc, dec)
    lay, total = _layout(CFG)
    assert blob[lay["info"]] == 1.0
    stamp = blob[lay["info"] + 1:lay["info"] + 4].view(np.uint32)
    assert stamp[0] == 0xCA5B0003
    assert int(stamp[1]) | (int(stamp[2]) << 32) == blob.size == L.packed_floats(CFG)
    w[7, 3] = 20000.0
    assert L.pack_weights(CFG, enc, dec)[lay["info"]] == 0.0


def test_mel_filterbank_matches_reference_fixture():
    """The library's own create_fb_matrix (data.py:21-57, float32, linspace(80, 7600, 257) bin
    quirk) against the matrix captured from the reference and against the oracle."""
    from golden_util import load_golden
    from oracle import casr_oracle as O
    G, _ = load_golden()
    fb = L.mel_filterbank()
    assert fb.shape == (257, 80)
    # float32 log10f / powf vs torch's float kernels: <= 1e-5 on weights <= 1 (same bound as the
    # oracle's own fixture test, tests/test_oracle_golden.py)
    np.testing.assert_allclose(fb, G["fb_matrix"], atol=2e-5, rtol=0)
    np.testing.assert_allclose(fb, O.create_fb_matrix(), atol=2e-5, rtol=0)
    assert ((fb > 0) == (G["fb_matrix"] > 0)).all()  # same filter supports


@pytest.mark.parametrize("n", [0, 100, 512, 513, 514, 672, 673, 24000, 128353, 10 ** 6])
def test_log_mel_frame_count(n):
    """torch.stft center=False on the pre-emphasised signal (n - 1 samples): 1 + (n-1-512)//160,
    and the reference raises below 513 samples (data.py:204) -> 0 here (plus a device flag)."""
    want = 1 + (n - 1 - 512) // 160 if n - 1 >= 512 else 0
    assert L.log_mel_frames(n) == want
