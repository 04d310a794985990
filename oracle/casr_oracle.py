"""CPU ORACLE — test infrastructure only. NOT part of the product path.

A float32 numpy restatement of the reference's inference path (shawnthu/chinese-asr),
used only by ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
``bench.py`` as the checker.  The product path (chinese-asr_amd/) never imports it.

Parity pinning: the restatement is checked against golden vectors captured from the
reference itself, imported in the build container with shims
(tests/golden/make_golden.py -> tests/golden/*.npz; tests/test_oracle_golden.py), and
against the reference's own encoder known-answer test (encoder.py:636-652:
110345.5 / 2048 / 28160).

Each function cites the reference lines it restates.
"""
import math

import numpy as np

F32 = np.float32
NEG_INF = F32(-np.inf)


# --------------------------------------------------------------------------------------
# front-end
# --------------------------------------------------------------------------------------
def create_fb_matrix(n_stft=257, f_min=80.0, f_max=7600.0, n_mels=80):
    """data.py:21-57 (including the quirk stft_freqs = linspace(f_min, f_max, n_stft),
    data.py:43; AudioBase uses f_min=80, f_max=7600, n_stft=257: data.py:378-380)."""
    def hz2mel(f):
        return F32(2595.0) * np.log10(F32(1.0) + (np.asarray(f, F32) / F32(700.0)))

    def mel2hz(m):
        return F32(700.0) * (F32(10.0) ** (m / F32(2595.0)) - F32(1.0))

    stft_freqs = np.linspace(f_min, f_max, n_stft, dtype=np.float64).astype(F32)
    m_min = F32(0.0) if f_min == 0 else hz2mel(f_min)
    m_max = hz2mel(f_max)
    m_pts = np.linspace(float(m_min), float(m_max), n_mels + 2, dtype=np.float64).astype(F32)
    f_pts = mel2hz(m_pts).astype(F32)
    f_diff = f_pts[1:] - f_pts[:-1]
    slopes = f_pts[None, :] - stft_freqs[:, None]
    down = (F32(-1.0) * slopes[:, :-2]) / f_diff[:-1]
    up = slopes[:, 2:] / f_diff[1:]
    return np.maximum(F32(0.0), np.minimum(down, up)).astype(F32)


def hann_window(n=400):
    """torch.hann_window(400), periodic (data.py:381-382)."""
    k = np.arange(n, dtype=np.float64)
    return (0.5 - 0.5 * np.cos(2.0 * math.pi * k / n)).astype(F32)


def log_mel(audio, preemphasis=0.97, n_fft=512, hop=160, win=400, fb=None, window=None):
    """data.py:167-224 (inference: no dither, no augmentation).
    audio: float32 [N] (soundfile float32 read).  Returns [L, 80] float32 with
    L = 1 + (N - 1 - n_fft) // hop; N - 1 < n_fft raises like torch.stft does."""
    audio = np.asarray(audio, F32)
    if preemphasis > 0:
        audio = audio[1:] - F32(preemphasis) * audio[:-1]                    # data.py:201-202
    n = audio.shape[0]
    if n < n_fft:
        raise RuntimeError("audio shorter than n_fft (torch.stft would raise, data.py:204)")
    window = hann_window(win) if window is None else window
    lpad = (n_fft - win) // 2
    w = np.zeros(n_fft, F32)
    w[lpad:lpad + win] = window                                            # centred, zero-padded
    nframes = 1 + (n - n_fft) // hop
    idx = np.arange(nframes)[:, None] * hop + np.arange(n_fft)[None, :]
    frames = audio[idx] * w[None, :]
    spec = np.fft.rfft(frames.astype(np.float64), n=n_fft, axis=1)        # center=False, onesided
    power = (spec.real.astype(F32) ** 2 + spec.imag.astype(F32) ** 2).astype(F32)  # data.py:220-221
    fb = create_fb_matrix() if fb is None else fb
    mel = (power @ fb).astype(F32)                                         # data.py:222
    mel[mel == 0] = np.finfo(np.float32).eps                               # data.py:223
    return np.log(mel).astype(F32)                                         # data.py:224


def delta_filters():
    """The three normalised 9-tap filters of add_delta_deltas (data.py:129-150)."""
    d = np.array([2, 1, 0, -1, -2], np.float64)
    dd = np.convolve(d, d, "full")
    stack = np.array([[0] * 4 + [1] + [0] * 4, [0] * 2 + list(d) + [0] * 2, list(dd)], np.float32)
    stack /= np.sqrt(np.sum(stack.astype(np.float32) ** 2, axis=1, keepdims=True)).astype(np.float32)
    return stack.astype(F32)  # [3, 9]


def add_delta_deltas(fbank):
    """data.py:129-164: zero-pad 4 frames each side, cross-correlate along time.
    fbank [L, 80] -> [3, L, 80]."""
    x = np.asarray(fbank, F32)
    L = x.shape[0]
    filt = delta_filters()
    xp = np.zeros((L + 8, x.shape[1]), F32)
    xp[4:4 + L] = x
    out = np.zeros((3, L, x.shape[1]), F32)
    for c in range(3):
        acc = np.zeros((L, x.shape[1]), F32)
        for k in range(9):
            if filt[c, k] != 0:
                acc += filt[c, k] * xp[k:k + L]
        out[c] = acc
    return out


def stack_frames(feat3):
    """data.py:242-249: [3, L, 80] -> [L//3, 720], out[j, c*240 + r*80 + m] = F[c, 3j+r, m]."""
    c, L, m = feat3.shape
    Lp = L // 3
    f = feat3[:, :3 * Lp].reshape(c, Lp, 3 * m)
    return np.ascontiguousarray(f.transpose(1, 0, 2).reshape(Lp, c * 3 * m))


def cmvn(x, eps=1e-6):
    """main.py:37 (eps 1e-6; the loader's batch_audio uses 1e-7, data.py:517-518):
    per-dimension (x - mean_t) / (std_t,unbiased + eps)."""
    x = np.asarray(x, F32)
    mean = x.mean(axis=0, dtype=np.float64).astype(F32)
    std = np.sqrt(((x.astype(np.float64) - mean) ** 2).sum(axis=0) / (x.shape[0] - 1)).astype(F32) \
        if x.shape[0] > 1 else np.full(x.shape[1], np.nan, F32)
    return ((x - mean) / (std + F32(eps))).astype(F32)


def features_from_fbank(fbank, eps=1e-6):
    """fbank [T, 80] -> encoder input [T//3, 720] (data.py:226-249 + main.py:37)."""
    return cmvn(stack_frames(add_delta_deltas(fbank)), eps)


# --------------------------------------------------------------------------------------
# network
# --------------------------------------------------------------------------------------
def _sigmoid(x):
    return (F32(1.0) / (F32(1.0) + np.exp(-x))).astype(F32)


def _lstm_cell(gates, c):
    """PyTorch LSTM gate order i, f, g, o."""
    H = c.shape[1]
    i = _sigmoid(gates[:, 0:H])
    f = _sigmoid(gates[:, H:2 * H])
    g = np.tanh(gates[:, 2 * H:3 * H])
    o = _sigmoid(gates[:, 3 * H:4 * H])
    c2 = (f * c + i * g).astype(F32)
    h2 = (o * np.tanh(c2)).astype(F32)
    return h2, c2


def _bilstm_layer(x, lens, wih, whh, bih, bhh, wih_r, whh_r, bih_r, bhh_r):
    """One packed bidirectional nn.LSTM layer (util.py:1249-1262 via get_rnn
    util.py:726-746).  x: [T, B, Din] (zeros past len).  Returns y [T, B, 2H] with zeros
    past each length, and final (h, c) per direction [2, B, H]."""
    T, B, _ = x.shape
    H = whh.shape[1]
    y = np.zeros((T, B, 2 * H), F32)
    hN = np.zeros((2, B, H), F32)
    cN = np.zeros((2, B, H), F32)
    for d, (Wi, Wh, bi, bh) in enumerate(((wih, whh, bih, bhh), (wih_r, whh_r, bih_r, bhh_r))):
        gx = (x.reshape(T * B, -1) @ Wi.T + bi).reshape(T, B, 4 * H).astype(F32)
        h = np.zeros((B, H), F32)
        c = np.zeros((B, H), F32)
        for s in range(T):
            act = s < lens
            if not act.any():
                break
            if d == 0:
                t = np.full(B, s)
            else:
                t = np.where(act, lens - 1 - s, 0)
            g = (gx[t, np.arange(B)] + (h @ Wh.T + bh)).astype(F32)
            h2, c2 = _lstm_cell(g, c)
            h = np.where(act[:, None], h2, h)
            c = np.where(act[:, None], c2, c)
            rows = np.nonzero(act)[0]
            y[t[rows], rows, d * H:(d + 1) * H] = h2[rows]
        hN[d], cN[d] = h, c
    return y, hN, cN


def encoder_forward(feats, lens, enc_sd, num_layers=4, residual=True):
    """RNNEncoder.forward (encoder.py:36-81) + RNN_RES.forward (util.py:1223-1324).
    feats: list of B arrays [T_b, D]; lens: [B] ints.  Returns (out [Tmax, B, 2H] f32 with
    zeros past len, (h [B, 2H], c [B, 2H]) = last layer [fw || bw] final states)."""
    lens = np.asarray(lens, np.int64)
    B = len(feats)
    T = int(lens.max())
    D = feats[0].shape[1]
    x = np.zeros((T, B, D), F32)
    for b, f in enumerate(feats):
        x[:lens[b], b] = f[:lens[b]]
    hN = cN = None
    for i in range(num_layers):
        p = f"rnn.rnn.{i}."
        y, hN, cN = _bilstm_layer(
            x, lens,
            enc_sd[p + "weight_ih_l0"], enc_sd[p + "weight_hh_l0"], enc_sd[p + "bias_ih_l0"], enc_sd[p + "bias_hh_l0"],
            enc_sd[p + "weight_ih_l0_reverse"], enc_sd[p + "weight_hh_l0_reverse"],
            enc_sd[p + "bias_ih_l0_reverse"], enc_sd[p + "bias_hh_l0_reverse"])
        x = (x + y).astype(F32) if (residual and i > 0) else y            # util.py:1284-1291
    h = np.concatenate([hN[0], hN[1]], axis=1)                             # encoder.py:67-72
    c = np.concatenate([cN[0], cN[1]], axis=1)
    return x, (h, c)


def mask_for_softmax(lens, T=None):
    """get_mask_for_softmax (util.py:131-142): [T, B], 0 valid, -inf padding."""
    lens = np.asarray(lens)
    T = int(lens.max()) if T is None else T
    m = np.zeros((T, len(lens)), F32)
    m[np.arange(T)[:, None] >= lens[None, :]] = NEG_INF
    return m


def compute_keys(enc, dec_sd):
    """BauAttn.compute_key_value (attention.py:67-78), map_enc False: values = enc."""
    return (enc @ dec_sd["attn_mechanism.W_enc"] + dec_sd["attn_mechanism.b_attn"]).astype(F32)


def attention(enc, mask, h, keys, dec_sd):
    """BauAttn.forward, heads == 1 (attention.py:91-95).  enc/keys [T, R, *], h [R, Hd]."""
    q = (h @ dec_sd["attn_mechanism.W_hidden"]).astype(F32)
    e = (np.tanh(keys + q[None]) * dec_sd["attn_mechanism.v"]).sum(axis=2, dtype=F32).astype(F32)
    z = (mask + e).astype(F32)
    z = z - z.max(axis=0, keepdims=True)
    p = np.exp(z).astype(F32)
    alpha = (p / p.sum(axis=0, keepdims=True, dtype=F32)).astype(F32)
    ctx = (alpha[..., None] * enc).sum(axis=0, dtype=F32).astype(F32)
    return ctx, alpha


def decoder_step(enc, mask, keys, token, h, c, ctx_prev, dec_sd):
    """RNNDecoder.forward (decoder.py:94-137) with input feeding: x = [embed(token) || ctx_prev],
    LSTMCell (util.py:1650-1661), attention, logit = proj([h || ctx])."""
    x = np.concatenate([dec_sd["embedding.weight"][token], ctx_prev], axis=1)
    g = (x @ dec_sd["cell.cell.0.weight_ih"].T + dec_sd["cell.cell.0.bias_ih"]
         + (h @ dec_sd["cell.cell.0.weight_hh"].T + dec_sd["cell.cell.0.bias_hh"])).astype(F32)
    h2, c2 = _lstm_cell(g, c)
    ctx, alpha = attention(enc, mask, h2, keys, dec_sd)
    logit = (np.concatenate([h2, ctx], axis=1) @ dec_sd["proj_linear.weight"].T
             + dec_sd["proj_linear.bias"]).astype(F32)
    return logit, h2, c2, ctx, alpha


def _log_softmax(logit):
    m = logit.max(axis=1, keepdims=True)
    lse = (m + np.log(np.exp(logit - m).sum(axis=1, keepdims=True, dtype=F32))).astype(F32)
    return (logit - lse).astype(F32)


def greedy_decode(feats, lens, enc_sd, dec_sd, sos=1, eos=2, max_len=40, temperature=1.0,
                  int2word=None, return_alignment=False):
    """Model.eval_one_batch_with_greedy (model.py:503-602).
    Returns dict(tokens=list of lists, score=list[float], text_len=int32[B],
    finished=bool[B], accum=f32[B], steps=int, logit_gap=min top1-top2 gap per step,
    alignment=list of [T, B] (optional), pred_text (if int2word))."""
    lens = np.asarray(lens, np.int64)
    B = len(feats)
    enc, (h, c) = encoder_forward(feats, lens, enc_sd)
    mask = mask_for_softmax(lens)
    keys = compute_keys(enc, dec_sd)
    tokens = np.full(B, sos, np.int64)
    ctx = np.zeros((B, enc.shape[2]), F32)
    finished = np.zeros(B, bool)
    final_lens = np.zeros(B, np.int32)
    accum = np.zeros(B, F32)
    outputs, alignments, gaps = [], [], []
    for l in range(max_len):
        logit, h, c, ctx, alpha = decoder_step(enc, mask, keys, tokens, h, c, ctx, dec_sd)
        alignments.append(alpha)
        logp = _log_softmax(logit)
        tokens = logp.argmax(axis=1)                                       # first max
        lp = logp[np.arange(B), tokens]
        top2 = np.partition(logp, -2, axis=1)[:, -2:]
        gaps.append((top2[:, 1] - top2[:, 0]).astype(np.float64))
        outputs.append(tokens.copy())
        cur = tokens == eos
        accum = (accum + ((~finished) & cur).astype(F32) * lp).astype(F32)  # model.py:567-576
        finished |= cur
        final_lens += (~finished).astype(np.int32)
        accum = (accum + (~finished).astype(F32) * lp).astype(F32)
        if finished.all():
            break
    outs = np.stack(outputs, axis=1)
    toks = [outs[b, :final_lens[b]].tolist() for b in range(B)]
    score = [0.0 if len(t) == 0 else float(accum[b]) / (int(final_lens[b]) + int(finished[b]))
             for b, t in enumerate(toks)]
    res = dict(tokens=toks, score=score, text_len=final_lens, finished=finished, accum=accum,
               steps=len(outputs), gaps=np.stack(gaps, axis=0), all_tokens=outs)
    if return_alignment:
        res["alignment"] = alignments
    if int2word is not None:
        res["pred_text"] = ["".join(int2word[e] for e in t) for t in toks]
    return res


def beam_decode(feats, lens, enc_sd, dec_sd, bmsz, sos=1, eos=2, pad=0, max_len=40,
                temperature=1.0, second_pass=False, lm_model=None, lm_weight=0.0,
                length_weight=0.0, int2word=None):
    """Model.eval_one_batch_with_beam (model.py:604-987), rules of SURVEY §3.2:
    l == 0 restricted to beam 0; finished recorded from the first k candidates;
    early stop once every utterance's rank-0 candidate has ever been EOS; active =
    first k non-EOS of the 2k; unfinished fallback adds length_weight*(l+1);
    second pass only for utterances with > 1 finished hypotheses.
    Returns dict(tokens, score, records, steps)."""
    lens = np.asarray(lens, np.int64)
    B = len(feats)
    k = bmsz
    V = dec_sd["proj_linear.weight"].shape[0]
    enc, (h, c) = encoder_forward(feats, lens, enc_sd)
    mask = mask_for_softmax(lens)
    keys = compute_keys(enc, dec_sd)
    # tile_batch (util.py:41-56): bb = b*k + j
    rep = np.repeat(np.arange(B), k)
    enc_t, mask_t, keys_t = enc[:, rep], mask[:, rep], keys[:, rep]
    h, c = h[rep], c[rep]
    ctx = np.zeros((B * k, enc.shape[2]), F32)
    hist = np.full((max_len + 1, B * k), pad, np.int64)
    hist[0] = sos
    score_buf = np.zeros(B * k, F32)
    bb_off = k * np.arange(B)
    records = {b: [] for b in range(B)}   # b -> list of (tokens, score) in (step, rank) order
    top_fin = np.zeros(B, bool)
    l = 0
    for l in range(max_len):
        logit, h, c, ctx, _ = decoder_step(enc_t, mask_t, keys_t, hist[l], h, c, ctx, dec_sd)
        logit = (logit / F32(temperature)).astype(F32)
        logp = (_log_softmax(logit) + score_buf[:, None]).astype(F32)
        scores = logp.reshape(B, k * V)
        if l == 0:
            scores = scores[:, :V]
        # torch.topk(..., 2k): sorted descending; ties resolved to the lower index
        order = np.argsort(-scores, axis=1, kind="stable")[:, :2 * k]
        cand_scores = np.take_along_axis(scores, order, axis=1)
        cand_beams = order // V                                            # model.py:866 (trunc)
        cand_tok = order % V
        for b in range(B):
            for j in range(k):
                if cand_tok[b, j] == eos:
                    src = b * k + cand_beams[b, j]
                    records[b].append((hist[1:l + 1, src].tolist(), float(cand_scores[b, j])))
        top_fin |= cand_tok[:, 0] == eos
        if top_fin.all():
            break
        key = np.arange(2 * k)[None, :] + (cand_tok == eos) * (2 * k)
        active = np.argsort(key, axis=1, kind="stable")[:, :k]
        sel_beams = np.take_along_axis(cand_beams, active, axis=1)
        bb = (sel_beams + bb_off[:, None]).reshape(-1)
        sel_tok = np.take_along_axis(cand_tok, active, axis=1).reshape(-1)
        h, c, ctx = h[bb], c[bb], ctx[bb]
        hist = hist[:, bb]
        hist[l + 1] = sel_tok
        score_buf = np.take_along_axis(cand_scores, active, axis=1).reshape(-1).astype(F32)
    best = {}
    for b in range(B):
        v = records[b]
        if not v:
            continue
        if second_pass and len(v) > 1:
            lm = [lm_model.score(" ".join(int2word[i] for i in t), bos=True) for t, _ in v]
            comb = [s + lm_weight * q + length_weight * len(t) for (t, s), q in zip(v, lm)]
            best[b] = v[int(np.argmax(comb))]
        elif second_pass:
            best[b] = v[0]
        else:
            best[b] = max(v, key=lambda e: e[1])                           # first max
    for b in range(B):
        if b in best:
            continue
        act = (score_buf + F32(lm_weight) * F32(0.0) + F32(length_weight * (l + 1))).astype(F32)
        seg = act[b * k:(b + 1) * k]
        j = int(np.argmax(seg))
        best[b] = (hist[1:l + 2, b * k + j].tolist(), float(seg[j]))
    toks = [best[b][0] for b in range(B)]
    res = dict(tokens=toks, score=[best[b][1] for b in range(B)], records=records, steps=l + 1)
    if int2word is not None:
        res["pred_text"] = ["".join(int2word[e] for e in t) for t in toks]
    return res
