"""CPU BASELINE PORT — bench/test infrastructure only. NOT part of the product path.

A torch-CPU restatement of the same inference path as oracle/casr_oracle.py, written with stock
torch CPU operators (multi-threaded nn.LSTM over packed sequences, as the reference's
RNN_RES.forward runs it: util.py:1249-1275; multi-threaded elementwise attention ops,
attention.py:91-95), so that bench.py's ``cpu_baseline`` times a CPU path that runs at the
reference's own speed on the same cores (measured ratio: tools/calibrate_cpu.py ->
profiles/r03/cpu_calibration.json).  The numpy oracle stays the parity checker: numpy runs its
elementwise work on one thread, which made it ~2.5x slower than the reference on 8 cores.

Only tests/ (tests/test_torch_port.py: tokens equal to the numpy oracle's and the reference
goldens) and bench.py's cpu_baseline leg use it.  Each function cites the reference lines it
follows, as casr_oracle.py does.
"""
import numpy as np
import torch
from torch.nn.utils.rnn import pack_sequence, pad_packed_sequence, PackedSequence

from . import casr_oracle as O

F32 = torch.float32


def features_from_fbank(fbank, eps=1e-6):
    """data.py:226-249 (deltas, 3-frame stacking) + main.py:37 (CMVN): fbank [T, 80] -> [T//3, 720]."""
    x = torch.as_tensor(np.asarray(fbank, np.float32))
    L, m = x.shape
    filt = torch.from_numpy(O.delta_filters())
    xp = torch.zeros(L + 8, m)
    xp[4:4 + L] = x
    out = torch.zeros(3, L, m)
    for c in range(3):                                      # data.py:151-164 (cross-correlation)
        for k in range(9):
            if float(filt[c, k]) != 0.0:
                out[c] += filt[c, k] * xp[k:k + L]
    Lp = L // 3
    f = out[:, :3 * Lp].reshape(3, Lp, 3 * m).transpose(0, 1).reshape(Lp, 9 * m)
    return (f - f.mean(dim=0)) / (f.std(dim=0) + eps)       # main.py:37


class TorchPort:
    """Weights from the reference state dicts (numpy); modules built like the reference's
    (encoder.py:17-34, decoder.py:18-54, attention.py:23-51)."""

    def __init__(self, enc_sd, dec_sd, num_layers=4, residual=True):
        t = {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in enc_sd.items()}
        self.lstms = []
        for i in range(num_layers):
            p = f"rnn.rnn.{i}."
            din = t[p + "weight_ih_l0"].shape[1]
            m = torch.nn.LSTM(din, t[p + "weight_hh_l0"].shape[1], 1, bidirectional=True)
            m.load_state_dict({k[len(p):]: v for k, v in t.items() if k.startswith(p)})
            self.lstms.append(m.eval())
        self.residual = residual
        d = {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in dec_sd.items()}
        self.emb = d["embedding.weight"]
        self.cell = torch.nn.LSTMCell(d["cell.cell.0.weight_ih"].shape[1], d["cell.cell.0.weight_hh"].shape[1])
        self.cell.load_state_dict({k[len("cell.cell.0."):]: v for k, v in d.items() if k.startswith("cell.cell.0.")})
        self.cell.eval()
        self.w_enc, self.b_attn = d["attn_mechanism.W_enc"], d["attn_mechanism.b_attn"]
        self.w_hidden, self.v = d["attn_mechanism.W_hidden"], d["attn_mechanism.v"]
        self.proj_w, self.proj_b = d["proj_linear.weight"], d["proj_linear.bias"]

    @torch.no_grad()
    def encode(self, feats):
        """RNNEncoder.forward (encoder.py:36-81) + RNN_RES.forward (util.py:1223-1324): packed
        bidirectional layers, residual on the packed data from layer 1 on, final state of the last
        layer [fw || bw].  Returns (enc [T, B, 512], h [B, 512], c [B, 512], lens [B])."""
        x = pack_sequence([torch.as_tensor(f) for f in feats], enforce_sorted=False)
        hN = cN = None
        for i, m in enumerate(self.lstms):
            y, (hN, cN) = m(x)
            if self.residual and i > 0:                     # util.py:1284-1291
                y = PackedSequence(y.data + x.data, y.batch_sizes, y.sorted_indices, y.unsorted_indices)
            x = y
        enc, lens = pad_packed_sequence(x)
        return enc, torch.cat([hN[0], hN[1]], 1), torch.cat([cN[0], cN[1]], 1), lens

    def step(self, enc, mask, keys, token, h, c, ctx):
        """RNNDecoder.forward (decoder.py:94-137): input feeding, LSTMCell, additive attention
        (attention.py:91-95), projection of [h || ctx]."""
        h, c = self.cell(torch.cat([self.emb[token], ctx], 1), (h, c))
        e = (torch.tanh(keys + (h @ self.w_hidden)[None]) * self.v).sum(2)
        alpha = torch.softmax(mask + e, dim=0)
        ctx = (alpha[..., None] * enc).sum(0)
        logit = torch.addmm(self.proj_b, torch.cat([h, ctx], 1), self.proj_w.t())
        return logit, h, c, ctx

    @staticmethod
    def mask(lens, T):
        m = torch.zeros(T, len(lens))                       # get_mask_for_softmax util.py:131-142
        m[torch.arange(T)[:, None] >= lens[None, :]] = float("-inf")
        return m

    @torch.no_grad()
    def greedy(self, feats, sos=1, eos=2, max_len=40):
        """Model.eval_one_batch_with_greedy (model.py:503-602).  Returns (tokens [B][...], score)."""
        enc, h, c, lens = self.encode(feats)
        B = enc.shape[1]
        mask = self.mask(lens, enc.shape[0])
        keys = enc @ self.w_enc + self.b_attn               # attention.py:67-78
        tok = torch.full((B,), sos, dtype=torch.long)
        ctx = torch.zeros(B, enc.shape[2])
        fin = torch.zeros(B, dtype=torch.bool)
        flen = torch.zeros(B, dtype=torch.int32)
        acc = torch.zeros(B)
        outs = []
        for _ in range(max_len):
            logit, h, c, ctx = self.step(enc, mask, keys, tok, h, c, ctx)
            logp = logit - torch.logsumexp(logit, 1, keepdim=True)
            lp, tok = logp.max(1)
            outs.append(tok)
            cur = tok == eos
            acc = acc + ((~fin) & cur).float() * lp          # model.py:567-576
            fin = fin | cur
            flen += (~fin).int()
            acc = acc + (~fin).float() * lp
            if bool(fin.all()):
                break
        o = torch.stack(outs, 1)
        toks = [o[b, :int(flen[b])].tolist() for b in range(B)]
        score = [0.0 if not t else float(acc[b]) / (int(flen[b]) + int(fin[b])) for b, t in enumerate(toks)]
        return toks, score

    @torch.no_grad()
    def beam(self, feats, k, sos=1, eos=2, pad=0, max_len=40, temperature=1.0, length_weight=0.0):
        """Model.eval_one_batch_with_beam (model.py:604-987) without second pass: the rules of
        casr_oracle.beam_decode on torch tensors.  Returns (tokens, score)."""
        enc, h, c, lens = self.encode(feats)
        B = enc.shape[1]
        V = self.proj_w.shape[0]
        rep = torch.arange(B).repeat_interleave(k)          # tile_batch util.py:41-56
        mask = self.mask(lens, enc.shape[0])[:, rep]
        keys = (enc @ self.w_enc + self.b_attn)[:, rep]
        enc = enc[:, rep]
        h, c = h[rep], c[rep]
        ctx = torch.zeros(B * k, enc.shape[2])
        hist = torch.full((max_len + 1, B * k), pad, dtype=torch.long)
        hist[0] = sos
        sbuf = torch.zeros(B * k)
        off = (k * torch.arange(B))[:, None]
        records = [[] for _ in range(B)]
        top_fin = torch.zeros(B, dtype=torch.bool)
        l = 0
        for l in range(max_len):
            logit, h, c, ctx = self.step(enc, mask, keys, hist[l], h, c, ctx)
            logp = torch.log_softmax(logit / temperature, 1) + sbuf[:, None]   # model.py:834-836
            scores = logp.view(B, k * V)
            if l == 0:
                scores = scores[:, :V]                      # model.py:862-863
            cs, order = torch.sort(scores, dim=1, descending=True, stable=True)
            cs, order = cs[:, :2 * k], order[:, :2 * k]
            cb, ct = order // V, order % V                  # model.py:866 (trunc)
            fe = ct[:, :k] == eos                           # model.py:874-889
            for b, j in fe.nonzero().tolist():
                records[b].append((hist[1:l + 1, b * k + int(cb[b, j])].tolist(), float(cs[b, j])))
            top_fin |= ct[:, 0] == eos                      # model.py:897-901
            if bool(top_fin.all()):
                break
            key = torch.arange(2 * k)[None] + (ct == eos).long() * (2 * k)
            act = torch.sort(key, dim=1, stable=True)[1][:, :k]  # model.py:904-909
            bb = (torch.gather(cb, 1, act) + off).reshape(-1)
            # model.py:913-926 reorders every per-row tensor, the per-utterance-invariant encoder
            # outputs, keys and mask included: the same copies here, so the timed work is the
            # reference's (40.7 % of its beam time)
            enc, mask, keys = enc[:, bb], mask[:, bb], keys[:, bb]
            h, c, ctx, hist = h[bb], c[bb], ctx[bb], hist[:, bb]
            hist[l + 1] = torch.gather(ct, 1, act).reshape(-1)
            sbuf = torch.gather(cs, 1, act).reshape(-1)
        toks, score = [], []
        for b in range(B):
            if records[b]:
                t, s = max(records[b], key=lambda e: e[1])  # model.py:765 (first max)
            else:                                           # model.py:961-972
                seg = sbuf[b * k:(b + 1) * k] + length_weight * (l + 1)
                j = int(torch.argmax(seg))
                t, s = hist[1:l + 2, b * k + j].tolist(), float(seg[j])
            toks.append(t)
            score.append(s)
        return toks, score
