"""wav -> log-mel HIP front-end (casr_log_mel) vs the reference's golden log-mel and the CPU
oracle (get_log_mel data.py:167-224), through the C ABI.

Tolerances: log-mel 1e-3 abs (fp32 FFT rounding in the reference vs fp64 here; the oracle itself
matches the reference at 5e-4), stacked delta features 3e-3 abs; frame counts exact.
"""
import numpy as np
import pytest
import torch

from golden_util import load_golden
from oracle import casr_oracle as O
from casr.config import CasrConfig
from casr.weights import synthetic_state_dicts

pytestmark = pytest.mark.gpu

G, META = load_golden()
CFG = CasrConfig()


@pytest.fixture(scope="module")
def eng():
    from casr.engine import Engine
    e = Engine(CFG, *synthetic_state_dicts(CFG, peaked=True))
    yield e
    e.close()


def synth_wav(n, seed):
    rs = np.random.RandomState(seed)
    t = np.arange(n) / 16000.0
    f0 = rs.uniform(100, 400)
    w = 0.4 * np.sin(2 * np.pi * f0 * t) * (1 + 0.5 * np.sin(2 * np.pi * 3 * t)) + 0.05 * rs.standard_normal(n)
    return w.astype(np.float32)


def test_log_mel_matches_reference_golden(eng):
    wav = G["wav0"]
    fb, frames = eng.log_mel(torch.from_numpy(wav[None]).cuda(), [wav.shape[0]])
    assert eng.device_flags() == 0
    ref = G["wav0_logmel"]
    assert int(frames[0]) == ref.shape[0] == fb.shape[1]
    np.testing.assert_allclose(fb[0].cpu().numpy(), ref, atol=1e-3, rtol=0)
    # -> delta / stacking without CMVN: what get_log_mel returns (data.py:226-249)
    feat, flen = eng.features(fb, frames, eps=-1.0)
    np.testing.assert_allclose(feat[0, :int(flen[0])].cpu().numpy(), G["wav0_features"], atol=3e-3, rtol=0)


def test_log_mel_ragged_batch_matches_oracle(eng):
    ns = [513, 673, 16000, 24000, 47999, 128353, 5000, 800]
    B, n_max = len(ns), max(ns)
    wav = np.zeros((B, n_max), np.float32)
    for b, n in enumerate(ns):
        wav[b, :n] = synth_wav(n, 100 + b)
    wav[3, 7000:7600] = 0.0  # a silent stretch
    fb, frames = eng.log_mel(torch.from_numpy(wav).cuda(), torch.tensor(ns, dtype=torch.int32))
    assert eng.device_flags() == 0
    fb = fb.cpu().numpy()
    for b, n in enumerate(ns):
        ref = O.log_mel(wav[b, :n])
        assert int(frames[b]) == ref.shape[0]
        np.testing.assert_allclose(fb[b, :ref.shape[0]], ref, atol=1e-3, rtol=0)
        assert (fb[b, ref.shape[0]:] == 0).all()


@pytest.mark.parametrize("golden", [True, False])
def test_log_mel_forms_bitwise_equal(eng, golden):
    """CASR_OPT_LOGMEL_Q16 (round 5): the 16-lanes-per-frame kernel (default: radix-4 stages 0-1 and
    2-3 in registers around one transpose) and the one-wave-per-frame kernel (three stage exchanges)
    run the same butterflies with the same twiddles in the same order, so their log-mel outputs are
    bitwise equal: on the reference's wav0 and on a ragged batch (padding frames, a silent stretch,
    the shortest valid signal of 513 samples)."""
    if golden:
        ns = [G["wav0"].shape[0]]
        wav = G["wav0"][None].astype(np.float32)
    else:
        ns = [513, 673, 16000, 24000, 47999, 5000, 800, 128353]
        wav = np.zeros((len(ns), max(ns)), np.float32)
        for b, n in enumerate(ns):
            wav[b, :n] = synth_wav(n, 300 + b)
        wav[4, 9000:9800] = 0.0
    w = torch.from_numpy(wav).cuda()
    outs = []
    try:
        for form in (1, 0):
            eng.set_option("LOGMEL_Q16", form)
            fb, frames = eng.log_mel(w, torch.tensor(ns, dtype=torch.int32))
            assert eng.device_flags() == 0
            outs.append((fb.cpu(), frames.cpu()))
    finally:
        eng.set_option("LOGMEL_Q16", 1)
    assert torch.equal(outs[0][1], outs[1][1])
    assert torch.equal(outs[0][0], outs[1][0])


def test_log_mel_short_audio_flag(eng):
    wav = torch.from_numpy(synth_wav(2000, 5)[None].repeat(2, 0)).cuda()
    fb, frames = eng.log_mel(wav, torch.tensor([2000, 400], dtype=torch.int32))
    assert int(frames[1]) == 0 and int(frames[0]) == 1 + (2000 - 1 - 512) // 160
    assert eng.device_flags() & 64


def test_wav_to_greedy_matches_oracle(eng):
    """The whole north-star chain from samples: log-mel -> delta/stack/CMVN (eps 1e-6,
    main.py:37) -> encoder -> greedy decode, identical tokens to the oracle chain."""
    ns = [24000, 36000, 16000]
    wav = np.zeros((3, max(ns)), np.float32)
    for b, n in enumerate(ns):
        wav[b, :n] = synth_wav(n, 300 + b)
    fb, frames = eng.log_mel(torch.from_numpy(wav).cuda(), ns)
    feat, flen = eng.features(fb, frames, eps=1e-6)
    eng.encode(feat, flen)
    out = eng.greedy()
    assert eng.device_flags() == 0
    enc_sd, dec_sd = synthetic_state_dicts(CFG, peaked=True)
    feats = [O.cmvn(O.stack_frames(O.add_delta_deltas(O.log_mel(wav[b, :n]))), 1e-6) for b, n in enumerate(ns)]
    r = O.greedy_decode(feats, [f.shape[0] for f in feats], enc_sd, dec_sd)
    np.testing.assert_array_equal(out["tokens"].cpu().numpy(), r["all_tokens"])


def _wav_file(path, x):
    import wave
    pcm = np.clip(np.round(x * 32768.0), -32768, 32767).astype(np.int16)
    with wave.open(str(path), "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(2)
        w.setframerate(16000)
        w.writeframes(pcm.tobytes())
    return pcm.astype(np.float32) / 32768.0  # what fast_read returns


def test_main_parse_and_asr_dropin(tmp_path):
    """main.parse / parse_batch / ASR(path) (main.py:27-102) on WAV files through the HIP chain,
    with weights round-tripped through the reference checkpoint format (model.py:347-370):
    the text equals the oracle chain's greedy decode of the same samples."""
    import main as MN
    import model as M
    from casr.vocab import load_vocab
    from casr.weights import save_checkpoint
    enc_sd, dec_sd = synthetic_state_dicts(CFG, peaked=True)
    ckpt = str(tmp_path / "w.ckpt")
    save_checkpoint(ckpt, enc_sd, dec_sd, args={"note": "synthetic"})
    asr = MN.ASR(ckpt=ckpt)
    i2w = load_vocab()[1]
    paths, samples = [], []
    for b, n in enumerate([24000, 40000, 12000]):
        p = tmp_path / f"u{b}.wav"
        samples.append(_wav_file(p, synth_wav(n, 500 + b)))
        paths.append(str(p))
    feats = [O.cmvn(O.stack_frames(O.add_delta_deltas(O.log_mel(s))), 1e-6) for s in samples]
    r = O.greedy_decode(feats, [f.shape[0] for f in feats], enc_sd, dec_sd)
    want = []
    for b in range(3):
        toks = r["all_tokens"][b]
        ids = []
        for t in toks:
            if t == CFG.eos:
                break
            ids.append(int(t))
        want.append("".join(i2w[i] for i in ids))
    assert [asr(p) for p in paths] == want
    assert MN.parse_batch(paths, asr.model, asr.audio_base) == want
    assert isinstance(M.Model().load(ckpt), dict)


def test_eval_loader_and_dataset_wer(tmp_path):
    """Batch I/O for dataset-level WER: manifest -> AudioDst (eval) ->
    AudioLoader batches through the HIP front-end with the loader's CMVN eps 1e-7
    (data.py:515-518) -> evaluate (model.py:240-261).  Features match the oracle chain; the
    dataset WER is the batch-size-weighted mean of the per-utterance WERs."""
    import data as D
    import model as M
    from casr.results import get_wer
    from casr.vocab import load_vocab
    w2i, i2w = load_vocab()
    ns = [24000, 40000, 12000, 30000, 20000]
    refs = ["你好世界", "今天天气很好", "谢谢", "我们", "中国人民"]
    lines, samples = [], []
    for b, n in enumerate(ns):
        p = tmp_path / f"u{b}.wav"
        samples.append(_wav_file(p, synth_wav(n, 700 + b)))
        lines.append(f"{p},{refs[b]}")
    man = tmp_path / "dev.csv"
    man.write_text("\n".join(lines))  # last line without newline: its text has no <unk>
    ab = D.AudioBase(manifests={"dev": str(man)})
    dst = D.AudioDst(ab, mode="eval", dev_or_test="dev")
    loader = D.AudioLoader(dst, batch_size=2)
    got, lens_all, texts = [], [], []
    for t, lens, text in loader.loader:
        assert isinstance(t, list) and lens.dtype == torch.int32
        got += [x.cpu().numpy() for x in t]
        lens_all += lens.tolist()
        texts += text
    assert len(got) == len(ns)
    for b, s in enumerate(samples):
        ref = O.cmvn(O.stack_frames(O.add_delta_deltas(O.log_mel(s))), 1e-7)
        assert got[b].shape == ref.shape and lens_all[b] == ref.shape[0]
        np.testing.assert_allclose(got[b], ref, atol=5e-3, rtol=0)
    assert texts[-1] == [w2i.get(ch, w2i["<unk>"]) for ch in refs[-1]]
    m = M.Model()
    m.load_state_dicts(*synthetic_state_dicts(CFG, peaked=True))
    wer, preds, rtexts = D.evaluate(m, loader, i2w)
    assert len(preds) == len(ns)
    per = [get_wer(p, r) for p, r in zip(preds, rtexts)]
    np.testing.assert_allclose(wer, np.mean(per), rtol=1e-12)
    # the same utterances one at a time give the same hypotheses (batch invariance)
    one = D.AudioLoader(dst, batch_size=1)
    assert D.evaluate(m, one, i2w)[1] == preds
