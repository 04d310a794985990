"""Host-side finalize rules (casr/results.py) against the reference semantics restated in the
oracle and the reference-captured goldens: greedy score/length (model.py:582-593), loop
length (model.py:578), finished-record ordering and second-pass selection (model.py:708-765)."""
import os

import numpy as np
import pytest

from golden_util import load_golden
from casr.results import (edit_distance, get_wer, greedy_outputs, greedy_steps, records_by_utterance,
                          second_pass_select)
from stub_lm import StubLM, pua_int2word

G, META = load_golden()


def test_greedy_outputs_rules():
    L = 6
    tokens = np.array([[5, 6, 2, 7, 2, 2],     # EOS at step 2 -> len 2
                       [2, 9, 9, 9, 9, 9],     # EOS at step 0 -> '' and 0.0
                       [4, 4, 4, 4, 4, 4]])    # never finishes -> len L
    out_len = np.array([2, 0, 6], np.int32)
    fin = np.array([True, True, False])
    accum = np.array([-3.0, -0.5, -12.0], np.float32)
    toks, score = greedy_outputs(tokens, out_len, fin, accum)
    assert toks == [[5, 6], [], [4] * 6]
    assert score[0] == -3.0 / 3 and score[1] == 0.0 and score[2] == -12.0 / 6
    assert greedy_steps(out_len, fin, L) == L
    assert greedy_steps(np.array([2, 0]), np.array([True, True]), L) == 3


def test_greedy_steps_match_golden():
    for name in ("plain", "peaked"):
        g = META[name]["greedy"]
        lens = np.array(g["text_len"])
        fin = lens < 40
        assert greedy_steps(lens, fin, 40) == g["steps"]


def test_records_order_and_first_max():
    B, L, k = 2, 4, 3
    rt = np.full((B, L, k, L), -1, np.int32)
    rs = np.zeros((B, L, k), np.float32)
    rv = np.zeros((B, L, k), np.uint8)
    # utterance 0: step 1 rank 2 (score -1.0), step 0 rank 0 (score -1.0): equal scores, the
    # earlier step must win (model.py:765 max keeps the first)
    rv[0, 1, 2] = 1; rs[0, 1, 2] = -1.0; rt[0, 1, 2, :1] = [7]
    rv[0, 0, 0] = 1; rs[0, 0, 0] = -1.0
    rv[1, 3, 1] = 1; rs[1, 3, 1] = -2.5; rt[1, 3, 1, :3] = [4, 5, 6]
    recs = records_by_utterance(rt, rs, rv)
    assert recs[0] == [([], -1.0), ([7], -1.0)]
    assert recs[1] == [([4, 5, 6], -2.5)]
    best = {b: max(v, key=lambda e: e[1]) for b, v in recs.items()}
    assert best[0] == ([], -1.0)


def test_second_pass_rule():
    i2w = pua_int2word(5004)
    lm = StubLM()
    recs = {0: [([10, 11], -3.0), ([10], -2.0), ([10, 11, 12, 13], -3.5)], 1: [([4], -9.0)]}
    sel = second_pass_select(recs, i2w, lm, 1.5, 1.5)
    comb = [s + 1.5 * lm.score(" ".join(i2w[i] for i in t), bos=True) + 1.5 * len(t) for t, s in recs[0]]
    assert sel[0] == recs[0][int(np.argmax(comb))]
    assert sel[1] == recs[1][0]  # a single finished hypothesis is taken as is


def test_second_pass_arrays_equals_record_lists():
    """second_pass_arrays (bench config 5 and the drop-in Model's beam path) chooses the same record
    per utterance and returns the same (tokens, logp) as second_pass_select over
    records_by_utterance, on random records (padding slots past each record's length hold -1, as
    the device leaves them), with no records, and with an int2word that does not cover the ids (the
    list form then runs)."""
    from casr.results import second_pass_arrays
    i2w = pua_int2word(5004)
    lm = StubLM()
    rs_ = np.random.RandomState(3)
    for B, L, k, p in ((16, 40, 16, 0.08), (8, 12, 4, 0.3), (4, 6, 2, 0.0)):
        rv = (rs_.rand(B, L, k) < p).astype(np.uint8)
        rt = np.full((B, L, k, L), -1, np.int32)
        for b, l, c in zip(*np.nonzero(rv)):
            rt[b, l, c, :l] = rs_.randint(0, 5004, size=l)
        rsc = rs_.randn(B, L, k).astype(np.float32)
        ref = second_pass_select(records_by_utterance(rt, rsc, rv), i2w, lm, 1.5, 1.5)
        assert second_pass_arrays(rt, rsc, rv, i2w, lm, 1.5, 1.5) == ref
        partial = {i: w for i, w in i2w.items() if i % 2}
        if ref:
            with pytest.raises(KeyError):  # the list form's lookup of a missing word, as the reference
                second_pass_arrays(rt, rsc, rv, partial, lm, 1.5, 1.5)


def test_parallel_rescorer_equals_second_pass_arrays():
    """casr.rescore.ParallelRescorer (config 5's host second pass over worker processes) returns the
    second_pass_arrays result exactly -- the same record per utterance, the same (tokens, logp) --
    on random records, with records split over several worker tasks (chunk smaller than the record
    count), and with no records."""
    from casr.results import second_pass_arrays
    from casr.rescore import ParallelRescorer
    i2w = pua_int2word(5004)
    pr = ParallelRescorer(StubLM, i2w, 5004, workers=2, chunk=37)
    try:
        rs_ = np.random.RandomState(5)
        for B, L, k, p in ((24, 40, 16, 0.06), (8, 12, 4, 0.3), (4, 6, 2, 0.0)):
            rv = (rs_.rand(B, L, k) < p).astype(np.uint8)
            rt = np.full((B, L, k, L), -1, np.int32)
            for b, l, c in zip(*np.nonzero(rv)):
                rt[b, l, c, :l] = rs_.randint(0, 5004, size=l)
            rsc = rs_.randn(B, L, k).astype(np.float32)
            assert pr.select(rt, rsc, rv, 1.5, 1.5) == second_pass_arrays(rt, rsc, rv, i2w, StubLM(), 1.5, 1.5)
        # exact ties (identical records: the first one wins), -inf and NaN scores (np.argmax takes the
        # first NaN), an utterance with one record (no LM call)
        B, L, k = 5, 10, 4
        rv = np.zeros((B, L, k), np.uint8)
        rt = np.full((B, L, k, L), -1, np.int32)
        rsc = rs_.randn(B, L, k).astype(np.float32)
        for b in range(4):
            for l, c in ((3, 0), (3, 1), (5, 2), (7, 3)):
                rv[b, l, c] = 1
                rt[b, l, c, :l] = (np.arange(l) * 7 + b) % 5004
        rt[0, 3, 1] = rt[0, 3, 0]
        rsc[0, 3, 1] = rsc[0, 3, 0]          # utterance 0: a tie between its first two records
        rsc[0, 5, 2] = rsc[0, 7, 3] = -50.0
        rsc[1, 5, 2] = -np.inf               # utterance 1: -inf in one record
        rsc[2, 5, 2] = np.nan                # utterance 2: a NaN record
        rv[4, 6, 1] = 1
        rt[4, 6, 1, :6] = 11                 # utterance 4: one record
        got = pr.select(rt, rsc, rv, 1.5, 1.5)
        want = second_pass_arrays(rt, rsc, rv, i2w, StubLM(), 1.5, 1.5)
        assert got.keys() == want.keys()
        for b in want:
            assert got[b][0] == want[b][0], b
            assert got[b][1] == want[b][1] or (np.isnan(got[b][1]) and np.isnan(want[b][1])), b
        assert np.isnan(got[2][1]) and got[0][0] == rt[0, 3, 0, :3].tolist()
    finally:
        pr.close()


def test_wer():
    assert edit_distance("abc", "abc") == 0
    assert edit_distance("", "abc") == 3
    assert edit_distance("kitten", "sitting") == 3
    assert get_wer("ab", "abcd") == 0.5


def test_checkpoint_roundtrip_with_reference_trainvar(tmp_path):
    """A checkpoint in the reference's own format (Model.save, model.py:347-355: state dicts,
    optimizer state, and ``args`` = a pickled util.TrainVar, util.py:2356) loads through the
    weights-only path: tensors bit-exact, the TrainVar fields readable, nothing executed."""
    import sys
    import types

    import numpy as np
    import torch

    from casr.config import CasrConfig
    from casr.weights import load_checkpoint, synthetic_state_dicts

    cfg = CasrConfig()
    enc_sd, dec_sd = synthetic_state_dicts(cfg, peaked=True)
    fake = types.ModuleType("util")  # what the reference pickles: util.TrainVar

    class TrainVar(object):
        def __init__(self, step, loss, best_wer, lr, duration, num_no_imprv):
            self.step, self.loss, self.best_wer = step, loss, best_wer
            self.lr, self.duration, self.num_no_imprv = lr, duration, num_no_imprv

    TrainVar.__module__, TrainVar.__qualname__ = "util", "TrainVar"
    fake.TrainVar = TrainVar
    saved = sys.modules.get("util")
    sys.modules["util"] = fake
    try:
        path = str(tmp_path / "ref.ckpt")
        torch.save({"encoder_state_dict": {k: torch.from_numpy(v) for k, v in enc_sd.items()},
                    "decoder_state_dict": {k: torch.from_numpy(v) for k, v in dec_sd.items()},
                    "optimizer_state_dict": {"state": {}, "param_groups": [{"lr": 1e-3, "params": [0, 1]}]},
                    "args": TrainVar(12000, 0.731, 0.06328, 1e-4, 3.5, 2)}, path)
    finally:
        if saved is None:
            del sys.modules["util"]
        else:
            sys.modules["util"] = saved
    e2, d2, args = load_checkpoint(path)
    for a, b in ((enc_sd, e2), (dec_sd, d2)):
        assert list(a) == list(b)
        for k in a:
            np.testing.assert_array_equal(a[k], b[k])
    assert args.step == 12000 and abs(args.best_wer - 0.06328) < 1e-12 and args.num_no_imprv == 2


def _brute_distance(a, b):
    """Levenshtein distance by plain recursion (tiny strings only): the definition."""
    from functools import lru_cache

    @lru_cache(maxsize=None)
    def d(i, j):
        if i == 0:
            return j
        if j == 0:
            return i
        return min(d(i - 1, j) + 1, d(i, j - 1) + 1, d(i - 1, j - 1) + (a[i - 1] != b[j - 1]))
    return d(len(a), len(b))


def test_wer_tuple_and_distance_definition():
    """get_wer(pred, ref, normalize, return_tuple) of util.py:237-262: the total equals the
    distance by definition; the (insert, delete, replace) split is one minimal edit script."""
    from casr.results import edit_ops
    rs = np.random.RandomState(3)
    for _ in range(200):
        a = "".join(rs.choice(list("abcd"), rs.randint(0, 7)))
        b = "".join(rs.choice(list("abcd"), rs.randint(1, 7)))
        dist = _brute_distance(a, b)
        assert edit_distance(a, b) == dist
        ins, dele, rep = edit_ops(a, b)
        assert ins + dele + rep == dist
        assert len(a) + ins - dele == len(b)  # the script turns pred into ref
        tot = get_wer(a, b, normalize=False, return_tuple=True)
        assert tot == (dist, ins, dele, rep)
        np.testing.assert_allclose(get_wer(a, b, return_tuple=True), [x / len(b) for x in tot])
        assert get_wer(a, b, normalize=False) == dist
    assert edit_ops("abc", "abxc") == (1, 0, 0)
    assert edit_ops("abxc", "abc") == (0, 1, 0)
    assert edit_ops("abc", "abd") == (0, 0, 1)


def test_manifest_and_eval_dataset_host(tmp_path):
    """get_wav_path_text_list_from_manifest (data.py:402-405) keeps the reference's parsing (text
    up to the next comma, trailing newline included, which maps to <unk>); AudioBase manifests feed
    AudioDst's eval / infer modes (data.py:409-466); train mode is out of scope."""
    import pytest
    import data as D
    man = tmp_path / "dev.csv"
    man.write_text("/a/u0.wav,你好\n/a/u1.wav,世界,extra\n")
    paths, texts = D.get_wav_path_text_list_from_manifest(str(man))
    assert paths == ["/a/u0.wav", "/a/u1.wav"]
    assert texts == ["你好\n", "世界"]
    ab = D.AudioBase(manifests={"dev": str(man)}, infer_paths=["/x.wav"])
    dst = D.AudioDst(ab, mode="eval", dev_or_test="dev")
    assert len(dst) == 2 and dst.text_list == texts
    unk = ab.word2int["<unk>"]
    ids = dst.text_ids(0)
    assert ids[-1] == unk and len(ids) == 3
    assert ids[:2] == [ab.word2int.get(ch, unk) for ch in "你好"]
    inf = D.AudioDst(ab, mode="infer", dev_or_test=None)
    assert inf.path_list == ["/x.wav"] and inf.text_list is None
    with pytest.raises(NotImplementedError):
        D.AudioDst(ab, mode="train")
    with pytest.raises(ValueError):
        D.AudioDst(D.AudioBase(), mode="eval", dev_or_test="test")
    loader = D.AudioLoader(dst, batch_size=1)
    assert len(loader) == 2 and loader.loader is loader


# ---------------------------------------------------------------- vocabulary (a13, data.py:373-374)
DICT_PKL = "/root/reference/dict.pkl"
DICT_PKL_SHA256 = "d81577bf8967efbfc587ad84e5653d95e2554ac980b469f1ca7814cce3b1d9d4"
VOCAB_JSON_SHA256 = "513ac53677949db69de2bfb3f28c68d7e65c5fa2a09639e79bfb180372bde1dc"


def test_vocab_json_pinned():
    """The committed vocab.json (what the drop-in ships) is the table parsed from the reference's
    dict.pkl in round 1: pinned by hash, 5004 contiguous ids with the reserved tokens first."""
    import hashlib
    from casr.vocab import VOCAB_JSON, load_vocab
    with open(VOCAB_JSON, "rb") as f:
        assert hashlib.sha256(f.read()).hexdigest() == VOCAB_JSON_SHA256
    w2i, i2w = load_vocab()
    assert len(i2w) == 5004 and sorted(i2w) == list(range(5004))
    assert [i2w[i] for i in range(4)] == ["<pad>", "<s>", "</s>", "<unk>"]
    assert all(w2i[w] == i for i, w in i2w.items())


@pytest.mark.skipif(not os.path.exists(DICT_PKL), reason="reference dict.pkl only in the build container")
def test_vocab_json_equals_reference_dict_pkl():
    """Every entry of vocab.json and of its word2int against the reference's dict.pkl itself,
    read by the opcode-level parser (nothing unpickled), whose bytes are pinned by sha256."""
    import hashlib
    from casr.vocab import load_dict_pkl, load_vocab
    with open(DICT_PKL, "rb") as f:
        assert hashlib.sha256(f.read()).hexdigest() == DICT_PKL_SHA256
    w2i_ref, i2w_ref = load_dict_pkl(DICT_PKL)
    w2i, i2w = load_vocab()
    assert i2w == i2w_ref
    assert w2i == w2i_ref
