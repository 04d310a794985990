"""Several batches in flight on one GPU (casr.pipeline.StreamPipeline, what bench.py's headline and
beam lines run): each batch's results equal a decode of that batch on one handle alone, bit for
bit, however the batches interleave on the device; and the sharded decoder (configs 4 / 5) over a
pipeline equals it over one Engine.  Ragged lengths, EOS-bias weights (rows finish early)."""
import numpy as np
import pytest
import torch

from golden_util import fbank_for
from casr.config import CasrConfig
from casr.lib import pack_weights
from casr.weights import synthetic_state_dicts

pytestmark = pytest.mark.gpu

CFG = CasrConfig()


def _batch(B, T, seed):
    rs = np.random.RandomState(seed)
    frames = rs.randint(60, T + 1, size=B).astype(np.int32)
    x = np.zeros((B, T, 80), np.float32)
    for b in range(B):
        x[b, :frames[b]] = fbank_for(seed * 1000 + b, int(frames[b]))
    return torch.from_numpy(x).cuda(), torch.from_numpy(frames).cuda()


@pytest.mark.parametrize("n", [2, 3])
def test_batches_in_flight_equal_serial(n):
    from casr.engine import Engine
    from casr.pipeline import StreamPipeline
    blob = torch.from_numpy(pack_weights(CFG, *synthetic_state_dicts(CFG, peaked=True))).cuda()
    batches = [_batch(B, 300, s) for s, B in enumerate((64, 96, 64, 40, 64, 96))]
    torch.cuda.synchronize()

    def greedy(e, fb, fr):
        e.encode_fbank(fb, fr)
        return {k: v for k, v in e.greedy().items() if torch.is_tensor(v)}

    def beam(e, fb, fr):
        e.encode_fbank(fb, fr)
        return e.beam(4, 0.0, 1.5)

    serial = Engine(CFG, packed=blob)
    try:
        want = [(greedy(serial, *b), beam(serial, *b)) for b in batches]
        want = [tuple({k: v.cpu() for k, v in d.items()} for d in w) for w in want]
        assert serial.device_flags() == 0
    finally:
        serial.close()
    pipe = StreamPipeline(CFG, blob, n=n)
    try:
        got = [(pipe.submit(lambda e, b=b: greedy(e, *b)), pipe.submit(lambda e, b=b: beam(e, *b))) for b in batches]
        torch.cuda.synchronize()
        assert pipe.device_flags() == 0
        got = [tuple({k: v.cpu() for k, v in d.items()} for d in g) for g in got]
    finally:
        pipe.close()
    for w, g in zip(want, got):
        for dw, dg in zip(w, g):
            assert dw.keys() == dg.keys()
            for k in dw:
                assert torch.equal(dw[k], dg[k]), k


def test_shard_decoder_over_pipeline_equals_engine():
    """BeamShardDecoder: a 300-utterance shard decoded as batches of <= 256 (256 + 44) with the
    batches on a two-handle pipeline, against the same decoder on one Engine; beam 8 + the second
    pass with the stub LM (config 5's chain): packed results identical."""
    from stub_lm import StubLM, pua_int2word
    from casr.distributed import BeamShardDecoder
    from casr.engine import Engine
    from casr.pipeline import StreamPipeline
    blob = torch.from_numpy(pack_weights(CFG, *synthetic_state_dicts(CFG, peaked=True))).cuda()
    fb, fr = _batch(300, 240, 7)
    torch.cuda.synchronize()
    i2w = pua_int2word(CFG.vocab)
    e = Engine(CFG, packed=blob)
    try:
        d1 = BeamShardDecoder(e, 8, StubLM(), i2w, 1.5, 1.5)
        want = d1.finish(d1.enqueue(fb, fr))
        assert d1.stats["batch_steps"] and len(d1.stats["batch_steps"]) == 2
        assert e.device_flags() == 0
    finally:
        e.close()
    pipe = StreamPipeline(CFG, blob, n=2)
    try:
        d2 = BeamShardDecoder(pipe, 8, StubLM(), i2w, 1.5, 1.5)
        got = d2.finish(d2.enqueue(fb, fr))
        assert pipe.device_flags() == 0
    finally:
        pipe.close()
    np.testing.assert_array_equal(got, want)


def test_full_chip_encoders_on_four_streams():
    """Four B = 256 encodes in flight on four handles / streams: every persistent layer wants all 256
    CUs, and its workgroups wait on each other, so two of them placed side by side could each hold
    part of the chip and wait forever (until the 2 s hand-off bound).  The library orders the
    persistent launches of a process per device (CASR_OPT_REC_COOP = 2, recurrence.hip): no guard
    bit, and every handle's encoder results equal the serial ones, over two rounds."""
    from casr.pipeline import StreamPipeline
    blob = torch.from_numpy(pack_weights(CFG, *synthetic_state_dicts(CFG, peaked=True))).cuda()
    fb, fr = _batch(256, 800, 11)
    torch.cuda.synchronize()
    pipe = StreamPipeline(CFG, blob, n=4)
    try:
        assert all(e.get_option("REC_COOP") == 2 for e in pipe.engines)
        e0 = pipe.engines[0]
        e0.encode_fbank(fb, fr)
        want = [t.cpu() for t in e0.encoder_results()]
        for _ in range(2):
            outs = [pipe.submit(lambda e: (e.encode_fbank(fb, fr), e.encoder_results())[1]) for _ in range(4)]
            torch.cuda.synchronize()
            assert pipe.device_flags() == 0
            for got in outs:
                for a, b in zip(want, got):
                    assert torch.equal(a, b.cpu())
    finally:
        pipe.close()
