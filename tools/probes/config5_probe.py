"""Where the BASELINE config-5 step (beam 16 + second pass, B = 128) spends its time: device
decode, records copy, host record assembly, LM rescoring.  Diagnostic only."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "chinese-asr_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import _StubLM, fbank_batch  # noqa: E402
from casr.config import CasrConfig  # noqa: E402
from casr.engine import Engine  # noqa: E402
from casr.results import records_by_utterance, second_pass_arrays, second_pass_select  # noqa: E402
from casr.weights import synthetic_state_dicts  # noqa: E402


def main():
    cfg = CasrConfig()
    dev = torch.device("cuda", 0)
    eng = Engine(cfg, *synthetic_state_dicts(cfg, peaked=True), device=dev)
    B, k, T = 128, 16, 800
    fb = torch.from_numpy(fbank_batch(0, B, T)).to(dev)
    fr = torch.full((B,), T, dtype=torch.int32, device=dev)
    i2w = {i: chr(0xE000 + i) for i in range(cfg.vocab)}
    lm = _StubLM()
    for it in range(3):
        t = [time.perf_counter()]
        feat, flen = eng.features(fb, fr)
        eng.encode(feat, flen)
        r = eng.beam(k, 1.5, 1.5)
        torch.cuda.synchronize()
        t.append(time.perf_counter())
        rt, rs, rv = (x.cpu().numpy() for x in eng.beam_records())
        t.append(time.perf_counter())
        recs = records_by_utterance(rt, rs, rv)
        t.append(time.perf_counter())
        second_pass_select(recs, i2w, lm, 1.5, 1.5)
        t.append(time.perf_counter())
        n = sum(len(v) for v in recs.values())
        print(f"iter {it}: device {1e3 * (t[1] - t[0]):.2f} ms, records copy {1e3 * (t[2] - t[1]):.2f} ms, "
              f"assembly {1e3 * (t[3] - t[2]):.2f} ms, rescoring {1e3 * (t[4] - t[3]):.2f} ms; "
              f"{n} records, steps {int(r['steps'].item())}", flush=True)
    # the bench's pipelined loop (bench.py config 5), per batch: enqueue, wait, host times
    pinned = [None, None]

    def enqueue(slot):
        t0 = time.perf_counter()
        eng.encode_fbank(fb, fr)
        r = eng.beam(k, 1.5, 1.5)
        dev_out = (r["tokens"], r["length"], r["steps"]) + tuple(eng.beam_records())
        if pinned[slot] is None:
            pinned[slot] = [torch.empty(x.shape, dtype=x.dtype, pin_memory=True) for x in dev_out]
        for h, x in zip(pinned[slot], dev_out):
            h.copy_(x, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        return slot, ev, time.perf_counter() - t0

    def finish(pend):
        slot, ev, te = pend
        t0 = time.perf_counter()
        ev.synchronize()
        t1 = time.perf_counter()
        toks, blen, steps, rt, rs, rv = (h.numpy().copy() for h in pinned[slot])
        t2 = time.perf_counter()
        second_pass_arrays(rt, rs, rv, i2w, lm, 1.5, 1.5)
        t3 = time.perf_counter()
        print(f"pipe: enqueue {1e3 * te:.2f} ms, wait {1e3 * (t1 - t0):.2f}, copy-out {1e3 * (t2 - t1):.2f}, "
              f"host {1e3 * (t3 - t2):.2f} ms", flush=True)

    if os.environ.get("FREEZE", "1") == "1":
        import gc
        gc.collect()
        gc.freeze()
    t0 = time.perf_counter()
    prev = None
    for i in range(6):
        cur = enqueue(i % 2)
        if prev is not None:
            finish(prev)
        prev = cur
    finish(prev)
    print(f"pipe: {1e3 * (time.perf_counter() - t0) / 6:.2f} ms per batch", flush=True)
    eng.profile(["features", "input_proj", "rec_step", "keys", "dec_lstm", "attention", "proj", "select"])
    feat, flen = eng.features(fb, fr)
    eng.encode(feat, flen)
    eng.beam(k, 1.5, 1.5)
    torch.cuda.synchronize()
    print({c: round(v[1], 3) for c, v in eng.profile_read().items()})


if __name__ == "__main__":
    main()
