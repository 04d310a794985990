"""Feasibility probe: does decoding the batch as two concurrent half-batch chains (two handles on
two streams, so one half's HBM-bound attention can run beside the other half's L2-bound decode
GEMMs) beat one full-batch decode?  Greedy, B = 256, T = 800, bench weights; chain B optionally
starts D clock cycles late (torch.cuda._sleep) so the halves run out of phase.
Prints ms per full-batch decode for: one B = 256 handle; two B = 128 handles on one stream;
two B = 128 handles on two streams with delays D."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "chinese-asr_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from casr.config import CasrConfig  # noqa: E402
from casr.engine import Engine  # noqa: E402
from casr.lib import pack_weights  # noqa: E402
from casr.weights import synthetic_state_dicts  # noqa: E402


def main():
    cfg = CasrConfig()
    dev = torch.device("cuda", 0)
    blob = torch.from_numpy(pack_weights(cfg, *synthetic_state_dicts(cfg, peaked=True, eos_bias=0.0))).to(dev)
    B, T = 256, 800
    fb = torch.from_numpy(np.stack([np.random.RandomState(1234 + b).standard_normal((T, 80)).astype(np.float32)
                                    for b in range(B)])).to(dev)
    fr = torch.full((B,), T, dtype=torch.int32, device=dev)
    graphs = os.environ.get("GRAPHS", "0") == "1"
    full = Engine(cfg, packed=blob, device=dev)
    halves = [Engine(cfg, packed=blob, device=dev) for _ in range(2)]
    for e in [full] + halves:
        e.set_graphs(graphs)
    print("graphs", graphs, flush=True)
    full.encode_fbank(fb, fr)
    for h, e in enumerate(halves):
        e.encode_fbank(fb[128 * h:128 * (h + 1)].contiguous(), fr[:128].contiguous())
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    N = 20

    def run_full():
        full.greedy()

    def run_seq():
        for e in halves:
            e.greedy()

    def run_par(delay):
        ev = torch.cuda.Event()
        ev.record()
        for i, (e, st) in enumerate(zip(halves, streams)):
            st.wait_event(ev)
            with torch.cuda.stream(st):
                if i == 1 and delay:
                    torch.cuda._sleep(delay)
                e.greedy()
        for st in streams:
            torch.cuda.current_stream().wait_stream(st)

    def timeit(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(N):
            fn()
        torch.cuda.synchronize()
        return 1000.0 * (time.perf_counter() - t0) / N

    res = {}
    for rnd in range(3):
        res.setdefault("full", []).append(timeit(run_full))
        res.setdefault("seq", []).append(timeit(run_seq))
        for d in (0, 20000, 50000, 100000):
            res.setdefault(f"par_d{d}", []).append(timeit(lambda: run_par(d)))
    for k, v in res.items():
        print(f"{k:>12s} ms/decode: " + " ".join(f"{x:.3f}" for x in v), flush=True)
    # the halves' tokens equal the full batch's
    a = full.greedy()["tokens"].cpu()
    b = torch.cat([e.greedy()["tokens"].cpu() for e in halves])
    print("tokens equal:", bool(torch.equal(a, b)))


if __name__ == "__main__":
    main()
