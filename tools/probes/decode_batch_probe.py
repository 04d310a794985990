"""Greedy decode time vs batch size on ONE handle (graphs on / off), then two handles alive:
does the decode of a half batch cost what its kernels cost?"""
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


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return 1000.0 * (time.perf_counter() - t0) / n


def main():
    cfg = CasrConfig()
    dev = torch.device("cuda", 0)
    blob = torch.from_numpy(pack_weights(cfg, *synthetic_state_dicts(cfg, peaked=True, eos_bias=0.0))).to(dev)
    T = 800
    fb = torch.from_numpy(np.stack([np.random.RandomState(1234 + b).standard_normal((T, 80)).astype(np.float32)
                                    for b in range(256)])).to(dev)
    fr = torch.full((256,), T, dtype=torch.int32, device=dev)
    e = Engine(cfg, packed=blob, device=dev)
    for B in (256, 128, 64, 32):
        e.encode_fbank(fb[:B].contiguous(), fr[:B].contiguous())
        g_on = timeit(e.greedy)
        e.set_graphs(False)
        g_off = timeit(e.greedy)
        e.set_graphs(True)
        e.profile(["dec_lstm", "attention", "proj", "select"])
        e.greedy()
        bd = {k: round(v[1], 3) for k, v in e.profile_read().items()}
        e.profile([])
        print(f"B={B}: greedy {g_on:.3f} ms (graphs) {g_off:.3f} ms (eager); classes {bd}", flush=True)
    e2 = Engine(cfg, packed=blob, device=dev)
    e.encode_fbank(fb[:128].contiguous(), fr[:128].contiguous())
    e2.encode_fbank(fb[128:].contiguous(), fr[:128].contiguous())
    print(f"two handles, B=128 each: e {timeit(e.greedy):.3f} e2 {timeit(e2.greedy):.3f} ms", flush=True)


if __name__ == "__main__":
    main()
