"""Phase breakdown of the persistent recurrence (diagnostics; GPU box).

Runs one encode of B utterances x T frames with CASR_REC_TRACE set, then reads the per-wave
timestamps of layer 0 (s_memrealtime, 100 MHz) written by rec_layer_kernel and prints median
phase times per step: sweep (step start -> h granules complete), mfma (-> after the LDS
barrier), cell (-> granule stored), the step period and the hand-off latency (latest producer
store of step s-1 in the row group -> this wave's sweep complete)."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "chinese-asr_amd"))


def main(B=256, T=800, path="/tmp/rec_trace.bin"):
    from casr.config import CasrConfig
    from casr.engine import Engine
    from casr.weights import synthetic_state_dicts
    cfg = CasrConfig()
    eng = Engine(cfg, *synthetic_state_dicts(cfg, peaked=True, eos_bias=0.0))
    fb = torch.from_numpy(np.random.RandomState(0).standard_normal((B, T, 80)).astype(np.float32)).cuda()
    feat, flen = eng.features(fb, torch.full((B,), T, dtype=torch.int32, device="cuda"))
    eng.encode(feat, flen)  # warm
    os.environ["CASR_REC_TRACE"] = path
    eng.encode(feat, flen)
    torch.cuda.synchronize()
    del os.environ["CASR_REC_TRACE"]
    raw = np.fromfile(path, dtype=np.uint32)
    nwg, nw, Tp, ne, npg = (int(x) for x in raw[:5].view(np.int32))
    tr = raw[5:].reshape(nwg, nw, Tp, ne).astype(np.int64)
    t = tr[..., :4] * 10.0 / 1000.0  # us
    t = t - t[..., 0:1, 0:1].min()
    ns = Tp - 1
    sweep = t[:, :, 1:, 1] - t[:, :, 1:, 0]
    mfma = t[:, :, 1:, 2] - t[:, :, 1:, 1]
    cell = t[:, :, 1:, 3] - t[:, :, 1:, 2]
    period = t[:, :, 2:, 0] - t[:, :, 1:-1, 0]
    passes = tr[:, :, 1:, 4]
    # grid order: blockIdx.x = npg unit blocks, then row groups, then directions
    ngrp = nwg // npg  # (row group, direction) groups of npg producer workgroups
    st = t[:, :, :, 3].max(axis=1).reshape(ngrp, npg, Tp)          # WG's last store per step
    done = t[:, :, :, 1].reshape(ngrp, npg, nw, Tp)
    lat = done[:, :, :, 1:] - st.max(axis=1)[:, None, None, :-1]
    # critical-path pieces: per workgroup and step, the last wave's sweep -> the barrier (MFMA of
    # that wave + partial exchange), the spread of the waves' sweep completions, and per group the
    # spread of its producers' stores
    crit = t[:, :, 1:, 2].min(axis=1) - t[:, :, 1:, 1].max(axis=1)
    spread = t[:, :, 1:, 1].max(axis=1) - t[:, :, 1:, 1].min(axis=1)
    gskew = st.max(axis=1) - st.min(axis=1)
    total = t[:, :, -1, 3].max() - t[:, :, 0, 0].min()
    print(f"grid {nwg} WGs x {nw} waves, Tp={Tp}; layer wall {total:.1f} us = {total / Tp:.2f} us/step")
    for name, a in (("sweep", sweep), ("mfma+barrier", mfma), ("cell+store", cell), ("period", period),
                    ("handoff (last producer store -> sweep done)", lat),
                    ("last wave's sweep -> barrier done (per WG)", crit),
                    ("sweep completion spread over a WG's waves", spread),
                    ("store spread over a group's producers", gskew[:, 1:])):
        q = np.percentile(a, [10, 50, 90])
        print(f"  {name:44s} p10 {q[0]:6.2f}  p50 {q[1]:6.2f}  p90 {q[2]:6.2f} us")
    print(f"  sweep passes p50 {np.median(passes):.0f}  p90 {np.percentile(passes, 90):.0f}  max {passes.max()}")
    eng.close()


if __name__ == "__main__":
    main()
