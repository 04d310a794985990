#!/usr/bin/env python
"""Container-only calibration of bench.py's CPU baseline (the timed CPU
stand-in must be within +-20% of the reference's own speed on the same cores).

The reference cannot travel to the GPU box, so bench.py times the torch-CPU port
(oracle/torch_port.py).  Here, where /root/reference exists, the reference, the torch port and the
numpy oracle (oracle/casr_oracle.py, the parity checker: for comparison) run on the same 8 cores
on the same workloads, one after the other, and the ratio port / reference goes to
profiles/r03/cpu_calibration.json, which bench.py quotes beside its cpu_baseline (``ref_ratio``,
``reference_equiv_value``).  Run it on an otherwise idle container.

The reference runs through the shims of tests/golden/make_golden.py (stub kenlm / Levenshtein /
soundfile, legacy integer division and stft; nothing written under /root/reference), with the
bench weights (synthetic recipe, proj x40, no EOS bias: all 40 decode steps).
Workloads: greedy B = 256, T = 800 (the headline) and beam 8 at B = 32, T = 800.
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path[:0] = [REPO, os.path.join(REPO, "chinese-asr_amd"), os.path.join(REPO, "tests", "golden")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import make_golden as MG  # noqa: E402  (the reference, imported with the shims)
from oracle import casr_oracle as O  # noqa: E402
from oracle import torch_port as TP  # noqa: E402
from casr.weights import synthetic_state_dicts  # noqa: E402

THREADS = 8
REPEAT = 3


def main():
    torch.set_num_threads(THREADS)
    try:
        from threadpoolctl import threadpool_limits
        threadpool_limits(THREADS)
    except Exception:
        pass
    enc_sd, dec_sd = synthetic_state_dicts(MG.CFG, peaked=True, eos_bias=0.0)
    m = MG.build_ref_model(enc_sd, dec_sd)
    dev = torch.device("cpu")
    out = {"threads": THREADS, "host": os.uname().nodename, "T": 800}
    for key, B, k in (("greedy", 256, 0), ("beam8", 32, 8)):
        fb = [MG.fbank_for(b, 800) for b in range(B)]
        ref_feats = [MG.ref_features(f)[1] for f in fb]
        lens = torch.tensor([f.shape[0] for f in ref_feats])
        port = TP.TorchPort(enc_sd, dec_sd)
        t_ref, t_port, t_np = [], [], []
        for _ in range(REPEAT):
            t0 = time.perf_counter()
            with torch.no_grad():
                if k:
                    m.eval_one_batch_with_beam(dev, k, ref_feats, lens, None, MG.PUA, second_pass=False,
                                               lm_model=None, lm_weight=0.0, length_weight=0.0)
                else:
                    m.eval_one_batch_with_greedy(dev, ref_feats, lens, MG.PUA, None)
            t_ref.append(time.perf_counter() - t0)
            # the torch port, timed as bench.py times it (features from fbank included)
            t0 = time.perf_counter()
            feats = [TP.features_from_fbank(f) for f in fb]
            if k:
                port.beam(feats, k)
            else:
                port.greedy(feats)
            t_port.append(time.perf_counter() - t0)
            # the numpy oracle (round-2 cpu_baseline), for comparison
            t0 = time.perf_counter()
            feats = [O.features_from_fbank(f) for f in fb]
            if k:
                O.beam_decode(feats, [f.shape[0] for f in feats], enc_sd, dec_sd, k)
            else:
                O.greedy_decode(feats, [f.shape[0] for f in feats], enc_sd, dec_sd)
            t_np.append(time.perf_counter() - t0)
        ref_ups, port_ups, np_ups = B / min(t_ref), B / min(t_port), B / min(t_np)
        out[key] = {"batch": B, "k": k or None, "reference_utt_s": ref_ups, "port_utt_s": port_ups,
                    "numpy_oracle_utt_s": np_ups, "port_over_reference": port_ups / ref_ups,
                    "numpy_oracle_over_reference": np_ups / ref_ups,
                    "reference_s": t_ref, "port_s": t_port, "numpy_oracle_s": t_np,
                    "note": f"{key} B={B} T=800 on {THREADS} container threads, best of {REPEAT}: the torch "
                            f"port runs at {port_ups / ref_ups:.2f}x the reference's speed (numpy oracle "
                            f"{np_ups / ref_ups:.2f}x)"}
        print(key, json.dumps(out[key]), flush=True)
    os.makedirs(os.path.join(REPO, "profiles", "r03"), exist_ok=True)
    with open(os.path.join(REPO, "profiles", "r03", "cpu_calibration.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
