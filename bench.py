#!/usr/bin/env python
"""North-star benchmark: utterances/s (+ RTF) of the MI355X casr path on synthetic fbank of
shape (B, T, F) = (256, 800, 80) per GPU, greedy decode (headline) and beam = 8 (the metric's
beam line, B = 256; BASELINE config 3, B = 128, beside it).

One step = features (delta/stack/CMVN, written straight as the encoder's layer-0 split-f16 image:
casr_encode_fbank) -> 4-layer BiLSTM encoder -> attention keys -> 40-step decode loop -> token
ids copied to the host, for one batch per GPU.  Inputs are
resident in HBM before the timed region.  Multi-GPU: one process per GPU (torchrun), rank 0
packs the weights and RCCL-broadcasts the packed blob over xGMI; utterance batches are
independent (no collective in the timed region except the start/stop barriers).
`python bench.py --gpus N` (N > 1, no WORLD_SIZE in the environment) relaunches itself under
torch.distributed.run with N ranks before touching the GPU; under a launcher, n_gpus is the live
world size and a mismatch with --gpus is refused.

Prints ONE JSON line on rank 0 (contract in the task statement).
"""
import argparse
import gc
import json
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "chinese-asr_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "utterances/sec + real-time factor, (B,T,F)=(256,800,80) greedy & beam=8"
PEAK_FP32_TFLOPS = 157.3    # MI355X_MICROARCH.md: FP32 matrix (= vector) peak, dense
PEAK_F16_TFLOPS = 2500.0    # MI355X_MICROARCH.md: BF16/F16 MFMA dense peak
# s16x3 (include/casr.h casr_set_precision): one f32 product = 3 f16 MFMA products, so the
# f32-equivalent ceiling of the split arithmetic is a third of the f16 peak
PEAK_S16X3_TFLOPS = PEAK_F16_TFLOPS / 3.0
PEAK_HBM_GBS = 8000.0       # MI355X_MICROARCH.md: HBM3E 8 TB/s spec
AUDIO_S_PER_UTT = 8.0       # 800 frames x 10 ms


def fbank_batch(first, B, T, F=80):
    return np.stack([np.random.RandomState(1234 + first + b).standard_normal((T, F)).astype(np.float32)
                     for b in range(B)])


def kernel_work(cls, B, Tp, R, V, T, fold=False):
    """Algorithmic work of ONE step's launches of a kernel class: (flops or bytes, bound).
    fold: the folded decode step (CASR_OPT_DEC_FOLD): the LSTMCell GEMM runs at
    decode step 0 only, the projection class is the fused [W_p ; W_ch] GEMM (the next step's gate
    columns at steps 0..38), the attention class also gathers the gates and the token's gate-table
    row and writes h / c (its q product is on-chip)."""
    H, C, HD, E, A, D = 256, 512, 512, 256, 128, 720
    if cls == "input_proj":
        return 2.0 * B * Tp * 8 * H * (D + 3 * C), "mfma"
    if cls == "rec_step":
        return 4 * 2.0 * B * Tp * 2 * 4 * H * H, "mfma"
    if cls == "keys":
        return 2.0 * B * Tp * A * C, "mfma"
    if cls == "dec_lstm":
        return (1 if fold else 40) * 2.0 * R * 4 * HD * (E + C + HD), "mfma"
    if cls == "proj":
        return (40 * 2.0 * R * V + (39 * 2.0 * R * 4 * HD if fold else 0)) * (C + HD), "mfma"
    if cls == "attention":   # keys + values streamed once per utterance per step
        cell = 39 * 4.0 * R * (2 * 4 * HD + HD + 3 * HD) if fold else 0.0
        return 40 * 4.0 * B * Tp * (A + C) + cell, "hbm"
    if cls == "select":      # the greedy select reads ProjA's per-block (max, sum, argmax) partials,
        return 40 * 4.0 * 3 * R * 64, "hbm"  # never the [R, V] logits (fused select: one launch)
    if cls == "features":    # fbank read + the layer-0 s16 row image written (Kp = 768: 4 B per column)
        return 4.0 * B * (T * 80 + Tp * 768), "hbm"
    return 0.0, "hbm"


# what one profiled "launch" of a class is (the unit achieved/avg_launch_us refer to; the rocprof
# kernel-trace average of the same kernel must agree: profiles/r01/)
LAUNCH_UNIT = {
    "rec_step": "rec_layer_kernel: one encoder layer, all Tp steps, both directions, B rows "
                "(per-step launches rec_step_kernel when the persistent grid does not fit)",
    "input_proj": "gemm16_bias_kernel (s16x3, 256x256 tiles) or gemm_nt_kernel<StoreBiasEpi> (f32) plus the "
                  "s16 split of the layer input: one layer's input projection, B*Tp rows",
    "proj": "dgemm_kernel<*,ProjA>: one decode step's vocabulary projection",
    "dec_lstm": "dgemm_kernel<*,DecLstmA>: one decode step's LSTMCell",
    "attention": "attention_kernel: one decode step",
}


def kernel_bytes(cls, B, Tp, R, V, fold=False, s16=True):
    """Algorithmic HBM bytes of ONE launch of a kernel class (compulsory reads + writes), to set
    beside the PMC-measured traffic; None where not tabulated.  Weights are the s16 images (4 B
    per element, like f32).  fold: as kernel_work."""
    H, C, D, A, E, HD = 256, 512, 720, 128, 256, 512
    VP = (V + 63) // 64 * 64
    if fold and cls == "attention":  # + gates and gate-table rows gathered, c read, h / c / h16 written
        return 4.0 * (B * Tp * (A + C) + R * (2 * 4 * HD + HD + 3 * HD))
    if fold and cls == "proj":       # fused image (vocabulary + gate tiles), [ctx | h] rows, gates written
        vt = (V + 15) // 16
        return 4.0 * ((vt * 16 + 4 * HD) * (C + HD) + R * (C + HD) + R * 4 * HD + 3 * R * 64 +
                      (R * V + R * vt if R > B else 0))
    if cls == "input_proj":  # average layer: X read, W_ih read, Gin written
        k = (D + 3 * C) / 4.0
        return 4.0 * (B * Tp * k + 8 * H * k + B * Tp * 8 * H)
    if cls == "rec_step":    # average layer: Gin read, layer output written, the residual input read
        # (layers 1-3), and the next layer's s16 row image written by the cells (the last layer's
        # feeds the keys GEMM; s16x3 only); the h exchange is on-chip traffic
        return 4.0 * B * Tp * (8 * H + C + 0.75 * C + (C if s16 else 0))
    if cls == "attention":
        return 4.0 * B * Tp * (A + C)
    if cls == "dec_lstm":    # W image, the gathered A rows, new h / c / h16 and the query partials
        return 4.0 * (4 * HD * (E + C + HD) + R * (E + C + HD) + 3 * R * HD + (HD // 16) * R * A)
    if cls == "proj":        # W image, [ctx | h] rows, per-block (max, sum, argmax) partials; beam: + logits
        return 4.0 * (VP * (C + HD) + R * (C + HD) + 3 * R * 64 + (R * V + R * (VP // 16) if R > B else 0))
    return None


class _StubLM:
    """Deterministic stand-in for kenlm.LanguageModel.score (main.py:82, model.py:755): KenLM and
    an LM file are absent offline.  Tokens arrive as private-use characters (id -> U+E000 + id).
    Every call does its own work (no per-word cache), so the host part of config 5 keeps the
    per-hypothesis cost pattern of a real LM call (tests/golden/stub_lm.py, the same function)."""

    def score(self, s, bos=True):
        ids = [ord(w) - 0xE000 for w in s.split(" ") if w]
        return -0.37 * len(ids) - 0.011 * sum(i % 97 for i in ids) - (0.5 if bos else 0.0)


# CPU port vs the reference itself on the same 8 container cores (tools/calibrate_cpu.py, committed
# result profiles/r03/cpu_calibration.json): port utt/s / reference utt/s
CPU_CALIBRATION = os.path.join(REPO, "profiles", "r03", "cpu_calibration.json")


def cpu_baseline(n_utt, T, beam_k=0):
    """The torch-CPU port of the reference path (oracle/torch_port.py: stock torch CPU operators,
    nn.LSTM over packed sequences like the reference's RNN_RES; tokens equal to the reference
    goldens, tests/test_torch_port.py) timed on this host's cores on a bounded sample of the same
    workload: greedy (beam_k = 0) or beam beam_k.  Its speed relative to the reference itself on
    the same cores was measured in the build container (profiles/r03/cpu_calibration.json)."""
    sys.path.insert(0, REPO)
    from oracle import torch_port as TP
    from casr.config import CasrConfig
    from casr.weights import synthetic_state_dicts
    enc_sd, dec_sd = synthetic_state_dicts(CasrConfig(), peaked=True, eos_bias=0.0)
    fb = fbank_batch(0, n_utt, T)
    port = TP.TorchPort(enc_sd, dec_sd)
    cores = torch.get_num_threads()
    t0 = time.perf_counter()
    feats = [TP.features_from_fbank(fb[b]) for b in range(n_utt)]
    if beam_k:
        port.beam(feats, beam_k)
    else:
        port.greedy(feats)
    dt = time.perf_counter() - t0
    mode = f"beam {beam_k}" if beam_k else "greedy"
    rec = {"value": n_utt / dt, "unit": "utt/s", "cores": int(cores), "kind": "port",
           "sample": f"{mode}, {n_utt} utterances x T={T} in one batch (all 40 steps), torch-CPU port "
                     f"(oracle/torch_port.py) on {cores} threads, {dt:.2f} s"}
    try:  # the port's speed relative to the reference's own CPU path, measured in the container
        cal = json.load(open(CPU_CALIBRATION))
        key = "beam8" if beam_k else "greedy"
        rec["ref_ratio"] = cal[key]["port_over_reference"]
        rec["ref_ratio_note"] = cal[key]["note"]
        rec["reference_equiv_value"] = rec["value"] / rec["ref_ratio"]
    except Exception:
        pass
    return rec


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def relaunch(n):
    """Run this script under torch.distributed.run with n ranks (one per GPU) and return its exit
    status.  Called before anything touches the GPU; device_count() does not initialise it."""
    import torch
    have = torch.cuda.device_count()
    if have < n:
        print(f"bench.py: --gpus {n} but only {have} GPU(s) visible", file=sys.stderr)
        return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--frames", type=int, default=800)
    ap.add_argument("--beam", type=int, default=8)
    ap.add_argument("--beam-batch", type=int, default=256,
                    help="per-GPU batch of the metric's beam line (BASELINE.json: B = 256, beam 8)")
    ap.add_argument("--config3-batch", type=int, default=128, help="BASELINE config 3: beam 8 at B = 128")
    ap.add_argument("--beam-steps", type=int, default=10)
    ap.add_argument("--no-beam", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-configs", action="store_true",
                    help="skip the BASELINE config 1 (one WAV via main.parse), config 2 (B=32 greedy) and "
                         "config 5 (beam 16 + LM) side lines")
    ap.add_argument("--sharded-batch", type=int, default=1024,
                    help="global batch of the BASELINE config 4 / 5 lines (partitioned over the ranks)")
    ap.add_argument("--rescore-workers", type=int, default=12,
                    help="host worker processes per rank for config 5's second-pass LM calls (0: in-process)")
    ap.add_argument("--cpu-sample", type=int, default=512)
    ap.add_argument("--cpu-beam-sample", type=int, default=64)
    ap.add_argument("--precision", default="s16x3", choices=["s16x3", "f32"],
                    help="MFMA arithmetic of the timed path (casr_set_precision)")
    ap.add_argument("--no-f32-compare", action="store_true",
                    help="skip the side measurement of the exact-f32 MFMA path")
    ap.add_argument("--streams", type=int, default=2,
                    help="greedy headline: batches in flight on the GPU (handles / HIP streams, casr.pipeline)")
    ap.add_argument("--beam-streams", type=int, default=2, help="batches in flight for the metric's beam line")
    ap.add_argument("--config2-streams", type=int, default=4,
                    help="BASELINE config 2's pipelined side measurement (its line itself is one batch in flight)")
    ap.add_argument("--no-s16x1", action="store_true",
                    help="skip config 2's opt-in s16x1 perf-arithmetic side measurement (libcasr_hip_s16x1.so)")
    ap.add_argument("--graphs", type=int, default=0,
                    help="1: hipGraph replay of the decode loop (casr_set_graphs); default 0: eager launches")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(relaunch(args.gpus))
    # config 5's host second pass on worker processes (casr.rescore): started here, before this
    # process initialises the GPU (a worker is a fresh interpreter; none of them touches the GPU)
    rescorer = None
    if not args.no_configs and args.sharded_batch > 0 and args.rescore_workers > 0:
        from casr.rescore import ParallelRescorer
        rescorer = ParallelRescorer(_StubLM, {i: chr(0xE000 + i) for i in range(5004)}, 5004,
                                    workers=args.rescore_workers)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but the launcher started {world} rank(s)", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)

    from casr.config import CasrConfig
    from casr.engine import Engine
    from casr.lib import pack_weights, packed_floats, load as load_lib
    from casr.weights import synthetic_state_dicts

    cfg = CasrConfig()
    load_lib()
    # ---- weights: pack on rank 0, RCCL broadcast of the packed blob
    t_w = time.perf_counter()
    packed = None
    if rank == 0:
        packed = torch.from_numpy(pack_weights(cfg, *synthetic_state_dicts(cfg, peaked=True, eos_bias=0.0))).to(dev)
    if dist is not None:
        from casr.distributed import broadcast_packed
        packed = broadcast_packed(packed, dev, expect_floats=packed_floats(cfg))
    torch.cuda.synchronize()
    weight_s = time.perf_counter() - t_w
    # batches in flight on this GPU (casr.pipeline.StreamPipeline): handle i mod n on stream i mod n;
    # handle 0 is the serial loop's (n = 1) and runs every instrumented single step
    from casr.pipeline import StreamPipeline
    pipe = StreamPipeline(cfg, packed, n=max(1, args.streams, args.beam_streams, args.config2_streams), device=dev)
    pipe.set_precision(args.precision)
    pipe.set_graphs(2 | (1 if args.graphs else 0))
    eng = pipe.engines[0]
    precision = eng.precision()  # effective (f32 if the blob's s16 images are unusable)

    B, T = args.batch, args.frames
    fb = torch.from_numpy(fbank_batch(rank * B, B, T)).to(dev)
    frames = torch.full((B,), T, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()

    # Each step ends with its token ids in host memory: copied into a ring of pinned buffers on the
    # step's stream, without a per-step host sync, so the host's launch work of step i+1 is not a
    # gap on the GPU between steps (the timed region's closing sync covers every copy).  The ring
    # has two slots per handle, so a slot is only ever written from one stream.
    pin = {}
    NPIN = 2 * pipe.n

    def to_host(t, tag):
        bufs = pin.get((tag, t.shape, t.dtype))
        if bufs is None:
            bufs = pin[(tag, t.shape, t.dtype)] = [[torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
                                                    for _ in range(NPIN)], 0]
        h = bufs[0][bufs[1] % NPIN]
        bufs[1] += 1
        h.copy_(t, non_blocking=True)
        return h

    def step_greedy(e=None):
        e = e or eng
        e.encode_fbank(fb, frames)  # features + encoder (casr_encode_fbank)
        out = e.greedy()
        return to_host(out["tokens"], "greedy")

    def barrier():
        if dist is not None:
            dist.barrier()

    flags = {}  # device guard bits read after every timed region (read and clear: all its steps)

    step_ms = {}  # per-step device span (HIP events on the step's stream around the step)

    def timed(fn, steps, tag, e=None, n=1):
        """Time exactly `steps` steps fn(engine), bracketed by barrier + synchronize (every
        stream); with n > 1 consecutive steps go to the pipeline's first n handles in turn, so up
        to n batches are in flight.  Returns the max over ranks of the wall time."""
        spans = []

        def one(h):
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            a.record()
            fn(h)
            b.record()
            spans.append((a, b))
        pipe.reset()
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            pipe.submit(one, n)
        torch.cuda.synchronize()
        barrier()
        dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
        if dist is not None:
            dist.all_reduce(dt, op=dist.ReduceOp.MAX)
        flags[tag] = e.device_flags() if e is not None else pipe.device_flags()
        step_ms[tag] = [a.elapsed_time(b) for a, b in spans]
        return float(dt.item())

    def step_stats(tag):
        v = sorted(step_ms.get(tag, []))
        if not v:
            return None
        return {"median": v[len(v) // 2] if len(v) % 2 else 0.5 * (v[len(v) // 2 - 1] + v[len(v) // 2]),
                "min": v[0], "max": v[-1], "n": len(v)}

    CLASSES = ["features", "input_proj", "rec_step", "keys", "dec_lstm", "attention", "proj", "select"]
    for _ in range(args.warmup):
        step_greedy()
    flags["warmup"] = eng.device_flags()
    # one instrumented step: per-class launch times -> dominant kernel
    eng.profile(CLASSES)
    step_greedy()
    breakdown = eng.profile_read()
    dominant = max(breakdown, key=lambda c: breakdown[c][1])
    # Timed regions of the same steps.  (1) Serial, one batch in flight, with the dominant class's
    # event pair around each of its launches, so `roofline` is the kernel's own launch duration (as
    # rocprof sees it in a serial run); the event records cost the step a few microseconds per launch
    # (an event timestamp waits for the previous kernel), so this pass times nothing else.  (2) The
    # same uninstrumented: `greedy_serial`, the latency.  (3) args.streams batches in flight (casr.pipeline),
    # uninstrumented: the line's `value`, the whole-job throughput.  (4) The same with the dominant
    # class's events: a launch there shares the chip with the other batch's kernels, so its span is
    # longer (roofline.pipelined_avg_launch_us) while the chip does more work per second.
    pipe.profile([dominant])
    dt_serial_prof = timed(step_greedy, args.steps, "greedy_serial_profiled", n=1)
    dom_launches, dom_ms = pipe.profile_read()[dominant]
    pipe.profile([])
    dt_serial = timed(step_greedy, args.steps, "greedy_serial", n=1)
    pl_dom = None
    if args.streams > 1:
        for _ in range(args.streams):  # every handle of the timed region warm
            pipe.submit(step_greedy, args.streams)
        flags["warmup_pipeline"] = pipe.device_flags()
        dt = timed(step_greedy, args.steps, "greedy", n=args.streams)
        pipe.profile([dominant])
        timed(step_greedy, args.steps, "greedy_pipelined_profiled", n=args.streams)
        pl_dom = pipe.profile_read()[dominant]
        pipe.profile([])
    else:
        dt = dt_serial

    Tp = T // 3
    value = B * world * args.steps / dt
    ms_step = 1000.0 * dt / args.steps
    def load_pmc(name):
        try:
            return json.load(open(os.path.join(REPO, "profiles", name)))
        except Exception:
            return {}
    # committed PMC passes (tools/probes/profile_r03.sh): greedy step, and beam 8 at B = 256
    pmc_greedy, pmc_beam = load_pmc("pmc_traffic.json"), load_pmc("pmc_traffic_beam.json")

    def roof(cls, launches, ms, steps, Bc, Rc, pmc=pmc_greedy, fold=False):
        """Achieved rate of one kernel class: algorithmic work of `steps` steps over its launches'
        summed duration, against the peak of its bound; PMC columns from the committed passes."""
        work, bound = kernel_work(cls, Bc, Tp, Rc, cfg.vocab, T, fold)
        if not work or not launches or ms <= 0:
            return None
        per_launch = work * steps / launches
        avg_s = ms / 1000.0 / launches
        if bound == "mfma":
            peak = PEAK_S16X3_TFLOPS if precision == "s16x3" else PEAK_FP32_TFLOPS
            ach, unit = per_launch / avg_s / 1e12, "TFLOP/s"
        else:
            ach, peak, unit = per_launch / avg_s / 1e9, PEAK_HBM_GBS, "GB/s"
        out = {"bound": bound, "achieved": ach, "peak": peak, "unit": unit, "frac": ach / peak,
               "launches": launches, "avg_launch_us": 1e6 * avg_s}
        rec_p = pmc.get(cls) or {}
        if rec_p.get("hbm_bytes"):
            out["traffic"] = float(rec_p["hbm_bytes"])
            alg = kernel_bytes(cls, Bc, Tp, Rc, cfg.vocab, fold, precision == "s16x3")
            if alg:
                out["traffic_over_algorithmic"] = out["traffic"] / alg
        if rec_p.get("mfma_busy") is not None:
            out["mfma_busy"] = rec_p["mfma_busy"]
        return out

    # the folded decode step ran when the instrumented step launched the LSTMCell GEMM once
    def folded(bd):
        return bd.get("dec_lstm", (0, 0.0))[0] == 1
    fold = folded(breakdown)
    dom = roof(dominant, dom_launches, dom_ms, args.steps, B, B, fold=fold)
    pl_roof = roof(dominant, pl_dom[0], pl_dom[1], args.steps, B, B, fold=fold) if pl_dom else None
    # every class of the instrumented step (one step: launches and ms of that step)
    kernels = {c: roof(c, n, ms, 1, B, B, fold=fold) for c, (n, ms) in breakdown.items()}
    achieved, peak, unit, bound = dom["achieved"], dom["peak"], dom["unit"], dom["bound"]
    avg_launch_s = dom["avg_launch_us"] / 1e6
    traffic = dom.get("traffic")

    def beam_line(Bb, k, steps, tag, n=1):
        fbb = torch.from_numpy(fbank_batch(rank * Bb, Bb, T)).to(dev)
        frb = torch.full((Bb,), T, dtype=torch.int32, device=dev)
        torch.cuda.synchronize()

        def step_beam(e=None):
            e = e or eng
            e.encode_fbank(fbb, frb)
            r = e.beam(k)
            return to_host(r["tokens"], tag)

        pipe.reset()
        for _ in range(n):
            pipe.submit(step_beam, n)
        flags[tag + "_warmup"] = pipe.device_flags()
        dtb = timed(step_beam, steps, tag, n=n)
        # one instrumented beam step after the timed region: per-class milliseconds
        eng.profile(CLASSES)
        step_beam()
        bd = eng.profile_read()
        eng.profile([])
        return {"k": k, "batch_per_gpu": Bb, "value": Bb * world * steps / dtb, "steps": steps,
                "batches_in_flight": n,
                "device_ms_per_step": step_stats(tag),
                "unit": "utt/s", "ms_per_step": 1000.0 * dtb / steps,
                "rtf": dtb / steps / (Bb * world * AUDIO_S_PER_UTT),
                "kernel_breakdown_ms": {c: round(v[1], 3) for c, v in bd.items()},
                "decode_step": "folded (2 launches + select)" if folded(bd) else "3 launches + select",
                "kernels": {c: roof(c, n, ms, 1, Bb, Bb * k, pmc_beam if Bb == 256 and k == 8 else {}, folded(bd))
                            for c, (n, ms) in bd.items()}}

    beam = config3 = None
    if not args.no_beam:
        # the metric's beam line: beam 8 at B = 256 per GPU (R = 2048 decode rows)
        beam = beam_line(args.beam_batch, args.beam, args.beam_steps, "beam", n=args.beam_streams)
        # BASELINE config 3: beam 8 at B = 128 per GPU (config 4 at --gpus 8: 1024 utterances)
        if not args.no_configs:
            # (one batch in flight: two measured slower at B = 128, profiles/r06/stream_sweep.log)
            config3 = beam_line(args.config3_batch, args.beam, args.beam_steps, "config3", n=1)
            config3["config"] = "BASELINE config 3 (config 4 at --gpus 8): beam 8, B=128/GPU, T=800"

    def s16x1_line(fbs, frs):
        """BASELINE config 2's opt-in perf arithmetic (include/casr.h CASR_PREC_S16X1, SURVEY 7(ii):
        one f16 MFMA per split product, the libcasr_hip_s16x1.so build) on the same B = 32 batch, one
        batch in flight.  Its token ids are compared with this line's s16x3 ones of the same batch
        (which tests/test_gpu_scale.py pins to the oracle on every row): reported, not claimed equal."""
        from casr.engine import Engine
        from casr.results import greedy_outputs
        Bs = fbs.shape[0]

        def run(e):
            e.encode_fbank(fbs, frs)
            return e.greedy()

        def seqs(o):
            o = {k: v.cpu().numpy() for k, v in o.items() if torch.is_tensor(v)}
            return greedy_outputs(o["tokens"], o["out_len"], o["finished"].astype(bool), o["accum"])[0]

        ref = seqs(run(eng))
        e1 = Engine(cfg, packed=packed, device=dev, arithmetic="s16x1")
        try:
            e1.set_graphs(2 | (1 if args.graphs else 0))
            assert e1.precision() == "s16x1", e1.precision()
            run(e1)
            e1.device_flags()
            barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                to_host(run(e1)["tokens"], "s16x1")
            torch.cuda.synchronize()
            barrier()
            dt1 = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
            if dist is not None:
                dist.all_reduce(dt1, op=dist.ReduceOp.MAX)
            flags["config2_s16x1"] = e1.device_flags()
            e1.profile(CLASSES)
            got = seqs(run(e1))
            bd1 = e1.profile_read()
            e1.profile([])
        finally:
            e1.close()
        same = sum(a == b for a, b in zip(ref, got))
        pos = sum(max(len(a), len(b)) for a, b in zip(ref, got))
        hit = sum(sum(x == y for x, y in zip(a, b)) for a, b in zip(ref, got))
        dt1 = float(dt1.item())
        return {"arithmetic": "s16x1 (hi.hi f16 MFMA only, f32 accumulate; opt-in, never the headline)",
                "value": Bs * world * args.steps / dt1, "unit": "utt/s", "ms_per_step": 1000.0 * dt1 / args.steps,
                "kernel_breakdown_ms": {c: round(v[1], 3) for c, v in bd1.items()},
                "token_agreement": {"against": "s16x3 token ids of the same batch (= the oracle's, "
                                               "tests/test_gpu_scale.py test_config2_greedy_b32_matches_oracle)",
                                    "utterances_identical": same, "utterances": len(ref),
                                    "token_positions_equal": hit, "token_positions": pos,
                                    "rate": hit / max(pos, 1)}}

    # BASELINE config 2: a B = 32 greedy batch (same weights, same step)
    small = None
    if not args.no_configs:
        Bs = 32
        fbs = torch.from_numpy(fbank_batch(rank * Bs, Bs, T)).to(dev)
        frs = torch.full((Bs,), T, dtype=torch.int32, device=dev)
        torch.cuda.synchronize()

        def step_small(e=None):
            e = e or eng
            e.encode_fbank(fbs, frs)
            return to_host(e.greedy()["tokens"], "small")

        step_small()
        dts = timed(step_small, args.steps, "config2")  # one batch in flight: the latency
        eng.profile(CLASSES)  # one instrumented step: where a B = 32 batch spends its time
        step_small()
        bds = eng.profile_read()
        eng.profile([])
        small = {"config": "BASELINE config 2: greedy, B=32/GPU, T=800", "batch_per_gpu": Bs,
                 "device_ms_per_step": step_stats("config2"),
                 "kernel_breakdown_ms": {c: round(v[1], 3) for c, v in bds.items()},
                 "value": Bs * world * args.steps / dts, "unit": "utt/s", "ms_per_step": 1000.0 * dts / args.steps,
                 "batches_in_flight": 1}
        nc2 = args.config2_streams
        if nc2 > 1:  # the same B = 32 batches with nc2 in flight (a B = 32 batch fills a quarter of the CUs)
            pipe.reset()
            for _ in range(nc2):
                pipe.submit(step_small, nc2)
            dtp = timed(step_small, max(args.steps, 2 * nc2), "config2_pipelined", n=nc2)
            nst = max(args.steps, 2 * nc2)
            small["pipelined"] = {"batches_in_flight": nc2, "value": Bs * world * nst / dtp, "unit": "utt/s",
                                  "ms_per_step": 1000.0 * dtp / nst,
                                  "device_ms_per_step": step_stats("config2_pipelined"),
                                  "note": "throughput with nc2 B = 32 batches in flight on nc2 handles / streams; "
                                          "ms_per_step is wall time per batch, device_ms_per_step each batch's own "
                                          "span (its latency under the overlap)".replace("nc2", str(nc2))}
        if precision == "s16x3" and not args.no_s16x1:
            small["s16x1_perf_mode"] = s16x1_line(fbs, frs)

    # BASELINE config 1: one 8 s WAV, greedy, through the drop-in main.parse (main.py:27-65):
    # 16 kHz samples on the host -> log-mel, delta / stack / CMVN -> encoder -> greedy -> text.
    # A latency: one utterance per call, the host-side Python of the reference's entry point
    # included (the reference runs this case on the CPU).
    single = None
    if not args.no_configs and rank == 0:
        import main as casr_main
        import model as casr_model
        from data import AudioBase
        m1 = casr_model.Model()
        m1.load_state_dicts(*synthetic_state_dicts(cfg, peaked=True, eos_bias=0.0))
        ab = AudioBase()
        wav = (0.1 * np.random.RandomState(99).standard_normal(int(AUDIO_S_PER_UTT * 16000) + 512)).astype(np.float32)
        text = casr_main.parse(wav, m1, ab, None, None)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        n1 = max(3, args.steps)
        for _ in range(n1):
            text = casr_main.parse(wav, m1, ab, None, None)
        dt1 = (time.perf_counter() - t1) / n1
        single = {"config": "BASELINE config 1: one 8 s WAV, greedy, via the drop-in main.parse (wav -> text)",
                  "latency_ms": 1000.0 * dt1, "rtf": dt1 / AUDIO_S_PER_UTT, "value": 1.0 / dt1,
                  "unit": "utt/s", "chars": len(text)}
        del m1

    # BASELINE configs 4 and 5 through the product's sharded call (casr.distributed.decode_sharded):
    # a global batch of --sharded-batch (1,024) utterances is partitioned over the world's ranks
    # (128 per GPU at --gpus 8, all 1,024 on one GPU at --gpus 1: fixed total work, "strong"), each
    # rank decodes its shard (BeamShardDecoder: features, encoder, beam; config 5 also the records to
    # the host and the second pass there) and the results are gathered as arrays onto every rank --
    # the gather is inside the timed region.  Config 5 uses the weights with the EOS bias (so
    # hypotheses finish and the second pass has records to rescore) and a deterministic stub LM
    # called once per hypothesis (KenLM and an LM file are absent offline; the reference also
    # scores on the host, model.py:749-763); its host part is reported beside the line.
    sharded = {}
    if not args.no_configs and args.sharded_batch > 0:
        from casr.distributed import BeamShardDecoder, decode_sharded, partition
        G = args.sharded_batch
        lens_g = [T // 3] * G
        my_idx = partition(lens_g, world)[rank]
        fb_sh = torch.from_numpy(np.stack([fbank_batch(int(i), 1, T)[0] for i in my_idx])).to(dev)
        fr_sh = torch.full((len(my_idx),), T, dtype=torch.int32, device=dev)
        gdev = dev if world > 1 else None
        names = [d.replace(" ", "_") for d in [torch.cuda.get_device_name(dev)]]
        dev_names = [None] * world
        if dist is not None:
            dist.all_gather_object(dev_names, (rank, names[0]))
        else:
            dev_names = [(0, names[0])]
        for tag, kk, lm_on in (("config4", args.beam, False), ("config5", 16, True)):
            # each rank's shard in batches of <= 256 with args.beam_streams of them in flight
            if lm_on:
                pipe5 = StreamPipeline(cfg, torch.from_numpy(pack_weights(cfg, *synthetic_state_dicts(cfg, peaked=True))).to(dev),
                                       n=max(1, args.beam_streams), device=dev)
                pipe5.set_precision(args.precision)
                e_sh = pipe5
            else:
                e_sh = pipe.limited(max(1, args.beam_streams))
            lm = _StubLM() if lm_on else None
            dec = BeamShardDecoder(e_sh, kk, lm, {i: chr(0xE000 + i) for i in range(cfg.vocab)} if lm_on else None,
                                   1.5 if lm_on else 0.0, 1.5 if lm_on else 0.0,
                                   rescorer=rescorer if lm_on else None)
            batches = lambda n: [(lens_g, lambda idx: (fb_sh, fr_sh))] * n
            for out in decode_sharded(batches(2), dec, device=gdev):
                pass
            flags[tag + "_warmup"] = e_sh.device_flags()
            nb = args.beam_steps
            gc.collect()
            gc.freeze()  # a serving process freezes its start-up heap (tools/probes/config5_probe.py)
            t_host = [0.0]
            fin = dec.finish

            def timed_finish(pend, fin=fin):
                t0 = time.perf_counter()
                r = fin(pend)
                t_host[0] += time.perf_counter() - t0
                return r
            dec.finish = timed_finish
            dts = timed(lambda h: [None for _ in decode_sharded(batches(nb), dec, device=gdev)], 1, tag, e=e_sh)
            gc.unfreeze()
            line = {"config": ("BASELINE config 4: beam 8" if not lm_on else
                               "BASELINE config 5: beam 16 + second-pass LM rescoring (stub LM, host)") +
                              f", {G} utterances sharded over {world} GPU(s), T={T}",
                    "k": kk, "global_batch": G, "batch_per_gpu": len(my_idx), "world_size": world,
                    "device_batch": min(dec.max_batch, len(my_idx)),
                    "devices": [n for _, n in sorted(dev_names)], "batches": nb,
                    "value": G * nb / dts, "unit": "utt/s", "ms_per_batch": 1000.0 * dts / nb,
                    "rtf": dts / nb / (G * AUDIO_S_PER_UTT), "scaling": "strong",
                    "decode_steps": dec.stats.get("steps"),
                    "entry_point": "casr.distributed.decode_sharded (partition -> BeamShardDecoder -> gather_arrays); "
                                   "the gather is inside the timed region",
                    "pipelined": "two global batches in flight: batch i's device work is enqueued before "
                                 "batch i-1's host part and gather",
                    "host_ms_per_batch_rank0": 1000.0 * t_host[0] / nb}
            if lm_on:
                line.update(records_per_batch_rank0=dec.stats.get("records"),
                            weights="synthetic recipe with the EOS bias (hypotheses finish before step 40)",
                            lm="deterministic stub, one call per hypothesis of every utterance with > 1 "
                               "(the reference's call pattern, model.py:755); a KenLM call costs more",
                            rescore_workers=(rescorer.workers if rescorer is not None else 0))
            sharded[tag] = line
            line["batches_in_flight"] = e_sh.n
            if lm_on:
                e_sh.close()

    # side measurement: the same greedy step on the exact-f32 MFMA path (not the headline)
    f32_cmp = None
    if precision == "s16x3" and not args.no_f32_compare:
        eng.set_precision("f32")
        step_greedy()
        dtf = timed(step_greedy, max(2, args.steps // 2), "f32", e=eng)  # one batch in flight
        nf = max(2, args.steps // 2)
        f32_cmp = {"value": B * world * nf / dtf, "unit": "utt/s", "ms_per_step": 1000.0 * dtf / nf}
        eng.set_precision(precision)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.cpu_sample, T)
        if beam is not None and args.cpu_beam_sample > 0:
            beam["cpu_baseline"] = cpu_baseline(args.cpu_beam_sample, T, beam_k=args.beam)
            beam["speedup_vs_cpu"] = beam["value"] / beam["cpu_baseline"]["value"]

    if rank == 0:
        rec = {
            "metric": METRIC, "value": value, "unit": "utt/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms_step, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f32" if precision == "f32" else "f32/s16x3",
            "arithmetic": ("f32 data and f32 accumulators; MFMA products " +
                           ("as s16x3: each f32 operand split into two f16 (hi + 2^-11 lo), 3 f16 MFMAs "
                            "per product (22 operand bits; measured error below the exact-f32 chain's)"
                            if precision == "s16x3" else "on exact-f32 v_mfma_f32_16x16x4_f32")),
            "data": "synthetic fbank RandomState(1234+b) (800x80); deterministic synthetic weights "
                    "(SURVEY 8d recipe, proj x40, no EOS bias: all 40 decode steps run)",
            "config": {"workload": f"greedy decode, B={B}/GPU, T={T}, F=80: features + 4-layer BiLSTM "
                                   f"encoder + 40-step attention decode, ids to host",
                       "global_batch": B * world, "seq_len": T, "parallelism": f"dp{world}"},
            "rtf": dt / args.steps / (B * world * AUDIO_S_PER_UTT),
            "batches_in_flight": args.streams,
            "greedy_serial": {"value": B * world * args.steps / dt_serial, "unit": "utt/s",
                              "ms_per_step": 1000.0 * dt_serial / args.steps,
                              "device_ms_per_step": step_stats("greedy_serial"),
                              "ms_per_step_with_dominant_events": 1000.0 * dt_serial_prof / args.steps,
                              "note": "the same steps with one batch in flight (the round-5 headline's loop); "
                                      "ms_per_step_with_dominant_events: the roofline's pass, an event pair "
                                      "around each launch of the dominant class"},
            "device_ms_per_step": step_stats("greedy"),
            "device_ms_note": "per timed step, HIP events on the compute stream around each step (device "
                              "time incl. any launch gaps; SURVEY 8d: median of the steps)",
            "decode_launch": "hipGraph replay" if args.graphs else "eager launches",
            "decode_step": "folded (2 launches per step: attention with the LSTM cell, fused projection | "
                           "gate GEMM)" if fold else "3 launches per step (LSTMCell, attention, projection)",
            "beam": beam,
            "config3_beam8_b128": config3,
            "roofline": {"kernel": dominant, "bound": bound, "achieved": achieved, "peak": peak,
                         "unit": unit, "frac": achieved / peak, "traffic": traffic,
                         "traffic_unit": "bytes per launch (PMC 2 x FETCH_SIZE + WRITE_SIZE)",
                         "algorithmic_bytes": kernel_bytes(dominant, B, Tp, B, cfg.vocab, fold, precision == "s16x3"),
                         "launches": dom_launches, "avg_launch_us": 1e6 * avg_launch_s,
                         "timed_region": "serial pass (one batch in flight) of the same greedy steps with this "
                                         "class's event pairs; the headline value is the uninstrumented pass with "
                                         "`batches_in_flight` batches in flight",
                         "pipelined_avg_launch_us": pl_roof["avg_launch_us"] if pl_roof else None,
                         "pipelined_frac": pl_roof["frac"] if pl_roof else None,
                         "launch": LAUNCH_UNIT.get(dominant, "one kernel launch"),
                         "peak_basis": ("f16 MFMA dense peak / 3 (s16x3 f32-equivalent)" if bound == "mfma" and
                                        precision == "s16x3" else "spec peak of the bound"),
                         **({"latency_bound": True, "per_step_us": 1e6 * avg_launch_s / Tp,
                             "note": "serial chain of Tp dependent steps per layer; per-step time is "
                                     "hand-off latency + MFMA + cell (DESIGN.md 3.2)"}
                            if dominant == "rec_step" else {}),
                         "kernels": kernels,
                         "kernels_note": "every kernel class of one instrumented greedy step (HIP events): "
                                         "achieved = algorithmic work / launch time; traffic / mfma_busy from "
                                         "the committed PMC passes (profiles/pmc_traffic.json)"},
            "config2_greedy_b32": small,
            "config1_single_wav": single,
            "config4_beam8_sharded": sharded.get("config4"),
            "config5_beam16_lm": sharded.get("config5"),
            "f32_exact_path": f32_cmp,
            "kernel_breakdown_ms": {k: round(v[1], 3) for k, v in breakdown.items()},
            "weights_bcast_s": weight_s,
            "device_flags": flags,
            "device_flags_clean": all(v == 0 for v in flags.values()),
            "cpu_baseline": cpu,
        }
        if cpu:
            rec["speedup_vs_cpu"] = value / cpu["value"]
        print(json.dumps(rec), flush=True)
    pipe.close()  # drain and free the handles now, not from __del__ at interpreter exit
    if rescorer is not None:
        rescorer.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
