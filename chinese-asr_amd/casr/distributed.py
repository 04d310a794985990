"""Utterance-level data parallelism across the GPUs of one node.

One process per GPU (torchrun).  Rank 0 packs the weights once and broadcasts the packed
blob (RCCL over xGMI with the "nccl" backend; gloo on CPU for tests).  Utterances are
independent, so a batch is partitioned by length (longest-processing-time greedy on T',
the encoder cost driver) and each rank decodes its share with no collective in the decode;
results are gathered to every rank in the original order.  The partition never changes a
result: decode is batch-invariant (tests/test_gpu_parity.py::test_batch_invariance...)."""
import os

import numpy as np
import torch


def env_rank():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def partition(lens, world):
    """Split utterance indices into `world` groups of near-equal total length (LPT greedy).
    Each group keeps the original relative order.  Returns a list of int arrays."""
    lens = np.asarray(lens, np.int64)
    order = np.argsort(-lens, kind="stable")
    load = np.zeros(world, np.int64)
    owner = np.empty(len(lens), np.int64)
    for i in order:
        r = int(np.argmin(load))
        owner[i] = r
        load[r] += lens[i]
    return [np.nonzero(owner == r)[0] for r in range(world)]


def broadcast_packed(packed, device, src=0, group=None, expect_floats=None):
    """Broadcast the packed weight blob from `src`.  `packed` is a tensor on rank src (ignored
    elsewhere).  Returns the blob on `device` on every rank.  With `expect_floats` (this rank's
    casr.lib.packed_floats(cfg)) every rank checks the blob size against its own build's layout
    before the payload moves: the per-rank verdicts are combined (all_reduce MAX), so when any
    rank's build disagrees (e.g. another library version) EVERY rank raises before the payload
    broadcast, and no rank is left waiting in it."""
    import torch.distributed as dist
    rank = dist.get_rank(group)
    n = torch.zeros(1, dtype=torch.int64, device=device)
    if rank == src:
        n[0] = packed.numel()
    dist.broadcast(n, src, group=group)
    bad = torch.zeros(1, dtype=torch.int32, device=device)
    if expect_floats is not None and int(n.item()) != int(expect_floats):
        bad[0] = 1
    dist.all_reduce(bad, op=dist.ReduceOp.MAX, group=group)
    if int(bad.item()):
        mine = "" if expect_floats is None else f"; this rank's layout has {int(expect_floats)}"
        raise ValueError(f"rank {rank}: broadcast blob has {int(n.item())} floats, and at least one rank's "
                         f"build expects another layout{mine}")
    if rank == src:
        buf = packed.to(device=device, dtype=torch.float32).contiguous()
    else:
        buf = torch.empty(int(n.item()), dtype=torch.float32, device=device)
    dist.broadcast(buf, src, group=group)
    return buf


def merge_shards(parts, n_total):
    """[(indices, results)] per shard -> the n_total results in the original utterance order.
    Every index in [0, n_total) must be covered exactly once."""
    out = [None] * n_total
    seen = np.zeros(n_total, np.int64)
    for idx, res in parts:
        if len(idx) != len(res):
            raise ValueError(f"shard has {len(idx)} indices but {len(res)} results")
        for i, r in zip(idx, res):
            out[int(i)] = r
            seen[int(i)] += 1
    if not (seen == 1).all():
        raise ValueError("shards do not cover every utterance exactly once")
    return out


def gather_results(local, indices, n_total, group=None):
    """all_gather the per-rank result lists; returns the list of n_total results in the
    original utterance order on every rank.  local[i] belongs to utterance indices[i]."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    parts = [None] * world
    dist.all_gather_object(parts, (list(map(int, indices)), list(local)), group=group)
    return merge_shards(parts, n_total)


# --------------------------------------------------------------------------------------------
# The sharded product call of BASELINE configs 4 and 5 (1,024 utterances over the node's GPUs,
# beam 8, or beam 16 + the second pass): partition -> per-rank decode -> gather.  One function
# serves bench.py --gpus N, the world-size-2 gloo test (per-rank decoder = the CPU oracle) and
# the single-GPU shard-by-shard tests (tests/test_gpu_scale.py), so all three run the same
# chain.  Results travel as fixed-size arrays, not Python objects: per utterance the token ids
# [max_len] int32, the length and the score (f32 bits), one all_gather per batch.
# --------------------------------------------------------------------------------------------
def _rank_world(group=None):
    """(rank, world size) of the process group, or (0, 1) when none is initialised (bench.py at
    --gpus 1 runs the same sharded call as a single shard)."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(group), dist.get_world_size(group)
    return 0, 1


def shard_sizes(lens, world):
    return [len(i) for i in partition(lens, world)]


def pack_results(tokens, length, score, max_len):
    """(tokens [n, >= max_len] int, length [n], score [n] f32) -> int32 [n, max_len + 2]: the
    token ids, the length, the score's f32 bits."""
    n = len(length)
    out = np.zeros((n, max_len + 2), np.int32)
    out[:, :max_len] = np.asarray(tokens)[:, :max_len]
    out[:, max_len] = np.asarray(length, np.int32)
    out[:, max_len + 1] = np.asarray(score, np.float32).view(np.int32)
    return out


def unpack_results(packed, max_len):
    packed = np.asarray(packed, np.int32)
    return (packed[:, :max_len].copy(), packed[:, max_len].copy(),
            packed[:, max_len + 1].copy().view(np.float32))


def merge_arrays(parts, n_total):
    """[(indices, packed [n_r, W])] per shard -> [n_total, W] in the original utterance order;
    every index in [0, n_total) must be covered exactly once (merge_shards' check)."""
    W = next(p.shape[1] for _, p in parts)
    out = np.zeros((n_total, W), np.int32)
    seen = np.zeros(n_total, np.int64)
    for idx, p in parts:
        idx = np.asarray(idx, np.int64)
        if len(idx) != p.shape[0]:
            raise ValueError(f"shard has {len(idx)} indices but {p.shape[0]} results")
        out[idx] = p
        np.add.at(seen, idx, 1)
    if not (seen == 1).all():
        raise ValueError("shards do not cover every utterance exactly once")
    return out


def gather_arrays(packed, lens, group=None, device=None):
    """all_gather of every rank's packed results (pack_results) into the global order.  Every
    rank recomputes the partition from the same lengths, so only the results move: one
    all_gather of [max shard, W] int32 per rank (on `device`: the rank's GPU under RCCL, the CPU
    under gloo).  Returns [len(lens), W] on every rank."""
    rank, world = _rank_world(group)
    shards = partition(lens, world)
    if world == 1:  # one process (no process group): nothing to exchange
        return merge_arrays([(shards[0], packed)], len(lens))
    import torch.distributed as dist
    m = max(len(s) for s in shards)
    W = packed.shape[1]
    dev = torch.device("cpu") if device is None else device
    buf = torch.zeros((m, W), dtype=torch.int32, device=dev)
    buf[:packed.shape[0]] = torch.from_numpy(np.ascontiguousarray(packed)).to(dev)
    allbuf = torch.empty((world * m, W), dtype=torch.int32, device=dev)
    dist.all_gather_into_tensor(allbuf, buf, group=group)
    allbuf = allbuf.cpu().numpy().reshape(world, m, W)
    return merge_arrays([(s, allbuf[r, :len(s)]) for r, s in enumerate(shards)], len(lens))


class BeamShardDecoder:
    """One rank's decode of its shard, the product path of BASELINE configs 4 / 5:
    casr_encode_fbank + casr_beam (model.py:604-987) and, with an LM, the finished-hypothesis
    records to the host and the second pass over them (second_pass_arrays, model.py:749-763;
    the rest keep the device's unfinished fallback / first max, :961-972), exactly as the drop-in
    Model.eval_one_batch_with_beam does.

    A shard larger than `max_batch` utterances is decoded as consecutive batches of at most that
    many (256: the largest batch whose encoder recurrence runs persistent, one workgroup per CU;
    beyond it the recurrence falls back to per-step launches, casr_recurrence_mode).  Like any
    batching of the reference's beam search, the batch a hypothesis is decoded in decides when the
    search stops (model.py:897-901), so the second pass sees the records of its own batch's steps.

    enqueue() puts every batch's device work and its copies into pinned host buffers on the
    stream and returns at once; finish() waits for one batch at a time and runs its host part, so
    the host part of one batch overlaps the device work of the next (two pinned slots per batch
    position)."""

    def __init__(self, engine, k, lm_model=None, int2word=None, lm_weight=0.0, length_weight=0.0,
                 keep_records=False, max_batch=256, rescorer=None):
        # engine: an Engine, or a casr.pipeline.StreamPipeline (or its limited() view), whose
        # handles then take the shard's batches in turn, several in flight
        self.engine, self.k = engine, int(k)
        self.keep_records = keep_records  # finish() keeps the last shard's record arrays (tests)
        self.last_records = None
        self.lm_model, self.int2word = lm_model, int2word
        self.lm_weight, self.length_weight = float(lm_weight), float(length_weight)
        self.max_len = engine.cfg.max_len
        self.max_batch = int(max_batch)
        self.rescorer = rescorer  # casr.rescore.ParallelRescorer: the LM calls on host worker processes
        self._slots = {}
        self._next = 0
        self.stats = {}

    def _batch(self, e, fbank, frames, key):
        e.encode_fbank(fbank, frames)
        r = e.beam(self.k, self.lm_weight, self.length_weight)
        dev_out = [r["tokens"], r["length"], r["score"], r["steps"]]
        if self.lm_model is not None:
            dev_out += list(e.beam_records())
        key = key + (tuple(tuple(x.shape) for x in dev_out),)
        bufs = self._slots.get(key)
        if bufs is None:
            bufs = self._slots[key] = [torch.empty(x.shape, dtype=x.dtype, pin_memory=True) for x in dev_out]
        for h, x in zip(bufs, dev_out):
            h.copy_(x, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()  # on the batch's stream
        return bufs, ev

    def enqueue(self, fbank, frames):
        n = int(fbank.shape[0])
        slot = self._next & 1
        self._next += 1
        submit = getattr(self.engine, "submit", None)
        pend = []
        for i, c0 in enumerate(range(0, n, self.max_batch)):
            c1 = min(n, c0 + self.max_batch)
            fn = (lambda e, c0=c0, c1=c1, i=i: self._batch(e, fbank[c0:c1], frames[c0:c1], (slot, i)))
            pend.append(submit(fn) if submit else fn(self.engine))
        return pend

    def _finish_batch(self, bufs, ev):
        from .results import second_pass_arrays
        ev.synchronize()  # this batch only (the guard bits are the caller's: reading them syncs the stream)
        toks, blen, score, steps = (b.numpy().copy() for b in bufs[:4])
        recs = None
        if self.lm_model is not None:
            rt, rs, rv = (b.numpy() for b in bufs[4:])
            if self.rescorer is not None:  # the same choice, LM calls spread over worker processes
                best = self.rescorer.select(rt, rs, rv, self.lm_weight, self.length_weight)
            else:
                best = second_pass_arrays(rt, rs, rv, self.int2word, self.lm_model, self.lm_weight,
                                          self.length_weight)
            self.stats["records"] = self.stats.get("records", 0) + int(np.count_nonzero(rv))
            if self.keep_records:
                recs = (rt.copy(), rs.copy(), rv.copy())
            for b, (t, s) in best.items():
                toks[b, :len(t)] = t
                blen[b] = len(t)
                score[b] = s
        return pack_results(toks, blen, score, self.max_len), int(steps[0]), recs

    def finish(self, pend):
        self.stats["records"] = 0
        parts, steps, recs = [], [], []
        for bufs, ev in pend:
            p, st, rc = self._finish_batch(bufs, ev)
            parts.append(p)
            steps.append(st)
            recs.append(rc)
        self.stats["steps"] = steps[-1]
        self.stats["batch_steps"] = steps
        if self.keep_records and self.lm_model is not None:
            self.last_records = tuple(np.concatenate([r[i] for r in recs]) for i in range(3))
        return np.concatenate(parts)


def decode_rank(lens, rank, world, load_shard, decoder):
    """The rank-local half of decode_sharded, unpipelined: (indices, packed results) of this
    rank's shard of one global batch (partition of `lens`; load_shard(indices) -> the decoder's
    inputs for those utterances)."""
    idx = partition(lens, world)[rank]
    return idx, decoder.finish(decoder.enqueue(*load_shard(idx)))


def decode_sharded(batches, decoder, group=None, device=None):
    """BASELINE configs 4 / 5 as one call per rank: for each global batch (lens, load_shard) of
    `batches` -> this rank's shard (partition of lens) -> decoder.enqueue(*load_shard(indices))
    -> decoder.finish -> gather_arrays.  Two batches in flight: batch i's device work is enqueued
    before batch i - 1's host part and gather run.  Yields, per global batch and on every rank,
    (tokens [N, max_len] int32, length [N] int32, score [N] f32) in the original utterance order.
    No collective runs inside the decode; the gather is the only exchange.  Without a process
    group the call runs as rank 0 of 1 (one shard, no exchange)."""
    rank, world = _rank_world(group)
    max_len = decoder.max_len
    prev = None
    for lens, load_shard in batches:
        idx = partition(lens, world)[rank]
        cur = (lens, decoder.enqueue(*load_shard(idx)))
        if prev is not None:
            yield unpack_results(gather_arrays(decoder.finish(prev[1]), prev[0], group, device), max_len)
        prev = cur
    if prev is not None:
        yield unpack_results(gather_arrays(decoder.finish(prev[1]), prev[0], group, device), max_len)
