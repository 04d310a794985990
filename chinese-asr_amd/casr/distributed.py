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
