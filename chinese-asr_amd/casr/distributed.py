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
    before receiving it: a rank running another library version fails here, not on the device."""
    import torch.distributed as dist
    rank = dist.get_rank(group)
    n = torch.zeros(1, dtype=torch.int64, device=device)
    if rank == src:
        n[0] = packed.numel()
    dist.broadcast(n, src, group=group)
    if expect_floats is not None and int(n.item()) != int(expect_floats):
        raise ValueError(f"rank {rank}: broadcast blob has {int(n.item())} floats, this build's layout "
                         f"has {int(expect_floats)}")
    if rank == src:
        buf = packed.to(device=device, dtype=torch.float32).contiguous()
    else:
        buf = torch.empty(int(n.item()), dtype=torch.float32, device=device)
    dist.broadcast(buf, src, group=group)
    return buf


def gather_results(local, indices, n_total, group=None):
    """all_gather the per-rank result lists; returns the list of n_total results in the
    original utterance order on every rank.  local[i] belongs to utterance indices[i]."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    parts = [None] * world
    dist.all_gather_object(parts, (list(map(int, indices)), list(local)), group=group)
    out = [None] * n_total
    for idx, res in parts:
        for i, r in zip(idx, res):
            out[i] = r
    return out
