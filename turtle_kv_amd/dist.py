"""Multi-GPU sharding of one checkpoint's leaf filters.

A checkpoint is thousands of independent leaf filters.  Rank r of W builds the contiguous
leaf range [r*P, min((r+1)*P, n_leaves)), P = ceil(n_leaves / W), into its own slice of a
fixed-stride global filter array: leaf s lives at byte s * stride, so each rank owns a
disjoint byte range ("disjoint bit-range" of the north star) and no keys move between GPUs.
The only exchange is one all-gather of the finished array (RCCL over xGMI when the process
group is "nccl"), which gives every rank -- or the host writer -- every filter page.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


@dataclass(frozen=True)
class Shard:
    rank: int
    world: int
    leaf_begin: int      # first global leaf index of this rank
    leaf_end: int        # one past the last
    leaves_per_rank: int
    key_begin: int       # first global key index of this rank
    key_end: int

    @property
    def n_leaves(self) -> int:
        return self.leaf_end - self.leaf_begin


def shard_leaves(leaf_key_counts, world: int, rank: int) -> Shard:
    counts = np.asarray(leaf_key_counts, dtype=np.int64)
    n = len(counts)
    per = -(-n // world) if n else 0
    b = min(n, rank * per)
    e = min(n, b + per)
    kb = int(counts[:b].sum())
    ke = kb + int(counts[b:e].sum())
    return Shard(rank, world, b, e, per, kb, ke)


def leaf_stride(kind: int, bits_per_key: int, max_leaf_keys: int, payload_capacity: int = 0) -> int:
    """Fixed per-leaf slot size (64-byte aligned) that fits the largest leaf's payload."""
    from .filters import plan_filters
    p = plan_filters(kind, [max_leaf_keys], bits_per_key, payload_capacity=payload_capacity)
    return (int(p.segs[0]["payload_bytes"]) + 63) // 64 * 64


def plan_shard(kind: int, leaf_key_counts, bits_per_key: int, shard: Shard, stride: int,
               payload_capacity: int = 0, src_page_ids=None):
    """The rank-local plan: its leaves, numbered globally, at fixed stride in a local slice of
    leaves_per_rank * stride bytes (padding leaves are left unwritten)."""
    from .filters import plan_filters
    counts = np.asarray(leaf_key_counts, dtype=np.uint64)[shard.leaf_begin:shard.leaf_end]
    if src_page_ids is None:
        src = np.arange(shard.leaf_begin, shard.leaf_end, dtype=np.uint64)
    else:
        src = np.asarray(src_page_ids, dtype=np.uint64)[shard.leaf_begin:shard.leaf_end]
    plan = plan_filters(kind, counts, bits_per_key, payload_capacity=payload_capacity,
                        out_stride=stride, src_page_ids=src)
    plan.total_out_bytes = shard.leaves_per_rank * stride
    return plan


def allgather_filters(local, gathered=None, group=None):
    """All-gather every rank's fixed-size slice into the global leaf-ordered array."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    if gathered is None:
        gathered = torch.empty(local.numel() * world, dtype=local.dtype, device=local.device)
    if local.is_cuda and dist.get_backend(group) != "nccl":
        # gloo (tests, CPU-only rehearsals): stage through host memory
        g = allgather_filters(local.cpu(), None, group)
        gathered.copy_(g)
        return gathered
    try:
        dist.all_gather_into_tensor(gathered, local, group=group)
    except (RuntimeError, NotImplementedError, AttributeError):
        parts = list(gathered.view(world, -1).unbind(0))
        dist.all_gather(parts, local, group=group)
    return gathered
