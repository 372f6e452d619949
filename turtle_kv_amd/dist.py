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


# ---------------------------------------------------------------------------------------
# Hash-range sharding of ONE monolithic Bloom filter (BASELINE config 5 read literally:
# "1B keys, Bloom @12, hash-range sharded across 8 GPUs, RCCL all-gather").  Unlike the leaf
# filters above, keys must move: every key's bits fall in the 64-byte block its h0 selects, so
# a rank can only build its byte range of the bitmap from the keys whose blocks fall there.
# Steps per build: route (reorder the rank's keys by owning rank: tkv_amq_bloom_route_records
# hashes each key once and ships its 12-byte bit record, k <= 8; tkv_amq_bloom_route ships the
# 16-byte key otherwise), one all-to-all of them (RCCL over xGMI), the rank's tile range built in
# LDS (tkv_amq_bloom_build_range_records / _build_range), then the all-gather of the bitmap
# ranges.
# ---------------------------------------------------------------------------------------
BLOOM_TILE_BLOCKS = 1024  # blocks per tile, as tkv_amq_bloom_route / _build_range cut them


def hash_shard_tiles(n_blocks: int, world: int) -> tuple[int, int]:
    """(T, q): the filter's tiles and the tiles per rank; rank r owns [r*q, min((r+1)*q, T))."""
    T = -(-int(n_blocks) // BLOOM_TILE_BLOCKS)
    return T, -(-T // world)


class HashShardedBloom:
    """One rank's side of a hash-range sharded build of one Bloom filter over the keys of all
    ranks (n_total_keys in all).  `build(keys)` returns the whole filter payload (header +
    bitmap, byte-identical to a one-GPU tkv_amq_build of the concatenated keys) on every rank.
    Buffers are allocated once and grown when a rank receives more keys than before."""

    def __init__(self, n_total_keys: int, bits_per_key: int, world: int, rank: int, device,
                 src_page_id: int = 0, group=None):
        import torch
        from . import abi
        from .filters import plan_filters
        self.world, self.rank, self.group, self.dev = world, rank, group, torch.device(device)
        self.plan = plan_filters(abi.BLOOM, [n_total_keys], bits_per_key, src_page_ids=[src_page_id])
        seg = self.plan.segs[0]
        self.n_blocks = int(seg["n_blocks"])
        self.payload_bytes = int(seg["payload_bytes"])
        T, q = hash_shard_tiles(self.n_blocks, world)
        # ranks past ceil(T / q) own no tile (e.g. T = 17 over 8 ranks: q = 3, ranks 6 and 7):
        # they route and exchange keys like the others, and their range build writes only the
        # filter header
        self.tile_begin, self.tile_end = min(T, rank * q), min(T, (rank + 1) * q)
        self.slice_bytes = q * BLOOM_TILE_BLOCKS * 64
        # the payload layout of tkv_amq_build (64-byte header, then the blocks), padded so every
        # rank's range is a slice of slice_bytes
        self.out = torch.zeros(64 + world * self.slice_bytes, dtype=torch.uint8, device=self.dev)
        self.gathered = torch.empty(world * self.slice_bytes, dtype=torch.uint8, device=self.dev)
        self.d_seg = self.plan.device_segs(self.dev)
        self.counts = torch.zeros(world, dtype=torch.int32, device=self.dev)
        self._bufs = {}
        # k <= 8 (bits_per_key <= 12): 12-byte bit records travel instead of the 16-byte keys,
        # hashed once by their sender (tkv_amq_bloom_route_records); the owner's range build
        # reads them without hashing (a range of <= 3,584 tiles: the record path's table)
        self.hash_count = int(seg["hash_count"])
        self.records = self.hash_count <= 8 and q <= 3584
        self.unit = 12 if self.records else 16  # bytes per routed key

    def _buf(self, name, nbytes):
        import torch
        b = self._bufs.get(name)
        if b is None or b.numel() < nbytes:
            b = torch.empty(max(nbytes, 16), dtype=torch.uint8, device=self.dev)
            self._bufs[name] = b
        return b

    def route(self, keys):
        """keys [n, 16] (or [n, 24] with bit records) uint8 on the device -> (routed [n, unit],
        send counts per rank, int64)."""
        import torch
        from . import abi
        from .filters import _ptr, _stream_handle
        L = abi.lib()
        kb = keys.shape[1] if keys.dim() == 2 else 0
        if not (kb == 16 or (kb == 24 and self.records)):
            # bit records (k <= 8) are routed from 16- or 24-byte keys
            # (tkv_amq_bloom_route_records_ex); keys themselves (k > 8) travel as 16 bytes only
            # (tkv_amq_bloom_route / _build_range; INTEGRATION.md key shapes)
            raise abi.TkvAmqError(abi.INVALID_ARGUMENT, "hash-range sharding takes [n, 16] uint8 "
                                  "keys, or [n, 24] at <= 12 bits/key, got shape "
                                  f"{tuple(keys.shape)}")
        n = keys.shape[0]
        u = self.unit
        routed = self._buf("routed", u * n)[:u * n].view(n, u)
        if self.records:
            ws = self._buf("route_ws", int(L.tkv_amq_bloom_route_records_ws_bytes(n, self.world)))
            abi.check(L.tkv_amq_bloom_route_records_ex(_ptr(keys), kb, n, _ptr(self.d_seg), self.n_blocks,
                                                       self.hash_count, self.world, _ptr(routed),
                                                       _ptr(self.counts), _ptr(ws), ws.numel(),
                                                       _stream_handle()), "tkv_amq_bloom_route_records_ex")
        else:
            ws = self._buf("route_ws", int(L.tkv_amq_bloom_route_ws_bytes(n, self.world)))
            abi.check(L.tkv_amq_bloom_route(_ptr(keys), n, _ptr(self.d_seg), self.n_blocks, self.world,
                                            _ptr(routed), _ptr(self.counts), _ptr(ws), ws.numel(),
                                            _stream_handle()), "tkv_amq_bloom_route")
        return routed, self.counts.to(dtype=torch.int64)

    def exchange(self, routed, send_counts):
        """All-to-all of the routed units (bit records or keys): returns the [m, unit] units
        this rank owns."""
        import torch
        import torch.distributed as dist
        u = self.unit
        gloo = dist.get_backend(self.group) != "nccl"
        sc = send_counts.cpu() if gloo else send_counts
        rc = torch.empty_like(sc)
        dist.all_to_all_single(rc, sc, group=self.group)
        send = [int(x) * u for x in sc.tolist()]
        recv = [int(x) * u for x in rc.tolist()]
        m = sum(recv) // u
        out = self._buf("recv", u * m)[:u * m]
        src = routed.reshape(-1)
        if gloo:  # CPU rehearsal: stage through host memory
            host = torch.empty(u * m, dtype=torch.uint8)
            dist.all_to_all_single(host, src.cpu(), recv, send, group=self.group)
            out.copy_(host)
        else:
            dist.all_to_all_single(out, src, recv, send, group=self.group)
        return out.view(m, u)

    def build_range(self, owned):
        """This rank's tile range of the filter from the keys it owns (into self.out)."""
        from . import abi
        from .filters import _ptr, _stream_handle
        L = abi.lib()
        m = owned.shape[0]
        ws = self._buf("build_ws", int(L.tkv_amq_bloom_build_range_ws_bytes(m, self.tile_begin,
                                                                             self.tile_end)))
        abi.check(L.tkv_amq_bloom_build_range(_ptr(owned), m, _ptr(self.d_seg), self.n_blocks,
                                              self.tile_begin, self.tile_end, _ptr(self.out),
                                              _ptr(ws), ws.numel(), _stream_handle()),
                  "tkv_amq_bloom_build_range")

    def build_range_records(self, recs):
        """This rank's tile range of the filter from the bit records it owns (into self.out)."""
        from . import abi
        from .filters import _ptr, _stream_handle
        L = abi.lib()
        m = recs.shape[0]
        ws = self._buf("build_ws", int(L.tkv_amq_bloom_build_range_records_ws_bytes(
            m, self.tile_begin, self.tile_end)))
        abi.check(L.tkv_amq_bloom_build_range_records(_ptr(recs), m, _ptr(self.d_seg), self.n_blocks,
                                                      self.hash_count, self.tile_begin, self.tile_end,
                                                      _ptr(self.out), _ptr(ws), ws.numel(),
                                                      _stream_handle()),
                  "tkv_amq_bloom_build_range_records")

    def build_owned(self, owned):
        """The range build from what exchange() returned (records or keys)."""
        if self.records:
            self.build_range_records(owned)
        else:
            self.build_range(owned)

    @property
    def _collective(self) -> bool:
        """route + all-to-all + all-gather whenever a process group exists (at world size 1
        too: that runs the RCCL code path on one GPU); alone, the range build is the filter."""
        import torch.distributed as dist
        return self.world > 1 or (dist.is_available() and dist.is_initialized())

    def local_build(self, keys):
        """route + exchange + range build: after it, this rank's byte range of the bitmap is final."""
        if not self._collective:
            self.build_range(keys)
            return
        routed, sc = self.route(keys)
        self.build_owned(self.exchange(routed, sc))

    def allgather(self):
        """Every rank's bitmap range -> the whole filter payload (header + bitmap) on every rank.
        Every rank's range build writes the header (also a rank that owns no tile)."""
        import torch
        if not self._collective:
            return self.out[:self.payload_bytes]
        r0 = 64 + self.rank * self.slice_bytes
        allgather_filters(self.out[r0:r0 + self.slice_bytes], self.gathered, self.group)
        return torch.cat([self.out[:64], self.gathered[:self.payload_bytes - 64]])

    def build(self, keys):
        self.local_build(keys)
        return self.allgather()
