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
# The all-gather overlapped with the build.  A contiguous leaf range per rank can only be
# gathered once the whole range is built (all_gather_into_tensor lands rank r's bytes at r's
# offset).  With block-cyclic ownership -- in round c rank r owns leaves [(c*W + r)*Q,
# (c*W + r + 1)*Q) -- round c's slots of all ranks are one contiguous piece of the leaf-ordered
# array, so each round is gathered straight into place on a communication stream while the
# next round builds: the step costs about max(build, gather) instead of their sum.
# ---------------------------------------------------------------------------------------
def cyclic_rounds(n_leaves: int, world: int, rank: int, chunk_leaves: int) -> list[tuple[int, int]]:
    """Rank `rank`'s leaf range in each round (empty ranges past the last leaf)."""
    q = max(1, int(chunk_leaves))
    rounds = -(-int(n_leaves) // (world * q)) if n_leaves else 0
    return [(min(n_leaves, (c * world + rank) * q), min(n_leaves, (c * world + rank + 1) * q))
            for c in range(rounds)]


class PipelinedLeafGather:
    """One rank's side of a checkpoint build whose filter array is all-gathered round by round
    while the next round builds (leaf s at s * stride of `gathered` on every rank, as
    allgather_filters gives).  `step(key_batches)` builds and gathers every round."""

    def __init__(self, kind: int, leaf_key_counts, bits_per_key: int, world: int, rank: int,
                 stride: int, chunk_leaves: int, device, payload_capacity: int = 0, group=None):
        import torch
        from .filters import plan_filters
        counts = np.asarray(leaf_key_counts, dtype=np.int64)
        self.world, self.rank, self.group, self.dev = world, rank, group, torch.device(device)
        self.stride, self.q = stride, max(1, int(chunk_leaves))
        self.n_leaves = len(counts)
        self.key_begin = np.concatenate([[0], np.cumsum(counts)])
        self.rounds = cyclic_rounds(self.n_leaves, world, rank, self.q)
        self.plans = []
        for b, e in self.rounds:
            if b == e:  # past the last leaf: this rank's slots of the round stay zero
                self.plans.append(None)
                continue
            p = plan_filters(kind, counts[b:e].astype(np.uint64), bits_per_key,
                             payload_capacity=payload_capacity, out_stride=stride,
                             src_page_ids=np.arange(b, e, dtype=np.uint64))
            self.plans.append(p)
        R = len(self.rounds)
        self.round_bytes = self.q * stride
        self.local = torch.zeros(max(1, R) * self.round_bytes, dtype=torch.uint8, device=self.dev)
        self.gathered = torch.zeros(max(1, R) * world * self.round_bytes, dtype=torch.uint8,
                                    device=self.dev)
        ws = max((p.workspace_bytes for p in self.plans if p is not None), default=0)
        self.ws = torch.empty(max(ws, 1), dtype=torch.uint8, device=self.dev)
        self.comm = torch.cuda.Stream(device=self.dev)

    def key_ranges(self) -> list[tuple[int, int]]:
        """Global key index range of each round's leaves (keys are laid out leaf after leaf)."""
        return [(int(self.key_begin[b]), int(self.key_begin[e])) for b, e in self.rounds]

    def _gather(self, c: int):
        rb, W = self.round_bytes, self.world
        allgather_filters(self.local[c * rb:(c + 1) * rb], self.gathered[c * W * rb:(c + 1) * W * rb],
                          self.group)

    def step(self, key_batches, build: bool = True, gather: bool = True, check: bool = False):
        """Build round c on the current stream; gather it on the communication stream once
        its build is done, while round c + 1 builds.  On return the current stream is ordered
        after every gather: work queued on it next sees the whole array (and may rebuild the
        slots).  check=True synchronises after each round's build to report VQF insert
        failures (build_all_filters' check); the default keeps the step asynchronous."""
        import torch
        from .filters import build_all_filters
        if len(key_batches) != len(self.rounds):
            raise ValueError(f"{len(key_batches)} key batches for {len(self.rounds)} rounds")
        cur = torch.cuda.current_stream(self.dev)
        self.comm.wait_stream(cur)  # the previous step's readers of `gathered` are done
        rb = self.round_bytes
        for c, kb in enumerate(key_batches):
            if build and self.plans[c] is not None:
                build_all_filters(self.plans[c], kb, out=self.local[c * rb:(c + 1) * rb],
                                  workspace=self.ws, check=check)
            if gather:
                ev = torch.cuda.Event()
                ev.record(cur)
                with torch.cuda.stream(self.comm):
                    self.comm.wait_event(ev)
                    self._gather(c)
        cur.wait_stream(self.comm)

    def filters(self):
        """The gathered leaf-ordered array (leaf s at s * stride), trimmed to the leaves."""
        return self.gathered[:self.n_leaves * self.stride]


# ---------------------------------------------------------------------------------------
# Hash-range sharding of ONE monolithic Bloom filter (BASELINE config 5 read literally:
# "1B keys, Bloom @12, hash-range sharded across 8 GPUs, RCCL all-gather").  Unlike the leaf
# filters above, keys must move: every key's bits fall in the 64-byte block its h0 selects, so
# a rank can only build its byte range of the bitmap from the keys whose blocks fall there.
# The filter's T tiles (tkv_amq_bloom_tile_blocks() blocks each) are cut into world * g parts
# of q tiles; rank r owns the g consecutive parts [r*g, (r+1)*g), a contiguous byte range of
# the bitmap.  g = 1 unless a rank's range exceeds what one range build takes (6,400 tiles:
# 800 MiB of filter per rank).  Steps per build, the same at every world size:
#   route     reorder the rank's keys by part (tkv_amq_bloom_route_records hashes each key once
#             and ships its 12-byte bit record, k <= 8; tkv_amq_bloom_route ships the 16-byte
#             key otherwise);
#   exchange  one all-to-all of them (RCCL over xGMI; at world size 1 a local copy);
#   build     each owned part built from its records (tkv_amq_bloom_build_range_records /
#             _build_range), part after part;
#   gather    the all-gather of the bitmap ranges.
# Without a process group (one GPU, no launcher) a filter of at most 6,400 tiles skips the
# route: the range build reads the keys and makes the same records itself.
# ---------------------------------------------------------------------------------------
BLOOM_TILE_BLOCKS = 2048        # tkv_amq_bloom_tile_blocks()
RECORD_RANGE_MAX_TILES = 6400   # tkv_amq_bloom_range_max_tiles(1): the partition's tile table
KEY_RANGE_MAX_TILES = 6400      # tkv_amq_bloom_range_max_tiles(0)
ROUTED_PART_TILES = 256         # the library's kRoutePartTiles: tiles per part of bit records
ROUTED_KEY_PART_TILES = 1600    # kRouteKeyPartTiles: tiles per part of routed 16-byte keys


def hash_shard_plan(n_blocks: int, world: int, records: bool = True) -> tuple[int, int, int]:
    """(T, g, q): the filter's tiles, the parts per rank and the tiles per part; part p owns
    tiles [p*q, min((p+1)*q, T)) and rank r parts [r*g, (r+1)*g).  Parts hold at most
    ROUTED_PART_TILES tiles of bit records (ROUTED_KEY_PART_TILES of routed keys), well under
    what one range build takes: the fewer tiles a part build spreads a batch of records over,
    the longer its stores' runs, and at most one tile per CU (kRoutePartTiles).  BASELINE
    config 5 (1B keys at 12 bits/key, 11,445 tiles) builds 45 parts of 255 tiles on one GPU,
    6 of 239 on each of eight."""
    T = -(-int(n_blocks) // BLOOM_TILE_BLOCKS)
    per_rank = -(-T // world)
    cap = (min(ROUTED_PART_TILES, RECORD_RANGE_MAX_TILES) if records
           else min(ROUTED_KEY_PART_TILES, KEY_RANGE_MAX_TILES))
    g = max(1, -(-per_rank // cap))
    q = -(-T // (world * g))
    return T, g, q


def hash_shard_tiles(n_blocks: int, world: int) -> tuple[int, int]:
    """(T, q): the filter's tiles and the tiles per part when each of `world` parts is one
    range build (the ABI's tkv_amq_bloom_route with n_parts = world)."""
    T = -(-int(n_blocks) // BLOOM_TILE_BLOCKS)
    return T, -(-T // world)


class ExactHashShardedBloom:
    """One rank's side of a hash-range sharded build of one Bloom filter over the keys of all
    ranks (n_total_keys in all), with an exchange sized by exact counts (two host
    synchronisations per build) and contiguous tile ranges per rank.  `build(keys)` returns the
    whole filter payload (header + bitmap, byte-identical to a one-GPU tkv_amq_build of the
    concatenated keys) on every rank.  HashShardedBloom uses it for k > 8 (16-byte keys travel)
    and when a pipelined step lost overflow entries (keys far from uniform).  Buffers are
    allocated once and grown when a rank receives more keys than before."""

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
        # k <= 8 (bits_per_key <= 12): 12-byte bit records travel instead of the 16-byte keys,
        # hashed once by their sender (tkv_amq_bloom_route_records); the owner's range builds
        # read them without hashing
        self.hash_count = int(seg["hash_count"])
        self.records = self.hash_count <= 8
        self.unit = 12 if self.records else 16  # bytes per routed key
        self.T, self.g, self.q = hash_shard_plan(self.n_blocks, world, self.records)
        self.n_parts = world * self.g
        # ranks past the last tile (e.g. T = 17 over 8 ranks: q = 3, ranks 6 and 7) route and
        # exchange keys like the others, and their range build writes only the filter header
        self.tile_begin = min(self.T, rank * self.g * self.q)
        self.tile_end = min(self.T, (rank + 1) * self.g * self.q)
        self.slice_bytes = self.g * self.q * BLOOM_TILE_BLOCKS * 64
        # the payload layout of tkv_amq_build (64-byte header, then the blocks), padded so every
        # rank's range is a slice of slice_bytes
        self.out = torch.zeros(64 + world * self.slice_bytes, dtype=torch.uint8, device=self.dev)
        self.gathered = torch.empty(world * self.slice_bytes, dtype=torch.uint8, device=self.dev)
        self.d_seg = self.plan.device_segs(self.dev)
        self.counts = torch.zeros(self.n_parts, dtype=torch.int32, device=self.dev)
        self._bufs = {}

    def _buf(self, name, nbytes):
        import torch
        b = self._bufs.get(name)
        if b is None or b.numel() < nbytes:
            b = torch.empty(max(nbytes, 16), dtype=torch.uint8, device=self.dev)
            self._bufs[name] = b
        return b

    def part_tiles(self, j: int) -> tuple[int, int]:
        """Tiles of this rank's j-th part."""
        b = min(self.T, self.tile_begin + j * self.q)
        return b, min(self.tile_end, b + self.q)

    def route(self, keys):
        """keys [n, 16] (or [n, 24] with bit records) uint8 on the device -> (routed [n, unit],
        per-part counts [n_parts], int64 on the device)."""
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
        P = self.n_parts
        if self.records:
            ws = self._buf("route_ws", int(L.tkv_amq_bloom_route_records_ws_bytes(n, P)))
            abi.check(L.tkv_amq_bloom_route_records_ex(_ptr(keys), kb, n, _ptr(self.d_seg), self.n_blocks,
                                                       self.hash_count, P, _ptr(routed),
                                                       _ptr(self.counts), _ptr(ws), ws.numel(),
                                                       _stream_handle()), "tkv_amq_bloom_route_records_ex")
        else:
            ws = self._buf("route_ws", int(L.tkv_amq_bloom_route_ws_bytes(n, P)))
            abi.check(L.tkv_amq_bloom_route(_ptr(keys), n, _ptr(self.d_seg), self.n_blocks, P,
                                            _ptr(routed), _ptr(self.counts), _ptr(ws), ws.numel(),
                                            _stream_handle()), "tkv_amq_bloom_route")
        return routed, self.counts.to(dtype=torch.int64)

    def exchange(self, routed, part_counts):
        """All-to-all of the routed units (bit records or keys).  Returns (owned [m, unit],
        sub [world, g]): the units this rank owns, sender after sender, each sender's ordered
        by part, and how many each sender sent for each of this rank's parts."""
        import torch
        import torch.distributed as dist
        u, W, g = self.unit, self.world, self.g
        gloo = dist.get_backend(self.group) != "nccl"
        pc = part_counts.cpu() if gloo else part_counts
        sub = torch.empty_like(pc)
        dist.all_to_all_single(sub, pc, group=self.group)  # [W*g] -> [sender][part]
        sub = sub.cpu().view(W, g)
        send = [int(x) * u for x in part_counts.cpu().view(W, g).sum(1).tolist()]
        recv = [int(x) * u for x in sub.sum(1).tolist()]
        m = sum(recv) // u
        src = routed.reshape(-1)
        if W == 1:  # every unit is this rank's own: nothing moves
            return src[:u * m].view(m, u), sub
        out = self._buf("recv", u * m)[:u * m]
        # this rank's own units are a device copy, not a message to itself (at world size 1 RCCL
        # moved 12 GB of records to the rank itself at under 1 GB/s)
        r = self.rank
        so, ro = sum(send[:r]), sum(recv[:r])
        out[ro:ro + recv[r]].copy_(src[so:so + send[r]])
        if gloo:  # CPU rehearsal: stage through host memory
            host = torch.empty(u * m, dtype=torch.uint8)
            dist.all_to_all_single(host, src.cpu(), recv, send, group=self.group)
            out.copy_(host)
        else:
            self._all_to_all_others(out, src, send, recv)
        return out.view(m, u), sub

    def _all_to_all_others(self, out, src, send, recv):
        """all_to_all_single of every peer's slice except this rank's own (already copied):
        the own split is sent as an empty message into a scratch view."""
        import torch.distributed as dist
        r = self.rank
        ins, outs = [], []
        so = ro = 0
        for d in range(self.world):
            ins.append(src[so:so + (0 if d == r else send[d])])
            outs.append(out[ro:ro + (0 if d == r else recv[d])])
            so += send[d]
            ro += recv[d]
        dist.all_to_all(outs, ins, group=self.group)

    def build_range(self, owned, t0=None, t1=None):
        """Tiles [t0, t1) (default: this rank's range) of the filter from 16-byte keys."""
        from . import abi
        from .filters import _ptr, _stream_handle
        L = abi.lib()
        t0 = self.tile_begin if t0 is None else t0
        t1 = self.tile_end if t1 is None else t1
        if owned.dim() != 2 or owned.shape[1] != 16:
            raise abi.TkvAmqError(abi.INVALID_ARGUMENT, "the range build takes [n, 16] uint8 keys, "
                                  f"got shape {tuple(owned.shape)}")
        m = owned.shape[0]
        ws = self._buf("build_ws", int(L.tkv_amq_bloom_build_range_ws_bytes(m, t0, t1)))
        abi.check(L.tkv_amq_bloom_build_range(_ptr(owned), m, _ptr(self.d_seg), self.n_blocks, t0, t1,
                                              _ptr(self.out), _ptr(ws), ws.numel(), _stream_handle()),
                  "tkv_amq_bloom_build_range")

    def build_range_records(self, recs, t0=None, t1=None):
        """Tiles [t0, t1) (default: this rank's range) of the filter from bit records."""
        from . import abi
        from .filters import _ptr, _stream_handle
        L = abi.lib()
        t0 = self.tile_begin if t0 is None else t0
        t1 = self.tile_end if t1 is None else t1
        m = recs.shape[0]
        ws = self._buf("build_ws", int(L.tkv_amq_bloom_build_range_records_ws_bytes(m, t0, t1)))
        abi.check(L.tkv_amq_bloom_build_range_records(_ptr(recs) if m else None, m, _ptr(self.d_seg),
                                                      self.n_blocks, self.hash_count, t0, t1,
                                                      _ptr(self.out), _ptr(ws), ws.numel(),
                                                      _stream_handle()),
                  "tkv_amq_bloom_build_range_records")

    def _build_part(self, units, j):
        t0, t1 = self.part_tiles(j)
        if self.records:
            self.build_range_records(units, t0, t1)
        else:
            self.build_range(units, t0, t1)

    def build_owned(self, owned, sub):
        """This rank's parts from what exchange() returned: part j's units are, for every
        sender, the sub[sender, j] units after that sender's parts < j."""
        import torch
        W, g = sub.shape
        if g == 1:
            self._build_part(owned, 0)
            return
        counts = sub.reshape(-1).tolist()
        starts = [0]
        for c in counts:
            starts.append(starts[-1] + int(c))
        for j in range(g):
            pieces = [owned[starts[s * g + j]:starts[s * g + j] + int(counts[s * g + j])] for s in range(W)]
            part = pieces[0] if W == 1 else torch.cat(pieces)
            self._build_part(part, j)

    @property
    def _collective(self) -> bool:
        """route + all-to-all + all-gather whenever a process group exists (at world size 1
        too: that runs the RCCL code path on one GPU); alone, the range build is the filter."""
        import torch.distributed as dist
        return self.world > 1 or (dist.is_available() and dist.is_initialized())

    def local_build(self, keys):
        """route + exchange + part builds: after it, this rank's byte range of the bitmap is
        final."""
        if not self._collective:
            if keys.dim() == 2 and keys.shape[1] == 16 and self.T <= KEY_RANGE_MAX_TILES:
                self.build_range(keys, 0, self.T)  # the partition makes the records itself
                return
            routed, pc = self.route(keys)  # (checks the key shape)
            self.build_owned(routed, pc.cpu().view(1, self.g))
            return
        routed, pc = self.route(keys)
        self.build_owned(*self.exchange(routed, pc))

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


class HashShardedBloom:
    """One rank's side of the pipelined hash-range sharded build of one Bloom filter over the
    keys of all ranks (n_total_keys in all; BASELINE config 5).  Per step (`step`):

      route     the rank's keys in `chunks` chunks (tkv_amq_bloom_route_blocks): every key
                hashed once into its 12-byte bit record, counting-sorted by part on chip and
                appended to its route workgroup's fixed-capacity region of the part's block
                (one block per part and chunk, in global part order, so round j -- part j of
                every rank -- is one slice);
      exchange  round j of chunk c in one all-to-all of equal splits (RCCL over xGMI) on the
                communication stream: every round of a chunk as soon as its route is done, the
                last chunk round by round -- no counts exchanged first, no host synchronisation;
      build     part j from the chunks x ranks blocks of its round, in place
                (tkv_amq_bloom_build_part_blocks: no regrouping copy), as soon as the last
                chunk's round j has landed -- while rounds j + 1, j + 2 are exchanged;
      gather    round j (part j of every rank: one contiguous byte range, parts being owned
                round-robin) all-gathered in place on the communication stream once this
                rank's part j is built, behind the exchange of round j + 2.

    `build(keys)` returns the whole filter payload (header + bitmap), byte-identical to a one-GPU
    tkv_amq_build of the concatenated keys, on every rank.  Without a process group (one GPU)
    a filter of at most 6,400 tiles with 16-byte keys is one range build (no route: the
    partition hashes the keys itself; `direct=False` keeps the route), and a larger one's route
    writes the part builds' input directly.  k > 8 (bits_per_key >= 13), a rank holding
    more keys than the plan's chunks take, and a step whose blocks lost overflow entries (`lost()`;
    keys far from uniform, e.g. one key repeated) go through ExactHashShardedBloom.  The receive
    buffer holds round j's blocks at [j][chunk][sender]."""

    def __init__(self, n_total_keys: int, bits_per_key: int, world: int, rank: int, device,
                 src_page_id: int = 0, group=None, chunks: int = 1, max_keys_per_rank=None,
                 direct: bool = True):
        import ctypes

        import torch
        from . import abi
        from .filters import plan_filters
        self.world, self.rank, self.group, self.dev = world, rank, group, torch.device(device)
        self.n_total_keys, self.bpk, self.src_page_id = n_total_keys, bits_per_key, src_page_id
        self.plan = plan_filters(abi.BLOOM, [n_total_keys], bits_per_key, src_page_ids=[src_page_id])
        seg = self.plan.segs[0]
        self.n_blocks = int(seg["n_blocks"])
        self.payload_bytes = int(seg["payload_bytes"])
        self.hash_count = int(seg["hash_count"])
        self.records = self.hash_count <= 8
        self.unit = 12 if self.records else 16
        self._exact = None
        self._exact_out = None
        self._fallback_out = None
        self.last_fallback = None
        if not self.records:
            self._exact = ExactHashShardedBloom(n_total_keys, bits_per_key, world, rank, device,
                                                src_page_id, group)
            self.T, self.g, self.q = self._exact.T, self._exact.g, self._exact.q
            return
        self.chunks = max(1, int(chunks))
        per_rank = int(max_keys_per_rank) if max_keys_per_rank else -(-n_total_keys // world)
        self.chunk_keys = max(1, -(-per_rank // self.chunks))
        rp = abi.RoutePlan()
        L = abi.lib()
        abi.check(L.tkv_amq_bloom_route_plan(self.chunk_keys, self.chunks, self.n_blocks,
                                             self.hash_count, world, ctypes.byref(rp)),
                  "tkv_amq_bloom_route_plan")
        self.rp = rp
        self.T, self.g, self.q = int(rp.n_tiles), int(rp.parts_per_rank), int(rp.part_tiles)
        self.n_parts = int(rp.n_parts)
        self.block_bytes = int(rp.block_bytes)
        self.part_bytes = int(rp.part_bytes)
        self.round_bytes = world * self.part_bytes
        # the filter payload, padded to whole rounds: part p's bitmap at 64 + p * part_bytes
        self.out = torch.zeros(64 + self.n_parts * self.part_bytes, dtype=torch.uint8, device=self.dev)
        C, W, B = self.chunks, world, self.block_bytes
        # round j's blocks at [j][chunk][sender]: part j's inputs are C * W consecutive blocks
        self.recv = torch.empty(self.g * C * W * B, dtype=torch.uint8, device=self.dev)
        # chunk c's send buffer: every part's block in global part order (round j's W blocks =
        # one slice); one rank routes straight into recv
        self.send = (None if world == 1 else
                     [torch.empty(self.n_parts * B, dtype=torch.uint8, device=self.dev)
                      for _ in range(C)])
        self.route_ws = torch.empty(int(rp.route_ws_bytes), dtype=torch.uint8, device=self.dev)
        self.part_ws = torch.empty(int(rp.part_ws_bytes), dtype=torch.uint8, device=self.dev)
        self.d_seg = self.plan.device_segs(self.dev)
        self.comm = torch.cuda.Stream(device=self.dev) if self.dev.type == "cuda" else None
        self.last_lost = None
        self.timeline = None
        self._direct = False
        self._direct_ok = direct   # one GPU, no process group, T <= 6,400: no route
        self._direct_ws = None

    @property
    def capacity(self) -> int:
        """The most keys one rank's step routes (chunks x chunk_keys)."""
        return self.chunks * self.chunk_keys if self._exact is None else 1 << 62

    # ---- ownership ------------------------------------------------------------------------
    def owned_parts(self) -> list[int]:
        """Global indices of this rank's parts (round-robin: part j * world + rank)."""
        return [j * self.world + self.rank for j in range(self.g)]

    def part_tiles(self, p: int) -> tuple[int, int]:
        b = min(self.T, p * self.q)
        return b, min(self.T, b + self.q)

    @property
    def _collective(self) -> bool:
        import torch.distributed as dist
        return self.world > 1 or (dist.is_available() and dist.is_initialized())

    @property
    def _gloo(self) -> bool:
        import torch.distributed as dist
        return dist.get_backend(self.group) != "nccl"

    def _exact_builder(self):
        """The exact exchange (built once, on first use: its buffers are reused)."""
        if self._exact is None:
            self._exact = ExactHashShardedBloom(self.n_total_keys, self.bpk, self.world, self.rank,
                                                self.dev, self.src_page_id, self.group)
        return self._exact

    # ---- the stages -----------------------------------------------------------------------
    def recv_round(self, j: int):
        """Round j's received blocks ([chunk][sender], C * W blocks)."""
        n = self.chunks * self.world * self.block_bytes
        return self.recv[j * n:(j + 1) * n]

    def route_chunk(self, keys, c: int):
        """Chunk c of this rank's keys ([n, 16] or [n, 24] uint8 on the device) into send[c]
        (world 1: into recv at [j][c])."""
        import ctypes

        from . import abi
        from .filters import _ptr, _stream_handle
        kb = keys.shape[1] if keys.dim() == 2 else 0
        if kb not in (16, 24):
            raise abi.TkvAmqError(abi.INVALID_ARGUMENT, "hash-range sharding takes [n, 16] or "
                                  f"[n, 24] uint8 keys, got shape {tuple(keys.shape)}")
        if keys.shape[0] > self.capacity:
            raise abi.TkvAmqError(abi.INVALID_ARGUMENT, f"{keys.shape[0]} keys on rank {self.rank}: "
                                  f"the plan routes at most {self.capacity} (max_keys_per_rank)")
        ck = self.chunk_keys
        part = keys[c * ck:(c + 1) * ck]
        n = part.shape[0]
        B = self.block_bytes
        if self.world == 1:
            dst, stride = self.recv[c * B:], self.chunks * B
        else:
            dst, stride = self.send[c], 0
        abi.check(abi.lib().tkv_amq_bloom_route_blocks(_ptr(part) if n else None, kb, n, _ptr(self.d_seg),
                                                       ctypes.byref(self.rp), _ptr(dst), stride,
                                                       _ptr(self.route_ws), self.route_ws.numel(),
                                                       _stream_handle()), "tkv_amq_bloom_route_blocks")

    def exchange(self, c: int, j: int):
        """All-to-all of round j of chunk c (one block of block_bytes per peer), on the current
        stream, into recv at [j][c][sender]."""
        import torch
        import torch.distributed as dist
        if self.world == 1:
            return  # routed straight into recv
        B, W, C = self.block_bytes, self.world, self.chunks
        dst = self.recv[(j * C + c) * W * B:(j * C + c + 1) * W * B]
        src = self.send[c][j * W * B:(j + 1) * W * B]
        if self._gloo:  # CPU rehearsal: stage through host memory
            host = torch.empty(W * B, dtype=torch.uint8)
            dist.all_to_all_single(host, src.cpu(), group=self.group)
            dst.copy_(host)
        else:
            dist.all_to_all_single(dst, src, group=self.group)

    def exchange_chunk(self, c: int):
        """Every round of chunk c."""
        for j in range(self.g):
            self.exchange(c, j)

    def build_part(self, j: int):
        """This rank's j-th part (global part j * world + rank) from its round's blocks."""
        import ctypes

        from . import abi
        from .filters import _ptr, _stream_handle
        L = abi.lib()
        S = self.chunks * self.world
        abi.check(L.tkv_amq_bloom_build_part_blocks(_ptr(self.recv_round(j)), S, _ptr(self.d_seg),
                                                    ctypes.byref(self.rp), j * self.world + self.rank,
                                                    _ptr(self.out), _ptr(self.part_ws),
                                                    self.part_ws.numel(), _stream_handle()),
                  "tkv_amq_bloom_build_part_blocks")

    def gather_round(self, j: int):
        """Round j (part j of every rank, contiguous) all-gathered in place."""
        import torch
        import torch.distributed as dist
        R = self.round_bytes
        rnd = self.out[64 + j * R:64 + (j + 1) * R]
        mine = rnd[self.rank * self.part_bytes:(self.rank + 1) * self.part_bytes]
        if self._gloo:
            host = torch.empty(R, dtype=torch.uint8)
            dist.all_gather_into_tensor(host, mine.cpu(), group=self.group)
            rnd.copy_(host)
        else:
            dist.all_gather_into_tensor(rnd, mine, group=self.group)

    # ---- the step -------------------------------------------------------------------------
    def step(self, keys, gather: bool = True, timeline: bool = False):
        """route -> exchange -> part builds (-> gathers), pipelined over two streams; on return
        the current stream is ordered after all of it (this rank's parts final, and with
        gather every part on every rank).  timeline=True records timing events at every stage
        boundary (`timeline_ms()` reads them after a synchronisation).

        Communication-stream order (the same on every rank): the rounds of chunks 0..C-2 as
        their routes finish, then X(0) X(1) X(2) G(0) X(3) G(1) ... X(g-1) G(g-3) G(g-2) G(g-1),
        X(j) the last chunk's round j and G(j) the gather of round j; the compute stream builds
        part j as soon as X(j) has landed."""
        import torch
        if self._exact is not None:
            self._exact.local_build(keys)
            if gather:
                self._exact_out = self._exact.allgather()
            return
        self.last_fallback = None
        coll = self._collective and self.comm is not None
        xch = coll and self.world > 1
        cur = torch.cuda.current_stream(self.dev)
        tl = {} if timeline else None

        def mark(name, stream):
            if tl is not None:
                e = torch.cuda.Event(enable_timing=True)
                e.record(stream)
                tl[name] = e

        mark("start", cur)
        self._direct = (self._direct_ok and not self._collective and self.T <= KEY_RANGE_MAX_TILES
                        and keys.dim() == 2
                        and keys.shape[1] == 16)
        if self._direct:
            # one GPU, no process group, a filter one partition takes whole: no route, no
            # blocks (the range build hashes the keys into its records itself)
            self._direct_build(keys)
            mark("build_direct", cur)
            mark("end", cur)
            self.timeline = tl
            return
        if coll:
            self.comm.wait_stream(cur)  # the previous step's readers are done
        C, g = self.chunks, self.g
        for c in range(C):
            self.route_chunk(keys, c)
            mark(f"route_{c}", cur)
            if xch:
                ev = torch.cuda.Event()
                ev.record(cur)
                with torch.cuda.stream(self.comm):
                    self.comm.wait_event(ev)
                    if c < C - 1:  # every round of an early chunk as soon as it is routed
                        self.exchange_chunk(c)
                        mark(f"exchange_chunk_{c}", self.comm)
        x_ev = [None] * g
        b_ev = [None] * g

        def exchange_last(j):  # the last chunk's round j, on the communication stream
            with torch.cuda.stream(self.comm):
                self.exchange(C - 1, j)
                mark(f"exchange_{j}", self.comm)
                x_ev[j] = torch.cuda.Event()
                x_ev[j].record(self.comm)

        def gather_after_build(j):
            with torch.cuda.stream(self.comm):
                self.comm.wait_event(b_ev[j])
                self.gather_round(j)
                mark(f"gather_{j}", self.comm)

        if xch:
            for j in range(min(2, g)):
                exchange_last(j)
        for j in range(g):
            if xch:
                cur.wait_event(x_ev[j])
            mark(f"build_{j}_start", cur)
            self.build_part(j)
            mark(f"build_{j}", cur)
            if coll and gather:
                b_ev[j] = torch.cuda.Event()
                b_ev[j].record(cur)
            if xch and j + 2 < g:
                exchange_last(j + 2)
            if coll and gather and j >= 1:
                gather_after_build(j - 1)
        if coll and gather and g:
            gather_after_build(g - 1)
        if coll:
            cur.wait_stream(self.comm)
        mark("end", cur)
        self.timeline = tl

    def _direct_build(self, keys):
        """The whole filter from the keys by one range build (tkv_amq_bloom_build_range)."""
        import torch

        from . import abi
        from .filters import _ptr, _stream_handle
        L = abi.lib()
        n = keys.shape[0]
        if keys.shape[0] > self.capacity:
            raise abi.TkvAmqError(abi.INVALID_ARGUMENT, f"{n} keys: the plan routes at most {self.capacity}")
        need = int(L.tkv_amq_bloom_build_range_ws_bytes(n, 0, self.T))
        if self._direct_ws is None or self._direct_ws.numel() < need:
            self._direct_ws = torch.empty(max(need, 1), dtype=torch.uint8, device=self.dev)
        abi.check(L.tkv_amq_bloom_build_range(_ptr(keys) if n else None, n, _ptr(self.d_seg), self.n_blocks, 0,
                                              self.T, _ptr(self.out), _ptr(self._direct_ws),
                                              self._direct_ws.numel(), _stream_handle()),
                  "tkv_amq_bloom_build_range")

    def timeline_ms(self) -> dict:
        """Milliseconds from the step's start to each recorded stage end (after a step with
        timeline=True and a synchronisation)."""
        if not self.timeline:
            return {}
        t0 = self.timeline["start"]
        return {k: round(t0.elapsed_time(e), 4) for k, e in self.timeline.items() if k != "start"}

    def local_build(self, keys):
        """route + exchange + part builds: this rank's parts of the bitmap are final."""
        self.step(keys, gather=False)

    def allgather(self):
        """Every round all-gathered (after local_build) -> the whole payload on every rank."""
        if not self.records:
            return self._exact.allgather()
        if self._collective:
            for j in range(self.g):
                self.gather_round(j)
        return self.filter()

    def filter(self):
        """The filter payload (header + bitmap) of the last step: a view of this builder's
        buffer, overwritten by its next step (build() returns a copy)."""
        if not self.records:
            return self._exact_out
        if self.last_fallback is not None:
            return self._fallback_out
        return self.out[:self.payload_bytes]

    def lost(self) -> bool:
        """Did any block of the last exchange lose overflow entries (synchronises)?"""
        import ctypes

        from . import abi
        from .filters import _ptr, _stream_handle
        if not self.records or self._direct:
            return False
        r = abi.lib().tkv_amq_bloom_blocks_lost(_ptr(self.recv), self.g * self.chunks * self.world,
                                                ctypes.byref(self.rp), _stream_handle())
        if r < 0:
            raise abi.TkvAmqError(-r, "tkv_amq_bloom_blocks_lost")
        self.last_lost = bool(r)
        return self.last_lost

    def _any_rank(self, flag: bool) -> bool:
        """MAX of a flag over the ranks (every rank takes the same path)."""
        import torch
        import torch.distributed as dist
        if not self._collective:
            return flag
        t = torch.tensor([1 if flag else 0], dtype=torch.int32,
                         device="cpu" if self._gloo else self.dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return bool(t.item())

    def build(self, keys):
        """The whole filter on every rank, as a new tensor.  A rank holding more keys than the
        plan's chunks take, or a step that lost overflow entries (each decided together by
        every rank), is built through the exact exchange instead."""
        if not self.records:
            self.step(keys, gather=True)
            return self._exact_out.clone()
        self.last_fallback = None
        if self._any_rank(keys.shape[0] > self.capacity):
            self.last_fallback = "keys_over_capacity"
        else:
            self.step(keys, gather=True)
            if self._any_rank(self.lost()):
                self.last_fallback = "overflow_lost"
        if self.last_fallback is not None:
            self._fallback_out = self._exact_builder().build(keys)
        return self.filter().clone()
