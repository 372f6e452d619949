"""CPU, world_size 2, 3 and 8 (gloo): the leaf-sharded multi-GPU layout.  Each rank builds its own
leaf range (here with the CPU oracle standing in for the GPU build, since the property
under test is the sharding/layout/all-gather logic), all-gathers its fixed-size slice, and
the gathered array must equal a single-process build of every leaf at the same stride."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def oracle_build(O, kind, keys, counts, bpk, cap, stride, leaf_ids, n_slots):
    counts = np.asarray(counts, dtype=np.int64)
    sb = np.concatenate([[0], np.cumsum(counts)]).astype(np.uint64)
    offs = (np.arange(len(counts)) * stride).astype(np.uint64)
    caps = np.full(len(counts), stride if kind == 0 else cap, np.uint64)
    out = np.zeros(n_slots * stride, np.uint8)
    st, out = O.build_segments(kind, keys, sb, bpk, offs, caps, 0,
                               src_page_id=np.asarray(leaf_ids, np.uint64), out=out)
    assert st == 0
    return out


def worker(rank, world, port, kind, result_q):
    import sys
    sys.path.insert(0, ROOT)
    from oracle import oracle as O
    from turtle_kv_amd import dist as tdist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    counts = [4096] * 9 + [1000]
    bpk, cap = (10, 0) if kind == 0 else (12, 16320)
    keys = O.gen_keys16(42, 0, sum(counts))
    if kind == 1:
        O.sort_segments(keys, np.concatenate([[0], np.cumsum(counts)]).astype(np.uint64))
    stride = tdist.leaf_stride(kind, bpk, max(counts), cap)
    sh = tdist.shard_leaves(counts, world, rank)
    plan = tdist.plan_shard(kind, counts, bpk, sh, stride, payload_capacity=cap)
    assert list(plan.segs["src_page_id"]) == list(range(sh.leaf_begin, sh.leaf_end))
    assert sh.n_leaves == 0 or int(plan.segs["key_begin"][0]) == 0
    local = oracle_build(O, kind, keys[sh.key_begin:sh.key_end], counts[sh.leaf_begin:sh.leaf_end],
                         bpk, cap, stride, range(sh.leaf_begin, sh.leaf_end), sh.leaves_per_rank)
    g = tdist.allgather_filters(torch.from_numpy(local))
    if rank == 0:
        full = oracle_build(O, kind, keys, counts, bpk, cap, stride, range(len(counts)),
                            sh.leaves_per_rank * world)
        result_q.put(bool(np.array_equal(g.numpy(), full)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("kind,world", [(0, 2), (1, 2), (0, 3), (1, 8)])
def test_sharded_allgather(kind, world):
    """world 3: ragged shards (4, 4, 2 leaves); world 8 (the driver's node size): ranks 5-7
    own no leaf and contribute an unwritten slice."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, kind, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=5) is True


def test_shard_ranges_cover_all_leaves():
    from turtle_kv_amd import dist as tdist
    counts = [16384] * 6103 + [8448]
    for world in (1, 2, 3, 4, 8):
        shards = [tdist.shard_leaves(counts, world, r) for r in range(world)]
        assert shards[0].leaf_begin == 0 and shards[-1].leaf_end == len(counts)
        for a, b in zip(shards, shards[1:]):
            assert a.leaf_end == b.leaf_begin and a.key_end == b.key_begin
        assert shards[-1].key_end == sum(counts)
        assert all(s.n_leaves <= s.leaves_per_rank for s in shards)


def test_hash_shard_tiles_cover_the_filter():
    """Hash-range sharding (config 5 read literally): the ranks' tile ranges are contiguous,
    disjoint and cover every tile.  With ceil(T/q) < ranks the last ranks own an empty range
    (T = 17 over 8 ranks: q = 3, ranks 6 and 7; 2 tiles over 8 ranks: ranks 2-7): they are
    accepted, and their range build writes the header only (GPU test
    test_gpu_hash_shard.py::test_empty_ranges_write_the_header)."""
    from turtle_kv_amd import abi
    from turtle_kv_amd.dist import BLOOM_TILE_BLOCKS as TB, ExactHashShardedBloom, hash_shard_tiles
    for nb, world in [(1, 1), (TB, 1), (TB + 1, 2), (93750, 8), (2_343_750, 8), (29297, 8),
                      (17 * TB, 8), (3000, 8)]:
        T, q = hash_shard_tiles(nb, world)
        assert T == -(-nb // TB)
        ranges = [(min(T, r * q), min(T, (r + 1) * q)) for r in range(world)]
        assert ranges[0][0] == 0 and ranges[-1][1] == T
        assert all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))
    T, q = hash_shard_tiles(17 * TB, 8)
    assert (T, q) == (17, 3)
    empty = [r for r in range(8) if min(T, r * q) == min(T, (r + 1) * q)]
    assert empty == [6, 7]
    hs = ExactHashShardedBloom(100_000, 12, 8, 5, "cpu")   # 2 tiles over 8 ranks: rank 5 owns none
    assert hs.T == 2 and hs.tile_begin == hs.tile_end == 2
    with pytest.raises(abi.TkvAmqError, match="got shape"):
        hs.route(torch.zeros((10, 20), dtype=torch.uint8))   # 16- or 24-byte keys only
    hk = ExactHashShardedBloom(100_000, 16, 8, 0, "cpu")    # k = 11: keys travel, 16 bytes only
    assert not hk.records
    with pytest.raises(abi.TkvAmqError, match="got shape"):
        hk.route(torch.zeros((10, 24), dtype=torch.uint8))
    with pytest.raises(abi.TkvAmqError, match="got shape"):
        hk.build_range(torch.zeros((10, 24), dtype=torch.uint8))   # the range build: 16 only


def test_hash_shard_parts_per_rank():
    """A rank's range is cut into g parts of at most 256 tiles of bit records
    (ROUTED_PART_TILES) or 1,600 of routed keys (ROUTED_KEY_PART_TILES), under the 6,400 of one
    range build's LDS tile table: BASELINE config 5 (1B keys at 12 bits/key, 11,445 tiles)
    builds 45 parts of 255 tiles on one rank, 23 of 249 on each of two, 6 of 239 on each of eight; the
    parts of all ranks tile the filter, and rank r's range is its parts' union."""
    from turtle_kv_amd.dist import (ROUTED_KEY_PART_TILES, ROUTED_PART_TILES, ExactHashShardedBloom,
                                    hash_shard_plan)
    nb_1b = -(-1_000_000_000 * 12 // 512)
    assert hash_shard_plan(nb_1b, 1) == (11445, 45, 255)
    assert hash_shard_plan(nb_1b, 2)[1:] == (23, 249)
    assert hash_shard_plan(nb_1b, 4)[1:] == (12, 239)
    assert hash_shard_plan(nb_1b, 8)[1:] == (6, 239)
    assert hash_shard_plan(nb_1b, 1, records=False) == (11445, 8, 1431)
    for nb in [1, 5000, nb_1b, 3 * nb_1b, 40_000_000 * 2048]:
        for world in [1, 2, 3, 8]:
            for rec in (True, False):
                T, g, q = hash_shard_plan(nb, world, rec)
                assert q <= (ROUTED_PART_TILES if rec else ROUTED_KEY_PART_TILES)
                parts = [(min(T, p * q), min(T, (p + 1) * q)) for p in range(world * g)]
                assert parts[0][0] == 0 and parts[-1][1] == T
                assert all(a[1] == b[0] for a, b in zip(parts, parts[1:]))
    hs = ExactHashShardedBloom(1_000_000_000, 12, 2, 1, "meta")
    assert (hs.g, hs.q, hs.tile_begin, hs.tile_end) == (23, 249, 5727, 11445)
    assert hs.part_tiles(0) == (5727, 5976) and hs.part_tiles(22) == (11205, 11445)


@pytest.mark.parametrize("world,chunks", [(1, 1), (2, 1), (8, 4), (3, 2)])
def test_pipelined_hash_shard_plan(world, chunks):
    """The pipelined form (tkv_amq_bloom_route_plan, a host function): the same parts as the
    exact form at config 5's size, owned round-robin (part p by rank p % world, so round j --
    part j of every rank -- is one contiguous byte range of the bitmap, gathered in place);
    every part is owned once; fixed-size blocks whose regions hold mean + 6 sigma + 16 records of
    a uniform hash; a rank's recv buffer holds chunks x world blocks."""
    from turtle_kv_amd.dist import HashShardedBloom, hash_shard_plan
    nb_1b = -(-1_000_000_000 * 12 // 512)
    owners = {}
    for r in range(world):
        hs = HashShardedBloom(1_000_000_000, 12, world, r, "meta", chunks=chunks)
        assert (hs.T, hs.g, hs.q) == hash_shard_plan(nb_1b, world)
        rp = hs.rp
        assert rp.n_parts == world * hs.g and rp.world == world and rp.n_chunks == chunks
        for p in hs.owned_parts():
            assert p % world == r and p not in owners
            owners[p] = r
        # round j's blocks at [j][chunk][sender]; a chunk's send buffer: every part's block
        assert hs.recv.numel() == hs.g * chunks * world * rp.block_bytes
        assert hs.recv_round(1).data_ptr() - hs.recv_round(0).data_ptr() == chunks * world * rp.block_bytes
        if world > 1:
            assert all(b.numel() == rp.n_parts * rp.block_bytes for b in hs.send)
        assert hs.out.numel() == 64 + rp.n_parts * rp.part_bytes >= hs.payload_bytes
        e = -(-hs.chunk_keys // rp.route_wgs) * min(hs.q * 2048, nb_1b) / nb_1b   # a region's share
        ns = 2 if world > 1 else 6   # (one rank sends nothing over xGMI: 6 sigma)
        assert e + ns * e ** 0.5 <= rp.region_cap <= e + ns * e ** 0.5 + 32
        assert rp.regions_off + 12 * rp.route_wgs * rp.region_cap <= rp.ovf_off
        assert rp.ovf_off + 16 * rp.ovf_cap <= rp.block_bytes and rp.block_bytes % 256 == 0
        # what crosses xGMI beside the records themselves: 2 sigma per region (the few records
        # past it travel as overflow entries), the overflow area and the counts (round 5's
        # 6-sigma regions: 14% at config 5's size on eight ranks)
        if world == 8:
            assert rp.block_bytes <= 1.07 * 12 * e * rp.route_wgs, (rp.block_bytes, 12 * e * rp.route_wgs)
    assert sorted(owners) == list(range(world * hs.g))
    tiles = sorted(hs.part_tiles(p) for p in owners)
    assert tiles[0][0] == 0 and tiles[-1][1] == hs.T
    assert all(a[1] == b[0] for a, b in zip(tiles, tiles[1:]))
    # k > 8: 16-byte keys travel through the exact form
    hk = HashShardedBloom(100_000, 16, world, 0, "cpu")
    assert not hk.records and hk._exact is not None


def test_build_owned_regroups_parts():
    """With g > 1 parts per rank the all-to-all delivers, per sender, that sender's units for
    each of this rank's parts in order; build_owned hands part j all senders' pieces of it."""
    from turtle_kv_amd.dist import ExactHashShardedBloom
    hs = ExactHashShardedBloom.__new__(ExactHashShardedBloom)
    got = []
    hs._build_part = lambda units, j: got.append((j, units.tolist()))
    W, g = 3, 2
    sub = torch.tensor([[2, 1], [0, 3], [1, 0]])     # sender s sent sub[s, j] units of part j
    owned = torch.arange(int(sub.sum()))
    hs.build_owned(owned, sub)
    # sender 0: [0 1 | 2], sender 1: [ | 3 4 5], sender 2: [6 | ]
    assert got == [(0, [0, 1, 6]), (1, [2, 3, 4, 5])]
    got.clear()
    hs.build_owned(owned[:5], torch.tensor([[5]]))
    assert got == [(0, [0, 1, 2, 3, 4])]


def test_cyclic_rounds_cover_leaves_in_order():
    """Round c of every rank, concatenated rank by rank, is one contiguous leaf range, and the
    rounds in order cover every leaf once: what lets each round's all-gather land in place."""
    from turtle_kv_amd import dist as tdist
    for n, world, q in [(10, 2, 2), (10, 3, 1), (6104, 8, 191), (7, 8, 1), (0, 2, 4), (5, 2, 8)]:
        per = [tdist.cyclic_rounds(n, world, r, q) for r in range(world)]
        assert len({len(p) for p in per}) == 1
        flat = [rng for c in range(len(per[0])) for r in range(world) for rng in [per[r][c]]]
        pos = 0
        for b, e in flat:
            assert b == pos or b == e == n
            pos = e
            assert e - b <= q
        assert pos == n


def cyclic_worker(rank, world, port, kind, q_leaves, result_q):
    """Rank r builds its block-cyclic rounds (the oracle standing in for the GPU build) and
    all-gathers round c into bytes [c*W*Q*stride, (c+1)*W*Q*stride) of the array, as
    PipelinedLeafGather does on its communication stream."""
    import sys
    sys.path.insert(0, ROOT)
    from oracle import oracle as O
    from turtle_kv_amd import dist as tdist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    counts = [4096] * 9 + [1000]
    bpk, cap = (10, 0) if kind == 0 else (12, 16320)
    keys = O.gen_keys16(42, 0, sum(counts))
    sb = np.concatenate([[0], np.cumsum(counts)])
    if kind == 1:
        O.sort_segments(keys, sb.astype(np.uint64))
    stride = tdist.leaf_stride(kind, bpk, max(counts), cap)
    rounds = tdist.cyclic_rounds(len(counts), world, rank, q_leaves)
    rb = q_leaves * stride
    gathered = torch.zeros(len(rounds) * world * rb, dtype=torch.uint8)
    for c, (b, e) in enumerate(rounds):
        local = np.zeros(rb, np.uint8)
        if e > b:
            local = oracle_build(O, kind, keys[sb[b]:sb[e]], counts[b:e], bpk, cap, stride,
                                 range(b, e), q_leaves)
        tdist.allgather_filters(torch.from_numpy(local), gathered[c * world * rb:(c + 1) * world * rb])
    if rank == 0:
        full = oracle_build(O, kind, keys, counts, bpk, cap, stride, range(len(counts)),
                            len(counts))
        result_q.put(bool(np.array_equal(gathered.numpy()[:len(counts) * stride], full)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("kind,world,q", [(0, 2, 2), (1, 2, 3), (0, 3, 1)])
def test_cyclic_round_allgather(kind, world, q):
    """The pipelined all-gather's layout: rounds gathered one by one give the leaf-ordered
    array a single-process build writes (ragged last round, ranks with empty rounds)."""
    ctx = mp.get_context("spawn")
    rq = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=cyclic_worker, args=(r, world, port, kind, q, rq))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert rq.get(timeout=5) is True


def test_hash_shard_build_falls_back_past_capacity():
    """a rank holding more keys than its plan's chunks take (an uneven split
    with the default max_keys_per_rank) must not lose keys: build() decides over every rank and
    takes the exact exchange; step() refuses such keys rather than routing a prefix of them."""
    from turtle_kv_amd import abi
    from turtle_kv_amd.dist import HashShardedBloom
    hs = HashShardedBloom(1_000_000, 12, 2, 0, "meta", chunks=2)
    assert hs.capacity == 2 * hs.chunk_keys == 500_000   # the even share of 2 ranks
    keys = torch.empty((600_000, 16), dtype=torch.uint8, device="meta")
    hs._any_rank = lambda flag: flag   # (no process group here: this rank's flag decides)
    calls = []

    class Exact:
        def build(self, k):
            calls.append(k.shape[0])
            return torch.zeros(8, dtype=torch.uint8)
    hs._exact_builder = lambda: Exact()

    def no_step(*a, **kw):
        raise AssertionError("the pipelined step must not run past the plan's capacity")
    hs.step = no_step
    out = hs.build(keys)
    assert hs.last_fallback == "keys_over_capacity" and calls == [600_000] and out.numel() == 8
    # another rank over capacity decides for this one too
    hs._any_rank = lambda flag: True
    hs.build(torch.empty((10, 16), dtype=torch.uint8, device="meta"))
    assert hs.last_fallback == "keys_over_capacity"
    # step() itself refuses (route_chunk) instead of dropping keys
    hs2 = HashShardedBloom(1_000_000, 12, 2, 0, "meta", chunks=2)
    with pytest.raises(abi.TkvAmqError):
        hs2.route_chunk(keys, 0)
