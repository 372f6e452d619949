"""Hash-range sharding of one monolithic Bloom filter (BASELINE config 5 read literally):
tkv_amq_bloom_route + tkv_amq_bloom_build_range through the C ABI on one GPU (the parts
played in turn), the rank-side orchestration (turtle_kv_amd.dist.HashShardedBloom) through
bench.py with two gloo ranks sharing the box's GPU, and the degenerate one-rank case.  The
assembled filter must equal the one-GPU monolithic build and the CPU oracle."""
import numpy as np
import pytest

from test_gpu_bench import SMALL, last_json, run_bench

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need a visible MI355X"
    return t


def _route(amq, torch, keys, plan, n_parts):
    from turtle_kv_amd.filters import _ptr, _stream_handle
    L = amq.abi.lib()
    n = keys.shape[0]
    nb = int(plan.segs[0]["n_blocks"])
    routed = torch.empty_like(keys)
    counts = torch.zeros(n_parts, dtype=torch.int32, device="cuda")
    ws = torch.empty(int(L.tkv_amq_bloom_route_ws_bytes(n, n_parts)), dtype=torch.uint8, device="cuda")
    amq.abi.check(L.tkv_amq_bloom_route(_ptr(keys), n, _ptr(plan.device_segs()), nb, n_parts,
                                        _ptr(routed), _ptr(counts), _ptr(ws), ws.numel(),
                                        _stream_handle()), "route")
    torch.cuda.synchronize()
    return routed, counts.cpu().numpy().astype(np.int64)


def _build_range(amq, torch, keys, plan, t0, t1, out):
    from turtle_kv_amd.filters import _ptr, _stream_handle
    L = amq.abi.lib()
    n = keys.shape[0]
    ws = torch.empty(max(1, int(L.tkv_amq_bloom_build_range_ws_bytes(n, t0, t1))), dtype=torch.uint8,
                     device="cuda")
    amq.abi.check(L.tkv_amq_bloom_build_range(_ptr(keys), n, _ptr(plan.device_segs()),
                                              int(plan.segs[0]["n_blocks"]), t0, t1, _ptr(out),
                                              _ptr(ws), ws.numel(), _stream_handle()), "build_range")


@pytest.mark.parametrize("n_keys,bpk,n_parts,dup", [(3_000_000, 12, 3, 0), (1_500_001, 10, 8, 0),
                                                   (700_000, 12, 1, 0), (2_000_000, 12, 4, 600_000),
                                                   (400_000, 16, 2, 0)])
def test_route_and_range_build_equal_monolithic(oracle, amq, torch, n_keys, bpk, n_parts, dup):
    """dup: that many copies of one key (its tile's regions overflow: the record path's
    overflow lists, applied with tile0 > 0 on most ranks); bpk 16: k = 11 > 8, the ranges
    partition the 16-byte keys themselves and hash them per tile."""
    from turtle_kv_amd.dist import hash_shard_tiles
    keys = amq.gen_keys16(11, 0, n_keys)
    if dup:
        keys[n_keys - dup:] = keys[n_keys // 3]
    plan = amq.plan_filters(0, [n_keys], bpk)
    nb = int(plan.segs[0]["n_blocks"])
    assert 64 * nb > 4 * 160 * 1024, "must take the tiled monolithic build"
    whole = amq.build_all_filters(plan, amq.KeyBatch.fixed(keys))
    routed, counts = _route(amq, torch, keys, plan, n_parts)
    assert counts.sum() == n_keys
    # the route is a permutation of the keys
    a = np.sort(keys.cpu().numpy().view("<u8").reshape(-1, 2), axis=0)
    b = np.sort(routed.cpu().numpy().view("<u8").reshape(-1, 2), axis=0)
    assert np.array_equal(a, b)
    T, q = hash_shard_tiles(nb, n_parts)
    out = torch.zeros(plan.total_out_bytes, dtype=torch.uint8, device="cuda")
    base = np.concatenate([[0], np.cumsum(counts)])
    for p in range(n_parts):
        part = routed[int(base[p]):int(base[p + 1])]
        _build_range(amq, torch, part, plan, min(T, p * q), min(T, (p + 1) * q), out)
    torch.cuda.synchronize()
    assert torch.equal(out, whole)
    st, ref = oracle.bloom_build(keys.cpu().numpy(), n_keys, bpk, src_page_id=0)
    assert st == 0 and out.cpu().numpy().tobytes() == ref.tobytes()


def test_range_build_ignores_keys_outside_its_tiles(amq, torch):
    """Handing a rank every key (not just the routed ones) builds the same range: keys of
    other ranks' tiles are skipped."""
    n = 2_000_000
    keys = amq.gen_keys16(12, 0, n)
    plan = amq.plan_filters(0, [n], 12)
    from turtle_kv_amd.dist import hash_shard_tiles
    T, q = hash_shard_tiles(int(plan.segs[0]["n_blocks"]), 4)
    whole = amq.build_all_filters(plan, amq.KeyBatch.fixed(keys))
    out = torch.zeros(plan.total_out_bytes, dtype=torch.uint8, device="cuda")
    _build_range(amq, torch, keys, plan, q, 2 * q, out)
    torch.cuda.synchronize()
    from turtle_kv_amd.dist import BLOOM_TILE_BLOCKS as TB
    lo, hi = 64 + 64 * TB * q, 64 + 64 * TB * 2 * q
    assert torch.equal(out[lo:hi], whole[lo:hi])
    assert torch.equal(out[:64], whole[:64])          # the header, from every range
    assert int(out[64:lo].count_nonzero()) == 0       # other ranges untouched
    assert int(out[hi:].count_nonzero()) == 0


def test_bench_hash_sharded_two_ranks_gloo():
    r = run_bench("--gpus", "2", "--backend", "gloo", "--workload", "bloom12hash",
                  "--keys-per-gpu", "2000000", *SMALL)
    assert r.returncode == 0, r.stderr[-4000:]
    d = last_json(r)
    assert d["n_gpus"] == 2 and d["config"]["total_keys"] == 4_000_000
    assert d["verified"] is True
    assert d["verify"]["equal_to_oracle"] and d["verify"]["header_ok"]
    assert d["config"]["chunks"] == 4 and d["config"]["allgather_in_step"] is True
    assert d["route_plan"]["overflow_lost"] is False
    b = d["step_breakdown_rank0_ms"]
    assert b["route"] > 0 and b["all_to_all"] > 0 and b["part_builds"] > 0 and b["allgather"] > 0


def test_bench_hash_sharded_one_rank():
    r = run_bench("--workload", "bloom12hash", "--keys-per-gpu", "3000000", *SMALL)
    assert r.returncode == 0, r.stderr[-4000:]
    d = last_json(r)
    assert d["n_gpus"] == 1 and d["verified"] is True


def test_empty_ranges_write_the_header(amq, torch):
    """T = 17 tiles over 8 ranks: q = 3, so ranks 6 and 7 own no tile.  They receive no keys
    from the route, and their range build still writes the whole filter header, so every
    rank's assembled result (its own header + the gathered ranges) equals the one-GPU build."""
    from turtle_kv_amd.dist import hash_shard_tiles
    n, world = 1_440_000, 8
    keys = amq.gen_keys16(13, 0, n)
    plan = amq.plan_filters(0, [n], 12)
    T, q = hash_shard_tiles(int(plan.segs[0]["n_blocks"]), world)
    assert (T, q) == (17, 3)
    whole = amq.build_all_filters(plan, amq.KeyBatch.fixed(keys))
    routed, counts = _route(amq, torch, keys, plan, world)
    assert counts[6] == 0 and counts[7] == 0 and counts.sum() == n
    base = np.concatenate([[0], np.cumsum(counts)])
    outs = []
    for r in range(world):
        out = torch.zeros(plan.total_out_bytes, dtype=torch.uint8, device="cuda")
        _build_range(amq, torch, routed[int(base[r]):int(base[r + 1])], plan, min(T, r * q),
                     min(T, (r + 1) * q), out)
        outs.append(out)
    torch.cuda.synchronize()
    for r in range(world):
        assert torch.equal(outs[r][:64], whole[:64]), f"rank {r}'s header"
    merged = outs[0].clone()
    for r in range(1, world):
        merged |= outs[r]
    assert torch.equal(merged, whole)


def _route_records(amq, torch, keys, plan, n_parts):
    from turtle_kv_amd.filters import _ptr, _stream_handle
    L = amq.abi.lib()
    n = keys.shape[0]
    seg = plan.segs[0]
    recs = torch.empty((n, 12), dtype=torch.uint8, device="cuda")
    counts = torch.zeros(n_parts, dtype=torch.int32, device="cuda")
    ws = torch.empty(int(L.tkv_amq_bloom_route_records_ws_bytes(n, n_parts)), dtype=torch.uint8,
                     device="cuda")
    amq.abi.check(L.tkv_amq_bloom_route_records(_ptr(keys), n, _ptr(plan.device_segs()),
                                                int(seg["n_blocks"]), int(seg["hash_count"]), n_parts,
                                                _ptr(recs), _ptr(counts), _ptr(ws), ws.numel(),
                                                _stream_handle()), "route_records")
    torch.cuda.synchronize()
    return recs, counts.cpu().numpy().astype(np.int64)


def _build_range_records(amq, torch, recs, plan, t0, t1, out):
    from turtle_kv_amd.filters import _ptr, _stream_handle
    L = amq.abi.lib()
    m = recs.shape[0]
    seg = plan.segs[0]
    ws = torch.empty(max(1, int(L.tkv_amq_bloom_build_range_records_ws_bytes(m, t0, t1))),
                     dtype=torch.uint8, device="cuda")
    amq.abi.check(L.tkv_amq_bloom_build_range_records(_ptr(recs) if m else None, m,
                                                      _ptr(plan.device_segs()), int(seg["n_blocks"]),
                                                      int(seg["hash_count"]), t0, t1, _ptr(out),
                                                      _ptr(ws), ws.numel(), _stream_handle()),
                  "build_range_records")


@pytest.mark.parametrize("n_keys,bpk,n_parts,dup", [(3_000_000, 12, 3, 0), (1_500_001, 10, 8, 0),
                                                   (700_000, 12, 1, 0), (2_000_000, 12, 4, 600_000),
                                                   (1_440_000, 12, 8, 0), (900_000, 5, 2, 0)])
def test_route_records_and_range_build_equal_monolithic(oracle, amq, torch, n_keys, bpk, n_parts, dup):
    """The record form of hash-range sharding (k <= 8): every key hashed once by its sender into
    a 12-byte bit record with its tile relative to its owner; each owner builds its tiles from
    the records alone.  Equal to the one-GPU build and the oracle: k = 8, 7 and 3, duplicate
    keys (one tile's regions overflow), ranks past the last tile (1.44M keys: 17 tiles over 8)."""
    from turtle_kv_amd.dist import hash_shard_tiles
    keys = amq.gen_keys16(21, 0, n_keys)
    if dup:
        keys[n_keys - dup:] = keys[n_keys // 3]
    plan = amq.plan_filters(0, [n_keys], bpk)
    assert int(plan.segs[0]["hash_count"]) <= 8
    whole = amq.build_all_filters(plan, amq.KeyBatch.fixed(keys))
    recs, counts = _route_records(amq, torch, keys, plan, n_parts)
    assert counts.sum() == n_keys
    T, q = hash_shard_tiles(int(plan.segs[0]["n_blocks"]), n_parts)
    out = torch.zeros(plan.total_out_bytes, dtype=torch.uint8, device="cuda")
    base = np.concatenate([[0], np.cumsum(counts)])
    for p in range(n_parts):
        _build_range_records(amq, torch, recs[int(base[p]):int(base[p + 1])], plan, min(T, p * q),
                             min(T, (p + 1) * q), out)
    torch.cuda.synchronize()
    assert torch.equal(out, whole)
    st, ref = oracle.bloom_build(keys.cpu().numpy(), n_keys, bpk, src_page_id=0)
    assert st == 0 and out.cpu().numpy().tobytes() == ref.tobytes()


@pytest.mark.parametrize("n_keys,bpk,n_parts,dup", [(1_200_000, 12, 3, 0), (900_001, 10, 8, 0),
                                                   (800_000, 12, 2, 300_000), (500_000, 5, 1, 0)])
def test_route_records_k24_equal_monolithic(oracle, amq, torch, n_keys, bpk, n_parts, dup):
    """Hash-range sharding of 24-byte keys (tkv_amq_bloom_route_records_ex): the sender hashes
    each key once into the same 12-byte records as for 16-byte keys, so the owners' range
    builds are unchanged.  Equal to the one-GPU build of the same keys and to the oracle."""
    from turtle_kv_amd.dist import hash_shard_tiles
    from turtle_kv_amd.filters import _ptr, _stream_handle
    L = amq.abi.lib()
    rng = np.random.default_rng(n_keys)
    kn = rng.integers(0, 256, (n_keys, 24), dtype=np.uint8)
    if dup:
        kn[n_keys - dup:] = kn[n_keys // 3]
    keys = torch.from_numpy(kn).cuda()
    plan = amq.plan_filters(0, [n_keys], bpk)
    seg = plan.segs[0]
    whole = amq.build_all_filters(plan, amq.KeyBatch.fixed(keys))
    recs = torch.empty((n_keys, 12), dtype=torch.uint8, device="cuda")
    counts = torch.zeros(n_parts, dtype=torch.int32, device="cuda")
    ws = torch.empty(int(L.tkv_amq_bloom_route_records_ws_bytes(n_keys, n_parts)), dtype=torch.uint8,
                     device="cuda")
    amq.abi.check(L.tkv_amq_bloom_route_records_ex(_ptr(keys), 24, n_keys, _ptr(plan.device_segs()),
                                                   int(seg["n_blocks"]), int(seg["hash_count"]), n_parts,
                                                   _ptr(recs), _ptr(counts), _ptr(ws), ws.numel(),
                                                   _stream_handle()), "route_records_ex")
    torch.cuda.synchronize()
    counts = counts.cpu().numpy().astype(np.int64)
    assert counts.sum() == n_keys
    T, q = hash_shard_tiles(int(seg["n_blocks"]), n_parts)
    out = torch.zeros(plan.total_out_bytes, dtype=torch.uint8, device="cuda")
    base = np.concatenate([[0], np.cumsum(counts)])
    for p in range(n_parts):
        _build_range_records(amq, torch, recs[int(base[p]):int(base[p + 1])], plan, min(T, p * q),
                             min(T, (p + 1) * q), out)
    torch.cuda.synchronize()
    assert torch.equal(out, whole)
    st, ref = oracle.bloom_build(kn, n_keys, bpk, src_page_id=0, stride=24)
    assert st == 0 and out.cpu().numpy().tobytes() == ref.tobytes()
    # key sizes other than 16 and 24 are refused
    counts_t = torch.zeros(n_parts, dtype=torch.int32, device="cuda")
    st = L.tkv_amq_bloom_route_records_ex(_ptr(keys), 20, n_keys, _ptr(plan.device_segs()),
                                          int(seg["n_blocks"]), int(seg["hash_count"]), n_parts,
                                          _ptr(recs), _ptr(counts_t), _ptr(ws), ws.numel(),
                                          _stream_handle())
    assert st == amq.abi.INVALID_ARGUMENT


def test_route_records_refuse_k_above_8(amq, torch):
    from turtle_kv_amd.filters import _ptr, _stream_handle
    L = amq.abi.lib()
    keys = amq.gen_keys16(22, 0, 1000)
    plan = amq.plan_filters(0, [1000], 16)     # k = 11
    ws = torch.empty(int(L.tkv_amq_bloom_route_records_ws_bytes(1000, 2)), dtype=torch.uint8, device="cuda")
    recs = torch.empty((1000, 12), dtype=torch.uint8, device="cuda")
    counts = torch.zeros(2, dtype=torch.int32, device="cuda")
    st = L.tkv_amq_bloom_route_records(_ptr(keys), 1000, _ptr(plan.device_segs()),
                                       int(plan.segs[0]["n_blocks"]), 11, 2, _ptr(recs), _ptr(counts),
                                       _ptr(ws), ws.numel(), _stream_handle())
    assert st == amq.abi.INVALID_ARGUMENT


@pytest.mark.parametrize("n_keys,bpk", [(1_200_000, 12), (700_000, 10)])
def test_hash_sharded_world1_24_byte_keys(oracle, amq, torch, n_keys, bpk):
    """HashShardedBloom without a process group (the first thing a caller tries) with [n, 24]
    keys: the range build reads 16-byte keys only, so the keys go through the record route
    (tkv_amq_bloom_route_records_ex) and the part builds; the filter equals the oracle's.
    Before round 4 such keys were read as 16-byte keys at a 16-byte stride."""
    from turtle_kv_amd.dist import HashShardedBloom
    rng = np.random.default_rng(n_keys)
    kn = rng.integers(0, 256, (n_keys, 24), dtype=np.uint8)
    hs = HashShardedBloom(n_keys, bpk, 1, 0, "cuda")
    filt = hs.build(torch.from_numpy(kn).cuda())
    torch.cuda.synchronize()
    st, ref = oracle.bloom_build(kn, n_keys, bpk, src_page_id=0, stride=24)
    assert st == 0 and filt.cpu().numpy().tobytes() == ref.tobytes()


def _pipelined_by_hand(amq, torch, keys_per_rank, bpk, chunks):
    """The pipelined hash-range build of `len(keys_per_rank)` ranks played on one GPU: each rank
    routes its chunks into its send blocks (tkv_amq_bloom_route_blocks), the all-to-all is done
    by block copies (recv block (c, s) of rank d = send block d of rank s's chunk c), each rank
    builds its round-robin parts (tkv_amq_bloom_build_part_blocks), and the filter is assembled
    from the parts' owners as the in-place all-gather of every round would."""
    from turtle_kv_amd.dist import HashShardedBloom
    W = len(keys_per_rank)
    n_total = sum(int(k.shape[0]) for k in keys_per_rank)
    mx = max(int(k.shape[0]) for k in keys_per_rank)
    hss = [HashShardedBloom(n_total, bpk, W, r, "cuda", chunks=chunks, max_keys_per_rank=mx) for r in range(W)]
    for r, hs in enumerate(hss):
        for c in range(chunks):
            hs.route_chunk(keys_per_rank[r], c)
    B = hss[0].block_bytes
    if W > 1:  # recv block [j][c][s] of rank d = rank s's chunk-c block of part j * W + d
        for d in range(W):
            for j in range(hss[0].g):
                for c in range(chunks):
                    for s_ in range(W):
                        i = (j * chunks + c) * W + s_
                        p = j * W + d
                        hss[d].recv[i * B:(i + 1) * B].copy_(hss[s_].send[c][p * B:(p + 1) * B])
    for hs in hss:
        for j in range(hs.g):
            hs.build_part(j)
    torch.cuda.synchronize()
    full = hss[0].out.clone()
    pb = hss[0].part_bytes
    for p in range(hss[0].n_parts):
        o = 64 + p * pb
        full[o:o + pb] = hss[p % W].out[o:o + pb]
        assert torch.equal(hss[p % W].out[:64], full[:64]), "every rank writes the header"
    return full[:hss[0].payload_bytes], hss


@pytest.mark.parametrize("n_keys,bpk,world,chunks,dup", [
    (3_000_000, 12, 1, 1, 0), (3_000_000, 12, 3, 2, 0), (1_500_001, 10, 8, 1, 0),
    (2_000_000, 12, 4, 3, 5_000), (1_440_000, 12, 8, 2, 0), (900_000, 5, 2, 1, 0),
    (40_000_000, 12, 2, 4, 0)])
def test_pipelined_blocks_equal_oracle(oracle, amq, torch, n_keys, bpk, world, chunks, dup):
    """The pipelined form against the oracle: k = 8, 7 and 3, ranks past the last tile (1.44M
    keys: 17 tiles over 8 ranks), ragged chunks and ranks, duplicate keys (their regions
    overflow: (record, part) entries through the blocks' overflow areas, within ovf_cap), and a
    size with several parts per rank."""
    keys = amq.gen_keys16(31, 0, n_keys)
    if dup:
        keys[n_keys - dup:] = keys[n_keys // 3]
    per = -(-n_keys // world)
    parts = [keys[r * per:min(n_keys, (r + 1) * per)] for r in range(world)]
    filt, hss = _pipelined_by_hand(amq, torch, parts, bpk, chunks)
    st, ref = oracle.bloom_build(keys.cpu().numpy(), n_keys, bpk, src_page_id=0)
    assert st == 0
    got = filt.cpu().numpy()
    if got.tobytes() != ref.tobytes():
        bad = np.nonzero(got != ref)[0]
        pytest.fail(f"{bad.size} bytes differ, first tiles {sorted({(int(b) - 64) // (64 * 2048) for b in bad[:1000]})[:8]}")
    # (5,000 copies of one key: ~3,300 records past their region, within a block's ovf_cap)
    assert not any(h.lost() for h in hss)
    if dup:
        h = hss[0]
        ovf = torch.stack([hs.recv.view(-1)[i * h.block_bytes + h.rp.ovf_n_off:
                                            i * h.block_bytes + h.rp.ovf_n_off + 4].view(torch.int32)
                           for hs in hss for i in range(h.g * h.chunks * h.world)]).sum()
        assert int(ovf) > 0, "the duplicates must have taken the overflow path"


def test_pipelined_blocks_24_byte_keys(oracle, amq, torch):
    rng = np.random.default_rng(5)
    n = 1_200_000
    kn = rng.integers(0, 256, (n, 24), dtype=np.uint8)
    keys = torch.from_numpy(kn).cuda()
    filt, _ = _pipelined_by_hand(amq, torch, [keys[:700_000], keys[700_000:]], 12, 2)
    st, ref = oracle.bloom_build(kn, n, 12, src_page_id=0, stride=24)
    assert st == 0 and filt.cpu().numpy().tobytes() == ref.tobytes()


def test_pipelined_blocks_report_lost_overflow(oracle, amq, torch):
    """One key repeated far past a block's overflow area: the blocks report the loss, and
    HashShardedBloom.build (one GPU, no process group) rebuilds through the exact exchange."""
    from turtle_kv_amd.dist import HashShardedBloom
    n = 30_000_000   # 344 tiles: two parts
    keys = amq.gen_keys16(32, 0, n)
    keys[n // 2:] = keys[7]
    hs = HashShardedBloom(n, 12, 1, 0, "cuda", direct=False)
    hs.step(keys)
    assert hs.lost()
    filt = HashShardedBloom(n, 12, 1, 0, "cuda", direct=False).build(keys)
    st, ref = oracle.bloom_build(keys.cpu().numpy(), n, 12, src_page_id=0)
    assert st == 0 and filt.cpu().numpy().tobytes() == ref.tobytes()


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _sharded_worker(rank, world, port, n_total, bpk, chunks, split, q):
    """One gloo rank on the box's one GPU: HashShardedBloom.build over this rank's keys (the
    real step: route chunks, the rounds' all-to-alls, part builds, round all-gathers on the
    communication stream); rank 0 checks the filter against the oracle."""
    import os
    import sys

    import torch
    import torch.distributed as dist
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import turtle_kv_amd as amq
    from turtle_kv_amd.dist import HashShardedBloom
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    bounds = [0] + [int(n_total * f) for f in split] + [n_total]
    k0, k1 = bounds[rank], bounds[rank + 1]
    keys = amq.gen_keys16(77, k0, k1 - k0)
    hs = HashShardedBloom(n_total, bpk, world, rank, "cuda", chunks=chunks)
    filt = hs.build(keys)
    hs2 = None
    if hs.last_fallback is None:  # the same step again, its stages timed
        hs.step(keys, timeline=True)
        torch.cuda.synchronize()
        hs2 = hs.timeline_ms()
        again = torch.equal(hs.filter(), filt)
    else:
        again = True
    res = None
    if rank == 0:
        from oracle import oracle as O
        O.build_oracle()
        allk = amq.gen_keys16(77, 0, n_total).cpu().numpy()
        st, ref = O.bloom_build(allk, n_total, bpk, src_page_id=0)
        res = (st == 0 and filt.cpu().numpy().tobytes() == ref.tobytes(), again, hs.last_fallback, hs2)
    dist.barrier()
    dist.destroy_process_group()
    if rank == 0:
        q.put(res)


@pytest.mark.parametrize("world,n_total,bpk,chunks,split,fallback", [
    (2, 3_000_000, 12, 2, (0.5,), None),               # even: the pipelined step
    (3, 2_500_001, 10, 3, (1 / 3, 2 / 3), None),        # ragged chunks, k = 7
    (2, 2_000_000, 12, 2, (0.6,), "keys_over_capacity"),  # rank 0 over its even share
])
def test_hash_sharded_step_gloo_ranks(world, n_total, bpk, chunks, split, fallback):
    """HashShardedBloom.build with `world` gloo ranks on the one GPU: the round-major exchange
    (chunks' rounds as routed, the last chunk round by round, part j built once its round has
    landed, round j gathered behind the exchange of round j + 2) gives the oracle's filter, and
    a rank holding more keys than the plan's chunks take sends every rank through the exact
    exchange.  (Parts per rank g = 1 at these sizes; config 5's g = 6 runs in the
    bench's 8-rank rehearsal.)"""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_sharded_worker, args=(r, world, port, n_total, bpk, chunks, split, q))
          for r in range(world)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(300)
    assert all(p.exitcode == 0 for p in ps), [p.exitcode for p in ps]
    ok, again, fb, tl = q.get(timeout=5)
    assert ok, "filter differs from the oracle"
    assert again and fb == fallback
    if fallback is None:  # every stage of the timed step was recorded, in stream order
        assert tl["route_0"] <= tl["build_0_start"] <= tl["build_0"] <= tl["end"], tl
        assert tl["exchange_0"] <= tl["build_0_start"] and tl["gather_0"] <= tl["end"], tl
