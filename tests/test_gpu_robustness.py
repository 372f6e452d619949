"""GPU: failure reporting, concurrency and edge cases of the C ABI (all against the oracle)."""
import threading

import numpy as np
import pytest
import xxhash

pytestmark = pytest.mark.gpu

VQF_SEED = 0x9D0924DC03E79A75


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available()
    return t


def overflow_keys(oracle, n=50):
    """Keys whose primary AND alternate bucket fall in block 0 of a 2-block, 8-bit VQF
    (R = 2 * 80 buckets): the 49th insert finds both candidate blocks full."""
    out = []
    i = 0
    while len(out) < n:
        k = oracle.gen_keys16(1234, i, 1)[0]
        i += 1
        h = xxhash.xxh64_intdigest(k.tobytes(), VQF_SEED)
        tag = h & 0xFF
        pi = (h >> 8) % 160
        ai = ((h ^ ((tag * 0x5BD1E995) & ((1 << 64) - 1))) >> 8) % 160
        if pi < 80 and ai < 80:
            out.append(k)
    return np.stack(out)


def test_vqf_block_overflow_is_reported(oracle, amq, torch):
    keys = overflow_keys(oracle)
    st, _, pl = oracle.vqf_build(keys, len(keys), 12, 32704)
    assert pl.nblocks == 2 and st == 13, "oracle: vqf_insert failure (filter_builder.hpp:211)"
    plan = amq.plan_filters(amq.VQF, [len(keys)], 12, payload_capacity=32704)
    with pytest.raises(amq.TkvAmqError) as e:
        amq.build_all_filters(plan, amq.KeyBatch.fixed(torch.from_numpy(keys).cuda()))
    assert e.value.status == amq.abi.INTERNAL
    # the per-leaf entry point logs and leaves the leaf without a filter (:323-325)
    assert amq.build_filter_for_leaf_in_job(12, 1, amq.KeyBatch.fixed(torch.from_numpy(keys).cuda())) is None
    # 48 of them fit exactly: no failure, bytes equal the oracle
    st, ref, pl = oracle.vqf_build(keys[:48], 48, 12, 32704)
    assert st == 0
    plan = amq.plan_filters(amq.VQF, [48], 12, payload_capacity=32704)
    out = amq.build_all_filters(plan, amq.KeyBatch.fixed(torch.from_numpy(keys[:48].copy()).cuda()))
    assert out.cpu().numpy()[:pl.payload_used].tobytes() == ref[:pl.payload_used].tobytes()


@pytest.mark.parametrize("n_leaves", [1, 64, 300, 800])
def test_vqf_failed_build_then_clean_build_on_one_workspace(oracle, amq, torch, n_leaves):
    """No memset precedes a VQF build: every decide-class kernel rewrites each leaf's nelts
    word (flags included).  A batch with one overflowing leaf reports Internal; the next,
    clean batch on the same workspace must report OK and equal the oracle.  1 / 64 leaves:
    vqf_ring_place; 300: its two-per-CU form; 800: vqf_decide."""
    bad = overflow_keys(oracle)
    rest = [oracle.gen_keys16(4000 + i, 0, 500) for i in range(n_leaves - 1)]
    counts = [len(bad)] + [500] * (n_leaves - 1)
    keys = np.concatenate([bad] + rest) if rest else bad
    plan = amq.plan_filters(amq.VQF, counts, 12, payload_capacity=32704)
    ws = torch.empty(plan.workspace_bytes, dtype=torch.uint8, device="cuda")
    with pytest.raises(amq.TkvAmqError) as e:
        amq.build_all_filters(plan, amq.KeyBatch.fixed(torch.from_numpy(keys).cuda()), workspace=ws)
    assert e.value.status == amq.abi.INTERNAL
    good = keys.copy()
    good[:len(bad)] = oracle.gen_keys16(999, 0, len(bad))
    out = amq.build_all_filters(plan, amq.KeyBatch.fixed(torch.from_numpy(good).cuda()), workspace=ws)
    o = out.cpu().numpy()
    sb = np.concatenate([[0], np.cumsum(counts)])
    for s in (0, n_leaves - 1):
        st, ref, pl = oracle.vqf_build(good[sb[s]:], counts[s], 12, 32704, src_page_id=s)
        seg = plan.segs[s]
        assert st == 0
        assert o[int(seg["out_offset"]):int(seg["out_offset"]) + pl.payload_used].tobytes() == \
            ref[:pl.payload_used].tobytes()


@pytest.mark.parametrize("kind", [0, 1])
def test_concurrent_streams_two_threads(oracle, amq, torch, kind):
    """The ABI is called concurrently from worker threads (build_all_pages); each call on its
    own stream must produce exactly its own filters."""
    results = {}

    def work(seed):
        counts = [16384] * 4 + [777]
        keys = oracle.gen_keys16(seed, 0, sum(counts))
        oracle.sort_segments(keys, np.concatenate([[0], np.cumsum(counts)]).astype(np.uint64))
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            plan = amq.plan_filters(kind, counts, 12, payload_capacity=32704)
            d = torch.from_numpy(keys).cuda()
            outs = [amq.build_all_filters(plan, amq.KeyBatch.fixed(d), stream=s) for _ in range(3)]
            s.synchronize()
        results[seed] = (plan, [o.cpu().numpy() for o in outs], keys, counts)

    ts = [threading.Thread(target=work, args=(sd,)) for sd in (5, 6)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for sd, (plan, outs, keys, counts) in results.items():
        # payload regions only: the 64-byte alignment padding between VQF payloads is never
        # written (like the unused tail of a reference page buffer)
        regions = [(int(g["out_offset"]), int(g["payload_bytes"])) for g in plan.segs]
        for o in outs[1:]:
            assert all(np.array_equal(outs[0][a:a + b], o[a:a + b]) for a, b in regions)
        sb = np.concatenate([[0], np.cumsum(counts)])
        for s_, c in enumerate(counts):
            if kind == 0:
                st, ref = oracle.bloom_build(keys[sb[s_]:], c, 12, src_page_id=s_)
                ref = ref.tobytes()
            else:
                st, ref, pl = oracle.vqf_build(keys[sb[s_]:], c, 12, 32704, src_page_id=s_)
                ref = ref[:pl.payload_used].tobytes()
            seg = plan.segs[s_]
            o = int(seg["out_offset"])
            assert outs[0][o:o + int(seg["payload_bytes"])].tobytes() == ref


def test_empty_and_no_filter_batches(oracle, amq, torch):
    keys = torch.zeros((0, 16), dtype=torch.uint8, device="cuda")
    for kind in (0, 1):
        plan = amq.plan_filters(kind, [], 12, payload_capacity=32704)
        amq.build_all_filters(plan, amq.KeyBatch.fixed(keys))
        plan = amq.plan_filters(kind, [0, 0], 12, payload_capacity=32704)
        out = amq.build_all_filters(plan, amq.KeyBatch.fixed(keys)).cpu().numpy()
        for s_ in range(2):   # empty leaves still get a valid (empty) filter page
            seg = plan.segs[s_]
            if kind == 0:
                st, ref = oracle.bloom_build(np.zeros((1, 16), np.uint8), 0, 12, src_page_id=s_)
                ref = ref.tobytes()
            else:
                st, ref, pl = oracle.vqf_build(np.zeros((1, 16), np.uint8), 0, 12, 32704, src_page_id=s_)
                ref = ref[:pl.payload_used].tobytes()
            o = int(seg["out_offset"])
            assert out[o:o + int(seg["payload_bytes"])].tobytes() == ref
    # bits_per_key == 0: no filters; every probe answers "maybe" (reject_page kUnknown)
    k = amq.gen_keys16(3, 0, 1000)
    for kind in (0, 1):
        plan = amq.plan_filters(kind, [1000], 0, payload_capacity=32704)
        out = amq.build_all_filters(plan, amq.KeyBatch.fixed(k))
        miss = amq.gen_keys16(4, 0, 1000)
        res = amq.probe_filters(plan, out, amq.KeyBatch.fixed(miss),
                                torch.zeros(1000, dtype=torch.int32, device="cuda"))
        assert bool(res.all())


def test_invalid_arguments(amq, torch):
    with pytest.raises(amq.TkvAmqError) as e:
        amq.plan_filters(amq.VQF, [100], 11, payload_capacity=32704)
    assert e.value.status == amq.abi.INVALID_ARGUMENT
    with pytest.raises(amq.TkvAmqError) as e:
        amq.plan_filters(amq.VQF, [100], 12, payload_capacity=100)
    assert e.value.status == amq.abi.RESOURCE_EXHAUSTED
    L = amq.abi.lib()
    # misaligned 16-byte keys are rejected, not read out of bounds
    buf = torch.zeros(33, dtype=torch.uint8, device="cuda")
    plan = amq.plan_filters(amq.BLOOM, [1], 10)
    st = L.tkv_amq_build(0, buf.data_ptr() + 1, None, 16, 1, plan.device_segs().data_ptr(), 1,
                         plan.max_seg_blocks, buf.data_ptr(), None, 0, None)
    assert st == amq.abi.INVALID_ARGUMENT


@pytest.mark.parametrize("kind,bpk,cap", [(0, 10, 0), (1, 12, 32704)])
def test_host_pipeline_matches_device_build(oracle, amq, torch, kind, bpk, cap):
    """build_filters_from_host (chunked H2D -> build -> D2H on three streams) writes the same
    filter pages as one device-resident build."""
    counts = [16384] * 37 + [999, 0, 16384]
    keys = oracle.gen_keys16(77, 0, sum(counts))
    if kind == 1:
        oracle.sort_segments(keys, np.concatenate([[0], np.cumsum(counts)]).astype(np.uint64))
    host = torch.from_numpy(keys).pin_memory()
    out, plan = amq.filters.build_filters_from_host(kind, counts, bpk, host, payload_capacity=cap,
                                                    chunk_keys=100_000)
    ref_plan = amq.plan_filters(kind, counts, bpk, payload_capacity=cap, out_stride=plan.segs[0]["out_offset"] * 0 + int(plan.segs[1]["out_offset"]))
    ref = amq.build_all_filters(ref_plan, amq.KeyBatch.fixed(torch.from_numpy(keys).cuda())).cpu().numpy()
    o = out.numpy()
    for g in plan.segs:
        a, b = int(g["out_offset"]), int(g["payload_bytes"])
        assert np.array_equal(o[a:a + b], ref[a:a + b])


@pytest.mark.parametrize("kind,bpk,cap", [(0, 10, 0), (1, 12, 32704)])
def test_host_pipeline_from_key_views(oracle, amq, torch, kind, bpk, cap):
    """run_views: keys gathered from EditView-like records (key at byte 8 of 40-byte records)
    by tkv_amq_stage_keys, chunk by chunk, give the same pages as run() on contiguous keys."""
    counts = [16384] * 9 + [123, 0, 5000]
    keys = oracle.gen_keys16(78, 0, sum(counts))
    if kind == 1:
        oracle.sort_segments(keys, np.concatenate([[0], np.cumsum(counts)]).astype(np.uint64))
    n, rec = len(keys), 40
    buf = np.zeros((n, rec), np.uint8)
    buf[:, 8:24] = keys
    views = amq.key_views(buf, np.arange(n, dtype=np.uint64) * rec + 8, 16)
    pipe = amq.HostFilterPipeline(kind, counts, bpk, payload_capacity=cap, chunk_keys=50_000)
    a = pipe.run_views(views).clone()
    b = pipe.run(torch.from_numpy(keys).pin_memory())
    assert torch.equal(a, b)


def test_build_records_reference_metrics(oracle, amq, torch):
    """A checked build folds its leaves into BloomFilterMetrics / QuotientFilterMetrics with a
    build latency, as build_{bloom,vqf}_filter do per leaf (filter_builder.hpp:139-147,198-202)."""
    counts = [16384, 777]
    keys = oracle.gen_keys16(5, 0, sum(counts))
    oracle.sort_segments(keys, np.concatenate([[0], np.cumsum(counts)]).astype(np.uint64))
    kb = amq.KeyBatch.fixed(torch.from_numpy(keys).cuda())
    for kind, m in ((amq.BLOOM, amq.BloomFilterMetrics.instance()),
                    (amq.VQF, amq.QuotientFilterMetrics.instance())):
        plan = amq.plan_filters(kind, counts, 12, payload_capacity=32704)
        c0, t0, l0 = m.item_count_stats.count, m.item_count_stats.total, m.build_page_latency.count
        amq.build_all_filters(plan, kb)
        assert m.item_count_stats.count == c0 + 2 and m.item_count_stats.total == t0 + sum(counts)
        assert m.build_page_latency.count == l0 + 2 and m.build_page_latency.total_usec > 0
        amq.build_all_filters(plan, kb, check=False)   # unchecked launches record nothing
        assert m.item_count_stats.count == c0 + 2


@pytest.mark.parametrize("kind", [0, 1])
def test_probe_leaf_index_out_of_range(oracle, amq, torch, kind):
    """A query naming a leaf outside the plan answers "maybe" (reject_page's kUnknown) on every
    probe path, and nothing outside the plan is read."""
    counts = [4096, 100]
    keys = oracle.gen_keys16(8, 0, sum(counts))
    oracle.sort_segments(keys, np.concatenate([[0], np.cumsum(counts)]).astype(np.uint64))
    kb = amq.KeyBatch.fixed(torch.from_numpy(keys).cuda())
    plan = amq.plan_filters(kind, counts, 12, payload_capacity=32704)
    filt = amq.build_all_filters(plan, kb)
    miss = amq.KeyBatch.fixed(amq.gen_keys16(9, 0, 1000))
    bad = torch.tensor([2, 3, 1 << 20, 0x7FFFFFF0] * 250, dtype=torch.int32, device="cuda")
    assert bool(amq.probe_filters(plan, filt, miss, bad).all())
    if kind == 0:
        qh = amq.bloom_query_hashes(miss, 32)
        assert bool(amq.bloom_probe_hashed(plan, filt, qh, 32, bad).all())
    else:
        assert bool(amq.vqf_probe_hashed(plan, filt, amq.vqf_hash_val(miss), bad).all())
    # in range, the same misses are mostly rejected
    good = torch.zeros(1000, dtype=torch.int32, device="cuda")
    assert int(amq.probe_filters(plan, filt, miss, good).sum()) < 100


@pytest.mark.parametrize("n_keys", [4_000_000, 1_300_000])
def test_vqf_round_plans_on_one_poisoned_workspace(oracle, amq, torch, n_keys):
    """PipelinedLeafGather builds differently sized round plans (41 / 40 leaves ... at fixed
    stride) one after another on ONE workspace.  Built that way on a workspace first filled
    with 0xFF, every round's leaves must equal a fresh whole-batch build of the same leaves on
    a zeroed workspace (no kernel may read state an earlier build of another plan left), and
    sampled leaves the oracle (an intermittent gathered-array mismatch)."""
    from turtle_kv_amd import dist as tdist
    cap = 32704
    counts = [16384] * (n_keys // 16384) + ([n_keys % 16384] if n_keys % 16384 else [])
    sb = np.concatenate([[0], np.cumsum(counts)]).astype(np.uint64)
    keys = oracle.gen_keys16(42, 0, int(sb[-1]))
    oracle.sort_segments(keys, sb, n_threads=8)
    d = torch.from_numpy(keys).cuda()
    stride = tdist.leaf_stride(1, 12, max(counts), cap)
    W, per_rank = 2, -(-len(counts) // 2)
    q = -(-per_rank // 3)
    rounds = []
    for r in range(W):
        for b, e in tdist.cyclic_rounds(len(counts), W, r, q):
            if b < e:
                rounds.append((b, e, amq.plan_filters(1, np.asarray(counts[b:e], np.uint64), 12,
                                                      payload_capacity=cap, out_stride=stride,
                                                      src_page_ids=np.arange(b, e, dtype=np.uint64))))
    ws = torch.full((max(p.workspace_bytes for *_, p in rounds),), 0xFF, dtype=torch.uint8, device="cuda")
    got = torch.zeros(len(counts) * stride, dtype=torch.uint8, device="cuda")
    for b, e, p in rounds:
        amq.build_all_filters(p, amq.KeyBatch.fixed(d[int(sb[b]):int(sb[e])]),
                              out=got[b * stride:e * stride], workspace=ws)
    full_plan = amq.plan_filters(1, counts, 12, payload_capacity=cap, out_stride=stride)
    fresh = torch.zeros(full_plan.total_out_bytes, dtype=torch.uint8, device="cuda")
    amq.build_all_filters(full_plan, amq.KeyBatch.fixed(d), out=fresh,
                          workspace=torch.zeros(full_plan.workspace_bytes, dtype=torch.uint8, device="cuda"))
    if not torch.equal(got, fresh):
        diff = torch.nonzero(got != fresh).flatten()
        pytest.fail(f"{diff.numel()} bytes differ, leaves {sorted({int(x) // stride for x in diff[:4096].tolist()})[:16]}")
    o = fresh.cpu().numpy()
    for s in (0, q - 1, q, len(counts) - 1):
        st, ref, pl = oracle.vqf_build(keys[int(sb[s]):], counts[s], 12, cap, src_page_id=s)
        assert st == 0
        assert o[s * stride:s * stride + pl.payload_used].tobytes() == ref[:pl.payload_used].tobytes()


@pytest.mark.parametrize("kind", [0, 1])
def test_verify_gather_names_the_wrong_leaf(oracle, amq, torch, kind, capsys):
    """VERDICT r05 (wrong gathered VQF array, round 4): a gathered array that differs from the
    single-process build is reported leaf by leaf -- its owning rank and round in the
    block-cyclic layout, which side equals the oracle, whether the keys each side built from are
    the oracle's, whether a lone rebuild reproduces the oracle -- and its bytes are kept.  Here
    one byte of leaf 5's gathered payload is flipped: the diagnosis must blame the gathered side
    (leaf 5 = round 1, rank 0 with 2 ranks and 2-leaf chunks) and clear the single build."""
    import json
    import os

    import bench
    counts = [4096] * 9 + [1000]
    bpk, cap = (10, 0) if kind == 0 else (12, 16320)
    from turtle_kv_amd import dist as tdist
    stride = tdist.leaf_stride(kind, bpk, max(counts), cap)
    plan = amq.plan_filters(kind, counts, bpk, payload_capacity=cap, out_stride=stride)
    keys = amq.gen_keys16(42, 0, sum(counts))
    if kind == 1:
        keys = bench.sort_segments_device(torch, keys, counts)
    good = torch.zeros(plan.total_out_bytes, dtype=torch.uint8, device="cuda")
    amq.build_all_filters(plan, amq.KeyBatch.fixed(keys), out=good)
    assert bench.verify_gather(torch, amq, kind, bpk, cap, counts, stride, good, 16,
                               torch.device("cuda"), layout=(2, 2)) is True
    bad = good.clone()
    bad[5 * stride + 100] ^= 0x40
    assert bench.verify_gather(torch, amq, kind, bpk, cap, counts, stride, bad, 16,
                               torch.device("cuda"), layout=(2, 2)) is False
    d = os.path.join(bench.ROOT, "gpurun_out", "verify_gather_fail")
    summary = json.load(open(os.path.join(d, "summary.json")))
    (row,) = summary["leaves"]
    assert (row["leaf"], row["rank"], row["round"]) == (5, 0, 1)
    assert row["gathered_equals_oracle"] is False and row["single_build_equals_oracle"] is True
    assert row["single_build_keys_equal_oracle"] is True and row["alone_equals_oracle"] == [True, True]
    z = np.load(os.path.join(d, "leaves.npz"))
    assert (z["leaf5_gathered"] != z["leaf5_oracle"]).sum() == 1
    assert "verify_gather diagnosis" in capsys.readouterr().err
