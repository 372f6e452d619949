"""GPU checks at bench scale: thousands of leaves laid out exactly as bench.py lays them out
(fixed per-leaf stride from turtle_kv_amd.dist, device-sorted keys for VQF).  Byte parity
with the oracle on sampled leaves, and no false negatives over every inserted key."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

S = 16384


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need a visible MI355X"
    return t


@pytest.mark.parametrize("n_full", [40, 6103])
def test_device_sort_matches_oracle(oracle, amq, torch, n_full):
    """bench.py sorts VQF leaves on the device; its order must be the oracle's memcmp order
    (at the bench's full 100M keys too)."""
    import bench
    counts = [S] * n_full + [8448, 3, 0, 1]
    n = sum(counts)
    keys = bench.sort_segments_device(torch, amq.gen_keys16(42, 0, n), counts).cpu().numpy()
    ref = oracle.gen_keys16(42, 0, n)
    oracle.sort_segments(ref, np.concatenate([[0], np.cumsum(counts)]).astype(np.uint64))
    assert np.array_equal(keys, ref)


@pytest.mark.parametrize("kind,bpk,cap,full", [(1, 12, 32704, 2000), (0, 10, 0, 2000),
                                               (1, 12, 32704, 6103)])
def test_bench_layout_no_false_negatives(oracle, amq, torch, kind, bpk, cap, full):
    import bench
    from turtle_kv_amd import dist as tdist
    counts = [S] * full + [8448]
    n = sum(counts)
    shard = tdist.shard_leaves(counts, 1, 0)
    stride = tdist.leaf_stride(kind, bpk, S, cap)
    plan = tdist.plan_shard(kind, counts, bpk, shard, stride, payload_capacity=cap)
    keys = amq.gen_keys16(42, 0, n)
    bkeys = bench.sort_segments_device(torch, keys, counts) if kind == 1 else keys
    out = amq.build_all_filters(plan, amq.KeyBatch.fixed(bkeys))
    seg = torch.repeat_interleave(torch.arange(len(counts), dtype=torch.int32, device="cuda"),
                                  torch.tensor(counts, device="cuda"))
    res = amq.probe_filters(plan, out, amq.KeyBatch.fixed(keys), seg).cpu().numpy()
    out_np = out.cpu().numpy()
    bad = np.nonzero(res == 0)[0]
    msg = ""
    if len(bad):
        sb = np.concatenate([[0], np.cumsum(counts)])
        leaf = int(np.searchsorted(sb, bad[0], side="right") - 1)
        msg = f"{len(bad)} false negatives, first key {int(bad[0])} in leaf {leaf}"
        hk = bkeys.cpu().numpy()
        lk = np.ascontiguousarray(hk[sb[leaf]:sb[leaf + 1]])
        o = int(plan.segs[leaf]["out_offset"])
        if kind == 1:
            st, pl, p = oracle.vqf_build(lk, len(lk), bpk, cap, src_page_id=leaf)
            ref = pl[:p.payload_used]
        else:
            st, ref = oracle.bloom_build(lk, len(lk), bpk, src_page_id=leaf)
        got = out_np[o:o + len(ref)]
        msg += f"; oracle build status {st}, leaf bytes equal: {np.array_equal(got, ref)}"
        st2, r2 = oracle.probe_segments(kind, out_np, plan.segs["out_offset"],
                                        keys.cpu().numpy()[bad[:64]], seg.cpu().numpy()[bad[:64]])
        msg += f"; oracle probe over GPU bytes of the first 64: {r2.tolist()}"
    assert len(bad) == 0, msg
    # sampled byte parity against the oracle, leaves spread over the whole array
    hk = bkeys.cpu().numpy()
    sb = np.concatenate([[0], np.cumsum(counts)])
    for leaf in [0, 1, 777, full - 1, full]:
        lk = np.ascontiguousarray(hk[sb[leaf]:sb[leaf + 1]])
        o = int(plan.segs[leaf]["out_offset"])
        if kind == 1:
            st, pl, p = oracle.vqf_build(lk, len(lk), bpk, cap, src_page_id=leaf)
            ref = pl[:p.payload_used]
        else:
            st, ref = oracle.bloom_build(lk, len(lk), bpk, src_page_id=leaf)
        assert st == 0
        assert out_np[o:o + len(ref)].tobytes() == ref.tobytes(), f"leaf {leaf}"
