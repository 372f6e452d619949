"""Seeded randomized parity: batches of random shape (leaf count across every kernel-selection
threshold, ragged and empty leaves, bits per key, key shape, page capacity) built through the
C ABI and compared leaf by leaf with the CPU oracle on a sample of leaves.  Each case is a
fixed seed, so a failure reproduces."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

# leaf counts around the kernel switches: Bloom split (< 256) / LDS (>= 256) / wide (< 2048);
# VQF ring (<= 768) / one wave per leaf (> 768)
LEAF_COUNTS = [1, 3, 63, 64, 255, 256, 700, 768, 769, 1100]


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need a visible MI355X"
    return t


def make_keys(rng, shape, n):
    if shape == 16:
        return rng.integers(0, 256, (n, 16), dtype=np.uint8), None, 16
    if shape == 24:
        return rng.integers(0, 256, (n, 24), dtype=np.uint8), None, 24
    # variable length, >= 6 bytes (duplicates of very short keys overflow a VQF block)
    lens = rng.integers(6, 48, n)
    offs = np.zeros(n + 1, np.int64)
    offs[1:] = np.cumsum(lens)
    return rng.integers(0, 256, int(offs[-1]), dtype=np.uint8), offs, 0


@pytest.mark.parametrize("case", range(20))
def test_random_batches_match_oracle(oracle, amq, torch, case):
    rng = np.random.default_rng(7000 + case)
    kind = case % 2
    n_leaves = LEAF_COUNTS[(case // 2) % len(LEAF_COUNTS)]
    shape = [16, 24, 0][case % 3]
    if kind == 0:
        bpk = int(rng.choice([1, 4, 7, 10, 12, 16, 24, 33]))
        cap = 0
    else:
        bpk = int(rng.choice([12, 13, 16, 20, 22, 28]))
        cap = int(rng.choice([8128, 16320, 32704, 65472]))
    # mostly small leaves (the sample is checked on the CPU), a few full ones, some empty
    counts = [int(c) for c in rng.integers(0, 1500, n_leaves)]
    for i in rng.choice(n_leaves, size=min(n_leaves, 3), replace=False):
        counts[int(i)] = int(rng.choice([0, 16384, 9000]))
    n = sum(counts)
    keys, offs, stride = make_keys(rng, shape, n)
    plan = amq.plan_filters(kind, counts, bpk, payload_capacity=cap)
    kt = torch.from_numpy(keys).cuda()
    kb = amq.KeyBatch.fixed(kt) if offs is None else amq.KeyBatch.variable(kt, torch.from_numpy(offs).cuda())
    out = amq.build_all_filters(plan, kb)
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    sb = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    sample = sorted({0, n_leaves - 1, *rng.choice(n_leaves, size=min(n_leaves, 12), replace=False).tolist()})
    for s in sample:
        b, c = int(sb[s]), counts[s]
        if offs is None:
            kp, o_s = keys[b:], None
        else:
            kp, o_s = keys[int(offs[b]):], (offs[b:b + c + 1] - offs[b]).astype(np.uint64)
        if kind == 0:
            st, ref = oracle.bloom_build(kp, c, bpk, src_page_id=s, offsets=o_s, stride=stride)
            ref = ref.tobytes()
        else:
            st, ref, p = oracle.vqf_build(kp, c, bpk, cap, src_page_id=s, offsets=o_s, stride=stride)
            ref = ref[:p.payload_used].tobytes()
        assert st == 0
        seg = plan.segs[s]
        got = o[int(seg["out_offset"]):int(seg["out_offset"]) + int(seg["payload_bytes"])].tobytes()
        assert got == ref, f"case {case}: kind {kind} bpk {bpk} cap {cap} shape {shape} leaf {s} of {n_leaves}"


@pytest.mark.parametrize("case", range(10))
def test_random_big_leaf_batches_match_oracle(oracle, amq, torch, case):
    """Batches holding one or two large leaves (TurtleKV leaves of small items, filter pages of
    64 KiB-1 MiB): Bloom images around the 160 KB LDS budget (split, one-workgroup and
    device-atomic paths), VQF leaves around 512 / 1,241 / 2,048 / 4,964 blocks (compact and
    8-byte records, one or several place workgroups per leaf, the unfused place, the LDS
    lane-mask table and the ballots).  The large leaves are always among those checked."""
    rng = np.random.default_rng(9100 + case)
    kind = case % 2
    n_leaves = [1, 5, 64, 300, 800][(case // 2) % 5]
    shape = [16, 0, 24][case % 3]
    if kind == 0:
        bpk = int(rng.choice([10, 12]))
        cap = 0
        big = [int(rng.choice([60000, 100000, 140000])) for _ in range(2)]
    else:
        bpk = int(rng.choice([12, 22]))
        cap = int(rng.choice([65472, 130944, 262080, 1048512]))
        big = [int(rng.choice([30000, 80000, 200000])) for _ in range(2)]
    counts = [int(c) for c in rng.integers(0, 800, n_leaves)]
    where = sorted({0, n_leaves - 1})
    for i, w in enumerate(where):
        counts[w] = big[i]
    n = sum(counts)
    keys, offs, stride = make_keys(rng, shape, n)
    plan = amq.plan_filters(kind, counts, bpk, payload_capacity=cap)
    kt = torch.from_numpy(keys).cuda()
    kb = amq.KeyBatch.fixed(kt) if offs is None else amq.KeyBatch.variable(kt, torch.from_numpy(offs).cuda())
    out = amq.build_all_filters(plan, kb)
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    sb = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    sample = sorted({*where, *rng.choice(n_leaves, size=min(n_leaves, 6), replace=False).tolist()})
    for s in sample:
        b, c = int(sb[s]), counts[s]
        if offs is None:
            kp, o_s = keys[b:], None
        else:
            kp, o_s = keys[int(offs[b]):], (offs[b:b + c + 1] - offs[b]).astype(np.uint64)
        if kind == 0:
            st, ref = oracle.bloom_build(kp, c, bpk, src_page_id=s, offsets=o_s, stride=stride)
            ref = ref.tobytes()
        else:
            st, ref, p = oracle.vqf_build(kp, c, bpk, cap, src_page_id=s, offsets=o_s, stride=stride)
            ref = ref[:p.payload_used].tobytes()
        assert st == 0
        seg = plan.segs[s]
        got = o[int(seg["out_offset"]):int(seg["out_offset"]) + int(seg["payload_bytes"])].tobytes()
        assert got == ref, (f"case {case}: kind {kind} bpk {bpk} cap {cap} shape {shape} leaf {s} "
                            f"of {n_leaves} ({c} keys, {int(seg['n_blocks'])} blocks)")


@pytest.mark.parametrize("case", range(8))
def test_random_tiled_leaf_batches_match_oracle(oracle, amq, torch, case):
    """Bloom batches whose leaves cross the tiled-build thresholds at random (a single filter
    past one LDS window; in a batch, 16/24-byte keys past 5 windows, other shapes past 16):
    2-12 leaves of 0-2.6M keys among small ones, random bits per key (k from 3 to 16), every
    key shape; every large leaf is checked, and a sample of the others."""
    rng = np.random.default_rng(9300 + case)
    shape = [16, 24, 0, 16][case % 4]
    bpk = int(rng.choice([5, 8, 10, 12, 14, 20]))
    n_big = int(rng.integers(1, 6)) if case != 0 else 1
    big = [int(rng.integers(200_000, 2_600_000)) for _ in range(n_big)]
    n_small = 0 if case == 0 else int(rng.integers(0, 40))
    counts = [int(c) for c in rng.integers(0, 20000, n_small)] + big
    rng.shuffle(counts)
    n = sum(counts)
    keys, offs, stride = make_keys(rng, shape, n)
    plan = amq.plan_filters(0, counts, bpk)
    kt = torch.from_numpy(keys).cuda()
    kb = amq.KeyBatch.fixed(kt) if offs is None else amq.KeyBatch.variable(kt, torch.from_numpy(offs).cuda())
    out = amq.build_all_filters(plan, kb)
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    sb = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    large = [i for i, c in enumerate(counts) if c >= 200_000]
    sample = sorted({*large, *rng.choice(len(counts), size=min(len(counts), 6), replace=False).tolist()})
    for s in sample:
        b, c = int(sb[s]), counts[s]
        if offs is None:
            kp, o_s = keys[b:], None
        else:
            kp, o_s = keys[int(offs[b]):], (offs[b:b + c + 1] - offs[b]).astype(np.uint64)
        st, ref = oracle.bloom_build(kp, c, bpk, src_page_id=s, offsets=o_s, stride=stride)
        assert st == 0
        seg = plan.segs[s]
        got = o[int(seg["out_offset"]):int(seg["out_offset"]) + int(seg["payload_bytes"])].tobytes()
        assert got == ref.tobytes(), f"case {case}: bpk {bpk} shape {shape} leaf {s} ({c} keys) of {len(counts)}"
