"""GPU parity: filters and probe answers from libtkv_amq (HIP, gfx950) must be byte-identical
to the CPU oracle (tkv-amq v1 spec) on the same seeded inputs; at full BASELINE sizes the
checks are size-independent properties (no false negatives, determinism, FPR equality).
Every call goes through the C ABI (include/tkv_amq.h) via ctypes."""
import hashlib
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
S = 16384
VQF_SEED = 0x9D0924DC03E79A75


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need a visible MI355X"
    return t


def seg_bounds(counts):
    return np.concatenate([[0], np.cumsum(counts)]).astype(np.uint64)


def oracle_per_segment(oracle, kind, keys_np, counts, bpk, cap=32704, src=None, stride=16,
                       offsets=None):
    """oracle payloads, one bytes object per segment"""
    out = []
    sb = seg_bounds(counts)
    for s, c in enumerate(counts):
        b = int(sb[s])
        sid = s if src is None else int(src[s])
        if offsets is not None:
            o = (offsets[b:b + c + 1] - offsets[b]).astype(np.uint64)
            kp = keys_np[int(offsets[b]):]
        else:
            o, kp = None, keys_np[b:]
        if kind == 0:
            st, pl = oracle.bloom_build(kp, c, bpk, src_page_id=sid, offsets=o, stride=stride)
            assert st == 0
            out.append(pl.tobytes() if bpk else b"")
        else:
            st, pl, plan = oracle.vqf_build(kp, c, bpk, cap, src_page_id=sid, offsets=o,
                                            stride=stride)
            assert st == 0, st
            out.append(pl[:plan.payload_used].tobytes() if bpk else b"")
    return out


def gpu_build(amq, torch, kind, keys_t, counts, bpk, cap=32704, src=None, offsets_t=None,
              check=True):
    plan = amq.plan_filters(kind, counts, bpk, payload_capacity=cap if kind == 1 else 0,
                            src_page_ids=src)
    kb = amq.KeyBatch.fixed(keys_t) if offsets_t is None else amq.KeyBatch.variable(keys_t, offsets_t)
    out = amq.build_all_filters(plan, kb, check=check)
    torch.cuda.synchronize()
    return plan, out.cpu().numpy()


def segment_bytes(plan, out_np, s):
    seg = plan.segs[s]
    o, n = int(seg["out_offset"]), int(seg["payload_bytes"])
    return out_np[o:o + n].tobytes()


def assert_same(plan, out_np, ref):
    for s, r in enumerate(ref):
        got = segment_bytes(plan, out_np, s)
        if got != r:
            a = np.frombuffer(got, np.uint8)
            b = np.frombuffer(r, np.uint8)
            n = min(len(a), len(b))
            diff = np.nonzero(a[:n] != b[:n])[0]
            raise AssertionError(f"segment {s}: len {len(a)} vs {len(b)}, first diff at "
                                 f"{diff[:8].tolist()}")


RAGGED = [16384, 1, 0, 777, 16384, 8448, 64, 63, 65, 2, 5000]


@pytest.mark.parametrize("bpk", [10, 12, 1, 5, 20, 33])
def test_bloom16_parity(oracle, amq, torch, bpk):
    counts = RAGGED
    keys = oracle.gen_keys16(42, 0, sum(counts))
    src = [1000 + i for i in range(len(counts))]
    ref = oracle_per_segment(oracle, 0, keys, counts, bpk, src=src)
    plan, out = gpu_build(amq, torch, 0, torch.from_numpy(keys).cuda(), counts, bpk, src=src)
    assert_same(plan, out, ref)


def test_bloom_config1_sha256(oracle, amq, torch):
    """BASELINE config 1 on the GPU: 1M x 16B keys @10 bpk, S = 16384 -> the golden SHA."""
    g = json.load(open(os.path.join(GOLDEN, "filters.json")))["config1_bloom10_1M"]
    n = g["n_keys"]
    counts = [S] * (n // S) + [n % S]
    keys = amq.gen_keys16(42, 0, n)
    plan = amq.plan_filters(0, counts, 10)
    out = amq.build_all_filters(plan, amq.KeyBatch.fixed(keys))
    assert plan.total_out_bytes == g["bytes"]
    assert hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest() == g["sha256"]


def test_gen_keys_match_oracle(oracle, amq, torch):
    k = amq.gen_keys16(42, 123456, 5000).cpu().numpy()
    assert np.array_equal(k, oracle.gen_keys16(42, 123456, 5000))


def test_bloom_fixed24_workload_keys(oracle, amq, torch):
    keys = [ln.strip().encode() for ln in open(os.path.join(GOLDEN, "workload_e_keys.txt")) if ln.strip()]
    blob = np.frombuffer(b"".join(keys), dtype=np.uint8).reshape(len(keys), 24).copy()
    plan, out = gpu_build(amq, torch, 0, torch.from_numpy(blob).cuda(), [len(keys)], 10, src=[7])
    assert segment_bytes(plan, out, 0) == open(os.path.join(GOLDEN, "workload_e_bloom10.bin"), "rb").read()
    plan, out = gpu_build(amq, torch, 1, torch.from_numpy(blob).cuda(), [len(keys)], 12, src=[7])
    assert segment_bytes(plan, out, 0) == open(os.path.join(GOLDEN, "workload_e_vqf12.bin"), "rb").read()


@pytest.mark.parametrize("kind", [0, 1])
def test_variable_length_keys(oracle, amq, torch, kind):
    rng = np.random.default_rng(11)
    counts = [3000, 0, 17, 4096]
    lens = rng.integers(0, 72, sum(counts))
    blob = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8)
    offs = np.zeros(len(lens) + 1, np.int64)
    offs[1:] = np.cumsum(lens)
    bpk = 10 if kind == 0 else 13
    ref = oracle_per_segment(oracle, kind, blob, counts, bpk, offsets=offs.astype(np.uint64))
    plan, out = gpu_build(amq, torch, kind, torch.from_numpy(blob).cuda(), counts, bpk,
                          offsets_t=torch.from_numpy(offs).cuda())
    assert_same(plan, out, ref)


@pytest.mark.parametrize("kind", [0, 1])
@pytest.mark.parametrize("tail", ["tiny", "every_length"])
def test_variable_length_key_windows(oracle, amq, torch, kind, tail):
    """Short keys are read as 32-byte windows through a buffer resource over their chunk or
    leaf, the window clamped into the key array: the array's last keys come through a shifted
    window and are realigned by 1..31 bytes (every length 0..31 ends the array here), and an
    array of fewer than 32 bytes takes the per-piece loads.  Bloom (64+ leaves: the length-
    sorted LDS build) and VQF (ring kernels) against the oracle."""
    rng = np.random.default_rng(23)
    if tail == "tiny":
        lens = np.array([0, 1, 2, 3, 4, 5, 6], np.int64)  # 21 bytes in all
        counts = [len(lens)] + [0] * 63
    else:
        body = rng.integers(6, 40, 5000)  # (many duplicates of very short keys would overflow
                                          # a VQF block, in the oracle too)
        lens = np.concatenate([body, np.arange(31, -1, -1), np.arange(0, 32)]).astype(np.int64)
        counts = [int(c) for c in rng.integers(0, 70, 63)]
        counts.append(len(lens) - sum(counts))
    blob = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8)
    offs = np.zeros(len(lens) + 1, np.int64)
    offs[1:] = np.cumsum(lens)
    bpk = 10 if kind == 0 else 12
    ref = oracle_per_segment(oracle, kind, blob, counts, bpk, offsets=offs.astype(np.uint64))
    plan, out = gpu_build(amq, torch, kind, torch.from_numpy(blob).cuda(), counts, bpk,
                          offsets_t=torch.from_numpy(offs).cuda())
    assert_same(plan, out, ref)


@pytest.mark.parametrize("big_leaf", [False, True])
def test_variable_length_keys_many_leaves(oracle, amq, torch, big_leaf):
    """Batches of >= 64 leaves take the per-leaf LDS build, bloom_build_lds<kKeyVar> (fewer
    leaves take the spread atomic path).  Empty leaves, a 45000-key leaf (big_leaf: a 56 KiB
    image), every short length, keys of >= 32 bytes, and the generic-k loop (5 bits/key ->
    k = 3)."""
    rng = np.random.default_rng(12)
    counts = [int(c) for c in rng.integers(0, 700, 70)]
    counts[3], counts[10], counts[11], counts[40] = 0, 4096, 9000, 513
    if big_leaf:
        counts[50] = 45000
    lens = rng.integers(0, 72, sum(counts))
    blob = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8)
    offs = np.zeros(len(lens) + 1, np.int64)
    offs[1:] = np.cumsum(lens)
    for bpk in (10, 12, 5):
        ref = oracle_per_segment(oracle, 0, blob, counts, bpk, offsets=offs.astype(np.uint64))
        plan, out = gpu_build(amq, torch, 0, torch.from_numpy(blob).cuda(), counts, bpk,
                              offsets_t=torch.from_numpy(offs).cuda())
        assert_same(plan, out, ref)


@pytest.mark.parametrize("n_leaves", [64, 300, 1023, 1024])
@pytest.mark.parametrize("shape", ["k16", "k24", "var"])
def test_bloom_leaf_kernel_widths(oracle, amq, torch, n_leaves, shape):
    """Below 1024 leaves each leaf's keys are split over several workgroups whose images are
    ORed by the last one (bloom_build_split); from 1024 leaves one workgroup per leaf
    (bloom_build_lds).  Both, every key shape, ragged leaves, against the oracle (sampled)."""
    rng = np.random.default_rng(n_leaves)
    counts = [int(c) for c in rng.integers(0, 3000, n_leaves)]
    counts[0], counts[1], counts[-1] = 0, 16384, 1
    n = sum(counts)
    offs = None
    if shape == "k16":
        keys, stride = oracle.gen_keys16(42, 0, n), 16
    elif shape == "k24":
        keys, stride = rng.integers(0, 256, (n, 24), dtype=np.uint8), 24
    else:
        lens = rng.integers(0, 40, n)
        keys, stride = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8), 0
        offs = np.zeros(n + 1, np.int64)
        offs[1:] = np.cumsum(lens)
    plan, out = gpu_build(amq, torch, 0, torch.from_numpy(keys).cuda(), counts, 10,
                          offsets_t=None if offs is None else torch.from_numpy(offs).cuda())
    sb = seg_bounds(counts)
    for s in sorted({0, 1, n_leaves - 1, *rng.integers(0, n_leaves, 12).tolist()}):
        b, c = int(sb[s]), counts[s]
        if offs is None:
            st, ref = oracle.bloom_build(keys[b:], c, 10, src_page_id=s, stride=stride)
        else:
            o = (offs[b:b + c + 1] - offs[b]).astype(np.uint64)
            st, ref = oracle.bloom_build(keys[int(offs[b]):], c, 10, src_page_id=s, offsets=o, stride=0)
        assert st == 0
        assert segment_bytes(plan, out, s) == ref.tobytes(), f"leaf {s}"


@pytest.mark.parametrize("counts", [[16384], [16384, 9000, 1, 0, 52000], [3000] * 200,
                                    [100000], [120000, 700, 0, 5]])
def test_bloom_split_matches_unsplit(oracle, amq, torch, counts):
    """The split build (workspace given) and the one-workgroup / atomic builds (no workspace)
    write the same bytes; the split one also equals the oracle (a 52K-key leaf: a 64 KiB
    image; 100K- and 120K-key leaves: 125 and 150 KB images, up to the 160 KB the split parts
    take in LDS)."""
    keys = oracle.gen_keys16(9, 0, sum(counts))
    kt = torch.from_numpy(keys).cuda()
    plan = amq.plan_filters(0, counts, 10)
    assert plan.workspace_bytes > 0
    a = amq.build_all_filters(plan, amq.KeyBatch.fixed(kt))
    L, F = amq.abi.lib(), amq.filters
    b = torch.zeros_like(a)
    st = L.tkv_amq_build(0, F._ptr(kt), None, 16, kt.shape[0], F._ptr(plan.device_segs()), plan.n_segs,
                         plan.max_seg_blocks, F._ptr(b), None, 0, F._stream_handle())
    assert st == 0
    torch.cuda.synchronize()
    an, bn = a.cpu().numpy(), b.cpu().numpy()
    sb = seg_bounds(counts)
    for s in range(len(counts)):
        assert segment_bytes(plan, an, s) == segment_bytes(plan, bn, s), f"leaf {s}"
        st, ref = oracle.bloom_build(keys[int(sb[s]):], counts[s], 10, src_page_id=s)
        assert segment_bytes(plan, an, s) == ref.tobytes(), f"leaf {s}"


def sorted_keys(oracle, seed, counts):
    keys = oracle.gen_keys16(seed, 0, sum(counts))
    oracle.sort_segments(keys, seg_bounds(counts))
    return keys


@pytest.mark.parametrize("bpk,cap", [(12, 32704), (13, 32704), (16, 32704), (22, 65472),
                                     (24, 65472), (32, 65472), (12, 16320), (12, 8128)])
def test_vqf_parity(oracle, amq, torch, bpk, cap):
    counts = RAGGED
    keys = sorted_keys(oracle, 42, counts)
    src = [500 + i for i in range(len(counts))]
    ref = oracle_per_segment(oracle, 1, keys, counts, bpk, cap=cap, src=src)
    plan, out = gpu_build(amq, torch, 1, torch.from_numpy(keys).cuda(), counts, bpk, cap=cap,
                          src=src)
    assert_same(plan, out, ref)


@pytest.mark.parametrize("bpk,cap", [(22, 65472), (32, 16320)])
def test_vqf_parity_fused_16bit_tags(oracle, amq, torch, bpk, cap):
    """16-bit tags (and, at 32 bpk in 16 KB pages, 8-bit truncated and 16-bit leaves in one
    batch) through the fused LDS place path: every leaf small enough that the batch's LDS
    image fits."""
    counts = [8000, 777, 5000, 1, 0, 64, 7000]
    keys = sorted_keys(oracle, 43, counts)
    src = [900 + i for i in range(len(counts))]
    ref = oracle_per_segment(oracle, 1, keys, counts, bpk, cap=cap, src=src)
    plan, out = gpu_build(amq, torch, 1, torch.from_numpy(keys).cuda(), counts, bpk, cap=cap,
                          src=src)
    assert plan.max_seg_blocks * 132 <= 80 * 1024, "batch should take the fused place"
    assert 16 in set(plan.segs["tag_bits"].tolist())
    assert_same(plan, out, ref)


def test_vqf_config1_sha256(oracle, amq, torch):
    g = json.load(open(os.path.join(GOLDEN, "filters.json")))["config1_vqf12_1M"]
    n = g["n_keys"]
    counts = [S] * (n // S) + [n % S]
    keys = sorted_keys(oracle, 42, counts)
    plan = amq.plan_filters(1, counts, 12, payload_capacity=32704, out_stride=32704)
    out = amq.build_all_filters(plan, amq.KeyBatch.fixed(torch.from_numpy(keys).cuda()))
    o = out.cpu().numpy()
    # the golden buffer has zero tails after each payload; the GPU writes payloads only
    for s in range(plan.n_segs):
        seg = plan.segs[s]
        o[int(seg["out_offset"]) + int(seg["payload_bytes"]):int(seg["out_offset"]) + 32704] = 0
    assert hashlib.sha256(o.tobytes()).hexdigest() == g["sha256"]


def test_vqf_unsorted_and_duplicate_keys(oracle, amq, torch):
    # insertion order matters for VQF: unsorted input and duplicate keys must still match
    counts = [16384, 9000]
    keys = oracle.gen_keys16(77, 0, sum(counts))
    keys[100:200] = keys[0:100]
    ref = oracle_per_segment(oracle, 1, keys, counts, 12)
    plan, out = gpu_build(amq, torch, 1, torch.from_numpy(keys).cuda(), counts, 12)
    assert_same(plan, out, ref)


@pytest.mark.parametrize("n_leaves", [40, 768, 769, 4097])
@pytest.mark.parametrize("shape", ["k16", "k24", "k20", "var"])
def test_vqf_decide_paths(oracle, amq, torch, n_leaves, shape):
    """Batches of up to 768 leaves (4,096 for keys read where they are hashed: 20-byte and
    variable-length ones) take vqf_decide_ring (producer waves locate and match each 64-key
    chunk, one decider wave replays the insertion order), larger ones vqf_decide (one wave
    per leaf); 16- and 24-byte keys are loaded ahead of their hash.  8- and 16-bit tags (12 / 22 bits per key), leaves of <= 512 and
    > 512 blocks (the producers' 9- and 11-bit matches, vqf_decide's LDS lane-mask table past
    512 blocks; a 30000-key leaf of ~740 blocks, placed in LDS), 4- and 8-byte key records,
    ragged leaves, every key shape, sampled against the oracle.  (The unfused place and the
    ballot matches: test_vqf_leaf_beyond_ring_blocks.)"""
    rng = np.random.default_rng(1000 + n_leaves)
    counts = [int(c) for c in rng.integers(0, 3000, n_leaves)]
    counts[0], counts[1], counts[2], counts[-1] = 0, 16384, 30000, 1
    n = sum(counts)
    offs = None
    if shape == "k16":
        keys, stride = oracle.gen_keys16(5, 0, n), 16
    elif shape in ("k24", "k20"):
        stride = int(shape[1:])
        keys = rng.integers(0, 256, (n, stride), dtype=np.uint8)
    else:  # >= 6 bytes: duplicates of very short keys would overflow a block (as in the oracle)
        lens = rng.integers(6, 40, n)
        keys, stride = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8), 0
        offs = np.zeros(n + 1, np.int64)
        offs[1:] = np.cumsum(lens)
    sb = seg_bounds(counts)
    for bpk in (12, 22):
        # (4,097 random leaves hold one whose 16-bit filter overflows -- vqf_insert fails in the
        # oracle too, as in the reference; the leaves compared are those the oracle builds)
        plan, out = gpu_build(amq, torch, 1, torch.from_numpy(keys).cuda(), counts, bpk, cap=65472,
                              offsets_t=None if offs is None else torch.from_numpy(offs).cuda(),
                              check=n_leaves < 4097)
        if bpk == 12:
            assert plan.segs["n_blocks"][2] > 512 and plan.segs["n_blocks"][1] <= 512
        else:
            assert plan.segs["n_blocks"][1] > 512 and 16 in set(plan.segs["tag_bits"].tolist())
        for s in sorted({0, 1, 2, n_leaves - 1, *rng.integers(0, n_leaves, 10).tolist()}):
            b, c = int(sb[s]), counts[s]
            if offs is None:
                st, ref, p = oracle.vqf_build(keys[b:], c, bpk, 65472, src_page_id=s, stride=stride)
            else:
                o = (offs[b:b + c + 1] - offs[b]).astype(np.uint64)
                st, ref, p = oracle.vqf_build(keys[int(offs[b]):], c, bpk, 65472, src_page_id=s,
                                              offsets=o, stride=0)
            if st != 0 and n_leaves == 4097:
                continue
            assert st == 0
            assert segment_bytes(plan, out, s) == ref[:p.payload_used].tobytes(), f"bpk {bpk} leaf {s}"


@pytest.mark.parametrize("shape", ["k20", "var", "var_long"])
def test_vqf_decide_odd_keys_all_leaves(oracle, amq, torch, shape):
    """Past 4,096 leaves, keys other than 16 or 24 bytes take vqf_decide, hashing each key in
    the leaf's chain.  EVERY leaf against the oracle (its batched build over the same key
    shape): 8-bit tags with 4-byte records, leaves past 512 blocks with 8-byte records, and keys
    of 32 bytes or more (var_long: XXH64's long path)."""
    rng = np.random.default_rng(77)
    n_leaves = 4200
    counts = [int(c) for c in rng.integers(0, 4000, n_leaves)]
    counts[0], counts[7], counts[100] = 0, 30000, 16384
    n = sum(counts)
    offs = None
    if shape == "k20":
        keys, stride = rng.integers(0, 256, (n, 20), dtype=np.uint8), 20
    else:
        lens = rng.integers(6, 40 if shape == "var" else 80, n)
        keys, stride = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8), 0
        offs = np.zeros(n + 1, np.int64)
        offs[1:] = np.cumsum(lens)
    plan, out = gpu_build(amq, torch, 1, torch.from_numpy(keys).cuda(), counts, 12, cap=65472,
                          offsets_t=None if offs is None else torch.from_numpy(offs).cuda())
    assert plan.segs["n_blocks"][7] > 512
    ref = np.zeros(len(out) + 65472, np.uint8)
    st = oracle.build_segments_ex(1, keys.reshape(-1), None if offs is None else offs.astype(np.uint64),
                                  stride, seg_bounds(counts), 12, plan.segs["out_offset"],
                                  np.full(n_leaves, 65472, np.uint64), ref,
                                  src_page_id=plan.segs["src_page_id"], n_threads=min(16, os.cpu_count()))
    assert st == 0
    for s_ in range(n_leaves):
        o, b = int(plan.segs["out_offset"][s_]), int(plan.segs["payload_bytes"][s_])
        if out[o:o + b].tobytes() != ref[o:o + b].tobytes():
            pytest.fail(f"leaf {s_} ({counts[s_]} keys) differs from the oracle")


@pytest.mark.parametrize("n_leaves", [1, 256, 257, 512])
@pytest.mark.parametrize("edge", ["b402", "tbl", "ring512", "ring960", "plain961"])
@pytest.mark.parametrize("bpk", [12, 22])
def test_vqf_ring_place_classes(oracle, amq, torch, n_leaves, edge, bpk):
    """Batches of <= 256 leaves whose largest leaf has <= 884 blocks take vqf_ring_place
    (decide and place in one workgroup per leaf, entries straight into the LDS image; <= 512
    blocks: the producers' LDS match tables), batches of up to 512 leaves of <= 420 blocks two
    such workgroups per CU (b402: the bench layout's 16K-key leaves), others vqf_decide_ring +
    vqf_place_fused.  The batch's largest leaf sits at each threshold (512 / 513 / 960 / 961
    blocks in 64 KiB pages), 8- and 16-bit tags; byte-equal to the oracle."""
    big = {12: {"b402": 16384, "tbl": 20889, "ring512": 20890, "ring960": 39167, "plain961": 39168},
           22: {"b402": 9000, "tbl": 11729, "ring512": 11730, "ring960": 21992, "plain961": 21993}}[bpk][edge]
    rng = np.random.default_rng(7 + n_leaves)
    counts = [big] + [int(c) for c in rng.integers(0, 3000, n_leaves - 1)]
    if n_leaves > 2:
        counts[1] = 0
    keys = oracle.gen_keys16(9, 0, sum(counts))
    plan, out = gpu_build(amq, torch, 1, torch.from_numpy(keys).cuda(), counts, bpk, cap=65472)
    want = {"b402": None, "tbl": 512, "ring512": 513, "ring960": 960, "plain961": 961}[edge]
    if want is not None:
        assert int(plan.segs["n_blocks"].max()) == want
    else:
        assert int(plan.segs["n_blocks"].max()) <= 420
    sb = seg_bounds(counts)
    for s in sorted({0, n_leaves - 1, *rng.integers(0, n_leaves, 4).tolist()}):
        st, ref, p = oracle.vqf_build(keys[int(sb[s]):], counts[s], bpk, 65472, src_page_id=s)
        assert st == 0
        assert segment_bytes(plan, out, s) == ref[:p.payload_used].tobytes(), f"leaf {s}"


@pytest.mark.parametrize("shape", ["k16", "k24", "k20", "var"])
@pytest.mark.parametrize("bpk", [12, 22])
@pytest.mark.parametrize("cap", [65472, 8128])
def test_vqf_ring_edges(oracle, amq, torch, shape, bpk, cap):
    """vqf_ring_place on the leaves where a decider step changes kind: 30 keys in one block
    (no key ever reaches the alternate-choice threshold), 40 keys in one block (the threshold
    is reached inside the first 64-key chunk; two blocks each at 16-bit tags), 1 and 0 keys,
    700, a 16,384-key leaf; 8- and 16-bit tags; in 8 KiB pages (cap 8128) the larger leaves
    keep only masked keys (hash_val_shift > 0); 16-, 24-, 20-byte and variable-length keys
    (the last two through vqf_locate_keys' located records).  Byte-equal to the oracle.  (The round-4 parallel-prefix variant of the ring,
    tools/patches/r04_vqf_loc_prefix_tile_loop.patch, was checked with these leaves.)"""
    counts = [30, 40, 1, 0, 700, 16384, 5000]
    n = sum(counts)
    rng = np.random.default_rng(11)
    offs = None
    if shape == "k16":
        keys, stride = oracle.gen_keys16(12, 0, n), 16
    elif shape in ("k24", "k20"):
        stride = int(shape[1:])
        keys = rng.integers(0, 256, (n, stride), dtype=np.uint8)
    else:
        lens = rng.integers(6, 40, n)
        keys, stride = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8), 0
        offs = np.zeros(n + 1, np.int64)
        offs[1:] = np.cumsum(lens)
    plan, out = gpu_build(amq, torch, 1, torch.from_numpy(keys).cuda(), counts, bpk, cap=cap,
                          offsets_t=None if offs is None else torch.from_numpy(offs).cuda())
    assert int(plan.segs["n_blocks"][:2].max()) <= 2  # (one block at 8-bit tags, two at 16)
    if cap == 8128:
        assert int(plan.segs["hash_val_shift"][5]) > 0
    if bpk == 22:
        assert 16 in set(plan.segs["tag_bits"].tolist())
    sb = seg_bounds(counts)
    for s in range(len(counts)):
        b, c = int(sb[s]), counts[s]
        if offs is None:
            st, ref, p = oracle.vqf_build(keys[b:], c, bpk, cap, src_page_id=s, stride=stride)
        else:
            o = (offs[b:b + c + 1] - offs[b]).astype(np.uint64)
            st, ref, p = oracle.vqf_build(keys[int(offs[b]):], c, bpk, cap, src_page_id=s,
                                          offsets=o, stride=0)
        assert st == 0
        assert segment_bytes(plan, out, s) == ref[:p.payload_used].tobytes(), f"leaf {s}"


@pytest.mark.parametrize("shape,n_leaves", [("var", 64), ("var", 65), ("k20", 32), ("k20", 33)])
def test_vqf_located_keys_threshold(oracle, amq, torch, shape, n_leaves):
    """Either side of the leaf counts up to which small VQF batches of variable-length (64)
    and 20-byte (32) keys are hashed and located on the whole chip before vqf_ring_place
    (kVqfLocMaxSegsVar/Fixed): ragged leaves, byte-equal to the oracle on a sample."""
    rng = np.random.default_rng(n_leaves)
    counts = rng.integers(0, 3000, n_leaves).tolist()
    counts[1] = 0
    n = sum(counts)
    offs = None
    if shape == "k20":
        keys, stride = rng.integers(0, 256, (n, 20), dtype=np.uint8), 20
    else:
        lens = rng.integers(1, 48, n)
        keys, stride = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8), 0
        offs = np.zeros(n + 1, np.int64)
        offs[1:] = np.cumsum(lens)
    plan, out = gpu_build(amq, torch, 1, torch.from_numpy(keys).cuda(), counts, 12, cap=65472,
                          offsets_t=None if offs is None else torch.from_numpy(offs).cuda())
    sb = seg_bounds(counts)
    for s in sorted({0, 1, n_leaves - 1, *rng.integers(0, n_leaves, 5).tolist()}):
        b, c = int(sb[s]), counts[s]
        if offs is None:
            st, ref, p = oracle.vqf_build(keys[b:], c, 12, 65472, src_page_id=s, stride=stride)
        else:
            o = (offs[b:b + c + 1] - offs[b]).astype(np.uint64)
            st, ref, p = oracle.vqf_build(keys[int(offs[b]):], c, 12, 65472, src_page_id=s,
                                          offsets=o, stride=0)
        assert st == 0
        assert segment_bytes(plan, out, s) == ref[:p.payload_used].tobytes(), f"leaf {s}"


@pytest.mark.parametrize("big", [100000, 260000])
@pytest.mark.parametrize("n_leaves", [4, 800])
@pytest.mark.parametrize("bpk", [12, 22])
def test_vqf_leaf_beyond_ring_blocks(oracle, amq, torch, n_leaves, big, bpk):
    """A 100000-key leaf in 1 MiB pages has 2451 blocks: more than the ring kernel's count
    table holds, so its wave 0 runs vqf_decide_body (block-id ballots, no LDS match table);
    in a batch of 800 leaves vqf_decide does the same.  Its LDS place is split over two
    workgroups per leaf; a 260000-key leaf (6373 blocks, beyond four) takes the unfused
    scatter + place.  At 22 bits/key: 16-bit tags, 4365 / 11349 blocks."""
    counts = [big, 500, 0, 16384] + [300] * (n_leaves - 4)
    keys = oracle.gen_keys16(6, 0, sum(counts))
    plan, out = gpu_build(amq, torch, 1, torch.from_numpy(keys).cuda(), counts, bpk, cap=1 << 20)
    assert plan.segs["n_blocks"][0] > 2048 and plan.segs["hash_val_shift"][0] == 0
    assert (plan.segs["n_blocks"][0] > 4964) == (big == 260000)
    sb = seg_bounds(counts)
    for s in sorted({0, 1, 2, 3, n_leaves - 1}):
        st, ref, p = oracle.vqf_build(keys[int(sb[s]):], counts[s], bpk, 1 << 20, src_page_id=s)
        assert st == 0
        assert segment_bytes(plan, out, s) == ref[:p.payload_used].tobytes(), f"leaf {s}"


@pytest.mark.parametrize("big,bpk,cap", [(700_000, 12, 4 << 20), (700_000, 22, 4 << 20),
                                         (7_000_000, 12, 16 << 20)])
def test_vqf_huge_leaf(oracle, amq, torch, big, bpk, cap):
    """Leaves past vqf_decide's u32 LDS count table (16,384 blocks), which round 2 refused:
    a 700K-key leaf (17,157 blocks at 12 bits/key, 30,553 with 16-bit tags at 22) keeps u8
    counts in LDS; a 7M-key leaf (171,569 blocks) keeps them in the workspace's block records
    (agent-scope atomics).  Both are placed by the multi-workgroup unfused place, in a batch
    with small leaves, and must equal the oracle byte for byte."""
    counts = [big, 500, 0, 16384] if big < 1_000_000 else [big, 3000]
    keys = oracle.gen_keys16(8, 0, sum(counts))
    plan, out = gpu_build(amq, torch, 1, torch.from_numpy(keys).cuda(), counts, bpk, cap=cap)
    nb = int(plan.segs["n_blocks"][0])
    assert nb > 16384 and (nb > 160 * 1024) == (big > 1_000_000)
    sb = seg_bounds(counts)
    for s in range(len(counts)):
        st, ref, p = oracle.vqf_build(keys[int(sb[s]):], counts[s], bpk, cap, src_page_id=s)
        assert st == 0
        assert segment_bytes(plan, out, s) == ref[:p.payload_used].tobytes(), f"leaf {s}"


def probe_inputs(oracle, n_keys, counts, n_miss):
    hits = np.arange(n_keys)
    seg_of = np.repeat(np.arange(len(counts)), counts)
    miss = oracle.gen_keys16(43, 0, n_miss)
    rng = np.random.default_rng(44)
    miss_seg = rng.integers(0, len(counts), n_miss)
    return hits, seg_of, miss, miss_seg


@pytest.mark.parametrize("kind,bpk", [(0, 10), (0, 12), (1, 12), (1, 24)])
def test_probe_parity(oracle, amq, torch, kind, bpk):
    counts = [S] * 8 + [8448, 0, 5]
    keys = sorted_keys(oracle, 42, counts) if kind else oracle.gen_keys16(42, 0, sum(counts))
    cap = 65472
    plan = amq.plan_filters(kind, counts, bpk, payload_capacity=cap if kind else 0)
    filt = amq.build_all_filters(plan, amq.KeyBatch.fixed(torch.from_numpy(keys).cuda()))
    n = sum(counts)
    _, seg_of, miss, miss_seg = probe_inputs(oracle, n, counts, 200000)
    q = np.concatenate([keys, miss])
    qs = np.concatenate([seg_of, miss_seg]).astype(np.uint32)
    res = amq.probe_filters(plan, filt, amq.KeyBatch.fixed(torch.from_numpy(q).cuda()),
                            torch.from_numpy(qs.astype(np.int32)).cuda()).cpu().numpy()
    # oracle probe over the GPU-built filter bytes (which equal the oracle's, tested above)
    st, ref = oracle.probe_segments(kind, filt.cpu().numpy(), plan.segs["out_offset"], q, qs)
    assert st == 0
    assert np.array_equal(res, ref)
    assert res[:n].all(), "false negative"
    fpr = res[n:].mean()
    assert fpr < (0.02 if kind == 0 else 0.01)
    if kind == 1:
        hv = amq.vqf_hash_val(amq.KeyBatch.fixed(torch.from_numpy(q).cuda()))
        res2 = amq.vqf_probe_hashed(plan, filt, hv, torch.from_numpy(qs.astype(np.int32)).cuda())
        assert np.array_equal(res2.cpu().numpy(), ref)


def test_vqf_hash_matches_xxhash(amq, torch):
    import xxhash
    keys = [ln.strip().encode() for ln in open(os.path.join(GOLDEN, "workload_e_keys.txt")) if ln.strip()]
    kb = amq.KeyBatch.from_host(keys[:1000])
    h = amq.vqf_hash_val(kb).cpu().numpy().view(np.uint64)
    assert [int(x) for x in h] == [xxhash.xxh64_intdigest(k, VQF_SEED) for k in keys[:1000]]
    h16 = amq.vqf_hash_val(amq.KeyBatch.fixed(amq.gen_keys16(1, 0, 1000))).cpu().numpy().view(np.uint64)
    k16 = amq.gen_keys16(1, 0, 1000).cpu().numpy()
    assert [int(x) for x in h16] == [xxhash.xxh64_intdigest(k.tobytes(), VQF_SEED) for k in k16]


@pytest.mark.parametrize("n,bpk,seed", [(600000, 10, 8), (3000000, 10, 9), (1500000, 12, 10),
                                         (1100000, 5, 11), (90000, 64, 12), (8_000_000, 10, 13),
                                         (14_000_000, 10, 14)])
def test_bloom_monolithic_partitioned(oracle, amq, torch, n, bpk, seed):
    """One filter of 16-byte keys larger than one LDS window (160 KB; tests/test_gpu_window.py
    has 2-4-window ones too): the hash-once record path (bloom_part_keys16 /
    bloom_tile), byte-identical to the oracle.  Covers a ragged last tile, k = 7 / 8 /
    generic <= 8 (12-byte bit records) and k = 44 (the keys themselves are partitioned and
    hashed per tile); below 128 tiles each tile's regions split over up to 16 tile workgroups
    and their partial images merged (6 tiles x 16, 29 x 8, 77 x 3), 134 tiles unsplit."""
    keys = oracle.gen_keys16(seed, 0, n)
    ref = oracle_per_segment(oracle, 0, keys, [n], bpk)
    plan, out = gpu_build(amq, torch, 0, torch.from_numpy(keys).cuda(), [n], bpk)
    assert plan.max_seg_blocks * 64 > 160 * 1024
    assert plan.workspace_bytes >= 16 * n  # the partitioned path's workspace
    assert_same(plan, out, ref)


@pytest.mark.parametrize("n,bpk,dup", [(600000, 10, 0), (1500000, 12, 0), (1100000, 5, 0),
                                       (400000, 14, 0), (90000, 64, 0), (700000, 10, 200000),
                                       (450000, 14, 150000)])
def test_bloom_monolithic_k24(oracle, amq, torch, n, bpk, dup):
    """One filter of 24-byte keys (TurtleKV's default key size) beyond one window: the record
    path's own partition kernel (bloom_part_keys24) hashes each key once into a 12-byte bit
    record; k > 8 (14 and 64 bits/key) keeps the first eight bits in the records and
    bloom_overflow sets the others; duplicates overflow the regions of one tile.
    Byte-identical to the oracle (round 2: device atomics)."""
    rng = np.random.default_rng(n + bpk)
    keys = rng.integers(0, 256, (n, 24), dtype=np.uint8)
    if dup:
        keys[n - dup:] = keys[n // 3]
    ref = oracle_per_segment(oracle, 0, keys, [n], bpk, stride=24)
    plan, out = gpu_build(amq, torch, 0, torch.from_numpy(keys).cuda(), [n], bpk)
    assert plan.max_seg_blocks * 64 > 4 * 160 * 1024
    assert_same(plan, out, ref)


def test_bloom_monolithic_duplicate_keys(oracle, amq, torch):
    """Every key identical (one tile receives the whole batch: its regions overflow and the
    overflow lists are applied with device atomics) and a few distinct ones."""
    n = 200000
    keys = np.repeat(oracle.gen_keys16(13, 0, 1), n, axis=0)
    keys[::50000] = oracle.gen_keys16(14, 0, len(keys[::50000]))
    ref = oracle_per_segment(oracle, 0, keys, [n], 10)
    plan, out = gpu_build(amq, torch, 0, torch.from_numpy(keys).cuda(), [n], 10)
    assert_same(plan, out, ref)


def sampled_tiles_equal_oracle(oracle, out, n, bpk, seed, n_random=6, extra_tiles=(), whole=False):
    """The header and sampled tiles of a GPU-built monolithic filter over gen_keys16(seed, 0, n)
    (the first, the last, six seeded-random ones and `extra_tiles`, e.g. both sides of every
    routed part boundary) against the oracle, which generates and hashes every key for them
    (oracle.bloom_sample_blocks); whole=True compares the whole bitmap (one window)."""
    from turtle_kv_amd.dist import BLOOM_TILE_BLOCKS as TB
    nb = int(oracle.lib().tkvo_bloom_block_count(n, bpk))
    T = -(-nb // TB)
    rng = np.random.default_rng(seed)
    tiles = sorted({0, T - 1, *[int(t) for t in rng.choice(T, size=min(n_random, T), replace=False)],
                    *[int(t) for t in extra_tiles if 0 <= t < T]})
    wins = [(0, nb)] if whole else [(t * TB, min(nb, (t + 1) * TB)) for t in tiles]
    st, got = oracle.bloom_sample_blocks(seed, 0, n, bpk, wins, n_threads=min(16, os.cpu_count()))
    assert st == 0
    for (lo, hi), ref in got.items():
        mine = out[64 + 64 * lo:64 + 64 * hi].cpu().numpy()
        if mine.tobytes() != ref.tobytes():
            bad = sorted({(lo + int(i) // 64) // TB for i in np.nonzero(mine != ref)[0][:100000]})
            pytest.fail(f"blocks [{lo}, {hi}) differ in tiles {bad[:16]} of {T}")
    k = int(oracle.lib().tkvo_bloom_hash_count(bpk))
    hdr = np.frombuffer(out[:64].cpu().numpy().tobytes(), dtype="<u8")
    assert [int(x) for x in hdr[:7]] == [0xCA6F49A0F3F8A4B0, 512 * nb, 0, 0, 8 * nb,
                                        nb | (k << 32) | (2 << 48), n]
    return T


@pytest.mark.parametrize("n,bpk,parts,whole", [(108_000_000, 10, 1, True), (1_750_000_000, 12, 79, False),
                                               (700_000_000, 64, 27, False),
                                               (600_000_000, 12, 27, True)])
def test_bloom_monolithic_large_sampled_oracle(oracle, amq, torch, n, bpk, parts, whole):
    """Full-size monolithic filters against the oracle: 108M keys at 10 bits/key (1,030 tiles:
    the partition reads the keys) and 600M keys at 12 bits/key (6,867 tiles: routed as 12-byte
    records into 27 parts) over the WHOLE bitmap; 1.75B keys at 12 bits/key (20,028 tiles,
    beyond one partition's 6,400-tile table: routed into 79 parts of <= 256 tiles, each built
    from its records, its count read on the device) and 700M keys at 64 bits/key (42,725 tiles,
    k = 44: the 16-byte keys themselves routed into 27 parts) on the header, eight sampled
    tiles and the tiles on both sides of every part boundary."""
    from turtle_kv_amd import abi
    L = abi.lib()
    seed = 16
    plan = amq.plan_filters(0, [n], bpk)
    T = -(-int(plan.max_seg_blocks) // int(L.tkv_amq_bloom_tile_blocks()))
    direct = T <= int(L.tkv_amq_bloom_range_max_tiles(0))
    assert direct == (parts == 1)
    if not direct:
        from turtle_kv_amd.dist import ROUTED_KEY_PART_TILES, ROUTED_PART_TILES
        assert -(-T // (ROUTED_PART_TILES if bpk <= 12 else ROUTED_KEY_PART_TILES)) == parts
    edges = []
    if not direct:
        q = -(-T // parts)
        edges = [t for j in range(1, parts) for t in (j * q - 1, j * q)]
    keys = amq.gen_keys16(seed, 0, n)
    out = amq.build_all_filters(plan, amq.KeyBatch.fixed(keys))
    del keys
    torch.cuda.synchronize()
    assert sampled_tiles_equal_oracle(oracle, out, n, bpk, seed, extra_tiles=edges, whole=whole) == T
    del out
    torch.cuda.empty_cache()


@pytest.mark.parametrize("shape", ["k16", "k24", "var"])
def test_bloom_big_leaves_in_lds(oracle, amq, torch, shape):
    """Batches of >= 64 leaves build leaf images of up to 160 KB in LDS (1024-thread
    workgroups above 32 KB; TurtleKV leaves of small items reach ~80K keys): a 100000-key leaf
    (125 KB at 10 bits/key, 150 KB at 12) and a 40000-key one among small leaves; at 14 bits/key
    the 100000-key leaf (175 KB) sends the batch to the window path (two windows)."""
    rng = np.random.default_rng(77)
    counts = [int(c) for c in rng.integers(0, 2000, 70)]
    counts[5], counts[40], counts[69] = 100000, 40000, 0
    n = sum(counts)
    offs = None
    if shape == "k16":
        keys, stride = oracle.gen_keys16(21, 0, n), 16
    elif shape == "k24":
        keys, stride = rng.integers(0, 256, (n, 24), dtype=np.uint8), 24
    else:
        lens = rng.integers(4, 40, n)
        keys, stride = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8), 0
        offs = np.zeros(n + 1, np.int64)
        offs[1:] = np.cumsum(lens)
    for bpk in (10, 12, 14):
        ref = oracle_per_segment(oracle, 0, keys, counts, bpk, stride=stride,
                                 offsets=None if offs is None else offs.astype(np.uint64))
        plan, out = gpu_build(amq, torch, 0, torch.from_numpy(keys).cuda(), counts, bpk,
                              offsets_t=None if offs is None else torch.from_numpy(offs).cuda())
        assert (plan.max_seg_blocks * 64 > 160 * 1024) == (bpk == 14)
        assert_same(plan, out, ref)


@pytest.mark.parametrize("big", [140000, 3_000_000])
def test_bloom_oversize_leaf_in_batch(oracle, amq, torch, big):
    """A multi-leaf batch holding a leaf beyond the LDS budget: a 175 KB image takes the
    window path (partial images in the workspace, merged); a 3.75 MB one (24 windows, more
    than the window path's 16) the tiled monolithic build of its own (tkv_amq_build_ex), the
    other leaves the batch kernels from a compacted leaf list."""
    counts = [big, 500, 16384]
    keys = oracle.gen_keys16(15, 0, sum(counts))
    ref = oracle_per_segment(oracle, 0, keys, counts, 10)
    plan, out = gpu_build(amq, torch, 0, torch.from_numpy(keys).cuda(), counts, 10)
    assert plan.workspace_bytes > 0
    assert_same(plan, out, ref)


@pytest.mark.parametrize("shape", ["k16", "k24", "var"])
def test_bloom_oversize_leaves_among_many(oracle, amq, torch, shape):
    """Several oversize leaves (past 16 windows) at the start, middle and end of a batch of
    small and window-sized leaves, 16- and 24-byte keys (the monolithic build, one leaf at a
    time) and variable-length keys (those leaves with device atomics, the rest batched)."""
    rng = np.random.default_rng(3)
    counts = [2_600_000] + [int(c) for c in rng.integers(0, 20000, 70)] + [3_100_000, 150_000] + \
             [int(c) for c in rng.integers(0, 3000, 30)] + [2_300_001]
    n = sum(counts)
    offs = None
    if shape == "k16":
        keys, stride = oracle.gen_keys16(41, 0, n), 16
    elif shape == "k24":
        keys, stride = rng.integers(0, 256, (n, 24), dtype=np.uint8), 24
    else:
        lens = rng.integers(8, 32, n)
        keys, stride = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8), 0
        offs = np.zeros(n + 1, np.int64)
        offs[1:] = np.cumsum(lens)
    ref = oracle_per_segment(oracle, 0, keys, counts, 10, stride=stride,
                             offsets=None if offs is None else offs.astype(np.uint64))
    plan, out = gpu_build(amq, torch, 0, torch.from_numpy(keys).cuda(), counts, 10,
                          offsets_t=None if offs is None else torch.from_numpy(offs).cuda())
    assert_same(plan, out, ref)


@pytest.mark.parametrize("shape,bpk,counts", [
    ("var", 10, [3_000_000, 500, 16384]),          # one 3M-key variable-length leaf
    ("var", 12, [16384, 2_700_000, 0, 1, 2_900_000, 77]),
    ("k20", 10, [3_000_000, 500, 16384]),          # a fixed stride other than 16 and 24
    ("k40", 8, [5_200_000, 3]),                    # keys of 32 bytes and more: hashed per seed
    ("var", 16, [3_000_000, 500]),                 # k > 8: device atomics (records hold 8 bits)
    ("var", 10, [2_700_000]),                      # one filter past the window path
    ("k20", 12, [2_200_000]),
])
def test_bloom_oversize_other_key_shapes(oracle, amq, torch, shape, bpk, counts):
    """Leaves past 16 LDS windows of variable-length or other fixed-size keys, in a batch and
    alone: each key hashed into its bit record (bloom_any_records), then the tiled build (round
    5: device atomics at 3.6 Gkeys/s), byte-equal to the oracle."""
    rng = np.random.default_rng(len(counts) * bpk)
    n = sum(counts)
    offs = None
    if shape == "var":
        lens = rng.integers(8, 32, n)
        lens[::97] = rng.integers(32, 48, lens[::97].size)   # some past XxhShort's 31 bytes
        keys, stride = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8), 0
        offs = np.zeros(n + 1, np.int64)
        offs[1:] = np.cumsum(lens)
    else:
        stride = int(shape[1:])
        keys = rng.integers(0, 256, (n, stride), dtype=np.uint8)
    ref = oracle_per_segment(oracle, 0, keys, counts, bpk, stride=stride,
                             offsets=None if offs is None else offs.astype(np.uint64))
    plan, out = gpu_build(amq, torch, 0, torch.from_numpy(keys).cuda(), counts, bpk,
                          offsets_t=None if offs is None else torch.from_numpy(offs).cuda())
    assert plan.max_seg_blocks > 16 * 160 * 1024 // 64
    assert_same(plan, out, ref)


@pytest.mark.parametrize("shape", ["var", "k16"])
def test_bloom_oversize_batch_side_stream_and_short_workspace(oracle, amq, torch, shape):
    """A batch of small leaves around one past the window path (tkv_amq_build_ex): built on a
    non-default caller stream and read after that stream alone is synchronised, and through
    the C ABI with a workspace 256 bytes short of the plan's (the Python entry refuses one; the
    library then takes whatever path still fits, down to device atomics).  Byte-equal either
    way, on output buffers poisoned beforehand."""
    from turtle_kv_amd import abi
    rng = np.random.default_rng(77)
    counts = [700, 3_000_000, 500, 16384, 0, 9000]
    n = sum(counts)
    if shape == "var":
        lens = rng.integers(8, 32, n)
        keys, stride = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8), 0
        offs = np.zeros(n + 1, np.int64)
        offs[1:] = np.cumsum(lens)
    else:
        keys, stride, offs = oracle.gen_keys16(77, 0, n), 16, None
    ref = oracle_per_segment(oracle, 0, keys, counts, 10, stride=stride,
                             offsets=None if offs is None else offs.astype(np.uint64))
    plan = amq.plan_filters(amq.BLOOM, counts, 10)
    keys_t = torch.from_numpy(keys).cuda()
    offs_t = None if offs is None else torch.from_numpy(offs).cuda()
    kb = amq.KeyBatch.fixed(keys_t) if offs_t is None else amq.KeyBatch.variable(keys_t, offs_t)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        out = torch.full((plan.total_out_bytes,), 0xA5, dtype=torch.uint8, device="cuda")
        amq.build_all_filters(plan, kb, out=out, stream=s, check=False)
    s.synchronize()
    assert_same(plan, out.cpu().numpy(), ref)
    ws = torch.full((plan.workspace_bytes,), 0xFF, dtype=torch.uint8, device="cuda")
    out2 = torch.full((plan.total_out_bytes,), 0x5A, dtype=torch.uint8, device="cuda")
    ptr = lambda t: None if t is None else t.data_ptr()
    st = abi.lib().tkv_amq_build_ex(plan.kind, keys_t.data_ptr(), ptr(offs_t), stride, n,
                                    plan.device_segs(keys_t.device).data_ptr(), plan.segs.ctypes.data,
                                    plan.n_segs, plan.max_seg_blocks, out2.data_ptr(), ws.data_ptr(),
                                    plan.workspace_bytes - 256, None)
    abi.check(st, "tkv_amq_build_ex")
    torch.cuda.synchronize()
    assert_same(plan, out2.cpu().numpy(), ref)


@pytest.mark.parametrize("shape,bpk,n_big", [("k16", 10, 35), ("k16", 16, 17), ("k24", 12, 17)])
def test_bloom_many_oversize_leaves(oracle, amq, torch, shape, bpk, n_big):
    """More oversize leaves than one multi-leaf launch holds (bloom_part_multi: 15 leaves), and
    (16-byte keys @10, 35 leaves of 2.1-2.3M keys, ~2.7 GB of partition workspace in all) more
    than its 2 GiB workspace budget: the launches split by count and by workspace; k > 8
    (@16: the 16-byte keys as records), 24-byte keys; small leaves between them."""
    rng = np.random.default_rng(bpk)
    first = 40960 * 512 // bpk + 1  # keys past 16 windows (40,960 blocks)
    counts = []
    for _ in range(n_big):
        counts += [int(first + rng.integers(0, 200_000)), int(rng.integers(0, 5000))]
    n = sum(counts)
    if shape == "k16":
        keys, stride = oracle.gen_keys16(bpk, 0, n), 16
    else:
        keys, stride = rng.integers(0, 256, (n, 24), dtype=np.uint8), 24
    ref = oracle_per_segment(oracle, 0, keys, counts, bpk, stride=stride)
    plan, out = gpu_build(amq, torch, 0, torch.from_numpy(keys).cuda(), counts, bpk)
    if n_big == 35:
        assert plan.workspace_bytes < 2.3e9   # the budget, not every leaf's workspace at once
    assert_same(plan, out, ref)


def test_reference_api_mirror(oracle, amq, torch):
    keys = sorted_keys(oracle, 3, [4000])
    kb = amq.KeyBatch.fixed(torch.from_numpy(keys).cuda())
    page = amq.build_filter_for_leaf_in_job(12, 4242, kb)          # default kind: VQF (config.hpp)
    assert page is not None and page.kind == amq.VQF
    vf = amq.PackedVqfFilter(page)
    vf.check_magic()
    assert vf.src_page_id == 4242 and vf.key_remainder_bits == 8
    q = amq.KeyQuery(kb)
    assert all(r == amq.BoolStatus.kFalse for r in q.reject_page(4242, page))
    assert all(r == amq.BoolStatus.kUnknown for r in q.reject_page(1, page))   # page id mismatch
    assert all(r == amq.BoolStatus.kUnknown for r in q.reject_page(4242, None))
    miss = amq.KeyBatch.fixed(torch.from_numpy(oracle.gen_keys16(99, 0, 4000)).cuda())
    rej = amq.KeyQuery(miss).reject_page(4242, page)
    assert sum(r == amq.BoolStatus.kTrue for r in rej) > 3900
    assert amq.build_filter_for_leaf_in_job(0, 1, kb) is None        # bpk 0: no filter
    bp = amq.build_bloom_filter_for_leaf(10, 9, kb)
    assert all(r == amq.BoolStatus.kFalse for r in q.reject_page(9, bp))


@pytest.mark.parametrize("kind,bpk", [(0, 10), (0, 12), (0, 20), (1, 12)])
def test_hash_once_probe_many(oracle, amq, torch, kind, bpk):
    """Multi-get fan-out: each query is hashed once (vqf_hash_val / BloomFilterQuery) and
    tested against several leaves' filters (one per level on its path).  Must equal probing
    every (query, leaf) pair from the raw key."""
    counts = [S] * 6 + [1234]
    keys = sorted_keys(oracle, 42, counts) if kind else oracle.gen_keys16(42, 0, sum(counts))
    plan = amq.plan_filters(kind, counts, bpk, payload_capacity=65472 if kind else 0)
    filt = amq.build_all_filters(plan, amq.KeyBatch.fixed(torch.from_numpy(keys).cuda()))
    nq, fan = 50000, 4
    q = np.concatenate([keys[:nq // 2], oracle.gen_keys16(43, 0, nq - nq // 2)])
    rng = np.random.default_rng(5)
    pair_query = np.repeat(np.arange(nq), fan).astype(np.int32)
    pair_leaf = rng.integers(0, len(counts), nq * fan).astype(np.int32)
    dq = amq.KeyBatch.fixed(torch.from_numpy(q).cuda())
    if kind == 0:
        qh = amq.bloom_query_hashes(dq, 32)
        got = amq.bloom_probe_hashed(plan, filt, qh, 32, torch.from_numpy(pair_leaf).cuda(),
                                     pair_query=torch.from_numpy(pair_query).cuda())
    else:
        hv = amq.vqf_hash_val(dq)
        got = amq.vqf_probe_hashed(plan, filt, hv, torch.from_numpy(pair_leaf).cuda(),
                                   pair_query=torch.from_numpy(pair_query).cuda())
    expand = amq.KeyBatch.fixed(torch.from_numpy(q[pair_query]).cuda())
    want = amq.probe_filters(plan, filt, expand, torch.from_numpy(pair_leaf).cuda())
    assert torch.equal(got, want)
    st, ref = oracle.probe_segments(kind, filt.cpu().numpy(), plan.segs["out_offset"],
                                    q[pair_query], pair_leaf.astype(np.uint32))
    assert np.array_equal(got.cpu().numpy(), ref)


def _bloom_seed(i):
    m = (1 << 64) - 1
    z = (0x243F6A8885A308D3 + i * 0x9E3779B97F4A7C15) & m
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & m
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & m
    return z ^ (z >> 31)


def test_variable_length_probe(oracle, amq, torch):
    """Probes of variable-length keys (0-71 bytes: the shared-lane short-key hash below 32
    bytes, the full XXH64 above): Bloom answers equal a python-xxhash evaluation of the
    tkv-amq v1 bit test; VQF hashes equal python-xxhash; raw-key and hash-once probes agree;
    no false negatives."""
    import xxhash
    rng = np.random.default_rng(21)
    counts = [3000, 17, 4096, 1]
    nq_miss = 3000
    # inserted keys 4-71 bytes (unique, as a leaf's keys are); miss queries 0-71 bytes
    lens = np.concatenate([rng.integers(4, 72, sum(counts)), rng.integers(0, 72, nq_miss)])
    blob = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8)
    offs = np.zeros(len(lens) + 1, np.int64)
    offs[1:] = np.cumsum(lens)
    n = sum(counts)
    kb = amq.KeyBatch.variable(torch.from_numpy(blob[:offs[n]].copy()).cuda(),
                               torch.from_numpy(offs[:n + 1].copy()).cuda())
    qb = amq.KeyBatch.variable(torch.from_numpy(blob).cuda(), torch.from_numpy(offs).cuda())
    seg_of_key = np.repeat(np.arange(len(counts)), counts)
    qseg = np.concatenate([seg_of_key, rng.integers(0, len(counts), nq_miss)]).astype(np.int32)
    key = lambda i: blob[offs[i]:offs[i + 1]].tobytes()
    for kind, bpk in ((0, 10), (1, 13)):
        plan = amq.plan_filters(kind, counts, bpk, payload_capacity=32704 if kind else 0)
        filt = amq.build_all_filters(plan, kb)
        res = amq.probe_filters(plan, filt, qb, torch.from_numpy(qseg).cuda()).cpu().numpy()
        assert res[:n].all(), "false negative"
        if kind == 0:
            f = filt.cpu().numpy()
            want = np.zeros(len(qseg), np.uint8)
            for i in range(len(qseg)):
                sg = plan.segs[qseg[i]]
                k = int(sg["hash_count"])
                h0 = xxhash.xxh64_intdigest(key(i), _bloom_seed(0))
                blk = (h0 * int(sg["n_blocks"])) >> 64
                base = int(sg["out_offset"]) + 64 + 64 * blk
                bits = [h0 & 511] + [xxhash.xxh64_intdigest(key(i), _bloom_seed(j)) & 511
                                     for j in range(1, k)]
                want[i] = all((f[base + (b >> 3)] >> (b & 7)) & 1 for b in bits)
            assert np.array_equal(res, want)
            qh = amq.bloom_query_hashes(qb, 32)
            got = amq.bloom_probe_hashed(plan, filt, qh, 32, torch.from_numpy(qseg).cuda())
            assert np.array_equal(got.cpu().numpy(), res)
        else:
            hv = amq.vqf_hash_val(qb).cpu().numpy().view(np.uint64)
            want_h = np.array([xxhash.xxh64_intdigest(key(i), VQF_SEED) for i in range(len(qseg))],
                              dtype=np.uint64)
            assert np.array_equal(hv, want_h)
            got = amq.vqf_probe_hashed(plan, filt, torch.from_numpy(hv.view(np.int64)).cuda(),
                                       torch.from_numpy(qseg).cuda())
            assert np.array_equal(got.cpu().numpy(), res)
