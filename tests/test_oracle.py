"""CPU-only: pin the oracle (test infrastructure) to the golden fixtures.

XXH64 is pinned to python-xxhash (libxxhash 0.8.2); the sizing tables to a pure-Python
restatement of tree/filter_builder.hpp:241-290; filter bytes are self-pinned SHA-256 of the
tkv-amq v1 spec (llfs / vqf absent: parity unpinned against them).
"""
import hashlib
import json
import os

import numpy as np
import pytest
import xxhash

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
VQF_SEED = 0x9D0924DC03E79A75


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def workload_keys():
    with open(os.path.join(GOLDEN, "workload_e_keys.txt")) as f:
        return [ln.strip().encode() for ln in f if ln.strip()]


def test_xxh64_golden(oracle):
    for v in load("xxh64.json"):
        data = bytes.fromhex(v["data"])
        assert oracle.xxh64(data, v["seed"]) == v["xxh64"], (len(data), v["seed"])


def test_vqf_hash_known_answer(oracle):
    # XXH64("user0123456789ab", 0x9d0924dc03e79a75)
    assert oracle.xxh64(b"user0123456789ab", VQF_SEED) == 0x76704C3C9F630896


def test_vqf_sizing_table(oracle):
    for c in load("sizing.json")["vqf"]:
        st, pl = oracle.vqf_plan(c["n"], c["bpk"], c["cap"])
        assert st == c["status"], c
        if st == 0 and c["tag_bits"]:
            got = dict(tag_bits=pl.tag_bits, hash_val_shift=pl.hash_val_shift, nslots=pl.nslots,
                       nblocks=pl.nblocks, filter_size=pl.filter_size,
                       payload_used=pl.payload_used)
            for k, v in got.items():
                assert v == c[k], (c, k, v)


def test_bloom_sizing_table(oracle):
    L = oracle.lib()
    for c in load("sizing.json")["bloom"]:
        assert L.tkvo_bloom_block_count(c["n"], c["bpk"]) == c["n_blocks"]
        assert L.tkvo_bloom_hash_count(c["bpk"]) == c["hash_count"]
        assert L.tkvo_bloom_payload_size(c["n"], c["bpk"]) == c["payload"]


def test_bits_per_key_clamp(oracle):
    L = oracle.lib()
    for c in load("sizing.json")["clamp"]:
        assert L.tkvo_tree_filter_bits_per_key(c["requested"], 1) == c["vqf"]
        assert L.tkvo_tree_filter_bits_per_key(c["requested"], 0) == c["bloom"]


def test_config1_filters_sha256(oracle):
    g = load("filters.json")
    n, S = 1_000_000, 16384
    keys = oracle.gen_keys16(42, 0, n)
    sb = np.array(list(range(0, n, S)) + [n], dtype=np.uint64)
    counts = np.diff(sb.astype(np.int64))
    sizes = np.array([oracle.lib().tkvo_bloom_payload_size(int(c), 10) for c in counts], np.uint64)
    offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64)
    st, out = oracle.build_segments(oracle.BLOOM, keys, sb, 10, offs, sizes, int(sizes.sum()))
    assert st == 0
    assert hashlib.sha256(out.tobytes()).hexdigest() == g["config1_bloom10_1M"]["sha256"]
    oracle.sort_segments(keys, sb)
    sizes = np.full(len(counts), 32704, np.uint64)
    offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64)
    st, out = oracle.build_segments(oracle.VQF, keys, sb, 12, offs, sizes, int(sizes.sum()))
    assert st == 0
    assert hashlib.sha256(out.tobytes()).hexdigest() == g["config1_vqf12_1M"]["sha256"]


def test_workload_e_filters(oracle):
    keys = workload_keys()
    assert len(keys) == 4096 and all(len(k) == 24 for k in keys)
    blob = np.frombuffer(b"".join(keys), dtype=np.uint8).reshape(len(keys), 24)
    st, b = oracle.bloom_build(blob, len(keys), 10, src_page_id=7, stride=24)
    assert st == 0
    assert b.tobytes() == open(os.path.join(GOLDEN, "workload_e_bloom10.bin"), "rb").read()
    st, v, pl = oracle.vqf_build(blob, len(keys), 12, 32704, src_page_id=7, stride=24)
    assert st == 0
    assert v[:pl.payload_used].tobytes() == open(os.path.join(GOLDEN, "workload_e_vqf12.bin"), "rb").read()


@pytest.mark.parametrize("bpk", [12, 16, 24])
def test_vqf_no_false_negatives_and_fpr(oracle, bpk):
    # the one property the reference's tests pin (tree/in_memory_node.test.cpp:101-131)
    n = 16384
    keys = oracle.gen_keys16(42, 0, n)
    st, f, pl = oracle.vqf_build(keys, n, bpk, 65472)
    assert st == 0
    for i in range(0, n, 7):
        assert oracle.vqf_is_present(f, xxhash.xxh64_intdigest(keys[i].tobytes(), VQF_SEED)) == 1
    miss = oracle.gen_keys16(43, 0, 20000)
    fp = sum(oracle.vqf_is_present(f, xxhash.xxh64_intdigest(m.tobytes(), VQF_SEED)) for m in miss)
    assert fp / 20000 < (0.01 if pl.tag_bits == 8 else 0.001)


def test_vqf_metadata_invariants(oracle):
    n = 16384
    keys = oracle.gen_keys16(5, 0, n)
    st, f, pl = oracle.vqf_build(keys, n, 12, 32704)
    assert st == 0 and pl.tag_bits == 8
    md = f[32:80].view("<u8")
    assert md[1] == 8 and md[3] == pl.nblocks and md[4] == n and md[5] == pl.nblocks * 48
    blocks = f[80:80 + 64 * pl.nblocks].reshape(-1, 64)
    total = 0
    for blk in blocks:
        lo, hi = blk[:16].view("<u8")
        pop = bin(int(lo)).count("1") + bin(int(hi)).count("1")
        c = 128 - pop if pop < 127 else (0 if (int(hi) >> 63) == 0 else 1)
        total += c
        assert pop >= 80
    assert total == n


def test_vqf_truncation_path(oracle):
    # more keys than the page can hold: hash_val_shift > 0 (filter_builder.hpp:277-290)
    n = 60000
    keys = oracle.gen_keys16(9, 0, n)
    st, f, pl = oracle.vqf_build(keys, n, 12, 16320)
    assert st == 0 and pl.hash_val_shift > 0
    mask = int(f[24:32].view("<u8")[0])
    assert mask == ((1 << 64) - 1) ^ ((1 << pl.hash_val_shift) - 1)
    for i in range(0, n, 13):
        h = xxhash.xxh64_intdigest(keys[i].tobytes(), VQF_SEED)
        assert oracle.vqf_is_present(f, h) == 1


def test_bloom_no_false_negatives_variable_keys(oracle):
    rng = np.random.default_rng(3)
    lens = rng.integers(0, 70, 3000)
    ks = [rng.integers(0, 256, L, dtype=np.uint8).tobytes() for L in lens]
    offs = np.zeros(len(ks) + 1, np.uint64)
    offs[1:] = np.cumsum(lens)
    blob = np.frombuffer(b"".join(ks), dtype=np.uint8).copy()
    st, b = oracle.bloom_build(blob, len(ks), 10, offsets=offs)
    assert st == 0
    assert all(oracle.bloom_query(b, k) == 1 for k in ks)


@pytest.mark.parametrize("n,bpk,cap", [(16384, 12, 32704), (8448, 12, 32704), (20000, 22, 131072),
                                       (5000, 30, 32704), (60000, 12, 32704), (1, 12, 32704),
                                       (0, 12, 32704), (700, 64, 32704)])
def test_vqf_bmi2_baseline(oracle, n, bpk, cap):
    """The CPU baseline bench.py times for VQF (oracle/tkv_amq_baseline.c: BMI2 select, POPCNT,
    unrolled XXH64 -- the instructions the reference's -mbmi2 -mavx2 build of vqf 0.2.4 uses,
    CMakeLists.txt:46-48) writes the literal oracle's bytes: 8- and 16-bit tags, hash
    truncation (60,000 keys on a 32 KiB page), one and zero keys, and the batched form."""
    keys = oracle.gen_keys16(100 + n, 0, max(n, 1))
    st, ref, pl = oracle.vqf_build(keys, n, bpk, cap)
    sb, got = oracle.vqf_build_baseline(keys, n, bpk, cap)
    assert st == sb == 0
    assert got[:pl.payload_used].tobytes() == ref[:pl.payload_used].tobytes()
    counts = [4000, 0, 16384, 777]
    allk = oracle.gen_keys16(7, 0, sum(counts))
    seg = np.concatenate([[0], np.cumsum(counts)]).astype(np.uint64)
    off = np.arange(len(counts), dtype=np.uint64) * 32768
    capa = np.full(len(counts), 32704, np.uint64)
    s1, a = oracle.build_segments(1, allk, seg, 12, off, capa, 32768 * len(counts), n_threads=3)
    s2, b = oracle.build_segments(1, allk, seg, 12, off, capa, 32768 * len(counts), n_threads=3,
                                  baseline=True)
    assert s1 == s2 == 0 and np.array_equal(a, b)


def test_vqf_bmi2_baseline_overflow(oracle):
    """A block overflow (keys whose primary and alternate buckets fall in block 0 of a 2-block
    filter) fails the baseline as it fails the oracle (vqf_insert, filter_builder.hpp:211)."""
    seed = 0x9D0924DC03E79A75
    out, i = [], 0
    while len(out) < 50:
        k = oracle.gen_keys16(1234, i, 1)[0]
        i += 1
        h = oracle.xxh64(k.tobytes(), seed)
        tag = h & 0xFF
        if (h >> 8) % 160 < 80 and ((h ^ ((tag * 0x5BD1E995) & ((1 << 64) - 1))) >> 8) % 160 < 80:
            out.append(k)
    keys = np.stack(out)
    st, _, _ = oracle.vqf_build(keys, 50, 12, 32704)
    sb, _ = oracle.vqf_build_baseline(keys, 50, 12, 32704)
    assert st == sb == 13
    st, ref, pl = oracle.vqf_build(keys[:48].copy(), 48, 12, 32704)
    sb, got = oracle.vqf_build_baseline(keys[:48].copy(), 48, 12, 32704)
    assert st == sb == 0 and got[:pl.payload_used].tobytes() == ref[:pl.payload_used].tobytes()


def test_whole_filter_window_equals_build(oracle):
    """bloom_sample_blocks with the one window [0, block_count) is the whole filter (the
    multithreaded whole-filter check of BASELINE config 5), and many small windows -- every
    part-boundary tile of a routed filter -- are found by their binary search."""
    import numpy as np
    n, bpk = 300_000, 12
    keys = oracle.gen_keys16(16, 0, n)
    st, ref = oracle.bloom_build(keys, n, bpk)
    assert st == 0
    nb = int(oracle.lib().tkvo_bloom_block_count(n, bpk))
    st, got = oracle.bloom_sample_blocks(16, 0, n, bpk, [(0, nb)], n_threads=4)
    assert st == 0 and got[(0, nb)].tobytes() == ref[64:].tobytes()
    wins = [(b, min(nb, b + 3)) for b in range(0, nb, 37)]
    st, got = oracle.bloom_sample_blocks(16, 0, n, bpk, wins, n_threads=4)
    assert st == 0
    for (a, b), v in got.items():
        assert v.tobytes() == ref[64 + 64 * a:64 + 64 * b].tobytes()
