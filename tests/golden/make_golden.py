"""Regenerate the committed golden fixtures in tests/golden/.

Sources, in decreasing order of independence from this repo's code:
  xxh64.json          python-xxhash 3.8.1 (libxxhash 0.8.2): pins XXH64 for the oracle and
                      the HIP kernels (the hash vqf_hash_val uses, vqf_filter_page_view.hpp:32-35)
  sizing.json         a third, pure-Python restatement of the turtle_kv sizing arithmetic
                      (tree/filter_builder.hpp:241-290, vqf_filter_page_view.hpp:39-59,
                      tree/tree_options.hpp:155-164) -- Python floats are IEEE doubles, so the
                      floor(n / load_factor) results are the reference's
  page_sizing.json    the same pure-Python restatement of TreeOptions filter page sizing
                      (tree/tree_options.hpp:177-258, tree_options.cpp:57-60,
                      tree/packed_leaf_page.hpp:307-311, core/packed_sizeof_edit.hpp:13-15);
                      sizeof(llfs::PackedArray<T>) = 8 is UNPINNED (llfs absent)
  workload_e_keys.txt the first 4096 distinct `user<20 digits>` keys of the reference's own
                      data/workloads/workload-e.txt (a data fixture, read once at generation
                      time; nothing reads /root/reference at test time)
  filters.json, *.bin filters built by the CPU oracle (tkv-amq v1 spec).  SELF-PINNED: llfs and
                      vqf are absent, so no reference output exists for filter bytes
                      ("parity unpinned" against llfs/vqf).

Run:  python tests/golden/make_golden.py [--workload /root/reference/data/workloads/workload-e.txt]
"""
from __future__ import annotations

import argparse
import hashlib
import json
import math
import os
import sys

import numpy as np
import xxhash

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402

VQF_SEED = 0x9D0924DC03E79A75
S = 16384


def sm64_mix(z):
    m = (1 << 64) - 1
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & m
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & m
    return z ^ (z >> 31)


def bloom_seed(i):
    return sm64_mix((0x243F6A8885A308D3 + i * 0x9E3779B97F4A7C15) & ((1 << 64) - 1))


def xxh_vectors():
    rng = np.random.default_rng(7)
    seeds = [0, 1, VQF_SEED, bloom_seed(0), bloom_seed(6), (1 << 64) - 1]
    out = []
    for L in list(range(0, 41)) + [47, 48, 63, 64, 65, 100, 255]:
        data = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
        for sd in seeds:
            out.append({"data": data.hex(), "seed": sd, "xxh64": xxhash.xxh64_intdigest(data, sd)})
    out.append({"data": b"user0123456789ab".hex(), "seed": VQF_SEED,
                "xxh64": xxhash.xxh64_intdigest(b"user0123456789ab", VQF_SEED)})
    return out


# ---- pure-Python restatement of the reference sizing ------------------------------------
def vqf_slots(t):
    return 48 if t == 8 else 28


def load_factor(t, bpk):
    return 0.0 if bpk == 0 else (10.2 / float(bpk) if t == 8 else 18.0 / float(bpk))


def required_size(t, nslots):
    s = vqf_slots(t)
    return 48 + 64 * ((nslots + s) // s)


def nslots_for_size(t, nbytes):
    if nbytes < 48 + 64:
        return 0
    return (nbytes - 48) // 64 * vqf_slots(t) - 1


def vqf_plan(n, bpk, cap):
    if bpk == 0:
        return {"status": 0, "tag_bits": 0}
    if bpk < 12:
        return {"status": 3}
    if cap < 32 + 48 + 64:
        return {"status": 8}
    max8, max16 = nslots_for_size(8, cap - 32), nslots_for_size(16, cap - 32)
    lf8, lf16 = load_factor(8, bpk), load_factor(16, bpk)
    n8, n16 = int(math.floor(float(n) / lf8)), int(math.floor(float(n) / lf16))
    shift = 0
    if lf16 <= 0.85 and n16 <= max16:
        t, ns = 16, n16
    elif n8 <= max8:
        t, ns = 8, n8
    else:
        shift = 1
        while float(n >> shift) / lf8 > float(max8):
            shift += 1
        t, ns = 8, max8
    nb = (ns + vqf_slots(t)) // vqf_slots(t)
    return {"status": 0, "tag_bits": t, "hash_val_shift": shift, "nslots": ns, "nblocks": nb,
            "filter_size": required_size(t, ns), "payload_used": 32 + required_size(t, ns)}


def bloom_plan(n, bpk):
    nb = max(1, -(-n * bpk // 512))
    k = min(32, max(1, int(bpk * 0.69314718055994530942 + 0.5)))
    return {"n_blocks": nb, "hash_count": k, "payload": 64 + 64 * nb}


def sizing():
    caps = [32704, 16320, 65472, 8128, 4032]
    ns = [0, 1, 2, 47, 48, 100, 1000, 4096, 8448, 12000, 16384, 20000, 30000, 60000]
    bpks = [0, 10, 12, 13, 16, 21, 22, 24, 32]
    vqf = [dict(n=n, bpk=b, cap=c, **vqf_plan(n, b, c)) for c in caps for n in ns for b in bpks]
    bloom = [dict(n=n, bpk=b, **bloom_plan(n, b)) for n in ns for b in [1, 4, 8, 10, 12, 16, 20, 33, 64]]
    clamp = [{"requested": r, "vqf": (0 if r == 0 else max(12, r)), "bloom": r}
             for r in [0, 1, 8, 10, 11, 12, 13, 16, 30]]
    return {"vqf": vqf, "bloom": bloom, "clamp": clamp}


# ---- TreeOptions filter page sizing, restated -------------------------------------------
PAGE_HEADER, LEAF_HEADER, PACKED_ARRAY = 64, 32, 8   # llfs::PackedPageHeader, PackedLeafPage, PackedArray
BLOOM_PAGE_HEADER, VQF_PAGE_HEADER = 64, 32 + 48     # tkv-amq v1 PackedBloomFilterPage; PackedVqfFilter


def log2_ceil(x):
    k = 0
    while (1 << k) < x:
        k += 1
    return k


def expected_items_per_leaf(leaf_size, key_hint, value_hint):
    leaf_data = leaf_size - (PAGE_HEADER + LEAF_HEADER + PACKED_ARRAY)
    return leaf_data // (4 + key_hint + 4 + 1 + value_hint)


def filter_page_size_log2(kind, leaf_size, key_hint, value_hint, bpk_set):
    bpk = bpk_set if kind == 0 else (0 if bpk_set == 0 else max(12, bpk_set))
    items = expected_items_per_leaf(leaf_size, key_hint, value_hint)
    if kind == 0:
        bits = -(-(items * bpk) // 512) * 512
        return log2_ceil(PAGE_HEADER + BLOOM_PAGE_HEADER + bits // 8)
    if bpk == 0:
        return 0
    s8 = int(math.ceil(float(items) / load_factor(8, bpk)))
    s16 = int(math.ceil(float(items) / load_factor(16, bpk)))
    return log2_ceil(max(required_size(8, s8), required_size(16, s16)) + PAGE_HEADER + VQF_PAGE_HEADER)


def page_sizing():
    rows = []
    for kind in (0, 1):
        for leaf_log2 in (12, 16, 18, 20, 21, 22, 24, 26):
            for kh, vh in ((24, 100), (16, 0), (8, 8), (64, 1000), (16, 16), (100, 4000)):
                for b in (0, 1, 8, 10, 12, 13, 16, 22, 32):
                    L = 1 << leaf_log2
                    rows.append({"kind": kind, "leaf_size": L, "key_size_hint": kh,
                                 "value_size_hint": vh, "bits_per_key": b,
                                 "leaf_data_size": L - (PAGE_HEADER + LEAF_HEADER + PACKED_ARRAY),
                                 "expected_items_per_leaf": expected_items_per_leaf(L, kh, vh),
                                 "filter_page_size_log2": filter_page_size_log2(kind, L, kh, vh, b)})
    return rows


def segments(n_keys, seg=S):
    b = list(range(0, n_keys, seg)) + [n_keys]
    return np.array(b, dtype=np.uint64)


def oracle_filters(kind, keys, seg_begin, bpk, cap):
    n_segs = len(seg_begin) - 1
    counts = np.diff(seg_begin.astype(np.int64))
    if kind == O.BLOOM:
        sizes = np.array([O.lib().tkvo_bloom_payload_size(int(c), bpk) for c in counts], np.uint64)
    else:
        sizes = np.full(n_segs, cap, np.uint64)
    offs = np.zeros(n_segs, np.uint64)
    offs[1:] = np.cumsum(sizes)[:-1]
    st, out = O.build_segments(kind, keys, seg_begin, bpk, offs, sizes, int(sizes.sum()))
    assert st == 0, st
    return out, offs, sizes


def filter_digests(workload_keys):
    res = {}
    # config 1: 1M x 16B keys (splitmix64 seed 42), S = 16384, Bloom @10, order irrelevant
    n = 1_000_000
    keys = O.gen_keys16(42, 0, n)
    sb = segments(n)
    out, _, _ = oracle_filters(O.BLOOM, keys, sb, 10, 0)
    res["config1_bloom10_1M"] = {"n_keys": n, "seg_keys": S, "bits_per_key": 10,
                                 "sha256": hashlib.sha256(out.tobytes()).hexdigest(),
                                 "bytes": int(out.size)}
    # same keys, sorted per segment (leaf order), VQF @12 in 32 KiB pages
    O.sort_segments(keys, sb)
    out, _, _ = oracle_filters(O.VQF, keys, sb, 12, 32704)
    res["config1_vqf12_1M"] = {"n_keys": n, "seg_keys": S, "bits_per_key": 12,
                               "payload_capacity": 32704,
                               "sha256": hashlib.sha256(out.tobytes()).hexdigest(),
                               "bytes": int(out.size)}
    # the reference's own workload keys (24 bytes), one leaf of 4096 keys
    blob = np.frombuffer(b"".join(workload_keys), dtype=np.uint8).reshape(len(workload_keys), -1)
    st, b = O.bloom_build(blob, len(workload_keys), 10, src_page_id=7, stride=24)
    assert st == 0
    b.tofile(os.path.join(HERE, "workload_e_bloom10.bin"))
    st, v, pl = O.vqf_build(blob, len(workload_keys), 12, 32704, src_page_id=7, stride=24)
    assert st == 0
    v[:pl.payload_used].tofile(os.path.join(HERE, "workload_e_vqf12.bin"))
    res["workload_e_bloom10"] = {"file": "workload_e_bloom10.bin",
                                 "sha256": hashlib.sha256(b.tobytes()).hexdigest()}
    res["workload_e_vqf12"] = {"file": "workload_e_vqf12.bin",
                               "sha256": hashlib.sha256(v[:pl.payload_used].tobytes()).hexdigest()}
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="/root/reference/data/workloads/workload-e.txt")
    args = ap.parse_args()
    O.build_oracle()
    kpath = os.path.join(HERE, "workload_e_keys.txt")
    if os.path.exists(args.workload):
        seen, keys = set(), []
        with open(args.workload) as f:
            for line in f:
                parts = line.split()
                if len(parts) >= 2 and parts[0] == "P" and parts[1] not in seen:
                    seen.add(parts[1])
                    keys.append(parts[1])
                    if len(keys) == 4096:
                        break
        keys.sort()
        with open(kpath, "w") as f:
            f.write("\n".join(keys) + "\n")
    with open(kpath) as f:
        wkeys = [ln.strip().encode() for ln in f if ln.strip()]
    with open(os.path.join(HERE, "xxh64.json"), "w") as f:
        json.dump(xxh_vectors(), f)
    with open(os.path.join(HERE, "sizing.json"), "w") as f:
        json.dump(sizing(), f)
    with open(os.path.join(HERE, "page_sizing.json"), "w") as f:
        json.dump(page_sizing(), f)
    with open(os.path.join(HERE, "filters.json"), "w") as f:
        json.dump(filter_digests(wkeys), f, indent=1)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
