"""CPU-only: the C-ABI library loads, exports every symbol include/tkv_amq.h declares, its
host-side planning matches the golden sizing tables and the oracle, and every device entry
point fails loudly (Unavailable) when no GPU is visible -- there is no CPU fallback."""
import json
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def header_symbols():
    src = open(os.path.join(ROOT, "include", "tkv_amq.h")).read()
    return sorted(set(re.findall(r"\b(tkv_amq_[a-z0-9_]+)\s*\(", src)))


def test_exports_match_header(amq):
    syms = header_symbols()
    assert sorted(amq.abi.EXPORTS) == syms
    out = subprocess.run(["nm", "-D", "--defined-only", amq.abi._build.LIB], capture_output=True,
                         text=True, check=True).stdout
    defined = set(re.findall(r" T (tkv_amq_\w+)", out))
    missing = [s for s in syms if s not in defined]
    assert not missing, missing
    L = amq.abi.lib()
    for s in syms:
        assert hasattr(L, s)


def test_library_is_gfx950(amq):
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-n", amq.abi._build.LIB],
                         capture_output=True, text=True)
    blob = open(amq.abi._build.LIB, "rb").read()
    assert b"gfx950" in blob


def test_version_and_status(amq):
    assert "tkv-amq" in amq.abi.version()
    assert amq.abi.lib().tkv_amq_status_string(8) == b"ResourceExhausted"


def test_plan_matches_golden_vqf(amq):
    g = json.load(open(os.path.join(GOLDEN, "sizing.json")))
    for c in g["vqf"]:
        if c["status"] != 0:
            with pytest.raises(amq.TkvAmqError) as e:
                amq.plan_filters(amq.VQF, [c["n"]], c["bpk"], payload_capacity=c["cap"])
            assert e.value.status == c["status"]
            continue
        p = amq.plan_filters(amq.VQF, [c["n"]], c["bpk"], payload_capacity=c["cap"])
        s = p.segs[0]
        if c["tag_bits"] == 0:
            assert s["tag_bits"] == 0 and s["payload_bytes"] == 0
            continue
        assert s["tag_bits"] == c["tag_bits"], c
        assert s["hash_val_shift"] == c["hash_val_shift"], c
        assert s["n_blocks"] == c["nblocks"], c
        assert s["payload_bytes"] == c["payload_used"], c
        R = c["nblocks"] * (80 if c["tag_bits"] == 8 else 36)
        assert int(s["mod_magic"]) == ((1 << 64) - 1) // R


def test_plan_matches_golden_bloom(amq):
    g = json.load(open(os.path.join(GOLDEN, "sizing.json")))
    for c in g["bloom"]:
        p = amq.plan_filters(amq.BLOOM, [c["n"]], c["bpk"])
        s = p.segs[0]
        assert s["n_blocks"] == c["n_blocks"] and s["hash_count"] == c["hash_count"]
        assert s["payload_bytes"] == c["payload"]


def test_clamp_and_load_factor(amq):
    g = json.load(open(os.path.join(GOLDEN, "sizing.json")))
    for c in g["clamp"]:
        assert amq.filter_bits_per_key(c["requested"], amq.VQF) == c["vqf"]
        assert amq.filter_bits_per_key(c["requested"], amq.BLOOM) == c["bloom"]
    assert amq.filter_bits_per_key(None, amq.VQF) == 12
    assert amq.vqf_filter_load_factor(8, 12) == 10.2 / 12
    assert amq.vqf_filter_load_factor(16, 24) == 18.0 / 24
    with pytest.raises(amq.TkvAmqError):
        amq.vqf_filter_load_factor(8, 10)


def test_batch_plan_layout(amq):
    counts = [16384] * 5 + [0, 1, 8448]
    p = amq.plan_filters(amq.VQF, counts, 12, payload_capacity=32704, src_page_ids=range(100, 108))
    s = p.segs
    assert list(s["key_begin"]) == list(np.concatenate([[0], np.cumsum(counts)[:-1]]))
    assert list(s["src_page_id"]) == list(range(100, 108))
    assert all(int(o) % 64 == 0 for o in s["out_offset"])
    ends = s["out_offset"] + s["payload_bytes"]
    assert all(ends[:-1] <= s["out_offset"][1:])
    assert p.total_out_bytes >= int(ends[-1])
    assert list(s["block_base"]) == list(np.concatenate([[0], np.cumsum(s["n_blocks"])[:-1]]))
    assert p.workspace_bytes >= 128 * int(s["n_blocks"].sum())
    assert p.max_seg_blocks == int(s["n_blocks"].max())
    # fixed stride (page-size slots), as used for the multi-GPU global layout
    p2 = amq.plan_filters(amq.BLOOM, counts, 10, out_stride=20544)
    assert list(p2.segs["out_offset"]) == [i * 20544 for i in range(len(counts))]
    with pytest.raises(amq.TkvAmqError):
        amq.plan_filters(amq.BLOOM, [100000], 10, out_stride=20544)


def test_hash_shard_constants_match_library(amq):
    """turtle_kv_amd.dist's tile geometry is the library's (tkv_amq_bloom_tile_blocks and the
    range builds' tile caps), and the monolithic workspace the plan asks for covers the
    routed form beyond one partition's tile table (the one-pass route's 12-byte records in
    their fixed-capacity regions, its overflow lists -- 16 bytes a key at worst -- and a part
    build's regions and overflow lists)."""
    from turtle_kv_amd import dist as tdist
    L = amq.abi.lib()
    assert L.tkv_amq_bloom_tile_blocks() == tdist.BLOOM_TILE_BLOCKS == 2048
    assert L.tkv_amq_bloom_range_max_tiles(1) == tdist.RECORD_RANGE_MAX_TILES
    assert L.tkv_amq_bloom_range_max_tiles(0) == tdist.KEY_RANGE_MAX_TILES
    direct = amq.plan_filters(amq.BLOOM, [100_000_000], 10)
    routed = amq.plan_filters(amq.BLOOM, [1_750_000_000], 12)
    assert direct.workspace_bytes >= 16 * 100_000_000
    assert routed.workspace_bytes >= (12 + 16) * 1_750_000_000
    # a range build past 6,400 tiles (the partition's LDS tile table) is refused
    assert L.tkv_amq_bloom_build_range_records_ws_bytes(1000, 0, 6400) > 0
    assert L.tkv_amq_bloom_build_range_records_ws_bytes(1000, 0, 6401) == 0
    assert L.tkv_amq_bloom_build_range_ws_bytes(1000, 5, 6405) > 0
    assert L.tkv_amq_bloom_build_range_ws_bytes(1000, 5, 6406) == 0


def test_device_calls_fail_loudly_without_gpu(amq):
    if amq.abi.lib().tkv_amq_device_count() > 0:
        pytest.skip("a GPU is visible")
    assert amq.abi.lib().tkv_amq_build(0, None, None, 16, 0, None, 0, 0, None, None, 0, None) == 14
    assert amq.abi.lib().tkv_amq_probe(0, None, None, 0, None, None, 16, 0, None, None, None) == 14
    with pytest.raises(amq.TkvAmqError):
        amq.gen_keys16(42, 0, 16)


def test_bench_splitmix_keys_match_oracle(oracle):
    """bench.py's elementwise key generator (shuffled probe queries) == the oracle's keys."""
    import numpy as np
    import torch
    import bench
    idx = torch.tensor([0, 1, 2, 77, 123456, 99_999_999], dtype=torch.int64)
    got = bench.splitmix_keys16(torch, 42, idx).numpy()
    for r, i in enumerate(idx.tolist()):
        assert np.array_equal(got[r], oracle.gen_keys16(42, i, 1)[0])
    seed = torch.tensor([43] * len(idx), dtype=torch.int64)
    got = bench.splitmix_keys16(torch, seed, idx).numpy()
    assert np.array_equal(got[3], oracle.gen_keys16(43, 77, 1)[0])
