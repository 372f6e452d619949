"""CPU: TreeOptions filter page sizing (tree/tree_options.hpp:177-258) and whole-page plans
(tkv_amq_plan_pages) through the C ABI, against the pure-Python restatement in
tests/golden/page_sizing.json (make_golden.py).  No device needed: planning is host code."""
import json
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_page_sizing_matches_golden(amq):
    L = amq.abi.lib()
    rows = json.load(open(os.path.join(GOLDEN, "page_sizing.json")))
    assert len(rows) == 864
    for r in rows:
        assert L.tkv_amq_leaf_data_size(r["leaf_size"]) == r["leaf_data_size"], r
        assert L.tkv_amq_expected_items_per_leaf(r["leaf_size"], r["key_size_hint"],
                                                 r["value_size_hint"]) == r["expected_items_per_leaf"], r
        got = L.tkv_amq_filter_page_size_log2(r["kind"], r["leaf_size"], r["key_size_hint"],
                                              r["value_size_hint"], r["bits_per_key"])
        assert got == r["filter_page_size_log2"], r


@pytest.mark.parametrize("kind", [0, 1])
def test_tree_options_defaults(amq, kind):
    """Defaults (tree_options.cpp:17-25, tree_options.hpp:57-59): 2 MiB leaves, 24 B keys,
    100 B values, 12 bits/key -> 15,767 items per leaf -> 32 KiB filter pages, 32,704 payload
    bytes (the capacity round 1 hard-coded)."""
    t = amq.TreeOptions.with_default_values(kind)
    assert t.leaf_size() == 2 << 20
    assert t.leaf_data_size() == (2 << 20) - 104
    assert t.expected_item_size() == 133
    assert t.expected_items_per_leaf() == 15767
    assert t.filter_bits_per_key() == 12
    assert t.filter_page_size_log2() == 15
    assert t.filter_page_size() == 32768
    assert t.filter_page_payload_size() == 32704


def test_tree_options_setters(amq):
    t = amq.TreeOptions(amq.VQF).set_filter_bits_per_key(10)
    assert t.filter_bits_per_key() == 12                # VQF clamp (:159-160)
    assert t.set_filter_bits_per_key(0).filter_bits_per_key() == 0
    t.set_filter_page_size(5000)                        # log2_ceil
    assert t.filter_page_size() == 8192
    b = amq.TreeOptions(amq.BLOOM).set_filter_bits_per_key(10)
    assert b.filter_bits_per_key() == 10
    b.set_leaf_size(1 << 16).set_key_size_hint(16).set_value_size_hint(16)
    assert b.expected_items_per_leaf() == (65536 - 104) // 41
    with pytest.raises(amq.TkvAmqError):
        amq.TreeOptions().set_leaf_size(3 << 20)       # must be a power of 2 (:106)


@pytest.mark.parametrize("kind,bpk", [(0, 10), (1, 12), (1, 22)])
def test_plan_pages_layout(amq, kind, bpk):
    """Leaf s owns page s; its payload starts after the 64-byte page header and fits the
    payload capacity page - 64 (the buffer the builder sizes against)."""
    log2 = amq.TreeOptions(kind).set_filter_bits_per_key(bpk).filter_page_size_log2()
    counts = [16384, 1, 0, 15767, 9000]
    p = amq.plan_filter_pages(kind, counts, bpk, log2, src_page_ids=[5, 6, 7, 8, 9])
    page = 1 << log2
    assert p.total_out_bytes == page * len(counts)
    for s, seg in enumerate(p.segs):
        assert int(seg["out_offset"]) == s * page + 64
        assert int(seg["page_flags"]) == amq.abi.PAGE_IMAGE | (log2 << 8)
        assert int(seg["payload_bytes"]) <= page - 64
    # the payload plan equals the packed plan at capacity page - 64
    q = amq.plan_filters(kind, counts, bpk, payload_capacity=page - 64, out_stride=page)
    for f in ("n_blocks", "hash_count", "tag_bits", "hash_val_shift", "payload_bytes", "mod_magic"):
        assert np.array_equal(p.segs[f], q.segs[f]), f


def test_plan_pages_rejects_bad_sizes(amq):
    with pytest.raises(amq.TkvAmqError):
        amq.plan_filter_pages(1, [100], 12, 5)          # page too small for any header
    with pytest.raises(amq.TkvAmqError) as e:
        amq.plan_filter_pages(0, [100000], 10, 12)      # 4 KiB page cannot hold 100K keys
    assert e.value.status == amq.abi.RESOURCE_EXHAUSTED


def test_vqf_large_leaves_plan(amq):
    """VQF leaves of any size the reference builds are planned: the round-2 cap of 16,384
    blocks is gone (vqf_decide keeps u8 counts in LDS up to 163,840 blocks and global counts
    beyond; GPU parity: test_gpu_parity.py::test_vqf_huge_leaf).  Only a filter past 2^24
    blocks (1 GiB) is refused, with ResourceExhausted."""
    ok = amq.plan_filters(1, [700000], 12, payload_capacity=4 << 20)
    assert ok.max_seg_blocks > 16384
    big = amq.plan_filters(1, [7_000_000], 12, payload_capacity=16 << 20)
    assert big.max_seg_blocks > 160 * 1024
    with pytest.raises(amq.TkvAmqError) as e:
        amq.plan_filters(1, [700_000_000], 12, payload_capacity=2 << 30)
    assert e.value.status == amq.abi.RESOURCE_EXHAUSTED
