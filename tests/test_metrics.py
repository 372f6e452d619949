"""CPU: the build metrics the reference records per leaf filter -- BloomFilterMetrics
(tree/filter_builder.hpp:39-56, updated at :139-147) and QuotientFilterMetrics (:156-172,
updated at :198-202) -- derived from a plan, checked against the reference's formulas over the
oracle's sizing."""
import numpy as np


def test_bloom_plan_stats(amq, oracle):
    counts = [16384, 5000, 0, 1]
    plan = amq.plan_filters(amq.BLOOM, counts, 10)
    st = amq.plan_filter_stats(plan)
    words = []
    for n in counts:
        nb = max(1, -(-n * 10 // 512))
        words.append(8 * nb)                      # PackedBloomFilter::word_count()
    words = np.array(words)
    assert st["word_count_stats"] == (4, int(words.sum()), int(words.min()), int(words.max()))
    assert st["byte_size_stats"][1] == int(8 * words.sum())
    assert st["bit_size_stats"][1] == int(64 * words.sum())
    assert st["item_count_stats"] == (4, sum(counts), 0, 16384)
    # bits_per_key 0: no filter, nothing recorded
    assert amq.plan_filter_stats(amq.plan_filters(amq.BLOOM, counts, 0))["item_count_stats"][0] == 0


def test_vqf_plan_stats_and_recording(amq, oracle):
    counts = [16384, 3000, 0]
    cap = 32704
    plan = amq.plan_filters(amq.VQF, counts, 12, payload_capacity=cap)
    st = amq.plan_filter_stats(plan)
    sizes, bpk = [], []
    for n in counts:
        _, _, pl = oracle.vqf_build(oracle.gen_keys16(1, 0, max(n, 1)), n, 12, cap)
        sizes.append(pl.filter_size)              # vqf_filter_size (filter_builder.hpp:194)
        if n:
            bpk.append((pl.filter_size * 8 + 4) // n)   # :202 (an empty leaf would divide by 0)
    assert st["byte_size_stats"] == (3, sum(sizes), min(sizes), max(sizes))
    assert st["bit_size_stats"][1] == 8 * sum(sizes)
    assert st["bits_per_key_stats"] == (2, sum(bpk), min(bpk), max(bpk))
    m = amq.QuotientFilterMetrics.instance()
    before = (m.byte_size_stats.count, m.byte_size_stats.total, m.build_page_latency.count)
    amq.record_filter_metrics(plan, latency_usec=300.0)
    assert m.byte_size_stats.count == before[0] + 3
    assert m.byte_size_stats.total == before[1] + sum(sizes)
    assert m.build_page_latency.count == before[2] + 3
