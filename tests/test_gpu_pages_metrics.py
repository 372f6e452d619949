"""GPU: whole filter-page images (tkv_amq_plan_pages), KeyQuery::Metrics counters from the
_ex probes, reject_page's page-id check, and the VQF workspace guards -- all against the
CPU oracle / oracle-derived expectations."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

S = 16384


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available()
    return t


def sorted_keys(oracle, seed, counts):
    keys = oracle.gen_keys16(seed, 0, sum(counts))
    oracle.sort_segments(keys, np.concatenate([[0], np.cumsum(counts)]).astype(np.uint64))
    return keys


@pytest.mark.parametrize("kind,bpk", [(0, 10), (1, 12), (1, 22)])
def test_page_images(oracle, amq, torch, kind, bpk):
    """Each leaf's page: header fields the builders set (layout_id, unused_begin =
    64 + 32 + filter_size for VQF, unused_end = page size; filter_builder.hpp:237,293-296),
    then the payload, byte-identical to the oracle at capacity page - 64."""
    t = amq.TreeOptions(kind).set_filter_bits_per_key(bpk)
    log2 = t.filter_page_size_log2()
    page = 1 << log2
    counts = [S, 9000, 1, 0, 15767]
    keys = sorted_keys(oracle, 42, counts) if kind else oracle.gen_keys16(42, 0, sum(counts))
    src = [300 + i for i in range(len(counts))]
    plan = amq.plan_filter_pages(kind, counts, bpk, log2, src_page_ids=src)
    out = torch.full((plan.total_out_bytes,), 0xAB, dtype=torch.uint8, device="cuda")
    amq.build_all_filters(plan, amq.KeyBatch.fixed(torch.from_numpy(keys).cuda()), out=out)
    o = out.cpu().numpy()
    b = 0
    for s, c in enumerate(counts):
        pg = o[s * page:(s + 1) * page]
        h = amq.page_header_fields(pg)
        if kind == 0:
            st, ref = oracle.bloom_build(keys[b:], c, bpk, src_page_id=src[s])
            ref = ref.tobytes()
        else:
            st, ref, pl = oracle.vqf_build(keys[b:], c, bpk, page - 64, src_page_id=src[s])
            ref = ref[:pl.payload_used].tobytes()
            assert h["unused_begin"] == 64 + 32 + pl.filter_size
        assert st == 0
        assert h["layout_id"] == ("vqf_filt" if kind else "bloomflt")
        assert h["unused_begin"] == 64 + len(ref)
        assert h["unused_end"] == page and h["size"] == page
        assert pg[64:64 + len(ref)].tobytes() == ref, f"leaf {s}"
        # the PageCache's own fields are left 0; the tail after unused_begin is not written
        assert not pg[:16].any() and not pg[24:28].any()
        assert (pg[64 + len(ref):] == 0xAB).all()
        b += c
    # probing through the page plan: no false negatives
    qs = torch.from_numpy(np.repeat(np.arange(len(counts)), counts).astype(np.int32)).cuda()
    res = amq.probe_filters(plan, out, amq.KeyBatch.fixed(torch.from_numpy(keys).cuda()), qs)
    assert bool(res.all())


def probe_setup(oracle, amq, torch, kind, bpk):
    counts = [S] * 6 + [8448, 0, 5]
    keys = sorted_keys(oracle, 42, counts) if kind else oracle.gen_keys16(42, 0, sum(counts))
    src = np.arange(900, 900 + len(counts), dtype=np.uint64)
    plan = amq.plan_filters(kind, counts, bpk, payload_capacity=32704 if kind else 0,
                            src_page_ids=src)
    filt = amq.build_all_filters(plan, amq.KeyBatch.fixed(torch.from_numpy(keys).cuda()))
    n = sum(counts)
    rng = np.random.default_rng(5)
    n_miss = 150000
    miss = oracle.gen_keys16(43, 0, n_miss)
    q = np.concatenate([keys, miss])
    seg_hit = np.repeat(np.arange(len(counts)), counts)
    # misses probe random leaves, a few of them outside the plan (no filter page)
    seg_miss = rng.integers(0, len(counts) + 2, n_miss)
    qs = np.concatenate([seg_hit, seg_miss]).astype(np.uint32)
    truth = np.concatenate([np.ones(n, np.uint8), np.zeros(n_miss, np.uint8)])
    # the leaf each query asks about: its own leaf, except every 7th miss asks about another
    page_ids = np.where(qs < len(counts), src[np.minimum(qs, len(counts) - 1)], 12345).astype(np.uint64)
    wrong = np.zeros(len(q), bool)
    wrong[n::7] = True
    page_ids[wrong] += 1000
    return plan, filt, counts, keys, q, qs, truth, page_ids, wrong


def expected_metrics(oracle, kind, plan, filt, q, qs, truth, page_ids, n_segs):
    inplan = qs < n_segs
    has = np.zeros(len(qs), bool)
    has[inplan] = plan.segs["n_keys"][qs[inplan]] >= 0  # every planned leaf has a filter (bpk > 0)
    src = np.zeros(len(qs), np.uint64)
    src[inplan] = plan.segs["src_page_id"][qs[inplan]]
    mism = has & (src != page_ids)
    checked = has & ~mism
    # oracle answer for the checked queries (over the GPU-built bytes, equal to the oracle's)
    qs_c = np.where(inplan, qs, 0).astype(np.uint32)
    st, ref = oracle.probe_segments(kind, filt.cpu().numpy(), plan.segs["out_offset"], q, qs_c)
    assert st == 0
    res = np.where(checked, ref, 1).astype(np.uint8)
    pos = checked & (ref == 1)
    m = {"total_filter_query_count": len(qs), "no_filter_page_count": int((~has).sum()),
         "page_id_mismatch_count": int(mism.sum()),
         "filter_reject_count": int((checked & (ref == 0)).sum()),
         "filter_positive_count": int(pos.sum()),
         "filter_false_positive_count": int((pos & (truth == 0)).sum())}
    return res, m


@pytest.mark.parametrize("kind,bpk", [(0, 10), (1, 12)])
def test_probe_metrics_and_page_id_check(oracle, amq, torch, kind, bpk):
    plan, filt, counts, keys, q, qs, truth, page_ids, wrong = probe_setup(oracle, amq, torch, kind, bpk)
    res_ref, m_ref = expected_metrics(oracle, kind, plan, filt, q, qs, truth, page_ids, len(counts))
    assert m_ref["page_id_mismatch_count"] > 0 and m_ref["no_filter_page_count"] > 0
    assert m_ref["filter_false_positive_count"] > 0
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    qb = amq.KeyBatch.fixed(d(q))
    pm = amq.ProbeMetrics()
    res = amq.probe_filters(plan, filt, qb, d(qs.astype(np.int32)), query_page_ids=d(page_ids.view(np.int64)),
                            truth=d(truth), metrics=pm)
    assert np.array_equal(res.cpu().numpy(), res_ref)
    assert pm.collect() == m_ref
    # counters accumulate across launches
    amq.probe_filters(plan, filt, qb, d(qs.astype(np.int32)), query_page_ids=d(page_ids.view(np.int64)),
                      truth=d(truth), metrics=pm)
    assert pm.collect() == {k: 2 * v for k, v in m_ref.items()}
    # without page ids and truth: no mismatches, false positives untouched
    pm.reset()
    res = amq.probe_filters(plan, filt, qb, d(qs.astype(np.int32)), metrics=pm)
    c = pm.collect()
    assert c["page_id_mismatch_count"] == 0 and c["filter_false_positive_count"] == 0
    assert c["total_filter_query_count"] == len(q)
    # the hashed (hash once, probe many) forms count the same
    qsd = d(qs.astype(np.int32))
    pm.reset()
    if kind == 1:
        hv = amq.vqf_hash_val(qb)
        r2 = amq.vqf_probe_hashed(plan, filt, hv, qsd, query_page_ids=d(page_ids.view(np.int64)),
                                  truth=d(truth), metrics=pm)
    else:
        qh = amq.bloom_query_hashes(qb, 32)
        r2 = amq.bloom_probe_hashed(plan, filt, qh, 32, qsd, query_page_ids=d(page_ids.view(np.int64)),
                                    truth=d(truth), metrics=pm)
    assert np.array_equal(r2.cpu().numpy(), res_ref)
    assert pm.collect() == m_ref


@pytest.mark.parametrize("kind,bpk", [(0, 10), (1, 12)])
def test_key_query_metrics(oracle, amq, torch, kind, bpk):
    """KeyQuery.reject_page updates KeyQuery.metrics() like the reference (:154-243) and the
    false-positive rate follows (:51-59)."""
    counts = [9000]
    keys = sorted_keys(oracle, 42, counts) if kind else oracle.gen_keys16(42, 0, 9000)
    kb = amq.KeyBatch.fixed(torch.from_numpy(keys).cuda())
    page = (amq.build_quotient_filter_for_leaf(bpk, 77, kb, 32704) if kind
            else amq.build_bloom_filter_for_leaf(bpk, 77, kb))
    miss = oracle.gen_keys16(43, 0, 20000)
    q = np.concatenate([keys[:1000], miss])
    truth = np.concatenate([np.ones(1000, np.uint8), np.zeros(20000, np.uint8)])
    kq = amq.KeyQuery(amq.KeyBatch.fixed(torch.from_numpy(q).cuda()))
    m = amq.KeyQuery.metrics()
    before = m.as_dict()
    r = kq.reject_page(77, page, truth=truth)
    assert all(x == amq.BoolStatus.kFalse for x in r[:1000])
    rejects = sum(x == amq.BoolStatus.kTrue for x in r)
    fps = sum(x == amq.BoolStatus.kFalse for x in r[1000:])
    assert kq.reject_page(78, page) == [amq.BoolStatus.kUnknown] * len(q)   # page-id mismatch
    assert kq.reject_page(77, None) == [amq.BoolStatus.kUnknown] * len(q)   # no filter page
    after = m.as_dict()
    delta = {k: after[k] - before[k] for k in after}
    assert delta["total_filter_query_count"] == 3 * len(q)
    assert delta["page_id_mismatch_count"] == len(q)
    assert delta["no_filter_page_count"] == len(q)
    assert delta["filter_reject_count"] == rejects
    assert delta["filter_positive_count"] == len(q) - rejects
    assert delta["filter_false_positive_count"] == fps
    assert 0 < m.filter_false_positive_rate() < 1
    # a page whose magic does not match its kind is refused (check_magic)
    wrong = amq.filters.FilterPage(1 - page.kind, page.payload, page.plan, 77)
    with pytest.raises(amq.TkvAmqError):
        kq.reject_page(77, wrong)


def test_vqf_workspace_guards(oracle, amq, torch):
    """A VQF workspace smaller than the plan needs is refused: by the host (Python, and the
    ABI's lower bound) or, past the host bound, by the device guard in every VQF kernel --
    never an out-of-bounds write."""
    counts = [S, S, 5000]
    keys = sorted_keys(oracle, 42, counts)
    kb = amq.KeyBatch.fixed(torch.from_numpy(keys).cuda())
    plan = amq.plan_filters(1, counts, 12, payload_capacity=32704)
    short = torch.empty(plan.workspace_bytes // 2, dtype=torch.uint8, device="cuda")
    with pytest.raises(amq.TkvAmqError) as e:
        amq.build_all_filters(plan, kb, workspace=short)
    assert e.value.status == amq.abi.INVALID_ARGUMENT
    # through the ABI: 1) below the host bound, 2) above it but short of the plan's need
    L = amq.abi.lib()
    F = amq.filters
    out = torch.zeros(plan.total_out_bytes, dtype=torch.uint8, device="cuda")
    ws = torch.zeros(plan.workspace_bytes, dtype=torch.uint8, device="cuda")
    segs = plan.device_segs()
    st = L.tkv_amq_build(1, F._ptr(kb.data), None, 16, kb.n, F._ptr(segs), plan.n_segs,
                         plan.max_seg_blocks, F._ptr(out), F._ptr(ws), 1024, F._stream_handle())
    assert st == amq.abi.INVALID_ARGUMENT
    host_bound = 256 + 128 * plan.max_seg_blocks + 8 * kb.n
    assert host_bound < plan.workspace_bytes - 64
    st = L.tkv_amq_build(1, F._ptr(kb.data), None, 16, kb.n, F._ptr(segs), plan.n_segs,
                         plan.max_seg_blocks, F._ptr(out), F._ptr(ws), host_bound, F._stream_handle())
    assert st == amq.abi.OK
    st = L.tkv_amq_build_check(1, F._ptr(ws), host_bound, F._stream_handle())
    assert st == amq.abi.INVALID_ARGUMENT
    assert not out.any(), "nothing written when the workspace is short"
    # the full workspace still builds the oracle's bytes
    amq.build_all_filters(plan, kb, out=out, workspace=ws)
    o = out.cpu().numpy()
    st, ref, pl = oracle.vqf_build(keys, S, 12, 32704, src_page_id=0)
    assert o[:pl.payload_used].tobytes() == ref[:pl.payload_used].tobytes()
