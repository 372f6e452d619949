"""Bloom leaves whose image exceeds one CU's LDS (160 KB) inside batches of any size: the
window path (bloom_build_window + bloom_split_merge).  Round 2 sent these leaves to device
atomics (~40x slower).  Every case is byte-compared with the CPU oracle, leaf by leaf:
the verdict's 70 x 200K-key batch at 12 bits/key, 2..16 windows per leaf, leaves of one
window mixed with leaves of several, every key shape (16-, 24-, 20-byte and variable-length
keys), k = 3 / 7 / 8 / 11 / 32, one filter alone (the window path for variable-length keys; 16-byte keys take the tiled build), and the
one-part fallback when the caller passes no workspace for partial images."""
import numpy as np
import pytest

from test_gpu_parity import assert_same, gpu_build, oracle_per_segment, seg_bounds, segment_bytes

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need a visible MI355X"
    return t


def windows(plan):
    return -(-int(plan.max_seg_blocks) * 64 // (160 * 1024))


def test_verdict_batch_70_leaves_200k_keys_12bpk(oracle, amq, torch):
    counts = [200_000] * 70
    keys = oracle.gen_keys16(31, 0, sum(counts))
    plan, out = gpu_build(amq, torch, 0, torch.from_numpy(keys).cuda(), counts, 12)
    assert windows(plan) == 2 and plan.workspace_bytes > 0   # two windows, partial images
    ref = oracle_per_segment(oracle, 0, keys, counts, 12)
    assert_same(plan, out, ref)


@pytest.mark.parametrize("big,bpk", [(140_000, 10), (300_000, 10), (1_000_000, 12),
                                     (2_000_000, 10), (350_000, 5), (60_000, 32), (100_000, 16)])
def test_window_counts_and_hash_counts(oracle, amq, torch, big, bpk):
    """2, 4, 10 and 16 windows (2M keys at 10 bits/key: 2.5 MB), k = 3 / 7 / 8 / 11 / 22, a
    ragged mix of big, small, one-key and empty leaves in one batch (16-byte keys: the leaves
    past 4 windows take the tiled build, the others the window path)."""
    rng = np.random.default_rng(big + bpk)
    counts = [int(c) for c in rng.integers(0, 3000, 12)]
    counts[0], counts[3], counts[7], counts[-1] = big, 1, 0, big // 3
    keys = oracle.gen_keys16(32, 0, sum(counts))
    plan, out = gpu_build(amq, torch, 0, torch.from_numpy(keys).cuda(), counts, bpk)
    assert 2 <= windows(plan) <= 16
    ref = oracle_per_segment(oracle, 0, keys, counts, bpk)
    assert_same(plan, out, ref)


@pytest.mark.parametrize("shape,bpk", [("k16", 16), ("k24", 10), ("k24", 14)])
def test_batch_tiled_past_five_windows(oracle, amq, torch, shape, bpk):
    """In a batch of 16- or 24-byte keys the leaves past 5 windows take the multi-leaf tiled
    build, the others the window / LDS paths: k = 11 (16-byte keys as records), 24-byte keys
    at k = 7 and at k = 10 (the bits past the eighth set by the overflow pass), ragged sizes
    around the threshold, small and empty leaves between."""
    rng = np.random.default_rng(bpk + len(shape))
    first = 5 * 2560 * 512 // bpk + 1   # keys past 5 windows of 2,560 blocks
    counts = [first + 50_000, 4000, 0, first - 1, 900_000, 17, first * 2, 2500]
    n = sum(counts)
    if shape == "k16":
        keys, stride = oracle.gen_keys16(bpk, 0, n), 16
    else:
        keys, stride = rng.integers(0, 256, (n, 24), dtype=np.uint8), 24
    plan, out = gpu_build(amq, torch, 0, torch.from_numpy(keys).cuda(), counts, bpk)
    assert windows(plan) > 5
    ref = oracle_per_segment(oracle, 0, keys, counts, bpk, stride=stride)
    assert_same(plan, out, ref)


@pytest.mark.parametrize("big", [1_000_000, 2_000_000])
def test_window_many_windows_variable_keys(oracle, amq, torch, big):
    """Variable-length keys keep the window path up to 16 windows in a batch (8 and 16 windows
    at 10 bits/key), beside small leaves."""
    rng = np.random.default_rng(big)
    counts = [big, 3000, 0, big // 2, 17]
    n = sum(counts)
    lens = rng.integers(8, 32, n)
    keys = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8)
    offs = np.zeros(n + 1, np.int64)
    offs[1:] = np.cumsum(lens)
    plan, out = gpu_build(amq, torch, 0, torch.from_numpy(keys).cuda(), counts, 10,
                          offsets_t=torch.from_numpy(offs).cuda())
    assert 8 <= windows(plan) <= 16
    ref = oracle_per_segment(oracle, 0, keys, counts, 10, stride=0, offsets=offs.astype(np.uint64))
    assert_same(plan, out, ref)


@pytest.mark.parametrize("shape", ["k24", "k20", "var"])
def test_window_key_shapes(oracle, amq, torch, shape):
    """24-byte keys move as their XxhFixed<24> state; 20-byte and variable-length keys (4-39
    bytes, the reference's KeyView ranges) as their index, re-hashed by the packed wave."""
    rng = np.random.default_rng(33)
    counts = [180_000, 700, 0, 260_000, 1, 5000]
    n = sum(counts)
    offs = None
    if shape in ("k24", "k20"):
        stride = int(shape[1:])
        keys = rng.integers(0, 256, (n, stride), dtype=np.uint8)
    else:
        lens = rng.integers(4, 40, n)
        keys, stride = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8), 0
        offs = np.zeros(n + 1, np.int64)
        offs[1:] = np.cumsum(lens)
    for bpk in (10, 12):
        plan, out = gpu_build(amq, torch, 0, torch.from_numpy(keys).cuda(), counts, bpk,
                              offsets_t=None if offs is None else torch.from_numpy(offs).cuda())
        assert windows(plan) >= 2
        ref = oracle_per_segment(oracle, 0, keys, counts, bpk, stride=stride,
                                 offsets=None if offs is None else offs.astype(np.uint64))
        assert_same(plan, out, ref)


@pytest.mark.parametrize("shape", ["k16", "var"])
@pytest.mark.parametrize("n,bpk", [(200_000, 10), (400_000, 5), (30_000, 64), (500_000, 10)])
def test_window_one_filter(oracle, amq, torch, n, bpk, shape):
    """One filter of 2-4 windows (the per-leaf call site's big leaf), k = 7, 3 and 32: 16-byte
    keys take the tiled build (a few tiles, each split over the chip), variable-length keys
    the window path, split into parts over the chip."""
    if shape == "k16":
        keys = oracle.gen_keys16(34, 0, n)
        plan, out = gpu_build(amq, torch, 0, torch.from_numpy(keys).cuda(), [n], bpk)
        ref = oracle_per_segment(oracle, 0, keys, [n], bpk)
    else:
        rng = np.random.default_rng(n + bpk)
        lens = rng.integers(8, 32, n)
        keys = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8)
        offs = np.zeros(n + 1, np.int64)
        offs[1:] = np.cumsum(lens)
        plan, out = gpu_build(amq, torch, 0, torch.from_numpy(keys).cuda(), [n], bpk,
                              offsets_t=torch.from_numpy(offs).cuda())
        ref = oracle_per_segment(oracle, 0, keys, [n], bpk, stride=0, offsets=offs.astype(np.uint64))
    assert 2 <= windows(plan) <= 4
    assert_same(plan, out, ref)


def test_window_without_workspace_one_part(oracle, amq, torch):
    """tkv_amq_build with no workspace: one part per leaf, windows written straight into the
    filters (no merge)."""
    from turtle_kv_amd.filters import _ptr, _stream_handle
    counts = [250_000, 3000, 90_000]
    keys = oracle.gen_keys16(35, 0, sum(counts))
    plan = amq.plan_filters(0, counts, 10)
    assert plan.workspace_bytes > 0
    kt = torch.from_numpy(keys).cuda()
    out = torch.zeros(plan.total_out_bytes, dtype=torch.uint8, device="cuda")
    amq.abi.check(amq.abi.lib().tkv_amq_build(0, _ptr(kt), None, 16, kt.shape[0],
                                              _ptr(plan.device_segs()), plan.n_segs,
                                              plan.max_seg_blocks, _ptr(out), None, 0,
                                              _stream_handle()), "build")
    torch.cuda.synchronize()
    assert_same(plan, out.cpu().numpy(), oracle_per_segment(oracle, 0, keys, counts, 10))


def test_window_page_images(oracle, amq, torch):
    """Whole filter pages (tkv_amq_plan_pages) of leaves past the LDS budget: the page header
    fields come from window 0 of part 0 (one part) or the merge (several)."""
    counts = [150_000] * 3 + [10]
    keys = oracle.gen_keys16(36, 0, sum(counts))
    log2 = 19  # 512 KiB pages
    plan = amq.plan_filter_pages(0, counts, 12, log2)
    out = amq.build_all_filters(plan, amq.KeyBatch.fixed(torch.from_numpy(keys).cuda()))
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    ref = oracle_per_segment(oracle, 0, keys, counts, 12)
    sb = seg_bounds(counts)
    for s in range(len(counts)):
        assert segment_bytes(plan, o, s) == ref[s], f"leaf {s}"
        page = o[s << log2:(s << log2) + 64]
        assert bytes(page[16:24]) == b"bloomflt"
        assert int(page[28:32].view(np.uint32)[0]) == 64 + int(plan.segs[s]["payload_bytes"])
        assert int(page[32:36].view(np.uint32)[0]) == 1 << log2
    del sb


def _window_parts(n_segs, n_keys, max_blocks):
    """A restatement of bloom_window_parts (tkv_amq_kernels.hip): the parts per leaf, so the
    test can check the plan's workspace (the partial images) and size a short one."""
    W = -(-64 * max_blocks // (160 * 1024))
    wblk = -(-max_blocks // W)
    per_cu = 2 if 64 * wblk <= 80 * 1024 else 1
    G = 256 * per_cu
    max_p = max(1, min(16, n_keys // n_segs // 4096))
    best, best_cost = 1, 1e30
    for p in range(1, max_p + 1):
        cost = -(-(n_segs * W * p) // G) / p + (0.03 * p if p > 1 else 0.0)
        if cost < best_cost - 1e-9:
            best, best_cost = p, cost
    return best


@pytest.mark.parametrize("form", ["parts", "short_workspace", "no_workspace"])
def test_window_workspace_forms(oracle, amq, torch, form):
    """The forms tkv_amq_build picks from the workspace it is given: partial images over
    several parts per leaf (the plan's workspace), and one part per leaf writing straight into
    the filters when the workspace is short or absent."""
    from turtle_kv_amd.filters import _ptr, _stream_handle
    counts = [200_000, 777, 90_000]
    n = sum(counts)
    keys = oracle.gen_keys16(37, 0, n)
    plan = amq.plan_filters(0, counts, 12)
    mb = int(plan.max_seg_blocks)
    P = _window_parts(len(counts), n, mb)
    assert P > 1 and plan.workspace_bytes == len(counts) * P * 64 * mb
    ws_bytes = {"parts": plan.workspace_bytes, "short_workspace": plan.workspace_bytes - 1,
                "no_workspace": 0}[form]
    kt = torch.from_numpy(keys).cuda()
    ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device="cuda")
    out = torch.zeros(plan.total_out_bytes, dtype=torch.uint8, device="cuda")
    amq.abi.check(amq.abi.lib().tkv_amq_build(0, _ptr(kt), None, 16, n, _ptr(plan.device_segs()),
                                              plan.n_segs, plan.max_seg_blocks, _ptr(out),
                                              _ptr(ws) if ws_bytes else None, ws_bytes,
                                              _stream_handle()), "build")
    torch.cuda.synchronize()
    assert_same(plan, out.cpu().numpy(), oracle_per_segment(oracle, 0, keys, counts, 12))
