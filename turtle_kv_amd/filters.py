"""Host-side mirror of TurtleKV's filter build/probe API over libtkv_amq (HIP, gfx950).

Reference interface (mathworks/turtle_kv, src/turtle_kv/...) and the function here that
replaces it:

  TreeOptions::filter_bits_per_key        tree/tree_options.hpp:155-164  -> filter_bits_per_key
  TreeOptions filter page sizing          tree/tree_options.hpp:166-258  -> TreeOptions
  vqf_hash_val                            vqf_filter_page_view.hpp:32-35 -> vqf_hash_val
  vqf_filter_load_factor<T>               vqf_filter_page_view.hpp:39-59 -> vqf_filter_load_factor
  build_bloom_filter_for_leaf             tree/filter_builder.hpp:109-152 -> build_bloom_filter_for_leaf
  build_quotient_filter_for_leaf          tree/filter_builder.hpp:221-301 -> build_quotient_filter_for_leaf
  build_filter_for_leaf_in_job            tree/filter_builder.hpp:307-331 -> build_filter_for_leaf_in_job
  TreeSerializeContext::build_all_pages   tree/tree_serialize_context.cpp:62-115 (the filter
                                          half of it)                     -> build_all_filters
  PackedVqfFilter::is_present             vqf_filter_page_view.hpp:113-125 -> PackedVqfFilter.is_present
  KeyQuery::reject_page                   tree/key_query.hpp:149-247      -> KeyQuery.reject_page
  KeyQuery::Metrics                       tree/key_query.hpp:36-60        -> KeyQueryMetrics
  FilterPageAlloc page + header fields    tree/filter_builder.hpp:58-105,231-237,293-296
                                                                          -> plan_filter_pages

Device memory, streams and multi-GPU plumbing come from PyTorch-ROCm; every filter
computation runs in the HIP kernels of libtkv_amq.so.  There is no CPU fallback: with no
GPU visible the device entry points raise TkvAmqError(Unavailable).
"""
from __future__ import annotations

import ctypes
import enum
import logging
import threading
import time
from dataclasses import dataclass, field

import numpy as np

from . import abi
from .abi import BLOOM, VQF, TkvAmqError

log = logging.getLogger("turtle_kv_amd")

# config.hpp:20-24 -- the reference compiles VQF in by default
TURTLE_KV_USE_BLOOM_FILTER = 0
TURTLE_KV_USE_QUOTIENT_FILTER = 1
DEFAULT_FILTER_KIND = VQF if TURTLE_KV_USE_QUOTIENT_FILTER else BLOOM

K_VQF_HASH_SEED = 0x9D0924DC03E79A75          # vqf_filter_page_view.hpp:26
K_MIN_QUOTIENT_FILTER_BITS_PER_KEY = 12       # vqf_filter_page_view.hpp:27
K_MAX_QUOTIENT_FILTER_LOAD_FACTOR = 0.85      # vqf_filter_page_view.hpp:28
K_DEFAULT_FILTER_BITS_PER_KEY = 12            # tree/tree_options.hpp:57
PACKED_PAGE_HEADER_BYTES = 64                 # llfs::PackedPageHeader (page payload offset)
VQF_MAGIC = 0x16015305E0F43A7D
BLOOM_MAGIC = 0xCA6F49A0F3F8A4B0


class BoolStatus(enum.Enum):
    """turtle_kv/import/bool_status.hpp: reject_page's tri-state result."""
    kFalse = 0
    kTrue = 1
    kUnknown = 2


def _torch():
    import torch
    return torch


def _stream_handle(stream=None):
    torch = _torch()
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def _hold(stream, *tensors):
    """Temporaries handed to a kernel launched on `stream` (a torch.cuda.Stream other than the
    current one): record that stream on them, so the caching allocator does not give their
    memory to other work before the kernel has read it."""
    torch = _torch()
    if stream is None or stream == torch.cuda.current_stream():
        return
    for t in tensors:
        if t is not None and getattr(t, "is_cuda", False):
            t.record_stream(stream)


def _ptr(t) -> ctypes.c_void_p | None:
    if t is None:
        return None
    if isinstance(t, np.ndarray):
        return ctypes.c_void_p(t.ctypes.data)
    return ctypes.c_void_p(t.data_ptr())


def _require_device():
    if abi.lib().tkv_amq_device_count() == 0:
        raise TkvAmqError(abi.UNAVAILABLE, "no HIP device visible")


# ---------------------------------------------------------------------------------------
# sizing
# ---------------------------------------------------------------------------------------
def filter_bits_per_key(requested: int | None, kind: int = DEFAULT_FILTER_KIND) -> int:
    """TreeOptions::filter_bits_per_key(): default 12; VQF clamps nonzero values to >= 12."""
    bpk = K_DEFAULT_FILTER_BITS_PER_KEY if requested is None else int(requested)
    return int(abi.lib().tkv_amq_filter_bits_per_key(kind, bpk))


def vqf_filter_load_factor(tag_bits: int, bits_per_key: int) -> float:
    if bits_per_key != 0 and bits_per_key < K_MIN_QUOTIENT_FILTER_BITS_PER_KEY:
        raise TkvAmqError(abi.INVALID_ARGUMENT, "vqf_filter_load_factor: bits_per_key < 12")
    if tag_bits not in (8, 16):
        raise TkvAmqError(abi.INVALID_ARGUMENT, "TAG_BITS must be 8 or 16")
    return float(abi.lib().tkv_amq_vqf_load_factor(tag_bits, bits_per_key))


def _log2_ceil(x: int) -> int:
    return max(0, (int(x) - 1).bit_length())


class TreeOptions:
    """The filter part of TreeOptions (tree/tree_options.hpp:43-395, tree_options.cpp:17-60):
    bits per key with the VQF clamp, and the filter page size derived from the leaf size and
    the key/value size hints.  `kind` stands for the compile-time filter switch (config.hpp:20-24)."""

    kDefaultFilterBitsPerKey = 12   # :57
    kDefaultKeySizeHint = 24        # :58
    kDefaultValueSizeHint = 100     # :59

    def __init__(self, kind: int = DEFAULT_FILTER_KIND):
        self.kind = kind
        self.leaf_size_log2_ = 21                  # 2 MiB (:384, with_default_values)
        self.filter_bits_per_key_ = None
        self.filter_page_size_log2_ = None
        self.key_size_hint_ = self.kDefaultKeySizeHint
        self.value_size_hint_ = self.kDefaultValueSizeHint

    @classmethod
    def with_default_values(cls, kind: int = DEFAULT_FILTER_KIND) -> "TreeOptions":
        return cls(kind)

    # leaf size
    def leaf_size(self) -> int:
        return 1 << self.leaf_size_log2_

    def set_leaf_size(self, size: int) -> "TreeOptions":
        self.leaf_size_log2_ = _log2_ceil(size)
        if self.leaf_size() != size:
            raise TkvAmqError(abi.INVALID_ARGUMENT, "leaf_size must be a power of 2")  # :106
        return self

    def set_leaf_size_log2(self, size_log2: int) -> "TreeOptions":
        self.leaf_size_log2_ = int(size_log2)
        return self

    def leaf_data_size(self) -> int:
        """leaf_max_space_from_size (tree/packed_leaf_page.hpp:307-311)."""
        return int(abi.lib().tkv_amq_leaf_data_size(self.leaf_size()))

    # bits per key
    def set_filter_bits_per_key(self, bits_per_key: int | None) -> "TreeOptions":
        self.filter_bits_per_key_ = bits_per_key
        return self

    def filter_bits_per_key(self) -> int:
        return filter_bits_per_key(self.filter_bits_per_key_, self.kind)

    # item size hints
    def key_size_hint(self) -> int:
        return self.key_size_hint_

    def set_key_size_hint(self, n_bytes: int) -> "TreeOptions":
        self.key_size_hint_ = int(n_bytes)
        return self

    def value_size_hint(self) -> int:
        return self.value_size_hint_

    def set_value_size_hint(self, n_bytes: int) -> "TreeOptions":
        self.value_size_hint_ = int(n_bytes)
        return self

    def expected_item_size(self) -> int:
        """PackedSizeOfEdit (core/packed_sizeof_edit.hpp:13-15) of a hint-sized edit."""
        return 4 + self.key_size_hint_ + 4 + 1 + self.value_size_hint_

    def expected_items_per_leaf(self) -> int:
        return int(abi.lib().tkv_amq_expected_items_per_leaf(self.leaf_size(), self.key_size_hint_,
                                                             self.value_size_hint_))

    # filter page size
    def set_filter_page_size_log2(self, size_log2: int) -> "TreeOptions":
        self.filter_page_size_log2_ = int(size_log2)
        return self

    def set_filter_page_size(self, size: int) -> "TreeOptions":
        return self.set_filter_page_size_log2(_log2_ceil(size))

    def filter_page_size_log2(self) -> int:
        if self.filter_page_size_log2_ is not None:
            return self.filter_page_size_log2_
        return int(abi.lib().tkv_amq_filter_page_size_log2(
            self.kind, self.leaf_size(), self.key_size_hint_, self.value_size_hint_,
            K_DEFAULT_FILTER_BITS_PER_KEY if self.filter_bits_per_key_ is None
            else int(self.filter_bits_per_key_)))

    def filter_page_size(self) -> int:
        return 1 << self.filter_page_size_log2()

    def filter_page_payload_size(self) -> int:
        """The payload buffer the filter builders size against: page size minus the llfs
        PackedPageHeader (filter_builder.hpp:231-244)."""
        return self.filter_page_size() - PACKED_PAGE_HEADER_BYTES


def vqf_required_size(tag_bits: int, nslots: int) -> int:
    return int(abi.lib().tkv_amq_vqf_required_size(tag_bits, nslots))


def vqf_nslots_for_size(tag_bits: int, nbytes: int) -> int:
    return int(abi.lib().tkv_amq_vqf_nslots_for_size(tag_bits, nbytes))


@dataclass
class FilterPlan:
    """Host plan of one batch of leaf filters (one build_all_pages queue)."""
    kind: int
    bits_per_key: int
    segs: np.ndarray                     # SEGMENT_DTYPE[n_segs]
    total_out_bytes: int
    workspace_bytes: int
    max_seg_blocks: int
    n_keys: int
    _device: dict = field(default_factory=dict, repr=False)
    _stats: dict | None = field(default=None, repr=False)

    @property
    def n_segs(self) -> int:
        return len(self.segs)

    def device_segs(self, device=None):
        """The plan uploaded to the device (cached per device)."""
        torch = _torch()
        dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        key = str(dev)
        if key not in self._device:
            host = torch.from_numpy(self.segs.view(np.uint8).reshape(-1).copy())
            self._device[key] = host.to(dev, non_blocking=False)
        return self._device[key]


def plan_filters(kind: int, seg_key_counts, bits_per_key: int, payload_capacity: int = 0,
                 out_stride: int = 0, src_page_ids=None) -> FilterPlan:
    """Restated build_{bloom,quotient}_filter_for_leaf sizing for every leaf of a batch."""
    counts = np.ascontiguousarray(np.asarray(seg_key_counts, dtype=np.uint64))
    n = len(counts)
    segs = np.zeros(n, dtype=abi.SEGMENT_DTYPE)
    src = None if src_page_ids is None else np.ascontiguousarray(np.asarray(src_page_ids, dtype=np.uint64))
    tot, ws, mb = ctypes.c_uint64(0), ctypes.c_uint64(0), ctypes.c_uint32(0)
    st = abi.lib().tkv_amq_plan(kind, _ptr(counts), _ptr(src), n, int(bits_per_key),
                                int(payload_capacity), int(out_stride), _ptr(segs),
                                ctypes.byref(tot), ctypes.byref(ws), ctypes.byref(mb))
    abi.check(st, "tkv_amq_plan")
    return FilterPlan(kind, int(bits_per_key), segs, int(tot.value), int(ws.value), int(mb.value),
                      int(counts.sum()) if n else 0)


def plan_filter_pages(kind: int, seg_key_counts, bits_per_key: int, page_size_log2: int,
                      src_page_ids=None) -> FilterPlan:
    """One whole filter page per leaf (tkv_amq_plan_pages): leaf s's page is bytes
    [s << log2, (s+1) << log2) of the output, a 64-byte page header then the payload, the
    buffer FilterPageAlloc hands the builder (filter_builder.hpp:70-88).  The build writes the
    header fields the builders set (layout_id, unused_begin, unused_end) and the page size."""
    counts = np.ascontiguousarray(np.asarray(seg_key_counts, dtype=np.uint64))
    n = len(counts)
    segs = np.zeros(n, dtype=abi.SEGMENT_DTYPE)
    src = None if src_page_ids is None else np.ascontiguousarray(np.asarray(src_page_ids, dtype=np.uint64))
    tot, ws, mb = ctypes.c_uint64(0), ctypes.c_uint64(0), ctypes.c_uint32(0)
    st = abi.lib().tkv_amq_plan_pages(kind, _ptr(counts), _ptr(src), n, int(bits_per_key),
                                      int(page_size_log2), _ptr(segs), ctypes.byref(tot),
                                      ctypes.byref(ws), ctypes.byref(mb))
    abi.check(st, "tkv_amq_plan_pages")
    return FilterPlan(kind, int(bits_per_key), segs, int(tot.value), int(ws.value), int(mb.value),
                      int(counts.sum()) if n else 0)


def page_header_fields(page: np.ndarray) -> dict:
    """The PackedPageHeader fields of one filter page image (offsets as in tkv_amq_plan_pages,
    llfs 0.42's layout: UNPINNED)."""
    b = np.asarray(page, dtype=np.uint8)
    u32 = b[:64].view("<u4")
    return {"layout_id": bytes(b[16:24]).rstrip(b"\0").decode("ascii", "replace"),
            "unused_begin": int(u32[7]), "unused_end": int(u32[8]), "size": int(u32[15])}


# ---------------------------------------------------------------------------------------
# keys
# ---------------------------------------------------------------------------------------
@dataclass
class KeyBatch:
    """Device-resident keys: fixed-length rows (`data` [n, L]) or variable-length bytes
    (`data` [total] + `offsets` int64 [n+1]), the flattened EditView key range the reference
    passes as `items` (core/merge_compactor.hpp:108-139)."""
    data: object
    n: int
    stride: int = 16
    offsets: object = None

    @staticmethod
    def fixed(t) -> "KeyBatch":
        assert t.dim() == 2 and t.dtype == _torch().uint8 and t.is_cuda and t.is_contiguous()
        return KeyBatch(t, t.shape[0], t.shape[1], None)

    @staticmethod
    def variable(data, offsets) -> "KeyBatch":
        torch = _torch()
        assert data.dtype == torch.uint8 and offsets.dtype == torch.int64
        return KeyBatch(data, offsets.numel() - 1, 0, offsets)

    @staticmethod
    def from_host(keys, device=None) -> "KeyBatch":
        """bytes-like list or [n, L] uint8 array -> device KeyBatch (H2D copy)."""
        torch = _torch()
        dev = device or "cuda"
        if isinstance(keys, np.ndarray) and keys.ndim == 2:
            return KeyBatch.fixed(torch.from_numpy(np.ascontiguousarray(keys)).to(dev))
        ks = [bytes(k) for k in keys]
        lens = {len(k) for k in ks}
        if len(lens) == 1 and ks:
            arr = np.frombuffer(b"".join(ks), dtype=np.uint8).reshape(len(ks), -1)
            return KeyBatch.fixed(torch.from_numpy(arr.copy()).to(dev))
        offs = np.zeros(len(ks) + 1, dtype=np.int64)
        np.cumsum([len(k) for k in ks], out=offs[1:])
        blob = np.frombuffer(b"".join(ks), dtype=np.uint8) if ks else np.zeros(0, np.uint8)
        data = torch.from_numpy(blob.copy() if len(blob) else np.zeros(1, np.uint8)).to(dev)
        return KeyBatch.variable(data, torch.from_numpy(offs).to(dev))


def key_views(buf: np.ndarray, offsets, lengths) -> np.ndarray:
    """tkv_amq_key_view records (KeyView = std::string_view {size, data}) for keys stored at
    byte `offsets[i]` (length `lengths[i]`) of host buffer `buf` -- the shape of the EditView
    key range the reference iterates (core/merge_compactor.hpp:107-139)."""
    offsets = np.asarray(offsets, dtype=np.uint64)
    v = np.empty(len(offsets), dtype=abi.KEY_VIEW_DTYPE)
    v["size"] = np.broadcast_to(np.asarray(lengths, dtype=np.uint64), offsets.shape)
    v["data"] = np.uint64(buf.ctypes.data) + offsets
    return v


def stage_keys(views, n: int | None = None, fixed_len: int = 16, out=None, view_stride: int = 16,
               n_threads: int = 0):
    """Gather viewed keys into one contiguous host buffer (tkv_amq_stage_keys, host threads).
    `views`: KEY_VIEW_DTYPE array or the address of the first view (then `n` and
    `view_stride` say how many and how far apart).  fixed_len > 0: returns `out` ([n,
    fixed_len] uint8, numpy or pinned torch); fixed_len == 0: returns (bytes, offsets[n+1])."""
    if isinstance(views, np.ndarray):
        assert views.dtype == abi.KEY_VIEW_DTYPE and views.flags.c_contiguous
        addr, n, view_stride = views.ctypes.data, len(views), abi.KEY_VIEW_DTYPE.itemsize
    else:
        addr = int(views)
    if fixed_len:
        if out is None:
            out = np.empty((n, fixed_len), dtype=np.uint8)
        cap = out.nbytes if isinstance(out, np.ndarray) else out.numel()
        st = abi.lib().tkv_amq_stage_keys(ctypes.c_void_p(addr), view_stride, n, fixed_len,
                                          _ptr(out), cap, None, n_threads)
        abi.check(st, "tkv_amq_stage_keys")
        return out
    sizes = np.ctypeslib.as_array((ctypes.c_uint64 * (2 * n)).from_address(addr)) if n and \
        view_stride == 16 else None
    total = int(sizes[0::2].sum()) if sizes is not None else (0 if n == 0 else None)
    if out is None:
        if total is None:
            raise TkvAmqError(abi.INVALID_ARGUMENT, "pass `out` for strided variable-length views")
        out = np.empty(max(total, 1), dtype=np.uint8)
    offs = np.empty(n + 1, dtype=np.uint64)
    cap = out.nbytes if isinstance(out, np.ndarray) else out.numel()
    st = abi.lib().tkv_amq_stage_keys(ctypes.c_void_p(addr), view_stride, n, 0, _ptr(out), cap,
                                      _ptr(offs), n_threads)
    abi.check(st, "tkv_amq_stage_keys")
    return out, offs


def gen_keys16(seed: int, first: int, n: int, device=None, stream=None):
    """Synthetic bench keys on the device (splitmix64 stream)."""
    torch = _torch()
    _require_device()
    out = torch.empty((n, 16), dtype=torch.uint8, device=device or "cuda")
    abi.check(abi.lib().tkv_amq_gen_keys16(seed, first, n, _ptr(out), _stream_handle(stream)),
              "tkv_amq_gen_keys16")
    return out


# ---------------------------------------------------------------------------------------
# build
# ---------------------------------------------------------------------------------------
# ---------------------------------------------------------------------------------------
# build metrics (BloomFilterMetrics, tree/filter_builder.hpp:39-56,136-147;
# QuotientFilterMetrics, :156-172,198-202)
# ---------------------------------------------------------------------------------------
class StatsMetric:
    """batt StatsMetric<u64>: count, total, min, max of the values it was updated with."""

    def __init__(self):
        self._lock = threading.Lock()
        self.count, self.total, self.min, self.max = 0, 0, None, None

    def merge(self, count: int, total: int, lo: int, hi: int) -> None:
        if count == 0:
            return
        with self._lock:
            self.count += count
            self.total += total
            self.min = lo if self.min is None else min(self.min, lo)
            self.max = hi if self.max is None else max(self.max, hi)

    def update(self, v: int) -> None:
        self.merge(1, int(v), int(v), int(v))

    @property
    def mean(self) -> float:
        return self.total / self.count if self.count else 0.0

    def __repr__(self):
        return f"StatsMetric(count={self.count}, total={self.total}, min={self.min}, max={self.max})"


class LatencyMetric:
    """LatencyMetric: count and total microseconds (per leaf filter, amortised over a batch)."""

    def __init__(self):
        self._lock = threading.Lock()
        self.count, self.total_usec = 0, 0

    def add(self, count: int, usec: float) -> None:
        with self._lock:
            self.count += count
            self.total_usec += int(usec)


class BloomFilterMetrics:
    """tree/filter_builder.hpp:39-56 (one process-wide instance, like Self::instance())."""
    _inst = None

    def __init__(self):
        self.word_count_stats = StatsMetric()
        self.byte_size_stats = StatsMetric()
        self.bit_size_stats = StatsMetric()
        self.bit_count_stats = StatsMetric()
        self.item_count_stats = StatsMetric()
        self.build_page_latency = LatencyMetric()

    @classmethod
    def instance(cls) -> "BloomFilterMetrics":
        if cls._inst is None:
            cls._inst = cls()
        return cls._inst


class QuotientFilterMetrics:
    """tree/filter_builder.hpp:156-172."""
    _inst = None

    def __init__(self):
        self.byte_size_stats = StatsMetric()
        self.bit_size_stats = StatsMetric()
        self.item_count_stats = StatsMetric()
        self.bits_per_key_stats = StatsMetric()
        self.build_page_latency = LatencyMetric()

    @classmethod
    def instance(cls) -> "QuotientFilterMetrics":
        if cls._inst is None:
            cls._inst = cls()
        return cls._inst


def _agg(v: np.ndarray):
    return (len(v), int(v.sum()), int(v.min()), int(v.max())) if len(v) else (0, 0, 0, 0)


def plan_filter_stats(plan: FilterPlan) -> dict:
    """The per-leaf values the reference records for every filter of a plan, aggregated
    (count, total, min, max), keyed by metric name.  Leaves without a filter (bits_per_key 0)
    record nothing; an empty VQF leaf skips bits_per_key (the reference would divide by
    zero, :202)."""
    if plan._stats is not None:
        return plan._stats
    segs = plan.segs
    n = segs["n_keys"].astype(np.int64)
    if plan.kind == BLOOM:
        has = segs["hash_count"] != 0
        words = 8 * segs["n_blocks"][has].astype(np.int64)        # PackedBloomFilter::word_count()
        st = {"word_count_stats": _agg(words), "byte_size_stats": _agg(8 * words),
              "bit_size_stats": _agg(64 * words),
              "bit_count_stats": _agg(512 * segs["n_blocks"][has].astype(np.int64)),  # header bit_count
              "item_count_stats": _agg(n[has])}
    else:
        has = segs["tag_bits"] != 0
        size = segs["payload_bytes"][has].astype(np.int64) - 32   # vqf_filter_size (:194)
        nz = n[has] > 0
        st = {"byte_size_stats": _agg(size), "bit_size_stats": _agg(8 * size),
              "item_count_stats": _agg(n[has]),
              "bits_per_key_stats": _agg((size[nz] * 8 + 4) // n[has][nz])}
    plan._stats = st
    return st


def record_filter_metrics(plan: FilterPlan, latency_usec: float | None = None) -> None:
    """Fold one built batch into BloomFilterMetrics / QuotientFilterMetrics, as the reference
    does per built leaf filter (filter_builder.hpp:139-147, :198-202)."""
    m = BloomFilterMetrics.instance() if plan.kind == BLOOM else QuotientFilterMetrics.instance()
    st = plan_filter_stats(plan)
    for name, agg in st.items():
        getattr(m, name).merge(*agg)
    if latency_usec is not None:
        leaves = st["item_count_stats"][0]
        if leaves:
            m.build_page_latency.add(leaves, latency_usec)


def build_all_filters(plan: FilterPlan, keys: KeyBatch, out=None, workspace=None, stream=None,
                      check: bool = True):
    """Build every planned filter into one device array (the filter half of
    TreeSerializeContext::build_all_pages).  Returns the output uint8 tensor."""
    torch = _torch()
    _require_device()
    if keys.n != plan.n_keys:
        raise TkvAmqError(abi.INVALID_ARGUMENT, f"plan covers {plan.n_keys} keys, got {keys.n}")
    dev = keys.data.device
    if out is None:
        out = torch.empty(max(plan.total_out_bytes, 1), dtype=torch.uint8, device=dev)
    elif out.numel() < plan.total_out_bytes:
        raise TkvAmqError(abi.INVALID_ARGUMENT,
                          f"output holds {out.numel()} bytes, the plan needs {plan.total_out_bytes}")
    if plan.workspace_bytes and workspace is None:
        workspace = torch.empty(plan.workspace_bytes, dtype=torch.uint8, device=dev)
    ws_bytes = 0 if workspace is None else workspace.numel() * workspace.element_size()
    if ws_bytes < plan.workspace_bytes:
        raise TkvAmqError(abi.INVALID_ARGUMENT,
                          f"workspace holds {ws_bytes} bytes, the plan needs {plan.workspace_bytes}")
    sh = _stream_handle(stream)
    t0 = time.perf_counter()
    # (_ex with the host plan: in a Bloom batch, leaves of 16- or 24-byte keys past 5 LDS windows
    # -- other key shapes past 16 -- take the tiled build, up to 40 such leaves per launch, and
    # the rest the batch kernels)
    L = abi.lib()
    if hasattr(L, "tkv_amq_build_ex"):
        st = L.tkv_amq_build_ex(plan.kind, _ptr(keys.data), _ptr(keys.offsets), keys.stride,
                                keys.n, _ptr(plan.device_segs(dev)), _ptr(plan.segs), plan.n_segs,
                                plan.max_seg_blocks, _ptr(out), _ptr(workspace), ws_bytes, sh)
        abi.check(st, "tkv_amq_build_ex")
    else:  # (an older library loaded through TKV_AMQ_LIB: the batch entry without the host plan)
        st = L.tkv_amq_build(plan.kind, _ptr(keys.data), _ptr(keys.offsets), keys.stride, keys.n,
                             _ptr(plan.device_segs(dev)), plan.n_segs, plan.max_seg_blocks,
                             _ptr(out), _ptr(workspace), ws_bytes, sh)
        abi.check(st, "tkv_amq_build")
    if check:
        # synchronous: the batch is known good, record its metrics with the build latency
        abi.check(abi.lib().tkv_amq_build_check(plan.kind, _ptr(workspace), ws_bytes, sh),
                  "vqf_insert (filter_builder.hpp:211)")
        record_filter_metrics(plan, (time.perf_counter() - t0) * 1e6)
    return out


class ProbeMetrics:
    """Device-side KeyQuery::Metrics counters (tkv_amq_probe_metrics) that probe launches add
    to; `collect()` reads them, `fold_into()` adds them to a host KeyQueryMetrics."""

    def __init__(self, device=None):
        torch = _torch()
        self.counts = torch.zeros(len(abi.PROBE_METRICS_FIELDS), dtype=torch.int64,
                                  device=device or "cuda")

    def reset(self) -> None:
        self.counts.zero_()

    def collect(self) -> dict:
        return dict(zip(abi.PROBE_METRICS_FIELDS, (int(v) for v in self.counts.cpu().tolist())))

    def fold_into(self, m: "KeyQueryMetrics", reset: bool = True) -> None:
        for k, v in self.collect().items():
            getattr(m, k).add(v)
        if reset:
            self.reset()


def _probe_opts(query_page_ids, truth, metrics):
    torch = _torch()
    keep = []
    pid = None
    if query_page_ids is not None:
        pid = query_page_ids.to(dtype=torch.int64).contiguous()
        keep.append(pid)
    tr = None
    if truth is not None:
        tr = truth.to(dtype=torch.uint8).contiguous()
        keep.append(tr)
    o = abi.ProbeOpts(None if pid is None else pid.data_ptr(), None if tr is None else tr.data_ptr(),
                      None if metrics is None else metrics.counts.data_ptr())
    return o, keep


def probe_filters(plan: FilterPlan, filters, queries: KeyBatch, query_seg, out=None, stream=None,
                  query_page_ids=None, truth=None, metrics: ProbeMetrics | None = None):
    """Batched KeyQuery filter test: result[i] = 0 iff the filter of segment query_seg[i]
    rejects queries[i] (reject_page == kTrue).  Optional, per query: the leaf page id asked
    about (a filter built for another page answers 1, kUnknown), the ground truth (1 = key is
    in the leaf) for the false-positive count, and device KeyQuery::Metrics counters."""
    torch = _torch()
    _require_device()
    dev = filters.device
    if out is None:
        out = torch.empty(queries.n, dtype=torch.uint8, device=dev)
    qs = query_seg.to(dtype=torch.int32)
    sh = _stream_handle(stream)
    if query_page_ids is None and truth is None and metrics is None:
        st = abi.lib().tkv_amq_probe(plan.kind, _ptr(filters), _ptr(plan.device_segs(dev)),
                                     plan.n_segs, _ptr(queries.data), _ptr(queries.offsets),
                                     queries.stride, queries.n, _ptr(qs), _ptr(out), sh)
    else:
        o, _keep = _probe_opts(query_page_ids, truth, metrics)
        st = abi.lib().tkv_amq_probe_ex(plan.kind, _ptr(filters), _ptr(plan.device_segs(dev)),
                                        plan.n_segs, _ptr(queries.data), _ptr(queries.offsets),
                                        queries.stride, queries.n, _ptr(qs), _ptr(out),
                                        ctypes.byref(o), sh)
        _hold(stream, *_keep)
    _hold(stream, qs)
    abi.check(st, "tkv_amq_probe")
    return out


def vqf_hash_val(keys: KeyBatch, stream=None):
    """vqf_hash_val for every key -> int64 tensor holding the u64 XXH64 bit patterns."""
    torch = _torch()
    _require_device()
    out = torch.empty(keys.n, dtype=torch.int64, device=keys.data.device)
    abi.check(abi.lib().tkv_amq_vqf_hash(_ptr(keys.data), _ptr(keys.offsets), keys.stride, keys.n,
                                         _ptr(out), _stream_handle(stream)), "tkv_amq_vqf_hash")
    return out


def vqf_probe_hashed(plan: FilterPlan, filters, hash_vals, query_seg, out=None, stream=None,
                     pair_query=None, query_page_ids=None, truth=None,
                     metrics: ProbeMetrics | None = None):
    """PackedVqfFilter::is_present for pre-hashed queries; pair i tests leaf query_seg[i]
    with hash_vals[pair_query[i]] (identity when pair_query is None).  The optional inputs
    are per pair, as in probe_filters."""
    torch = _torch()
    _require_device()
    dev = filters.device
    n = query_seg.numel()
    if out is None:
        out = torch.empty(n, dtype=torch.uint8, device=dev)
    qs = query_seg.to(dtype=torch.int32)
    pq = None if pair_query is None else pair_query.to(dtype=torch.int32)
    o, _keep = _probe_opts(query_page_ids, truth, metrics)
    abi.check(abi.lib().tkv_amq_vqf_probe_hashed_ex(_ptr(filters), _ptr(plan.device_segs(dev)),
                                                    plan.n_segs, _ptr(hash_vals), _ptr(pq), n,
                                                    _ptr(qs), _ptr(out), ctypes.byref(o),
                                                    _stream_handle(stream)),
              "tkv_amq_vqf_probe_hashed")
    _hold(stream, qs, pq, *_keep)
    return out


def bloom_query_hashes(keys: KeyBatch, k_max: int, stream=None):
    """BloomFilterQuery<KeyView> cache for a batch of queries (tree/key_query.hpp:78,97):
    one record per query (h0 + k_max-1 bit indices), computed once."""
    torch = _torch()
    _require_device()
    stride = int(abi.lib().tkv_amq_bloom_query_stride(k_max))
    out = torch.empty(max(keys.n, 1) * stride, dtype=torch.uint8, device=keys.data.device)
    abi.check(abi.lib().tkv_amq_bloom_hash(_ptr(keys.data), _ptr(keys.offsets), keys.stride, keys.n,
                                           k_max, _ptr(out), _stream_handle(stream)),
              "tkv_amq_bloom_hash")
    return out


def bloom_probe_hashed(plan: FilterPlan, filters, query_hashes, k_max: int, query_seg, out=None,
                       stream=None, pair_query=None, query_page_ids=None, truth=None,
                       metrics: ProbeMetrics | None = None):
    """PackedBloomFilter::query(BloomFilterQuery) for (query, leaf) pairs."""
    torch = _torch()
    _require_device()
    dev = filters.device
    n = query_seg.numel()
    if out is None:
        out = torch.empty(n, dtype=torch.uint8, device=dev)
    qs = query_seg.to(dtype=torch.int32)
    pq = None if pair_query is None else pair_query.to(dtype=torch.int32)
    o, _keep = _probe_opts(query_page_ids, truth, metrics)
    abi.check(abi.lib().tkv_amq_bloom_probe_hashed_ex(_ptr(filters), _ptr(plan.device_segs(dev)),
                                                      plan.n_segs, _ptr(query_hashes), k_max,
                                                      _ptr(pq), n, _ptr(qs), _ptr(out),
                                                      ctypes.byref(o), _stream_handle(stream)),
              "tkv_amq_bloom_probe_hashed")
    _hold(stream, qs, pq, *_keep)
    return out


# ---------------------------------------------------------------------------------------
# single-leaf API (the reference's per-leaf entry points)
# ---------------------------------------------------------------------------------------
@dataclass
class FilterPage:
    """A built filter page payload on the device plus its one-segment plan."""
    kind: int
    payload: object          # device uint8 tensor (page payload bytes)
    plan: FilterPlan
    leaf_page_id: int

    @property
    def filter_size(self) -> int:
        return int(self.plan.segs[0]["payload_bytes"])

    def unused_begin(self) -> int:
        """filter_page_header->unused_begin (filter_builder.hpp:293-294)."""
        return PACKED_PAGE_HEADER_BYTES + self.filter_size


def _build_one(kind: int, bpk: int, leaf_page_id: int, keys: KeyBatch,
               page_payload_bytes: int) -> FilterPage | None:
    if bpk == 0:
        return None  # filter_builder.hpp:115-117 / :227-229
    plan = plan_filters(kind, [keys.n], bpk, payload_capacity=page_payload_bytes,
                        src_page_ids=[leaf_page_id])
    out = build_all_filters(plan, keys)
    return FilterPage(kind, out, plan, leaf_page_id)


def build_bloom_filter_for_leaf(filter_bits_per_key: int, leaf_page_id: int, keys: KeyBatch,
                                page_payload_bytes: int = 0) -> FilterPage | None:
    return _build_one(BLOOM, filter_bits_per_key, leaf_page_id, keys, page_payload_bytes)


def build_quotient_filter_for_leaf(filter_bits_per_key: int, leaf_page_id: int, keys: KeyBatch,
                                   page_payload_bytes: int) -> FilterPage | None:
    return _build_one(VQF, filter_bits_per_key, leaf_page_id, keys, page_payload_bytes)


def build_filter_for_leaf_in_job(filter_bits_per_key: int, leaf_page_id: int, keys: KeyBatch,
                                 page_payload_bytes: int | None = None,
                                 kind: int = DEFAULT_FILTER_KIND) -> FilterPage | None:
    """Like the reference: a failed build is logged and the leaf gets no filter
    (filter_builder.hpp:323-325).  The payload capacity defaults to the filter page of the
    default TreeOptions for this bits/key (TreeOptions.filter_page_payload_size)."""
    if page_payload_bytes is None:
        page_payload_bytes = (TreeOptions(kind).set_filter_bits_per_key(filter_bits_per_key)
                              .filter_page_payload_size())
    try:
        if kind == BLOOM:
            return build_bloom_filter_for_leaf(filter_bits_per_key, leaf_page_id, keys,
                                               page_payload_bytes)
        return build_quotient_filter_for_leaf(filter_bits_per_key, leaf_page_id, keys,
                                              page_payload_bytes)
    except TkvAmqError as e:
        if e.status == abi.UNAVAILABLE:
            raise
        log.warning("Failed to build filter: %s", e)
        return None


class PackedVqfFilter:
    """View of a VQF filter page payload in device memory (vqf_filter_page_view.hpp:63-126)."""

    def __init__(self, page: FilterPage):
        if page.kind != VQF:
            raise TkvAmqError(abi.INVALID_ARGUMENT, "not a VQF filter page")
        self.page = page
        hdr = page.payload[:80].cpu().numpy().view("<u8")
        self.magic, self.src_page_id, self.hash_seed, self.hash_mask = (int(x) for x in hdr[:4])
        self.key_remainder_bits = int(hdr[5])

    def check_magic(self) -> None:
        if self.magic != VQF_MAGIC:
            raise TkvAmqError(abi.INTERNAL, "PackedVqfFilter magic mismatch")

    def is_present(self, hash_vals):
        """Batched is_present(hash_val): uint8 tensor, 1 = maybe present."""
        torch = _torch()
        hv = hash_vals if hasattr(hash_vals, "data_ptr") else torch.tensor(
            np.asarray(hash_vals, dtype=np.uint64).view(np.int64), device=self.page.payload.device)
        qs = torch.zeros(hv.numel(), dtype=torch.int32, device=hv.device)
        return vqf_probe_hashed(self.page.plan, self.page.payload, hv, qs)


class _Count:
    """FastCountMetric<u64>."""

    def __init__(self):
        self._lock = threading.Lock()
        self.value = 0

    def add(self, n: int) -> None:
        with self._lock:
            self.value += int(n)

    def get(self) -> int:
        return self.value

    def __repr__(self):
        return str(self.value)


class KeyQueryMetrics:
    """KeyQuery::Metrics, the filter counters (tree/key_query.hpp:36-60).  reject_page updates
    total / no-filter / load-failed / page-id-mismatch / reject (:154,157,183,210,231,243);
    the caller's leaf search updates positive / false positive (key_query.cpp:41,77): the
    batched device probes count those when given a ProbeMetrics (and ground truth)."""

    def __init__(self):
        self.total_filter_query_count = _Count()
        self.no_filter_page_count = _Count()
        self.filter_page_load_failed_count = _Count()
        self.page_id_mismatch_count = _Count()
        self.filter_reject_count = _Count()
        self.filter_positive_count = _Count()
        self.filter_false_positive_count = _Count()

    def filter_false_positive_rate(self) -> float:
        positives = self.filter_positive_count.get()
        if positives == 0:
            return -1.0
        return self.filter_false_positive_count.get() / positives

    def as_dict(self) -> dict:
        return {k: v.get() for k, v in vars(self).items() if isinstance(v, _Count)}


class KeyQuery:
    """KeyQuery (tree/key_query.hpp:33-253) for a batch of point-query keys.  The hashes are
    computed once per query and reused for every filter probed: the VQF hash_val
    (key_query.hpp:82) and the Bloom BloomFilterQuery cache (:78,97)."""

    BLOOM_K_MAX = 32
    _metrics = KeyQueryMetrics()

    @classmethod
    def metrics(cls) -> KeyQueryMetrics:
        """The process-wide counters (KeyQuery::metrics(), :64-68)."""
        return cls._metrics

    def __init__(self, keys: KeyBatch):
        self.keys = keys
        self.hash_val = vqf_hash_val(keys)
        self.bloom_query = bloom_query_hashes(keys, self.BLOOM_K_MAX)

    def reject_page(self, page_id_to_reject: int, filter_page: FilterPage | None,
                    truth=None) -> list:
        """Per key: kTrue = filter says definitely absent; kFalse = maybe present;
        kUnknown = no filter page, or it belongs to another leaf (key_query.hpp:156-159,207-232).
        `truth` (optional, 1 = key is in the leaf): counts the positives that are false, as the
        caller's leaf search does (key_query.cpp:41,77)."""
        torch = _torch()
        m = self.metrics()
        n = self.keys.n
        m.total_filter_query_count.add(n)
        if filter_page is None:
            m.no_filter_page_count.add(n)
            return [BoolStatus.kUnknown] * n
        hdr = filter_page.payload[:32].cpu().numpy().view("<u8")
        magic = int(hdr[0])
        want = VQF_MAGIC if filter_page.kind == VQF else BLOOM_MAGIC
        if magic != want:  # check_magic (:194, vqf_filter_page_view.hpp:97-100)
            raise TkvAmqError(abi.INTERNAL, "filter page magic mismatch")
        src = int(hdr[2]) if filter_page.kind == BLOOM else int(hdr[1])
        if src != page_id_to_reject:
            m.page_id_mismatch_count.add(n)
            return [BoolStatus.kUnknown] * n
        dev = filter_page.payload.device
        qs = torch.zeros(n, dtype=torch.int32, device=dev)
        pm = ProbeMetrics(dev)
        tr = None if truth is None else torch.as_tensor(np.asarray(truth, dtype=np.uint8), device=dev)
        if filter_page.kind == VQF:
            present = vqf_probe_hashed(filter_page.plan, filter_page.payload, self.hash_val, qs,
                                       truth=tr, metrics=pm)
        else:
            present = bloom_probe_hashed(filter_page.plan, filter_page.payload, self.bloom_query,
                                         self.BLOOM_K_MAX, qs, truth=tr, metrics=pm)
        c = pm.collect()
        m.filter_reject_count.add(c["filter_reject_count"])
        m.filter_positive_count.add(c["filter_positive_count"])
        if truth is not None:
            m.filter_false_positive_count.add(c["filter_false_positive_count"])
        return [BoolStatus.kFalse if p else BoolStatus.kTrue for p in present.cpu().tolist()]


# ---------------------------------------------------------------------------------------
# host-resident keys -> host filter pages (keys come from host
# checkpoint buffers and the filters return to host page memory)
# ---------------------------------------------------------------------------------------
class HostFilterPipeline:
    """Host-resident keys -> host filter pages for one batch shape (a checkpoint's leaves).

    Chunks of whole leaves flow H2D -> build -> D2H on three streams (copy-in, build,
    copy-out), double-buffered, so PCIe transfers in both directions overlap the kernels.
    Plans, device buffers and per-chunk plan uploads are prepared once in the constructor;
    run() only enqueues copies and builds.  Output: the batch's filter pages at a fixed
    per-leaf stride (leaf s at byte s * out_stride)."""

    def __init__(self, kind: int, leaf_key_counts, bits_per_key: int, payload_capacity: int = 0,
                 out_stride: int = 0, chunk_keys: int = 8 << 20, src_page_ids=None,
                 key_bytes: int = 16, device=None):
        torch = _torch()
        _require_device()
        self.kind, self.dev = kind, torch.device(device or "cuda")
        self.key_bytes = key_bytes
        counts = np.asarray(leaf_key_counts, dtype=np.int64)
        if out_stride == 0:
            biggest = int(counts.max()) if len(counts) else 0
            p1 = plan_filters(kind, [biggest], bits_per_key, payload_capacity=payload_capacity)
            out_stride = (int(p1.segs[0]["payload_bytes"]) + 63) // 64 * 64 or 64
        self.out_stride = out_stride
        self.plan = plan_filters(kind, counts, bits_per_key, payload_capacity=payload_capacity,
                                 out_stride=out_stride, src_page_ids=src_page_ids)
        bounds, acc = [0], 0
        for i, c in enumerate(counts):
            acc += int(c)
            if acc >= chunk_keys:
                bounds.append(i + 1)
                acc = 0
        if bounds[-1] != len(counts):
            bounds.append(len(counts))
        self.key_begin = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
        self.chunks = list(zip(bounds, bounds[1:]))
        self.plans = [plan_filters(kind, counts[b0:b1], bits_per_key,
                                   payload_capacity=payload_capacity, out_stride=out_stride,
                                   src_page_ids=self.plan.segs["src_page_id"][b0:b1])
                      for b0, b1 in self.chunks]
        max_keys = max((int(self.key_begin[b1] - self.key_begin[b0]) for b0, b1 in self.chunks), default=1)
        max_leaves = max((b1 - b0 for b0, b1 in self.chunks), default=1)
        ws_bytes = max((p.workspace_bytes for p in self.plans), default=0)
        self.d_keys = [torch.empty((max(max_keys, 1), key_bytes), dtype=torch.uint8, device=self.dev)
                       for _ in range(2)]
        self.d_out = [torch.empty(max(max_leaves * out_stride, 1), dtype=torch.uint8, device=self.dev)
                      for _ in range(2)]
        self.d_ws = [torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=self.dev) for _ in range(2)]
        for p in self.plans:
            p.device_segs(self.dev)
        self.s_in, self.s_run, self.s_out = (torch.cuda.Stream(self.dev) for _ in range(3))
        # failed leaves by cause: [0] inserts that overflowed a block (TKV_AMQ_VQF_FLAG_OVERFLOW,
        # bit 31), [1] a workspace smaller than the plan (TKV_AMQ_VQF_FLAG_WORKSPACE, bit 30)
        self.fail = torch.zeros(2, dtype=torch.int32, device=self.dev)
        torch.cuda.synchronize(self.dev)

    def new_host_output(self):
        return _torch().empty(self.plan.total_out_bytes, dtype=_torch().uint8, pin_memory=True)

    def _fold_flags(self, slot: int, chunk) -> None:
        """Add the chunk's failed-leaf counts (the flag bits of each leaf's nelts word in the VQF
        workspace, tkv_amq_build_check's source) to self.fail, on the device: bit 31 (an insert
        overflowed its block) and bit 30 (the workspace was short) counted apart, so each is
        reported as tkv_amq_build_check reports it."""
        torch = _torch()
        b0, b1 = chunk
        w = self.d_ws[slot][64:64 + 4 * (b1 - b0)].view(torch.int32)
        self.fail[0].add_((w < 0).sum(dtype=torch.int32))                  # bit 31
        self.fail[1].add_((((w >> 30) & 1) != 0).sum(dtype=torch.int32))  # bit 30

    def run_views(self, views, host_out=None, view_stride: int = 16, n_threads: int = 16,
                  check: bool = True):
        """Keys given as tkv_amq_key_view records (the EditView key range; KEY_VIEW_DTYPE
        array or the address of the first view).  Each chunk's keys are gathered into a
        pinned staging buffer by host threads just before its H2D copy is enqueued, so the
        gather of chunk c+1 overlaps the copies and build of chunk c.  The threads are a
        persistent pool, each running tkv_amq_stage_keys on a slice (ctypes releases the GIL),
        so no threads are created per chunk."""
        import concurrent.futures
        torch = _torch()
        if isinstance(views, np.ndarray):
            assert views.dtype == abi.KEY_VIEW_DTYPE and views.flags.c_contiguous
            addr, view_stride = views.ctypes.data, abi.KEY_VIEW_DTYPE.itemsize
        else:
            addr = int(views)
        n_keys = int(self.key_begin[-1])
        if getattr(self, "_h_stage", None) is None or self._h_stage.shape[0] < n_keys:
            self._h_stage = torch.empty((max(n_keys, 1), self.key_bytes), dtype=torch.uint8,
                                        pin_memory=True)
        h = self._h_stage
        if getattr(self, "_pool", None) is None or self._pool_threads != n_threads:
            self._pool = concurrent.futures.ThreadPoolExecutor(max(1, n_threads))
            self._pool_threads = n_threads

        def one(a, b):
            stage_keys(addr + a * view_stride, b - a, self.key_bytes, out=h[a:b],
                       view_stride=view_stride, n_threads=1)

        def stage(k0, k1):
            if k1 <= k0:
                return
            parts = max(1, min(n_threads, (k1 - k0) // 16384))
            cuts = [k0 + (k1 - k0) * i // parts for i in range(parts + 1)]
            for f in [self._pool.submit(one, a, b) for a, b in zip(cuts, cuts[1:])]:
                f.result()

        return self.run(h, host_out, check, stage=stage)

    def run(self, host_keys, host_out=None, check: bool = True, stage=None):
        """`stage(k0, k1)`, if given, fills host_keys[k0:k1] before that chunk's H2D copy is
        enqueued (run_views)."""
        torch = _torch()
        t_run = time.perf_counter()
        if host_out is None:
            host_out = self.new_host_output()
        n = len(self.chunks)
        ev_in = [torch.cuda.Event() for _ in range(n)]
        ev_run = [torch.cuda.Event() for _ in range(n)]
        ev_out = [torch.cuda.Event() for _ in range(n)]
        st = self.out_stride
        self.s_run.wait_stream(torch.cuda.current_stream(self.dev))
        with torch.cuda.stream(self.s_run):
            self.fail.zero_()
        for c, (b0, b1) in enumerate(self.chunks):
            slot = c & 1
            k0, k1 = int(self.key_begin[b0]), int(self.key_begin[b1])
            if stage is not None:
                stage(k0, k1)
            with torch.cuda.stream(self.s_in):
                if c >= 2:
                    self.s_in.wait_event(ev_run[c - 2])       # slot's keys no longer read
                self.d_keys[slot][:k1 - k0].copy_(host_keys[k0:k1], non_blocking=True)
                ev_in[c].record(self.s_in)
            with torch.cuda.stream(self.s_run):
                self.s_run.wait_event(ev_in[c])
                if c >= 2:
                    self.s_run.wait_event(ev_out[c - 2])      # slot's output copied out
                    if self.kind == VQF:                      # fold chunk c-2's failure flags
                        self._fold_flags(slot, self.chunks[c - 2])
                build_all_filters(self.plans[c], KeyBatch.fixed(self.d_keys[slot][:k1 - k0]),
                                  out=self.d_out[slot], workspace=self.d_ws[slot],
                                  stream=self.s_run, check=False)
                ev_run[c].record(self.s_run)
            with torch.cuda.stream(self.s_out):
                self.s_out.wait_event(ev_run[c])
                nbytes = (b1 - b0) * st
                host_out[b0 * st:b0 * st + nbytes].copy_(self.d_out[slot][:nbytes], non_blocking=True)
                ev_out[c].record(self.s_out)
        if self.kind == VQF:
            with torch.cuda.stream(self.s_run):
                for c in range(max(0, n - 2), n):
                    self._fold_flags(c & 1, self.chunks[c])
        self.s_out.synchronize()
        if check and self.kind == VQF:
            self.s_run.synchronize()
            overflow, short_ws = (int(x) for x in self.fail.tolist())
            if short_ws:  # as tkv_amq_build_check: the plan's workspace was not given
                raise TkvAmqError(abi.INVALID_ARGUMENT, f"vqf build: workspace smaller than the plan "
                                                        f"({short_ws} leaves)")
            if overflow:
                raise TkvAmqError(abi.INTERNAL, "vqf_insert (filter_builder.hpp:211)")
        if check or self.kind == BLOOM:
            record_filter_metrics(self.plan, (time.perf_counter() - t_run) * 1e6)
        return host_out


def build_filters_from_host(kind: int, leaf_key_counts, bits_per_key: int, host_keys,
                            payload_capacity: int = 0, out_stride: int = 0, host_out=None,
                            chunk_keys: int = 8 << 20, src_page_ids=None, device=None):
    """One-shot HostFilterPipeline: returns (host_out, plan of the whole batch)."""
    torch = _torch()
    if not isinstance(host_keys, torch.Tensor):
        host_keys = torch.from_numpy(np.ascontiguousarray(host_keys))
    pipe = HostFilterPipeline(kind, leaf_key_counts, bits_per_key, payload_capacity, out_stride,
                              chunk_keys, src_page_ids, host_keys.shape[1], device)
    return pipe.run(host_keys, host_out), pipe.plan
