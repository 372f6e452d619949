"""ctypes binding of the C ABI declared in include/tkv_amq.h (libtkv_amq.so).

This is the only way the Python host side reaches the filter kernels.  There is no CPU
fallback: if the library is missing or no GPU is visible, device entry points raise.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import _build

OK = 0
INVALID_ARGUMENT = 3
RESOURCE_EXHAUSTED = 8
INTERNAL = 13
UNAVAILABLE = 14

BLOOM = 0
VQF = 1

STATUS_NAMES = {OK: "OK", INVALID_ARGUMENT: "InvalidArgument",
                RESOURCE_EXHAUSTED: "ResourceExhausted", INTERNAL: "Internal",
                UNAVAILABLE: "Unavailable"}


class TkvAmqError(RuntimeError):
    """A non-OK status from libtkv_amq (mirrors batt::Status propagation)."""

    def __init__(self, status: int, what: str):
        super().__init__(f"{what}: {STATUS_NAMES.get(status, status)}")
        self.status = status


class Segment(ctypes.Structure):
    """tkv_amq_segment (64 bytes)."""
    _fields_ = [
        ("out_offset", ctypes.c_uint64),
        ("n_blocks", ctypes.c_uint32),
        ("hash_count", ctypes.c_uint16),
        ("tag_bits", ctypes.c_uint8),
        ("hash_val_shift", ctypes.c_uint8),
        ("mod_magic", ctypes.c_uint64),
        ("key_begin", ctypes.c_uint64),
        ("src_page_id", ctypes.c_uint64),
        ("block_base", ctypes.c_uint64),
        ("n_keys", ctypes.c_uint32),
        ("payload_bytes", ctypes.c_uint32),
        ("bits_per_key", ctypes.c_uint32),
        ("page_flags", ctypes.c_uint32),
    ]


assert ctypes.sizeof(Segment) == 64

SEGMENT_DTYPE = np.dtype([
    ("out_offset", "<u8"), ("n_blocks", "<u4"), ("hash_count", "<u2"), ("tag_bits", "u1"),
    ("hash_val_shift", "u1"), ("mod_magic", "<u8"), ("key_begin", "<u8"), ("src_page_id", "<u8"),
    ("block_base", "<u8"), ("n_keys", "<u4"), ("payload_bytes", "<u4"), ("bits_per_key", "<u4"),
    ("page_flags", "<u4")])
PAGE_IMAGE = 0x1  # TKV_AMQ_PAGE_IMAGE


class ProbeOpts(ctypes.Structure):
    """tkv_amq_probe_opts (device pointers, any may be NULL)."""
    _fields_ = [("d_query_page_id", ctypes.c_void_p), ("d_truth", ctypes.c_void_p),
                ("d_metrics", ctypes.c_void_p)]


# tkv_amq_probe_metrics: KeyQuery::Metrics counters (tree/key_query.hpp:36-60), u64 each
PROBE_METRICS_FIELDS = ("total_filter_query_count", "no_filter_page_count",
                        "page_id_mismatch_count", "filter_reject_count", "filter_positive_count",
                        "filter_false_positive_count")
assert SEGMENT_DTYPE.itemsize == 64

# every symbol include/tkv_amq.h declares
EXPORTS = [
    "tkv_amq_version", "tkv_amq_status_string", "tkv_amq_device_count",
    "tkv_amq_filter_bits_per_key", "tkv_amq_vqf_load_factor", "tkv_amq_vqf_required_size",
    "tkv_amq_vqf_nslots_for_size", "tkv_amq_plan", "tkv_amq_build", "tkv_amq_build_check",
    "tkv_amq_probe", "tkv_amq_vqf_hash", "tkv_amq_vqf_probe_hashed", "tkv_amq_gen_keys16",
    "tkv_amq_bloom_query_stride", "tkv_amq_bloom_hash", "tkv_amq_bloom_probe_hashed",
    "tkv_amq_stage_keys", "tkv_amq_leaf_data_size", "tkv_amq_expected_items_per_leaf",
    "tkv_amq_filter_page_size_log2", "tkv_amq_plan_pages", "tkv_amq_probe_ex",
    "tkv_amq_vqf_probe_hashed_ex", "tkv_amq_bloom_probe_hashed_ex",
    "tkv_amq_bloom_route_ws_bytes", "tkv_amq_bloom_route", "tkv_amq_bloom_build_range_ws_bytes",
    "tkv_amq_bloom_build_range", "tkv_amq_bloom_route_records_ws_bytes", "tkv_amq_bloom_route_records",
    "tkv_amq_bloom_build_range_records_ws_bytes", "tkv_amq_bloom_build_range_records",
    "tkv_amq_bloom_route_records_ex", "tkv_amq_bloom_tile_blocks", "tkv_amq_bloom_range_max_tiles",
    "tkv_amq_bloom_route_plan", "tkv_amq_bloom_route_blocks", "tkv_amq_bloom_build_part_blocks",
    "tkv_amq_bloom_blocks_lost", "tkv_amq_build_ex",
]


class RoutePlan(ctypes.Structure):
    """tkv_amq_route_plan: the pipelined hash-range build's parts, route workgroups and block
    layout (include/tkv_amq.h)."""
    _fields_ = [(n, ctypes.c_uint32) for n in (
        "n_tiles", "n_parts", "parts_per_rank", "part_tiles", "world", "n_chunks", "route_wgs",
        "region_cap", "ovf_cap", "hash_count")] + [(n, ctypes.c_uint64) for n in (
        "chunk_keys", "block_bytes", "counts_off", "ovf_n_off", "regions_off", "ovf_off",
        "route_ws_bytes", "part_ws_bytes", "part_bytes", "n_blocks")]


assert ctypes.sizeof(RoutePlan) == 120

# tkv_amq_key_view (libstdc++ std::string_view layout)
KEY_VIEW_DTYPE = np.dtype([("size", "<u8"), ("data", "<u8")])

_lib = None


def experiment_lib():
    """TKV_AMQ_LIB names an experiment build of the library (kernel A/B timing).  It is taken
    only together with TKV_AMQ_EXPERIMENT=1, so a stray variable cannot put an experiment
    library behind the tests, smoke() or the bench."""
    path = os.environ.get("TKV_AMQ_LIB")
    if not path:
        return None
    if os.environ.get("TKV_AMQ_EXPERIMENT") != "1":
        raise RuntimeError("TKV_AMQ_LIB is set but TKV_AMQ_EXPERIMENT is not 1: experiment "
                           "libraries are loaded only on purpose")
    return path


def lib(build_if_missing: bool = True):
    """Load libtkv_amq.so (building it in-tree if absent and hipcc is available)."""
    global _lib
    if _lib is not None:
        return _lib
    path = experiment_lib() or _build.LIB
    if not os.path.exists(path):
        if not build_if_missing:
            raise RuntimeError(f"libtkv_amq.so not built ({path}); run __graft_entry__.build()")
        _build.build()
    L = ctypes.CDLL(path)
    u64, u32, i32, vp, dbl = (ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p,
                              ctypes.c_double)
    L.tkv_amq_version.restype = ctypes.c_char_p
    L.tkv_amq_version.argtypes = []
    L.tkv_amq_status_string.restype = ctypes.c_char_p
    L.tkv_amq_status_string.argtypes = [i32]
    L.tkv_amq_device_count.restype = i32
    L.tkv_amq_device_count.argtypes = []
    L.tkv_amq_filter_bits_per_key.restype = u64
    L.tkv_amq_filter_bits_per_key.argtypes = [i32, u64]
    L.tkv_amq_vqf_load_factor.restype = dbl
    L.tkv_amq_vqf_load_factor.argtypes = [i32, u64]
    L.tkv_amq_vqf_required_size.restype = u64
    L.tkv_amq_vqf_required_size.argtypes = [i32, u64]
    L.tkv_amq_vqf_nslots_for_size.restype = u64
    L.tkv_amq_vqf_nslots_for_size.argtypes = [i32, u64]
    L.tkv_amq_plan.restype = i32
    L.tkv_amq_plan.argtypes = [i32, vp, vp, u32, u32, u64, u64, vp,
                               ctypes.POINTER(u64), ctypes.POINTER(u64), ctypes.POINTER(u32)]
    L.tkv_amq_build.restype = i32
    L.tkv_amq_build.argtypes = [i32, vp, vp, u32, u64, vp, u32, u32, vp, vp, u64, vp]
    if hasattr(L, "tkv_amq_build_ex"):
        L.tkv_amq_build_ex.restype = i32
        L.tkv_amq_build_ex.argtypes = [i32, vp, vp, u32, u64, vp, vp, u32, u32, vp, vp, u64, vp]
    L.tkv_amq_build_check.restype = i32
    L.tkv_amq_build_check.argtypes = [i32, vp, u64, vp]
    L.tkv_amq_probe.restype = i32
    L.tkv_amq_probe.argtypes = [i32, vp, vp, u32, vp, vp, u32, u64, vp, vp, vp]
    L.tkv_amq_vqf_hash.restype = i32
    L.tkv_amq_vqf_hash.argtypes = [vp, vp, u32, u64, vp, vp]
    L.tkv_amq_vqf_probe_hashed.restype = i32
    L.tkv_amq_vqf_probe_hashed.argtypes = [vp, vp, u32, vp, vp, u64, vp, vp, vp]
    L.tkv_amq_bloom_query_stride.restype = u32
    L.tkv_amq_bloom_query_stride.argtypes = [u32]
    L.tkv_amq_bloom_hash.restype = i32
    L.tkv_amq_bloom_hash.argtypes = [vp, vp, u32, u64, u32, vp, vp]
    L.tkv_amq_bloom_probe_hashed.restype = i32
    L.tkv_amq_bloom_probe_hashed.argtypes = [vp, vp, u32, vp, u32, vp, u64, vp, vp, vp]
    L.tkv_amq_gen_keys16.restype = i32
    L.tkv_amq_gen_keys16.argtypes = [u64, u64, u64, vp, vp]
    L.tkv_amq_stage_keys.restype = i32
    L.tkv_amq_stage_keys.argtypes = [vp, u64, u64, u32, vp, u64, vp, i32]
    if path != _build.LIB and not hasattr(L, "tkv_amq_probe_ex"):
        _lib = L  # an older experiment build (A/B timing): the round-1 entry points only
        return L
    L.tkv_amq_leaf_data_size.restype = u64
    L.tkv_amq_leaf_data_size.argtypes = [u64]
    L.tkv_amq_expected_items_per_leaf.restype = u64
    L.tkv_amq_expected_items_per_leaf.argtypes = [u64, u32, u32]
    L.tkv_amq_filter_page_size_log2.restype = u32
    L.tkv_amq_filter_page_size_log2.argtypes = [i32, u64, u32, u32, u64]
    L.tkv_amq_plan_pages.restype = i32
    L.tkv_amq_plan_pages.argtypes = [i32, vp, vp, u32, u32, u32, vp,
                                     ctypes.POINTER(u64), ctypes.POINTER(u64), ctypes.POINTER(u32)]
    popts = ctypes.POINTER(ProbeOpts)
    L.tkv_amq_probe_ex.restype = i32
    L.tkv_amq_probe_ex.argtypes = [i32, vp, vp, u32, vp, vp, u32, u64, vp, vp, popts, vp]
    L.tkv_amq_vqf_probe_hashed_ex.restype = i32
    L.tkv_amq_vqf_probe_hashed_ex.argtypes = [vp, vp, u32, vp, vp, u64, vp, vp, popts, vp]
    L.tkv_amq_bloom_probe_hashed_ex.restype = i32
    L.tkv_amq_bloom_probe_hashed_ex.argtypes = [vp, vp, u32, vp, u32, vp, u64, vp, vp, popts, vp]
    if hasattr(L, "tkv_amq_bloom_route"):
        L.tkv_amq_bloom_route_ws_bytes.restype = u64
        L.tkv_amq_bloom_route_ws_bytes.argtypes = [u64, u32]
        L.tkv_amq_bloom_route.restype = i32
        L.tkv_amq_bloom_route.argtypes = [vp, u64, vp, u32, u32, vp, vp, vp, u64, vp]
        L.tkv_amq_bloom_build_range_ws_bytes.restype = u64
        L.tkv_amq_bloom_build_range_ws_bytes.argtypes = [u64, u32, u32]
        L.tkv_amq_bloom_build_range.restype = i32
        L.tkv_amq_bloom_build_range.argtypes = [vp, u64, vp, u32, u32, u32, vp, vp, u64, vp]
        L.tkv_amq_bloom_route_records_ws_bytes.restype = u64
        L.tkv_amq_bloom_route_records_ws_bytes.argtypes = [u64, u32]
        L.tkv_amq_bloom_route_records.restype = i32
        L.tkv_amq_bloom_route_records.argtypes = [vp, u64, vp, u32, u32, u32, vp, vp, vp, u64, vp]
        L.tkv_amq_bloom_route_records_ex.restype = i32
        L.tkv_amq_bloom_route_records_ex.argtypes = [vp, u32, u64, vp, u32, u32, u32, vp, vp, vp, u64, vp]
        L.tkv_amq_bloom_build_range_records_ws_bytes.restype = u64
        L.tkv_amq_bloom_build_range_records_ws_bytes.argtypes = [u64, u32, u32]
        L.tkv_amq_bloom_build_range_records.restype = i32
        L.tkv_amq_bloom_build_range_records.argtypes = [vp, u64, vp, u32, u32, u32, u32, vp, vp, u64, vp]
    if hasattr(L, "tkv_amq_bloom_route_plan"):
        prp = ctypes.POINTER(RoutePlan)
        L.tkv_amq_bloom_route_plan.restype = i32
        L.tkv_amq_bloom_route_plan.argtypes = [u64, u32, u32, u32, u32, prp]
        L.tkv_amq_bloom_route_blocks.restype = i32
        L.tkv_amq_bloom_route_blocks.argtypes = [vp, u32, u64, vp, prp, vp, u64, vp, u64, vp]
        L.tkv_amq_bloom_build_part_blocks.restype = i32
        L.tkv_amq_bloom_build_part_blocks.argtypes = [vp, u32, vp, prp, u32, vp, vp, u64, vp]
        L.tkv_amq_bloom_blocks_lost.restype = i32
        L.tkv_amq_bloom_blocks_lost.argtypes = [vp, u32, prp, vp]
    if hasattr(L, "tkv_amq_bloom_tile_blocks"):
        L.tkv_amq_bloom_tile_blocks.restype = u32
        L.tkv_amq_bloom_tile_blocks.argtypes = []
        L.tkv_amq_bloom_range_max_tiles.restype = u32
        L.tkv_amq_bloom_range_max_tiles.argtypes = [i32]
    _lib = L
    return L


def check(status: int, what: str) -> None:
    if status != OK:
        raise TkvAmqError(status, what)


def version() -> str:
    return lib().tkv_amq_version().decode()
