"""ctypes loader for the CPU oracle (TEST INFRASTRUCTURE ONLY).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module, and only as the checker or as the timed CPU baseline.  The product
package ``turtle_kv_amd`` never imports it.

The C source (``tkv_amq_oracle.c``) restates TurtleKV's filter path; see its header for
the reference file:line map and the parity status (Bloom/VQF layouts parity-unpinned
against llfs/vqf, which are absent from /root/reference).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libtkv_amq_oracle.so")
_NATIVE_PATH = os.path.join(_HERE, "build", "native", "libtkv_amq_oracle.so")
_lib = None
_native = None

VQF_HASH_SEED = 0x9D0924DC03E79A75
BLOOM, VQF = 0, 1


class VqfPlan(ctypes.Structure):
    _fields_ = [
        ("tag_bits", ctypes.c_uint32),
        ("hash_val_shift", ctypes.c_uint32),
        ("nslots", ctypes.c_uint64),
        ("nblocks", ctypes.c_uint64),
        ("filter_size", ctypes.c_uint64),
        ("payload_used", ctypes.c_uint64),
    ]


def build_oracle() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def build_native() -> str:
    """The reference's own flags (-O3 -march=native -mbmi2 -mavx2, CMakeLists.txt:46-48),
    compiled for the CPU this runs on (bench.py's cpu_baseline leg, on the GPU box's host)."""
    subprocess.run(["make", "-s", "-C", _HERE, "native"], check=True)
    return _NATIVE_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build_oracle()
        _lib = _load(_LIB_PATH)
    return _lib


def native_lib():
    """The oracle built with -march=native on this host (None if that build fails: the
    portable build is then the baseline, and bench.py says so)."""
    global _native
    if _native is None:
        try:
            build_native()
            _native = _load(_NATIVE_PATH)
        except (OSError, subprocess.CalledProcessError):
            return None
    return _native


def _load(path):
    L = ctypes.CDLL(path)
    u64, u32, vp, i32 = ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int
    L.tkvo_xxh64.restype = u64
    L.tkvo_xxh64.argtypes = [vp, ctypes.c_size_t, u64]
    L.tkvo_splitmix64_at.restype = u64
    L.tkvo_splitmix64_at.argtypes = [u64, u64]
    L.tkvo_gen_keys16.argtypes = [u64, u64, u64, vp]
    L.tkvo_sort_keys16_segments.argtypes = [vp, vp, u32, i32]
    L.tkvo_bloom_hash_count.restype = u32
    L.tkvo_bloom_hash_count.argtypes = [u32]
    L.tkvo_bloom_seed.restype = u64
    L.tkvo_bloom_seed.argtypes = [u32]
    L.tkvo_bloom_block_count.restype = u32
    L.tkvo_bloom_block_count.argtypes = [u64, u32]
    L.tkvo_bloom_payload_size.restype = u64
    L.tkvo_bloom_payload_size.argtypes = [u64, u32]
    L.tkvo_bloom_build_payload.restype = i32
    L.tkvo_bloom_build_payload.argtypes = [vp, vp, u32, u64, u32, u64, vp, u64]
    L.tkvo_bloom_query_payload.restype = i32
    L.tkvo_bloom_query_payload.argtypes = [vp, vp, ctypes.c_size_t]
    L.tkvo_bloom_sample_blocks_gen16.restype = i32
    L.tkvo_bloom_sample_blocks_gen16.argtypes = [u64, u64, u64, u32, vp, vp, u32, vp, i32]
    L.tkvo_vqf_load_factor.restype = ctypes.c_double
    L.tkvo_vqf_load_factor.argtypes = [i32, u64]
    L.tkvo_vqf_required_size.restype = u64
    L.tkvo_vqf_required_size.argtypes = [i32, u64]
    L.tkvo_vqf_nslots_for_size.restype = u64
    L.tkvo_vqf_nslots_for_size.argtypes = [i32, u64]
    L.tkvo_vqf_plan_segment.restype = i32
    L.tkvo_vqf_plan_segment.argtypes = [u64, u64, u64, ctypes.POINTER(VqfPlan)]
    L.tkvo_vqf_build_payload.restype = i32
    L.tkvo_vqf_build_payload.argtypes = [vp, vp, u32, u64, u64, u64, vp, u64,
                                         ctypes.POINTER(VqfPlan)]
    L.tkvo_vqf_is_present_payload.restype = i32
    L.tkvo_vqf_is_present_payload.argtypes = [vp, u64]
    L.tkvo_tree_filter_bits_per_key.restype = u64
    L.tkvo_tree_filter_bits_per_key.argtypes = [u64, i32]
    L.tkvo_build_segments.restype = i32
    L.tkvo_build_segments.argtypes = [i32, vp, vp, u32, u32, vp, vp, vp, vp, i32]
    L.tkvo_build_segments_ex.restype = i32
    L.tkvo_build_segments_ex.argtypes = [i32, vp, vp, u32, vp, u32, u32, vp, vp, vp, vp, i32]
    L.tkvb_vqf_build_payload16.restype = i32
    L.tkvb_vqf_build_payload16.argtypes = [vp, u64, u64, u64, vp, u64]
    L.tkvb_vqf_build_segments.restype = i32
    L.tkvb_vqf_build_segments.argtypes = [vp, vp, u32, u32, vp, vp, vp, vp, i32]
    L.tkvo_probe_segments.restype = i32
    L.tkvo_probe_segments.argtypes = [i32, vp, vp, vp, vp, u64, vp, i32]
    return L


def _p(a: np.ndarray | None):
    return None if a is None else ctypes.c_void_p(a.ctypes.data)


def xxh64(data: bytes, seed: int) -> int:
    buf = np.frombuffer(data, dtype=np.uint8) if data else np.zeros(1, np.uint8)
    return lib().tkvo_xxh64(_p(buf), len(data), seed)


def gen_keys16(seed: int, first: int, n: int) -> np.ndarray:
    out = np.empty((n, 16), dtype=np.uint8)
    lib().tkvo_gen_keys16(seed, first, n, _p(out))
    return out


def sort_segments(keys: np.ndarray, seg_begin: np.ndarray, n_threads: int = 8) -> None:
    seg_begin = np.ascontiguousarray(seg_begin, dtype=np.uint64)
    lib().tkvo_sort_keys16_segments(_p(keys), _p(seg_begin), len(seg_begin) - 1, n_threads)


def bloom_build(keys, n: int, bpk: int, src_page_id: int = 0, offsets=None, stride: int = 16,
                L=None):
    L = L or lib()
    cap = L.tkvo_bloom_payload_size(n, bpk)
    out = np.zeros(cap, dtype=np.uint8)
    st = L.tkvo_bloom_build_payload(_p(keys), _p(offsets), stride, n, bpk, src_page_id,
                                       _p(out), cap)
    return st, out


def bloom_sample_blocks(seed: int, first: int, n: int, bpk: int, windows, n_threads: int = 8):
    """The 64-byte blocks of the block windows [(b0, b1), ...] (ascending, disjoint) of the
    Bloom filter over gen_keys16(seed, first, n), without the key array or the whole filter.
    Returns (status, {(b0, b1): bytes})."""
    windows = sorted(windows)
    b0 = np.ascontiguousarray([w[0] for w in windows], dtype=np.uint64)
    b1 = np.ascontiguousarray([w[1] for w in windows], dtype=np.uint64)
    out = np.zeros(int(64 * (b1 - b0).sum()), dtype=np.uint8)
    st = lib().tkvo_bloom_sample_blocks_gen16(seed, first, n, bpk, _p(b0), _p(b1), len(windows),
                                             _p(out), n_threads)
    res, off = {}, 0
    for (a, b) in windows:
        res[(a, b)] = out[off:off + 64 * (b - a)]
        off += 64 * (b - a)
    return st, res


def bloom_query(payload: np.ndarray, key: bytes) -> int:
    kb = np.frombuffer(key, dtype=np.uint8).copy() if key else np.zeros(1, np.uint8)
    return lib().tkvo_bloom_query_payload(_p(payload), _p(kb), len(key))


def vqf_plan(n: int, bpk: int, payload_capacity: int):
    pl = VqfPlan()
    st = lib().tkvo_vqf_plan_segment(n, bpk, payload_capacity, ctypes.byref(pl))
    return st, pl


def vqf_build(keys, n: int, bpk: int, payload_capacity: int, src_page_id: int = 0,
              offsets=None, stride: int = 16):
    out = np.zeros(payload_capacity, dtype=np.uint8)
    pl = VqfPlan()
    st = lib().tkvo_vqf_build_payload(_p(keys), _p(offsets), stride, n, bpk, src_page_id,
                                     _p(out), payload_capacity, ctypes.byref(pl))
    return st, out, pl


def vqf_build_baseline(keys16, n: int, bpk: int, payload_capacity: int, src_page_id: int = 0,
                       L=None):
    """tkv_amq_baseline.c's BMI2 VQF build (the CPU baseline bench.py times)."""
    out = np.zeros(payload_capacity, dtype=np.uint8)
    st = (L or lib()).tkvb_vqf_build_payload16(_p(keys16), n, bpk, src_page_id, _p(out), payload_capacity)
    return st, out


def vqf_is_present(payload: np.ndarray, hash_val: int) -> int:
    return lib().tkvo_vqf_is_present_payload(_p(payload), hash_val)


def build_segments(kind: int, keys16: np.ndarray, seg_begin: np.ndarray, bpk: int,
                   out_offset: np.ndarray, out_capacity: np.ndarray, total_bytes: int,
                   src_page_id: np.ndarray | None = None, n_threads: int = 8,
                   out: np.ndarray | None = None, L=None, baseline: bool = False):
    """The oracle over a batch of 16-byte-key leaves (baseline=True, VQF: the BMI2 baseline)."""
    seg_begin = np.ascontiguousarray(seg_begin, dtype=np.uint64)
    out_offset = np.ascontiguousarray(out_offset, dtype=np.uint64)
    out_capacity = np.ascontiguousarray(out_capacity, dtype=np.uint64)
    if out is None:
        out = np.zeros(total_bytes, dtype=np.uint8)
    if kind == VQF and baseline:
        st = (L or lib()).tkvb_vqf_build_segments(_p(keys16), _p(seg_begin), len(seg_begin) - 1, bpk,
                                                  _p(src_page_id), _p(out), _p(out_offset),
                                                  _p(out_capacity), n_threads)
        return st, out
    st = (L or lib()).tkvo_build_segments(kind, _p(keys16), _p(seg_begin), len(seg_begin) - 1, bpk,
                                   _p(src_page_id), _p(out), _p(out_offset), _p(out_capacity),
                                   n_threads)
    return st, out


def build_segments_ex(kind: int, keys: np.ndarray, offsets: np.ndarray | None, stride: int,
                      seg_begin: np.ndarray, bpk: int, out_offset: np.ndarray,
                      out_capacity: np.ndarray, out: np.ndarray,
                      src_page_id: np.ndarray | None = None, n_threads: int = 8):
    """The oracle over a batch of leaves of any key shape (fixed `stride`, or variable-length
    keys through `offsets`, indexed by global key), into `out` at out_offset."""
    seg_begin = np.ascontiguousarray(seg_begin, dtype=np.uint64)
    out_offset = np.ascontiguousarray(out_offset, dtype=np.uint64)
    out_capacity = np.ascontiguousarray(out_capacity, dtype=np.uint64)
    if offsets is not None:
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    if src_page_id is not None:
        src_page_id = np.ascontiguousarray(src_page_id, dtype=np.uint64)
    return lib().tkvo_build_segments_ex(kind, _p(keys), _p(offsets), stride, _p(seg_begin),
                                        len(seg_begin) - 1, bpk, _p(src_page_id), _p(out),
                                        _p(out_offset), _p(out_capacity), n_threads)


def probe_segments(kind: int, filters: np.ndarray, out_offset: np.ndarray,
                   queries16: np.ndarray, query_seg: np.ndarray, n_threads: int = 8, L=None,
                   out: np.ndarray | None = None):
    out_offset = np.ascontiguousarray(out_offset, dtype=np.uint64)
    query_seg = np.ascontiguousarray(query_seg, dtype=np.uint32)
    res = np.zeros(len(query_seg), dtype=np.uint8) if out is None else out
    st = (L or lib()).tkvo_probe_segments(kind, _p(filters), _p(out_offset), _p(queries16),
                                   _p(query_seg), len(query_seg), _p(res), n_threads)
    return st, res
