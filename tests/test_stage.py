"""CPU: host key staging (tkv_amq_stage_keys) -- the EditView key range of
build_filter_for_leaf_in_job (core/merge_compactor.hpp:107-139) gathered into one contiguous
host buffer.  Checked against numpy gathers; needs no device."""
import ctypes

import numpy as np
import pytest


def edit_buffer(rng, n, key_len, val_len=24):
    """n edits laid out as [key | value] records, like leaf-page items: key i at i*rec."""
    rec = key_len + val_len
    buf = rng.integers(0, 256, n * rec, dtype=np.uint8)
    return buf, rec


@pytest.mark.parametrize("n,threads", [(1, 0), (5000, 1), (200_001, 0), (300_000, 7)])
def test_stage_fixed16_from_strided_records(amq, n, threads):
    rng = np.random.default_rng(n)
    buf, rec = edit_buffer(rng, n, 16)
    views = amq.key_views(buf, np.arange(n, dtype=np.uint64) * rec, 16)
    got = amq.stage_keys(views, fixed_len=16, n_threads=threads)
    want = buf.reshape(n, rec)[:, :16]
    assert np.array_equal(got, want)


def test_stage_views_read_in_place_at_edit_stride(amq):
    """&edits[0].key with stride sizeof(EditView): views embedded in larger records."""
    n = 70_000
    rng = np.random.default_rng(3)
    keys = rng.integers(0, 256, (n, 24), dtype=np.uint8)
    edit = np.dtype([("size", "<u8"), ("data", "<u8"), ("vsize", "<u8"), ("vdata", "<u8")])
    edits = np.zeros(n, dtype=edit)
    edits["size"] = 24
    edits["data"] = np.uint64(keys.ctypes.data) + np.arange(n, dtype=np.uint64) * 24
    got = amq.stage_keys(edits.ctypes.data, n, fixed_len=24, view_stride=edit.itemsize)
    assert np.array_equal(got, keys)


@pytest.mark.parametrize("n", [0, 1, 9999, 150_000])
def test_stage_variable_length(amq, n):
    rng = np.random.default_rng(n + 1)
    lens = rng.integers(0, 40, n).astype(np.uint64)
    blob = rng.integers(0, 256, int(lens.sum()) + 64, dtype=np.uint8)
    # keys scattered in the blob in a shuffled order (views need not be in address order)
    starts = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64) if n else np.zeros(0, np.uint64)
    perm = rng.permutation(n)
    views = amq.key_views(blob, starts[perm], lens[perm])
    data, offs = amq.stage_keys(views, fixed_len=0)
    assert offs[0] == 0 and int(offs[-1]) == int(lens.sum())
    for j in range(0, n, max(1, n // 500)):
        i = perm[j]
        want = blob[int(starts[i]):int(starts[i] + lens[i])]
        assert np.array_equal(data[int(offs[j]):int(offs[j + 1])], want)


def test_stage_errors(amq):
    L = amq.abi.lib()
    buf = np.zeros(64, np.uint8)
    v = amq.key_views(buf, [0, 16, 32], [16, 16, 15])     # one key of the wrong length
    with pytest.raises(amq.TkvAmqError) as e:
        amq.stage_keys(v, fixed_len=16)
    assert e.value.status == amq.abi.INVALID_ARGUMENT
    v = amq.key_views(buf, [0, 16, 32], 16)
    small = np.zeros((2, 16), np.uint8)                    # does not fit
    assert L.tkv_amq_stage_keys(ctypes.c_void_p(v.ctypes.data), 16, 3, 16,
                                ctypes.c_void_p(small.ctypes.data), small.nbytes, None, 0) == 8
    with pytest.raises(amq.TkvAmqError) as e:               # variable length, too small
        amq.stage_keys(v, fixed_len=0, out=np.zeros(40, np.uint8))
    assert e.value.status == amq.abi.RESOURCE_EXHAUSTED
    assert L.tkv_amq_stage_keys(None, 16, 3, 16, ctypes.c_void_p(small.ctypes.data), 64, None, 0) == 3
    assert L.tkv_amq_stage_keys(ctypes.c_void_p(v.ctypes.data), 8, 3, 16,   # stride < view
                                ctypes.c_void_p(small.ctypes.data), 64, None, 0) == 3
