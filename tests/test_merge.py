"""sg_merge_ts (csrc/sg_merge.cpp): the host merge of per-shard match runs into timestamp order (north_star:
per-partition output merged back in timestamp order on the host; the order MultiProcessStreamReceiver.java:
119-121 hands StateEvents on).  Against numpy's stable sort of the same records by (ts, run, index), serial and
parallel (merge path), with heavy timestamp ties, empty runs and one run.  Host code only: runs without a GPU."""
import ctypes as C
import importlib

import numpy as np
import pytest

sa = importlib.import_module("siddhi-1_amd")


def _lib():
    lib = sa.load_hip_library()
    lib.sg_merge_ts.argtypes = [C.c_uint32, C.POINTER(C.c_void_p), C.POINTER(C.c_uint64), C.c_uint32, C.c_void_p]
    lib.sg_merge_ts.restype = C.c_int
    return lib


def _merge(runs, threads):
    lib = _lib()
    k = len(runs)
    ptrs = (C.c_void_p * max(1, k))(*[r.ctypes.data if len(r) else None for r in runs])
    lens = (C.c_uint64 * max(1, k))(*[len(r) for r in runs])
    total = sum(len(r) for r in runs)
    out = np.zeros(max(1, total), dtype=np.uint64)
    assert lib.sg_merge_ts(k, ptrs, lens, threads, out.ctypes.data) == 0
    return out[:total]


def _expected(runs):
    ts = np.concatenate([r for r in runs]) if runs else np.zeros(0, np.int64)
    run = np.concatenate([np.full(len(r), i, np.uint64) for i, r in enumerate(runs)])
    idx = np.concatenate([np.arange(len(r), dtype=np.uint64) for r in runs])
    o = np.lexsort((idx, run, ts))
    return (run[o] << np.uint64(48)) | idx[o]


def _runs(rng, k, n, spread):
    return [np.sort(rng.integers(0, spread, size=int(rng.integers(0, n + 1)))).astype(np.int64) for _ in range(k)]


@pytest.mark.parametrize("threads", [1, 4, 16])
@pytest.mark.parametrize("k,n,spread", [(2, 1000, 50), (8, 50_000, 1000), (8, 50_000, 10**9), (5, 200_000, 7),
                                        (1, 100_000, 100), (16, 30_000, 3)])
def test_merge_equals_stable_sort(k, n, spread, threads):
    rng = np.random.default_rng(k * 1000 + n + spread % 97 + threads)
    runs = _runs(rng, k, n, spread)
    np.testing.assert_array_equal(_merge(runs, threads), _expected(runs))


def test_merge_empty_and_negative_timestamps():
    runs = [np.zeros(0, np.int64), np.array([-5, -5, 3], np.int64), np.zeros(0, np.int64),
            np.array([-9, -5, 3, 3], np.int64)]
    np.testing.assert_array_equal(_merge(runs, 4), _expected(runs))
    assert len(_merge([np.zeros(0, np.int64)] * 3, 2)) == 0


def test_merge_parallel_cuts_inside_a_tie():
    """one timestamp everywhere: every parallel cut falls inside the tie, which must stay in (run, index) order"""
    runs = [np.full(70_000, 42, np.int64) for _ in range(4)]
    np.testing.assert_array_equal(_merge(runs, 8), _expected(runs))
