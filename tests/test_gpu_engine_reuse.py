"""Engines created one after another in one process (the bench, the runtime's re-created apps, the test
suite): a new engine's device memory may be the freed memory of the previous one, so its zeroed state must
be in place, in stream order, before its first batch runs.  Regression: the general engine zeroed its
state blocks with a null-stream memset that its non-blocking stream did not wait for; the second engine
of a 2^20-key C3_min1 run read the first one's stale state and its batch kernel never finished."""
import importlib

import numpy as np
import pytest

from test_gpu_parity import _same

sa = importlib.import_module("siddhi-1_amd")
synth = importlib.import_module("siddhi-1_amd.synth")

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("query,cap", [("C3_MIN1_QUERY", 8), ("C2_QUERY", 64)])
def test_second_engine_starts_from_zeroed_state(query, cap):
    K, B = 1 << 20, 1 << 22
    app = sa.parse_app(getattr(synth, query))
    cq = sa.compile_query(app, app.queries[0], sa.StringDictionary())
    data = [synth.stock_ticks(b * B, B, K, seed=31 + b) for b in range(2)]
    runs = []
    for _ in range(2):
        e = sa.NativeEngine(sa.load_hip_library(), "sg_", cq.ir, n_keys=K, max_batch=B, partial_capacity=cap,
                            match_capacity=2 * B)
        out = []
        for b, d in enumerate(data):
            e.push(0, b * B, d["ts"], [d["symbol"], d["price"], d["volume"]], None, d["key"])
            out.append(e.poll())
        runs.append(out)
        e.close()
    assert sum(len(m) for m in runs[0]) > 0
    for x, y in zip(*runs):
        _same(x, y)


def test_partial_capacity_below_register_window():
    """partial_capacity below the two-state kernel's register window (12 slots): the window is clamped to
    the capacity, so a key that outgrows it spills into its slab in bounds and the engine reports
    SG_ERR_CAPACITY (an earlier build wrote the whole window past the slab: an illegal address)"""
    K, B = 4096, 1 << 16
    app = sa.parse_app(synth.C2_QUERY)
    cq = sa.compile_query(app, app.queries[0], sa.StringDictionary())
    d = synth.stock_ticks(0, B, K, seed=5, rate_per_ms=64)
    e = sa.NativeEngine(sa.load_hip_library(), "sg_", cq.ir, n_keys=K, max_batch=B, partial_capacity=4,
                        match_capacity=1 << 20)
    with pytest.raises(sa.EngineError) as ex:
        e.push(0, 0, d["ts"], [d["symbol"], d["price"], d["volume"]], None, d["key"])
        e.poll()
    assert ex.value.code == -4   # SG_ERR_CAPACITY
