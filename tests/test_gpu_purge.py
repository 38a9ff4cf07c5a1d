"""Partition purge on the device (sg_reset_keys) against the oracle (sgo_reset_keys), bit-exact, on
both kernels: the two-state kernel's per-key header and the general engine's state blocks (count
chains, SEQUENCE, absent-state timers).  Property as in test_purge.py: keys reset between two batches
behave exactly like keys never seen before."""
import importlib

import numpy as np
import pytest

from oracle_backend import build_oracle
from test_gpu_general import ABSENT, _burst_stream
from test_gpu_parity import _same
from test_purge import SHAPES, reset_property

sa = importlib.import_module("siddhi-1_amd")

pytestmark = pytest.mark.gpu


def _hip(ir, nk):
    return sa.NativeEngine(sa.load_hip_library(), "sg_", ir, n_keys=nk, max_batch=8192, partial_capacity=64,
                           match_capacity=1 << 20)


@pytest.mark.parametrize("shape", sorted(SHAPES))
def test_gpu_reset_equals_never_seen_and_oracle(shape):
    ma, mb = reset_property(shape, _hip)
    _same(ma, mb)
    assert len(ma) > 0
    lib = build_oracle()
    mo, _ = reset_property(shape, lambda ir, nk: sa.NativeEngine(lib, "sgo_", ir, n_keys=nk))
    _same(ma, mo)


@pytest.mark.parametrize("shape", sorted(ABSENT))
def test_gpu_reset_with_timers(shape):
    """keys reset mid-stream lose their armed absent-state timers (the schedulers' per-key state is
    cleaned too); the device and the oracle agree match for match"""
    n_keys = 64
    q = ABSENT[shape]
    app = sa.parse_app(q)
    cq = sa.compile_query(app, app.queries[0], sa.StringDictionary())
    gpu = sa.NativeEngine(sa.load_hip_library(), "sg_", cq.ir, n_keys=n_keys, max_batch=4096, partial_capacity=48,
                          match_capacity=1 << 20)
    ora = sa.NativeEngine(build_oracle(), "sgo_", cq.ir, n_keys=n_keys)
    d = _burst_stream(1200, n_keys, seed=13)
    ts = d["ts"]
    bounds = np.concatenate([[0], np.nonzero(np.diff(ts))[0] + 1, [len(ts)]])
    two = "S1" in q
    for e in (gpu, ora):
        e.advance_time(int(ts[0]) - 5)
    _same(gpu.poll(), ora.poll())
    rng = np.random.default_rng(3)
    total = 0
    for i in range(len(bounds) - 1):
        lo, hi = int(bounds[i]), int(bounds[i + 1])
        for e in (gpu, ora):
            e.advance_time(int(ts[lo]))
        mg = gpu.poll()
        _same(mg, ora.poll())
        total += len(mg)
        if i % 97 == 50:
            keys = rng.choice(n_keys, 16, replace=False).astype(np.uint32)
            for e in (gpu, ora):
                e.reset_keys(keys)
        stream = (cq.stream_index("S1") if (i % 3) else cq.stream_index("S2")) if two else 0
        sl = slice(lo, hi)
        for e in (gpu, ora):
            e.push(stream, lo, ts[sl], [d["symbol"][sl], d["price"][sl], d["volume"][sl]], None, d["key"][sl])
        mg = gpu.poll()
        _same(mg, ora.poll())
        total += len(mg)
    for e in (gpu, ora):
        e.advance_time(int(ts[-1]) + 1000)
    mg = gpu.poll()
    _same(mg, ora.poll())
    assert total + len(mg) > 0
    assert gpu.stats()["partials_live"] == ora.stats()["partials_live"]


def test_gpu_reset_key_range():
    q = SHAPES["two_state"]
    app = sa.parse_app(q)
    cq = sa.compile_query(app, app.queries[0], sa.StringDictionary())
    e = _hip(cq.ir, 16)
    with pytest.raises(sa.EngineError) as ex:
        e.reset_keys(np.array([3, 16], dtype=np.uint32))
    assert ex.value.code == -1
    e.reset_keys(np.array([], dtype=np.uint32))
