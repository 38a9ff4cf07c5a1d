"""ShardedEngine (tests/sharded_model.py, a Python model of csrc/sg_sharded.cpp): one engine per device, keys sharded by key % N, matches merged
back into the single engine's order.  CPU: N oracle engines against one oracle engine on the same
streams (two-state, count, SEQUENCE, absent with playback timers, purge, snapshot/restore), bit-exact;
the same through the runtime API.  The device version is in test_gpu_sharded.py."""
import importlib

import numpy as np
import pytest

from oracle_backend import build_oracle
from test_purge import SHAPES as PSHAPES
from sharded_model import ShardedEngine

sa = importlib.import_module("siddhi-1_amd")
synth = importlib.import_module("siddhi-1_amd.synth")

STOCK = "define stream S (symbol string, price float, volume int);\n"
SHAPES = dict(PSHAPES)
SHAPES["absent_playback"] = ("@app:playback " + STOCK + "partition with (symbol of S) begin from every e1=S[price>20] "
                             "-> not S[price>e1.price] for 30 milliseconds within 60 milliseconds "
                             "select e1.price as a insert into O; end;")


def same(a, b):
    assert len(a) == len(b), (len(a), len(b))
    for f in ("trigger_seq", "key", "ts", "chain_len"):
        assert np.array_equal(getattr(a, f), getattr(b, f)), f
    w = min(a.slot_seq.shape[2], b.slot_seq.shape[2])
    assert np.array_equal(a.slot_seq[:, :, :w], b.slot_seq[:, :, :w])


def run_property(shape, lib, prefix, devices, cabi=False):
    """cabi: the sharded engine is the C-ABI's own fan-out (sg_config.n_devices, one handle), else the Python
    ShardedEngine over N engines"""
    app = sa.parse_app(SHAPES[shape])
    cq = sa.compile_query(app, app.queries[0], sa.StringDictionary())
    K = 300
    mk = lambda: sa.NativeEngine(lib, prefix, cq.ir, n_keys=K, max_batch=1 << 14, partial_capacity=64,
                                 match_capacity=1 << 20)
    one = mk()

    def mk_sharded():
        if cabi:
            return sa.NativeEngine(lib, prefix, cq.ir, n_keys=K, max_batch=1 << 14, partial_capacity=64,
                                   match_capacity=1 << 20, devices=devices)
        return ShardedEngine(lib, prefix, cq.ir, n_keys=K, devices=devices, max_batch=1 << 14,
                                partial_capacity=64, match_capacity=1 << 20)
    shd = mk_sharded()
    playback = "playback" in SHAPES[shape]
    seq, total = 0, 0
    for b in range(4):
        d = synth.stock_ticks(seq, 5000, K, seed=70 + b, rate_per_ms=4)
        if playback:   # one key per millisecond: distinct timer due times
            d = synth.burst_ticks(seq, 5000, K, 1, t0=1_000_000)
        for e in (one, shd):
            if playback:
                e.advance_time(int(d["ts"][-1]))
        if playback:
            ma, mb = one.poll(), shd.poll()
            same(ma, mb)
            total += len(ma)
        if b == 2:   # purge a third of the keys, snapshot and restore the sharded engine
            ids = np.arange(0, K, 3, dtype=np.uint32)
            for e in (one, shd):
                e.reset_keys(ids)
            if hasattr(lib, prefix + "snapshot"):   # (the oracle has no snapshot)
                img = shd.snapshot()
                shd.close()
                shd = mk_sharded()
                shd.restore(img)
        for e in (one, shd):
            e.push(0, seq, d["ts"], [d["symbol"], d["price"], d["volume"]], None, d["key"])
        ma, mb = one.poll(), shd.poll()
        same(ma, mb)
        total += len(ma)
        seq += 5000
    assert total > 0
    so, ss = one.stats(), shd.stats()
    assert so["partials_live"] == ss["partials_live"]
    if not hasattr(lib, prefix + "snapshot"):   # (a restored engine's counters start afresh)
        assert so["matches"] == ss["matches"]
    one.close()
    shd.close()


@pytest.mark.parametrize("shape", sorted(SHAPES))
def test_sharded_oracle_equals_single(shape):
    run_property(shape, build_oracle(), "sgo_", devices=(0, 0, 0))


def test_sharded_runtime_api():
    from oracle_backend import build_oracle as bo
    lib = bo()
    app = (STOCK + "partition with (symbol of S) begin @info(name='q') from every e1=S[price>20] -> "
           "e2=S[price>e1.price] within 1 sec select e1.symbol as s, e1.price as p1, e2.price as p2 "
           "insert into O; end;")

    def run(factory):
        rt = sa.SiddhiAppRuntime(app, factory, n_keys=64)
        got = []
        rt.addCallback("O", lambda evs: got.append([tuple(e.data) for e in evs]))
        rt.start()
        h = rt.getInputHandler("S")
        rng = np.random.default_rng(4)
        for i in range(400):
            h.send(sa.Event(1000 + i, [f"K{int(rng.integers(0, 20))}", float(np.float32(10 + 30 * rng.random())), 1]))
        rt.shutdown()
        return got

    single = run(lambda ir, nk: sa.NativeEngine(lib, "sgo_", ir, n_keys=nk, max_batch=64))
    sharded = run(lambda ir, nk: ShardedEngine(lib, "sgo_", ir, n_keys=nk, devices=(0, 0, 0, 0), max_batch=64))
    assert single == sharded and len(single) > 10
