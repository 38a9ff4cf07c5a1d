"""On-device projection of the select list (QuerySelector.processNoGroupBy,
QuerySelector.java:162-206) against the host projection of the same matches, bit-exact: the C2 select
(e1.symbol, e1.price, e2.price, e2.price - e1.price: float32 without FMA), the two-stream shape (e1 of
another stream: its attributes travel as captures), arithmetic with nulls and /0, count / SEQUENCE /
absent shapes on the general kernel.  The reference KATs (test_gpu_kat) check the device projection
against the reference's own expected rows."""
import importlib

import numpy as np
import pytest

sa = importlib.import_module("siddhi-1_amd")
cp = importlib.import_module("siddhi-1_amd.compiler")
synth = importlib.import_module("siddhi-1_amd.synth")

pytestmark = pytest.mark.gpu

STOCK = "define stream S (symbol string, price float, volume int);\n"
APPS = {
    "c2": synth.C2_QUERY.replace("@info(name = 'query1')", "@info(name = 'query1')"),
    "two_streams": ("define stream S1 (symbol string, price float, volume int);\n"
                    "define stream S2 (symbol string, price double, volume long);\n"
                    "partition with (symbol of S1, symbol of S2) begin @info(name='query1') "
                    "from every e1=S1[price>20] -> e2=S2[price>e1.price] within 1 sec "
                    "select e1.symbol as s, e1.volume as v1, e2.volume - e1.volume as dv, e2.price * e1.price as pp "
                    "insert into O; end;"),
    "arith_nulls": (STOCK + "partition with (symbol of S) begin @info(name='query1') "
                    "from every e1=S[price>25] -> e2=S[price>e1.price] within 1 sec "
                    "select e2.volume / (e1.volume % 3) as q, e1.price / (e2.price - e2.price) as z, "
                    "e2.volume is null as nv, ifThenElse(e1.volume > 1000, e1.price, e2.price) as pick, "
                    "e1.volume * 1L + 7 as l insert into O; end;"),
    "count": (STOCK + "partition with (symbol of S) begin @info(name='query1') "
              "from every e1=S[price>20]<2:5> -> e2=S[price>e1[last].price] within 1 sec "
              "select e1[0].price as p0, e1[last].price as pl, e1[1].volume as v1, e2.price - e1[0].price as d "
              "insert into O; end;"),
    "sequence": (STOCK + "partition with (symbol of S) begin @info(name='query1') "
                 "from every e1=S[price>20], e2=S[price>e1.price] select e1.symbol as s, e2.price - e1.price as d "
                 "insert into O; end;"),
    "absent": ("@app:playback " + STOCK + "partition with (symbol of S) begin @info(name='query1') "
               "from every e1=S[price>20] -> not S[price>e1.price] for 30 milliseconds "
               "select e1.symbol as s, e1.price * 2.0 as p2 insert into O; end;"),
}


def run(app, device_projection, n_keys=512, n=6000, nb=3, nulls=False):
    lib = sa.load_hip_library()

    def factory(ir, nk):
        return sa.NativeEngine(lib, "sg_", ir, n_keys=nk, max_batch=1 << 14, partial_capacity=64,
                               match_capacity=1 << 20)

    if not device_projection:
        saved = cp.projection_program
        cp.projection_program = lambda *a: None
    try:
        rt = sa.SiddhiAppRuntime(app, factory, n_keys=n_keys)
    finally:
        if not device_projection:
            cp.projection_program = saved
    assert all(q.device_projection == device_projection for q in rt.queries)
    got = []
    rt.addCallback("query1", lambda ts, cur, exp: got.extend((e.timestamp, tuple(e.data)) for e in cur or []))
    rt.start()
    streams = list(rt.app.streams)
    rng = np.random.default_rng(5)
    seq = 0
    for b in range(nb):
        if "playback" in app:
            d = synth.burst_ticks(seq, n, n_keys, 1, t0=1_000_000)
        else:
            d = synth.stock_ticks(seq, n, n_keys, seed=90 + b, rate_per_ms=8)
        for s in streams:
            evs = []
            for i in range(n):
                if len(streams) > 1 and (i % 2) != streams.index(s):
                    continue
                vol = int(d["volume"][i])
                price = float(d["price"][i])
                if nulls and rng.random() < 0.05:
                    vol = None
                evs.append(sa.Event(int(d["ts"][i]), [f"K{int(d['key'][i])}", price, vol]))
            rt.getInputHandler(s).send(evs)
        seq += n
    rt.shutdown()
    return got


def bits(rows):
    out = []
    for ts, data in rows:
        out.append((ts, tuple(("f", np.float32(x).view(np.uint32).item()) if isinstance(x, np.float32) else
                              ("d", np.float64(x).view(np.uint64).item()) if isinstance(x, float) else x
                              for x in data)))
    return out


@pytest.mark.parametrize("name", sorted(APPS))
def test_device_projection_equals_host(name):
    app = APPS[name]
    dev = run(app, True, nulls=(name == "arith_nulls"))
    host = run(app, False, nulls=(name == "arith_nulls"))
    assert len(dev) == len(host) and len(dev) > 0
    assert bits(dev) == bits(host)
