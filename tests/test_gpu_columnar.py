"""The columnar host API on the HIP engine with the select list projected on the device: send_columns +
ColumnarQueryCallback give the rows send(Event[]) + QueryCallback give (STRING, float, int items, `having`,
dictionary-encoded symbols)."""
import importlib

import numpy as np
import pytest

from test_columnar_api import C2, STOCK, CatCols, Cols, Rows, _norm

sa = importlib.import_module("siddhi-1_amd")
synth = importlib.import_module("siddhi-1_amd.synth")

pytestmark = pytest.mark.gpu

HAVING = STOCK + ("partition with (symbol of S) begin @info(name = 'q') from every e1=S[price>20] -> "
                  "e2=S[price>e1.price] within 1 sec select e1.symbol as sym, e2.price - e1.price as d "
                  "having d > 2.5 insert into O; end;")


@pytest.mark.parametrize("app", [C2, HAVING], ids=["c2", "having"])
@pytest.mark.parametrize("categorical,out_cat", [(False, False), (True, False), (True, True)])
def test_gpu_columnar_equals_rows(app, categorical, out_cat):
    pd = pytest.importorskip("pandas") if categorical else None
    n_keys, n = 4096, 50000
    out = {}
    for columnar in (False, True):
        rt = sa.SiddhiManager(n_keys=n_keys, max_batch=n).createSiddhiAppRuntime(app)
        assert rt.queries[0].device_projection
        cb = (CatCols() if out_cat else Cols()) if columnar else Rows()
        rt.addCallback("q", cb)
        rt.start()
        h = rt.getInputHandler("S")
        cats = pd.Index([f"K{k}" for k in range(n_keys)]) if categorical else None
        for b in range(3):
            d = synth.stock_ticks(b * n, n, n_keys, seed=90 + b, rate_per_ms=16)
            names = [f"K{k}" for k in d["key"].tolist()]
            if columnar:
                sym = pd.Categorical.from_codes(d["key"].astype(np.int64), categories=cats) if categorical \
                    else np.array(names)
                h.send_columns(d["ts"], [sym, d["price"], d["volume"]])
            else:
                h.send([sa.Event(t, [s, p, v]) for t, s, p, v in
                        zip(d["ts"].tolist(), names, d["price"].tolist(), d["volume"].tolist())])
        rt.shutdown()
        out[columnar] = cb.rows
    assert len(out[False]) > 0
    assert _norm(out[True]) == _norm(out[False])


def test_gpu_categorical_string_output_nulls():
    """string_columns = "categorical" on the device projection: null STRING items as code -1, the
    values the object-array callback gets beside it"""
    pytest.importorskip("pandas")
    app = ("define stream S (symbol string, price float, venue string);\n"
           "partition with (symbol of S) begin @info(name = 'q') from every e1=S[price>20] -> "
           "e2=S[price>e1.price] within 1 sec select e1.symbol as sym, e2.venue as venue, "
           "e2.price - e1.price as d insert into O; end;")
    rt = sa.SiddhiManager(n_keys=64, max_batch=4096).createSiddhiAppRuntime(app)
    assert rt.queries[0].device_projection
    obj, cat = Cols(), CatCols()
    rt.addCallback("q", obj)
    rt.addCallback("q", cat)
    rt.start()
    h = rt.getInputHandler("S")
    for b in range(3):
        d = synth.stock_ticks(b * 4000, 4000, 23, seed=60 + b, rate_per_ms=4)
        sym = np.array([f"K{k}" for k in d["key"].tolist()])
        venue = np.array([None if v % 7 == 0 else f"V{v % 5}" for v in d["volume"].tolist()], dtype=object)
        h.send_columns(d["ts"], [sym, d["price"], venue])
    rt.shutdown()
    assert len(obj.rows) > 0 and cat.rows == obj.rows and cat.calls == obj.calls
    assert any(r[1][1] is None for r in obj.rows) and any(r[1][1] is not None for r in obj.rows)
