"""InputHandler.send_columns / ColumnarQueryCallback (the columnar additions to the host API) against the
reference-shaped path they shortcut: the same events sent as send(Event[]) give the same callbacks,
row for row, for partitioned and unpartitioned queries, nulls, null partition keys (dropped), host-side
aggregators (not applied twice when both callback kinds listen), playback timers, the broadcast of an
unkeyed stream inside a partition and @purge (both take the row path inside)."""
import importlib

import numpy as np
import pytest

from oracle_backend import oracle_factory, oracle_manager

sa = importlib.import_module("siddhi-1_amd")
synth = importlib.import_module("siddhi-1_amd.synth")

STOCK = "define stream S (symbol string, price float, volume int);\n"
C2 = STOCK + ("partition with (symbol of S) begin @info(name = 'q') from every e1=S[price>20] -> "
              "e2=S[price>e1.price] within 1 sec select e1.symbol as sym, e1.price as p1, e2.price as p2, "
              "e2.volume - e1.volume as dv insert into O; end;")


class Rows(sa.QueryCallback):
    def __init__(self):
        self.rows = []

    def receive(self, timestamp, in_events, remove_events):
        self.rows += [(e.timestamp, tuple(e.data)) for e in in_events]


class Cols(sa.ColumnarQueryCallback):
    def __init__(self):
        self.rows = []
        self.calls = 0

    def receive_columns(self, timestamps, columns, trigger_seq):
        self.calls += 1
        names = list(columns)
        vals = []
        for nm in names:
            c = columns[nm]
            if np.ma.isMaskedArray(c):
                vals.append([None if m else x for x, m in zip(c.data.tolist(), np.ma.getmaskarray(c).tolist())])
            elif type(c).__name__ == "Categorical":   # string_columns = "categorical"
                assert self.string_columns == "categorical"
                cats = list(c.categories)
                vals.append([None if k < 0 else cats[k] for k in np.asarray(c.codes).tolist()])
            else:
                vals.append(c.tolist())
        assert len(trigger_seq) == len(timestamps)
        self.rows += list(zip(timestamps.tolist(), map(tuple, zip(*vals))))


class CatCols(Cols):
    """STRING items delivered dictionary-encoded (pandas.Categorical)"""
    string_columns = "categorical"


def _norm(rows):
    out = []
    for ts, data in rows:
        out.append((int(ts), tuple(None if v is None else (float(v) if isinstance(v, (float, np.floating)) else
                                                          (v if isinstance(v, str) else int(v))) for v in data)))
    return out


def _stream(n, n_keys, seed, nulls=False, null_keys=False):
    d = synth.stock_ticks(0, n, n_keys, seed=seed, rate_per_ms=4)
    sym = np.array([f"K{k}" for k in d["key"].tolist()])
    price = d["price"]
    events_price = price.tolist()
    mprice = price
    if nulls:
        mask = (d["volume"] % 13) == 0
        mprice = np.ma.MaskedArray(price, mask=mask)
        events_price = [None if m else p for p, m in zip(price.tolist(), mask.tolist())]
    syms = sym.tolist()
    sym_col = sym
    if null_keys:
        syms = [None if (i % 17) == 5 else s for i, s in enumerate(syms)]
        sym_col = np.array(syms, dtype=object)
    events = [sa.Event(t, [s, p, v]) for t, s, p, v in zip(d["ts"].tolist(), syms, events_price, d["volume"].tolist())]
    return d["ts"], [sym_col, mprice, d["volume"]], events


def _run(app, chunks, columnar, both=False, query="q"):
    rt = oracle_manager().createSiddhiAppRuntime(app)
    rows, cols = Rows(), Cols()
    if not columnar or both:
        rt.addCallback(query, rows)
    if columnar:
        rt.addCallback(query, cols)
    rt.start()
    h = rt.getInputHandler("S")
    for ts, colv, events in chunks:
        if columnar:
            h.send_columns(ts, colv)
        else:
            h.send(events)
    rt.shutdown()
    return rows.rows, cols.rows, cols.calls


@pytest.mark.parametrize("nulls,null_keys", [(False, False), (True, False), (False, True)])
def test_send_columns_equals_send_events(nulls, null_keys):
    chunks = [_stream(3000, 97, seed=s, nulls=nulls, null_keys=null_keys) for s in (1, 2, 3)]
    # the chunks continue one stream: shift each chunk's timestamps after the previous one's
    shift = 0
    fixed = []
    for ts, colv, events in chunks:
        ts = ts + shift
        events = [sa.Event(e.timestamp + shift, e.data) for e in events]
        shift = int(ts[-1]) + 1 - int(chunks[0][0][0])
        fixed.append((ts, colv, events))
    ref, _, _ = _run(C2, fixed, columnar=False)
    got_rows, got_cols, calls = _run(C2, fixed, columnar=True, both=True)
    assert len(ref) > 0
    assert _norm(got_rows) == _norm(ref)
    assert _norm(got_cols) == _norm(ref)
    assert calls == 3


def test_columns_as_dict_and_lists():
    ts, colv, events = _stream(2000, 31, seed=9)
    ref, _, _ = _run(C2, [(ts, colv, events)], columnar=False)
    d = {"symbol": colv[0].tolist(), "price": colv[1], "volume": colv[2]}
    _, got, _ = _run(C2, [(ts, d, events)], columnar=True)
    assert _norm(got) == _norm(ref) and len(ref) > 0


def test_host_aggregators_not_applied_twice():
    app = STOCK + ("partition with (symbol of S) begin @info(name = 'q') from every e1=S[price>20] -> "
                   "e2=S[price>e1.price] select e1.symbol as sym, count() as n, sum(e2.volume) as sv "
                   "insert into O; end;")
    chunk = _stream(2500, 13, seed=4)
    ref, _, _ = _run(app, [chunk], columnar=False)
    rows, cols, _ = _run(app, [chunk], columnar=True, both=True)
    assert len(ref) > 0 and _norm(rows) == _norm(ref) and _norm(cols) == _norm(ref)


def test_unpartitioned_and_playback_timers():
    app = ("@app:playback\n" + STOCK + "@info(name = 'q') from every e1=S[price>38] -> not S[price>e1.price] "
           "for 5 milliseconds select e1.price as p insert into O;")
    d = synth.stock_ticks(0, 400, 1, seed=5, rate_per_ms=1)
    sym = np.array(["X"] * 400)
    events = [sa.Event(t, ["X", p, v]) for t, p, v in zip(d["ts"].tolist(), d["price"].tolist(), d["volume"].tolist())]
    chunks = [(d["ts"][i:i + 100], [sym[i:i + 100], d["price"][i:i + 100], d["volume"][i:i + 100]], events[i:i + 100])
              for i in range(0, 400, 100)]
    ref, _, _ = _run(app, chunks, columnar=False)
    _, got, _ = _run(app, chunks, columnar=True)
    assert len(ref) > 0 and _norm(got) == _norm(ref)


def test_broadcast_and_purge_take_the_row_path():
    app = ("define stream S (symbol string, price float, volume int);\n"
           "define stream T (price float);\n"
           "@purge(enable='true', interval='1 sec', idle.period='1 hour')\n"
           "partition with (symbol of S) begin @info(name = 'q') from every e1=S[price>20] -> e2=T[price>e1.price] "
           "select e1.symbol as sym, e2.price as p insert into O; end;")
    rt_rows = {}
    for columnar in (False, True):
        rt = oracle_manager().createSiddhiAppRuntime(app)
        cb = Cols() if columnar else Rows()
        rt.addCallback("q", cb)
        rt.start()
        hs, ht = rt.getInputHandler("S"), rt.getInputHandler("T")
        for i in range(5):
            d = synth.stock_ticks(i * 200, 200, 11, seed=6, rate_per_ms=1)
            syms = np.array([f"K{k}" for k in d["key"].tolist()])
            if columnar:
                hs.send_columns(d["ts"], [syms, d["price"], d["volume"]])
                ht.send_columns(d["ts"][-1:] + 1, [np.array([35.0], dtype=np.float32)])
            else:
                hs.send([sa.Event(t, [s, p, v]) for t, s, p, v in
                         zip(d["ts"].tolist(), syms.tolist(), d["price"].tolist(), d["volume"].tolist())])
                ht.send([sa.Event(int(d["ts"][-1]) + 1, [35.0])])
        rt.shutdown()
        rt_rows[columnar] = cb.rows
    assert len(rt_rows[False]) > 0
    assert _norm(rt_rows[True]) == _norm(rt_rows[False])


def test_bad_columns_rejected():
    rt = oracle_manager().createSiddhiAppRuntime(C2)
    rt.start()
    h = rt.getInputHandler("S")
    with pytest.raises(ValueError):
        h.send_columns(np.arange(3), [np.array(["a", "b", "c"]), np.zeros(3, np.float32)])
    with pytest.raises(ValueError):
        h.send_columns(np.arange(3), [np.array(["a", "b"]), np.zeros(3, np.float32), np.zeros(3, np.int32)])
    rt.shutdown()


def test_categorical_columns():
    """dictionary-encoded STRING columns (pandas.Categorical): ids interned once per category set, null
    codes (-1) as null values / dropped partition keys, same callbacks as send(Event[])"""
    pd = pytest.importorskip("pandas")
    cats = pd.Index([f"K{k}" for k in range(23)])
    chunks = []
    base = 0
    for s in range(3):
        d = synth.stock_ticks(base, 1500, 23, seed=20 + s, rate_per_ms=4)
        codes = d["key"].astype(np.int64)
        codes[::41] = -1                                   # null partition key: the event is dropped
        col = pd.Categorical.from_codes(codes, categories=cats)
        syms = [None if c < 0 else f"K{c}" for c in codes.tolist()]
        events = [sa.Event(t, [k, p, v]) for t, k, p, v in
                  zip(d["ts"].tolist(), syms, d["price"].tolist(), d["volume"].tolist())]
        chunks.append((d["ts"], [col, d["price"], d["volume"]], events))
        base += 1500
    ref, _, _ = _run(C2, chunks, columnar=False)
    _, got, _ = _run(C2, chunks, columnar=True)
    assert len(ref) > 0 and _norm(got) == _norm(ref)


def test_categorical_id_maps_affine_and_gathered():
    """category sets whose ids form one contiguous run map codes with an add (from id 0, and from a later
    base once other keys hold the first ids); a reordered / overlapping set takes the gather: all three
    give send(Event[])'s callbacks"""
    pd = pytest.importorskip("pandas")
    sets = [pd.Index([f"K{k}" for k in range(23)]),                 # fresh ids 0..22: affine, base 0
            pd.Index([f"K{k}" for k in reversed(range(23))]),       # same keys reversed: gathered
            pd.Index([f"N{k}" for k in range(23)])]                 # fresh ids 23..45: affine, base 23
    chunks = []
    base = 0
    for s, cats in enumerate(sets):
        d = synth.stock_ticks(base, 1500, 23, seed=30 + s, rate_per_ms=4)
        codes = d["key"].astype(np.int64)
        col = pd.Categorical.from_codes(codes, categories=cats)
        syms = [cats[c] for c in codes.tolist()]
        events = [sa.Event(t, [k, p, v]) for t, k, p, v in
                  zip(d["ts"].tolist(), syms, d["price"].tolist(), d["volume"].tolist())]
        chunks.append((d["ts"], [col, d["price"], d["volume"]], events))
        base += 1500
    ref, _, _ = _run(C2, chunks, columnar=False)
    _, got, _ = _run(C2, chunks, columnar=True)
    assert len(ref) > 0 and _norm(got) == _norm(ref)


def test_categorical_string_output():
    """ColumnarQueryCallback.string_columns = "categorical": STRING items arrive as pandas.Categorical
    (null: code -1) with the values the object-array callback gets, beside it on the same query"""
    pytest.importorskip("pandas")
    app = ("define stream S (symbol string, price float, venue string);\n"
           "partition with (symbol of S) begin @info(name = 'q') from every e1=S[price>20] -> "
           "e2=S[price>e1.price] within 1 sec select e1.symbol as sym, e2.venue as venue, "
           "e2.price - e1.price as d insert into O; end;")
    rt = oracle_manager().createSiddhiAppRuntime(app)
    obj, cat = Cols(), CatCols()
    rt.addCallback("q", obj)
    rt.addCallback("q", cat)
    rt.start()
    h = rt.getInputHandler("S")
    for b in range(3):
        ts, colv, _ = _stream(1500, 23, seed=40 + b)
        venue = np.array([None if v % 7 == 0 else f"V{v % 5}" for v in colv[2].tolist()], dtype=object)
        h.send_columns(ts + b * 10_000, [colv[0], colv[1], venue])
    rt.shutdown()
    assert len(obj.rows) > 0 and cat.rows == obj.rows and cat.calls == obj.calls
    assert any(r[1][1] is None for r in obj.rows) and any(r[1][1] is not None for r in obj.rows)


@pytest.mark.parametrize("purge", [False, True])
def test_bytes_string_columns(purge):
    """numpy bytes ('S') STRING columns behave as the same str values sent as Event objects: the partition
    keys, a STRING attribute projected on the host (e1.symbol), and the rows the event store keeps"""
    app = C2 if not purge else ("@purge(enable='true', interval='10 sec', idle.period='1 hour')\n" + C2)
    ts, colv, events = _stream(2500, 19, seed=31)
    bcol = np.char.encode(colv[0], "utf-8")
    assert bcol.dtype.kind == "S"
    ref, _, _ = _run(app, [(ts, colv, events)], columnar=False)
    rows, cols, _ = _run(app, [(ts, [bcol, colv[1], colv[2]], events)], columnar=True, both=True)
    assert len(ref) > 0
    assert _norm(rows) == _norm(ref) and _norm(cols) == _norm(ref)
    assert all(isinstance(r[1][0], str) for r in rows)


def test_restore_drops_dictionary_derived_caches():
    """a categorical column sent after restoring an older snapshot maps its categories through the
    restored dictionaries, not through ids cached before the restore"""
    pd = pytest.importorskip("pandas")
    app = STOCK + ("partition with (symbol of S) begin @info(name = 'q') from every e1=S[price>20] -> "
                   "e2=S[price>e1.price] within 1 sec select e1.symbol as sym, e2.price as p insert into O; end;")

    def run(with_detour):
        rt = oracle_manager().createSiddhiAppRuntime(app)
        cb = Rows()
        rt.addCallback("q", cb)
        rt.start()
        h = rt.getInputHandler("S")
        # the oracle engine has no device image: the engine part of the snapshot is a fresh engine's
        # (nothing was sent before the snapshot), so only the host runtime's restore is exercised
        make = oracle_factory()
        for qr in rt.queries:
            qr.engine.snapshot = lambda: b""

            def restore(img, qr=qr):   # a fresh engine, as the image of the fresh engine would give
                qr.engine = make(qr.cq.ir, qr.n_keys)
                qr.engine.snapshot = lambda: b""
            qr.engine.restore = restore
        snap = rt.snapshot()
        cats = pd.Index([f"K{k}" for k in range(11)])
        if with_detour:   # keys interned (and their ids cached for `cats`), then thrown away by the restore
            cats0 = pd.Index([f"Z{k}" for k in range(7)])
            for c, n in ((cats0, 7), (cats, 11)):
                d = synth.stock_ticks(0, 500, n, seed=41, rate_per_ms=4)
                h.send_columns(d["ts"], [pd.Categorical.from_codes(d["key"].astype(np.int64), categories=c),
                                         d["price"], d["volume"]])
            rt.restore(snap)
            cb.rows.clear()
        # the same keys through a plain str column, then through the categorical column: both must reach
        # the keys' one set of partials
        d = synth.stock_ticks(1000, 1600, 11, seed=42, rate_per_ms=4)
        h.send_columns(d["ts"][:800] + 10_000, [np.array([f"K{k}" for k in d["key"][:800].tolist()]),
                                                d["price"][:800], d["volume"][:800]])
        h.send_columns(d["ts"][800:] + 10_000, [pd.Categorical.from_codes(d["key"][800:].astype(np.int64),
                                                                          categories=cats),
                                                d["price"][800:], d["volume"][800:]])
        rt.shutdown()
        return cb.rows

    ref = run(False)
    assert len(ref) > 0 and _norm(run(True)) == _norm(ref)
