"""The hot-key pipeline (p2_jit.hip k_hot_*: a key with far more events than its batch's average has its partials
advanced all at once instead of by one lane) against the oracle, bit-exact, with the exact work counters.

Zipf(s=1.1) partition keys (the head keys thousands of events per batch), one key holding half the stream, an
unpartitioned query (the single key is the whole batch), the register window forced small and the LDS region
forced small (the staged pass hands the hot keys over from every path: LDS-split tiles, tiles split in HBM,
workgroups left whole to the HBM pass), projections of e1's captures (their raw slots filled by the pipeline),
and the runs the pipeline gives back to the HBM pass: timestamps out of order inside a hot key's run, a batch
older than the partials carried in.  Reference: StreamPreStateProcessor.java:118-129 / :308-403 and
PatternMultiProcessStreamReceiver.java:31-51 (the walk the pipeline decomposes)."""
import importlib

import numpy as np
import pytest

from test_gpu_parity import SHAPES, _same

sa = importlib.import_module("siddhi-1_amd")
synth = importlib.import_module("siddhi-1_amd.synth")
native = importlib.import_module("siddhi-1_amd.native")

pytestmark = pytest.mark.gpu

COLS = ["symbol", "price", "volume"]
STATS = ("partials_live", "partials_created", "partials_scanned", "matches", "keys_touched", "live_at_batch_start")
UNPART = ("define stream S (symbol string, price float, volume int);\n"
          "from every e1=S[price>20] -> e2=S[price>e1.price] within 1 sec select e1.price as a insert into O;")


def _pair(query, n_keys, n, cap=256):
    """the engine under test, the oracle, and a lane-walk engine (SG_HOT_MIN=0) for the work counters the oracle
    does not keep"""
    import os
    from test_gpu_parity import build_oracle
    app = sa.parse_app(query)
    cq = sa.compile_query(app, app.queries[0], sa.StringDictionary())

    def mk():
        return sa.NativeEngine(sa.load_hip_library(), "sg_", cq.ir, n_keys=n_keys, max_batch=n, partial_capacity=cap,
                               match_capacity=1 << 22)
    gpu = mk()
    saved = os.environ.get("SG_HOT_MIN")
    os.environ["SG_HOT_MIN"] = "0"
    try:
        lane = mk()
    finally:
        if saved is None:
            os.environ.pop("SG_HOT_MIN")
        else:
            os.environ["SG_HOT_MIN"] = saved
    ora = sa.NativeEngine(build_oracle(), "sgo_", cq.ir, n_keys=n_keys)
    return cq, gpu, ora, lane


def _zipf(seq, n, n_keys, seed, rate):
    d = synth.zipf_ticks(seq, n, n_keys, seed=seed, rate_per_ms=rate)
    return d


def _run(gpu, ora, lane, batches, keyed=True):
    for seq, d in batches:
        for e in (gpu, ora, lane):
            e.push(0, seq, d["ts"], [d[c] for c in COLS], None, d["key"] if keyed else None)
        mg = gpu.poll()
        _same(mg, ora.poll())
        _same(mg, lane.poll())
    sg, so, sl = gpu.stats(), ora.stats(), lane.stats()
    for f in ("partials_live", "matches"):
        assert sg[f] == so[f], (f, sg[f], so[f])
    for f in STATS:
        assert sg[f] == sl[f], (f, sg[f], sl[f])
    assert "k_hot_prep" not in lane.describe()
    return sg


@pytest.mark.parametrize("shape", ["c2_every_within", "every_no_within", "int_long_double", "arith_null_div"])
def test_hot_zipf_keys_bit_exact(shape, monkeypatch):
    monkeypatch.setenv("SG_HOT_MIN", "64")
    n_keys, n = 1 << 14, 1 << 16
    cq, gpu, ora, lane = _pair(SHAPES[shape], n_keys, n)
    batches = [(b * n, _zipf(b * n, n, n_keys, 40 + b, 64)) for b in range(3)]
    sg = _run(gpu, ora, lane, batches)
    assert sg["matches"] > 0
    assert "k_hot_prep" in gpu.describe(), gpu.describe()
    for e in (gpu, ora, lane):
        e.close()


@pytest.mark.parametrize("env", [{"SGD_REG_SLOTS": "2"}, {"SGD_STAGE_CHUNKS": "64"}, {"SG_NO_FUSED": "1"}])
def test_hot_keys_from_every_staged_path(env, monkeypatch):
    """hot keys handed over from the LDS-split tiles, from tiles split in HBM (LDS region forced small), from the
    sorted grouping's workgroups left whole to the HBM pass, with the register window stopping most other keys"""
    monkeypatch.setenv("SG_HOT_MIN", "64")
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    n_keys, n = 1 << 14, 1 << 16
    cq, gpu, ora, lane = _pair(SHAPES["c2_every_within"], n_keys, n)
    batches = [(b * n, _zipf(b * n, n, n_keys, 50 + b, 64)) for b in range(3)]
    _run(gpu, ora, lane, batches)
    for e in (gpu, ora, lane):
        e.close()


def test_hot_one_key_half_the_stream(monkeypatch):
    """one key with half of every batch (~32K events), carried-in partials across 4 batches, the hottest key's
    matches compared on their own as well"""
    monkeypatch.setenv("SG_HOT_MIN", "256")
    n_keys, n = 4096, 1 << 16
    cq, gpu, ora, lane = _pair(SHAPES["c2_every_within"], n_keys, n)
    rng = np.random.default_rng(3)
    batches = []
    for b in range(4):
        d = synth.stock_ticks(b * n, n, n_keys, seed=60 + b, rate_per_ms=32)
        d["key"][rng.random(n) < 0.5] = 1234
        d["symbol"] = d["key"].copy()
        batches.append((b * n, d))
    hot = 0
    for seq, d in batches:
        for e in (gpu, ora, lane):
            e.push(0, seq, d["ts"], [d[c] for c in COLS], None, d["key"])
        mg, mo = gpu.poll(), ora.poll()
        _same(mg, mo)
        _same(mg, lane.poll())
        sel = mg.key == 1234
        hot += int(sel.sum())
        assert np.array_equal(mg.trigger_seq[sel], mo.trigger_seq[mo.key == 1234])
    assert hot > 1000
    for f in STATS:
        assert gpu.stats()[f] == lane.stats()[f], f
    for e in (gpu, ora, lane):
        e.close()


def test_hot_unpartitioned_query(monkeypatch):
    """no partition: the single key's run is the whole batch"""
    monkeypatch.setenv("SG_HOT_MIN", "256")
    n = 1 << 15
    cq, gpu, ora, lane = _pair(UNPART, 1, n)
    batches = [(b * n, synth.stock_ticks(b * n, n, 1, seed=70 + b, rate_per_ms=16)) for b in range(3)]
    sg = _run(gpu, ora, lane, batches, keyed=False)
    assert sg["matches"] > 1000
    assert "k_hot_prep" in gpu.describe()
    for e in (gpu, ora, lane):
        e.close()


def test_hot_runs_given_back_to_the_hbm_pass(monkeypatch):
    """a hot key whose timestamps go backwards inside the batch, and a batch whose timestamps precede the partials
    carried in: the pipeline leaves them to the HBM pass, still exact"""
    monkeypatch.setenv("SG_HOT_MIN", "64")
    n_keys, n = 1 << 12, 1 << 15
    cq, gpu, ora, lane = _pair(SHAPES["c2_every_within"], n_keys, n)
    batches = []
    for b in range(4):
        d = _zipf(b * n, n, n_keys, 80 + b, 64)
        if b == 1:  # out of order inside the batch
            sw = np.arange(0, n - 1, 97)
            d["ts"][sw], d["ts"][sw + 1] = d["ts"][sw + 1].copy(), d["ts"][sw].copy()
        if b == 3:  # older than the partials carried in from batch 2
            d["ts"] = d["ts"] - 200
        batches.append((b * n, d))
    _run(gpu, ora, lane, batches)
    for e in (gpu, ora, lane):
        e.close()


def test_hot_keys_with_projection(monkeypatch):
    """device projection of e1's captures and e2's attributes: the pipeline's raw slots carry the captures"""
    monkeypatch.setenv("SG_HOT_MIN", "64")
    app = ("define stream S (symbol string, price float, volume int);\n"
           "partition with (symbol of S) begin @info(name='query1') "
           "from every e1=S[price>20] -> e2=S[price>e1.price] within 1 sec "
           "select e1.symbol as s, e1.price as p1, e1.volume as v1, e2.price - e1.price as d insert into O; end;")
    lib = sa.load_hip_library()
    cp = importlib.import_module("siddhi-1_amd.compiler")

    def run(device):
        rt_factory = (lambda ir, nk: sa.NativeEngine(lib, "sg_", ir, n_keys=nk, max_batch=1 << 14,
                                                     partial_capacity=256, match_capacity=1 << 20))
        saved = cp.projection_program
        if not device:
            cp.projection_program = lambda *a: None
        try:
            rt = sa.SiddhiAppRuntime(app, rt_factory, n_keys=256)
        finally:
            cp.projection_program = saved
        got = []
        rt.addCallback("query1", lambda ts, cur, exp: got.extend((e.timestamp, tuple(e.data)) for e in cur or []))
        rt.start()
        h = rt.getInputHandler("S")
        n = 8000
        for b in range(3):
            d = synth.zipf_ticks(b * n, n, 256, seed=90 + b, rate_per_ms=16)
            h.send([sa.Event(int(d["ts"][i]), [f"K{int(d['key'][i])}", float(d["price"][i]), int(d["volume"][i])])
                    for i in range(n)])
        rt.shutdown()
        return got

    dev, host = run(True), run(False)
    assert len(dev) == len(host) and len(dev) > 0
    assert [(t, tuple(np.float32(x).view(np.uint32).item() if isinstance(x, np.float32) else x for x in r))
            for t, r in dev] == [(t, tuple(np.float32(x).view(np.uint32).item() if isinstance(x, np.float32) else x
                                           for x in r)) for t, r in host]


def test_giant_tiles_switch_to_the_sorted_grouping(monkeypatch):
    """a key with 70 % of 2^17-event batches: its tile (> SGD_BIG_TILE events) would be split by one workgroup in
    the fused grouping; once a batch reports it, the engine groups the next batches with the sorted passes (the
    hot key still to the pipeline), exact throughout"""
    monkeypatch.setenv("SG_HOT_MIN", "256")
    n_keys, n = 1 << 14, 1 << 17
    cq, gpu, ora, lane = _pair(SHAPES["c2_every_within"], n_keys, n)
    rng = np.random.default_rng(9)
    batches = []
    for b in range(5):
        d = synth.stock_ticks(b * n, n, n_keys, seed=110 + b, rate_per_ms=64)
        d["key"][rng.random(n) < 0.7] = 4321
        d["symbol"] = d["key"].copy()
        batches.append((b * n, d))
    _run(gpu, ora, lane, batches)
    desc = gpu.describe()
    assert "per 8-bit digit" in desc and "k_hot_prep" in desc, desc
    for e in (gpu, ora, lane):
        e.close()


def test_hot_many_survivors(monkeypatch):
    """a hot key whose partials only expire (f1 never holds): ~160 live at every batch end, more than one wave of
    survivors (k_hot_final_big orders them), carried across batches"""
    monkeypatch.setenv("SG_HOT_MIN", "64")
    q = ("define stream S (symbol string, price float, volume int);\n"
         "partition with (symbol of S) begin from every e1=S[price>10] -> e2=S[price>e1.price + 100.0] "
         "within 200 milliseconds select e1.price as a insert into O; end;")
    n_keys, n = 4096, 1 << 16
    cq, gpu, ora, lane = _pair(q, n_keys, n)
    rng = np.random.default_rng(21)
    batches = []
    for b in range(3):
        d = synth.stock_ticks(b * n, n, n_keys, seed=130 + b, rate_per_ms=16)
        d["key"][rng.random(n) < 0.05] = 77
        d["symbol"] = d["key"].copy()
        batches.append((b * n, d))
    sg = _run(gpu, ora, lane, batches)
    assert sg["partials_live"] > 64
    for e in (gpu, ora, lane):
        e.close()


@pytest.mark.slow
@pytest.mark.parametrize("kind", ["zipf", "walk"])
def test_c2_variants_at_bench_size_key_subset(kind):
    """the bench's C2 variants at their size (2^20 keys, two 2^24-event batches): Zipf(s=1.1) keys — key 0 is the
    hottest (~12 % of every batch, to the hot-key pipeline) and is in the subset — and per-key random-walk prices
    (longer-lived partials, register-window spills).  Oracle on keys % 64 == 0 with the same arrival seqs, plus
    size-independent properties of every match."""
    from test_gpu_parity import _engines
    n_keys, batch, mod = 1 << 20, 1 << 24, 64
    cq, gpu, ora = _engines(synth.C2_QUERY, n_keys, batch, cap=256, mcap=1 << 24)
    walk = synth.RandomWalk(n_keys) if kind == "walk" else None
    seq, hot = 0, 0
    for b in range(2):
        if kind == "zipf":
            d = synth.zipf_ticks(seq, batch, n_keys)
        else:
            d = synth.stock_ticks(seq, batch, n_keys)
            d["price"] = walk.step(d["key"], seq)
        gpu.push(0, seq, d["ts"], [d[c] for c in COLS], None, d["key"])
        mg = gpu.poll()
        idx = np.nonzero((d["key"] % mod) == 0)[0]
        starts = np.concatenate([[0], np.nonzero(np.diff(idx) != 1)[0] + 1])
        ends = np.concatenate([starts[1:], [len(idx)]])
        for s, t in zip(starts, ends):
            sl = idx[s:t]
            ora.push(0, seq + int(sl[0]), d["ts"][sl], [d[c][sl] for c in COLS], None, d["key"][sl])
        mo = ora.poll()
        keep = (mg.key % mod) == 0
        assert int(keep.sum()) == len(mo) and len(mo) > 0
        assert np.array_equal(mg.trigger_seq[keep], mo.trigger_seq)
        assert np.array_equal(mg.slot_seq[keep], mo.slot_seq)
        hot += int((mg.key == 0).sum())
        trig = mg.trigger_seq.astype(np.int64) - seq
        e1 = mg.slot_seq[:, 0, 0].astype(np.int64)
        assert np.all(np.diff(mg.trigger_seq.astype(np.int64)) >= 0)
        assert np.all(e1 < mg.trigger_seq.astype(np.int64))
        cur = e1 >= seq
        p1, p2 = d["price"][e1[cur] - seq], d["price"][trig[cur]]
        assert np.all(p1 > 20) and np.all(p2 > p1)
        assert np.all(d["key"][trig] == mg.key)
        seq += batch
    st = gpu.stats()
    if kind == "zipf":
        assert hot > 1000 and st["hot_keys"] > 0 and "k_hot_prep" in gpu.describe()
    gpu.close()
    ora.close()


@pytest.mark.parametrize("exmax", ["48", "400"])
def test_hot_partials_given_back_above_exmax(exmax, monkeypatch):
    """several hot keys carrying ~160 live partials each into every batch, with the pipeline's flat index space for
    carried-in partials (hot_exmax, SG_HOT_EXMAX) smaller than their sum: k_hot_scan's second pass gives the keys
    past the limit back to the HBM pass (p2_jit.hip hot_scan_pass), still exact against the oracle and the lane walk"""
    monkeypatch.setenv("SG_HOT_MIN", "64")
    monkeypatch.setenv("SG_HOT_EXMAX", exmax)
    q = ("define stream S (symbol string, price float, volume int);\n"
         "partition with (symbol of S) begin from every e1=S[price>10] -> e2=S[price>e1.price + 100.0] "
         "within 200 milliseconds select e1.price as a insert into O; end;")
    n_keys, n = 4096, 1 << 16
    cq, gpu, ora, lane = _pair(q, n_keys, n)
    rng = np.random.default_rng(31)
    batches = []
    for b in range(4):
        d = synth.stock_ticks(b * n, n, n_keys, seed=150 + b, rate_per_ms=16)
        u = rng.random(n)
        for i, k in enumerate((77, 78, 79, 80, 81)):
            d["key"][(u >= 0.04 * i) & (u < 0.04 * (i + 1))] = k
        d["symbol"] = d["key"].copy()
        batches.append((b * n, d))
    sg = _run(gpu, ora, lane, batches)
    assert sg["partials_live"] > 5 * 64
    assert "k_hot_prep" in gpu.describe()
    for e in (gpu, ora, lane):
        e.close()


def test_hot_pipeline_from_the_first_batch_and_buffers_given_back(monkeypatch):
    """the first batch an engine sees runs the hot-key pipeline (a Zipf head key left to one HBM-pass lane is
    quadratic in its run), and after SGD_HOT_IDLE (8) batches in a row without a hot key the pipeline's buffers
    are freed (stream-ordered: the device pool's used bytes fall back); a later hot batch allocates them again,
    bit-exact with the oracle throughout"""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")

    def pool_used():   # the pipeline's buffers are stream-ordered allocations from the device's default pool
        pool, v = ctypes.c_void_p(), ctypes.c_uint64()
        assert hip.hipDeviceGetDefaultMemPool(ctypes.byref(pool), 0) == 0
        assert hip.hipMemPoolGetAttribute(pool, 0x7, ctypes.byref(v)) == 0   # hipMemPoolAttrUsedMemCurrent
        return v.value

    monkeypatch.setenv("SG_HOT_MIN", "64")
    n_keys, n = 1 << 14, 1 << 18
    cq, gpu, ora, lane = _pair(SHAPES["c2_every_within"], n_keys, n)
    seq = 0

    def push(d):
        nonlocal seq
        for e in (gpu, ora, lane):
            e.push(0, seq, d["ts"], [d[c] for c in COLS], None, d["key"])
        mg = gpu.poll()
        _same(mg, ora.poll())
        _same(mg, lane.poll())
        seq += len(d["ts"])

    gpu.synchronize()
    used0 = pool_used()
    push(_zipf(seq, n, n_keys, 70, 64))
    assert gpu.stats()["hot_keys"] > 0, "the first batch did not run the pipeline"
    used_hot = pool_used()
    assert used_hot - used0 > 20 << 20, (used0, used_hot)   # B + hot_exmax slots x 40 B + 3 x B words
    for b in range(10):
        push(synth.stock_ticks(seq, 1 << 14, n_keys, seed=80 + b, rate_per_ms=64))
    gpu.synchronize()
    used_idle = pool_used()
    assert used_hot - used_idle > 20 << 20, (used_hot, used_idle)
    h0 = gpu.stats()["hot_keys"]
    push(_zipf(seq, n, n_keys, 71, 64))
    push(_zipf(seq, n, n_keys, 72, 64))
    assert gpu.stats()["hot_keys"] > h0
    sg, so = gpu.stats(), ora.stats()
    for f in ("partials_live", "matches"):
        assert sg[f] == so[f], (f, sg[f], so[f])
    for e in (gpu, ora, lane):
        e.close()
