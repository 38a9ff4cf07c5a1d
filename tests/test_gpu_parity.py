"""HIP engine parity with the CPU oracle (bit-exact match tuples), through the C-ABI.

* every transcribed reference KAT whose query shape runs on the device (others must be rejected
  at engine creation with SG_ERR_UNSUPPORTED — never silently);
* seeded random streams over many keys, several batches (state carried across batches), for every
  two-state shape / filter type / receiver kind the device supports;
* the BASELINE configuration size (1,048,576 keys, 2^24-event batches) checked against the oracle on
  a key subset (keys are independent, PartitionStateHolder.java:43-49) plus size-independent
  properties of every emitted match.
"""
import importlib

import numpy as np
import pytest

from kat_runner import load_cases, run_case
from oracle_backend import build_oracle

sa = importlib.import_module("siddhi-1_amd")
synth = importlib.import_module("siddhi-1_amd.synth")

pytestmark = pytest.mark.gpu

SG_ERR_UNSUPPORTED = -2


def hip_manager(n_keys=1024):
    lib = sa.load_hip_library()

    def make(ir, nk):
        return sa.NativeEngine(lib, "sg_", ir, n_keys=nk, max_batch=4096, partial_capacity=64,
                               match_capacity=1 << 16)
    return sa.SiddhiManager(engine_factory=make, n_keys=n_keys)


from test_oracle_kat import KNOWN_UNSUPPORTED, SLOW

KATS = [(f, c) for f, c in load_cases() if "skip" not in c and f"{f}::{c['name']}" not in SLOW]


@pytest.mark.parametrize("fc", KATS, ids=[f"{f}::{c['name']}" for f, c in KATS])
def test_gpu_kat(fc):
    """every transcribed reference KAT through the HIP engine (two-state kernel or general engine)"""
    f, case = fc
    if f"{f}::{case['name']}" in KNOWN_UNSUPPORTED:
        pytest.skip(KNOWN_UNSUPPORTED[f"{f}::{case['name']}"])
    try:
        ok, msg = run_case(case, hip_manager())
    except sa.EngineError as ex:
        if ex.code == SG_ERR_UNSUPPORTED:
            pytest.skip(f"shape not on the device yet: {ex}")
        raise
    except (sa.SiddhiAppCreationException, sa.SiddhiParserException) as ex:
        pytest.skip(f"outside the pattern path: {ex}")
    assert ok, msg


# ------------------------------------------------------------------------------------------------
def _engines(query, n_keys, max_batch, cap=64, mcap=1 << 22):
    app = sa.parse_app(query)
    cq = sa.compile_query(app, app.queries[0], sa.StringDictionary())
    gpu = sa.NativeEngine(sa.load_hip_library(), "sg_", cq.ir, n_keys=n_keys, max_batch=max_batch,
                          partial_capacity=cap, match_capacity=mcap)
    ora = sa.NativeEngine(build_oracle(), "sgo_", cq.ir, n_keys=n_keys)
    return cq, gpu, ora


def _same(mg, mo):
    """bit-exact match records; slot chains compared up to their lengths (engines may pad the
    chain dimension differently: entries past chain_len are SG_NULL_SEQ)"""
    assert len(mg) == len(mo), (len(mg), len(mo))
    assert np.array_equal(mg.trigger_seq, mo.trigger_seq)
    assert np.array_equal(mg.key, mo.key)
    assert np.array_equal(mg.ts, mo.ts)
    assert np.array_equal(mg.chain_len, mo.chain_len)
    w = min(mg.slot_seq.shape[2], mo.slot_seq.shape[2])
    assert np.array_equal(mg.slot_seq[:, :, :w], mo.slot_seq[:, :, :w])
    for m in (mg, mo):
        assert np.all(m.slot_seq[:, :, w:] == np.uint64(0xFFFFFFFFFFFFFFFF))


STOCK = "define stream S (symbol string, price float, volume int);\n"
TWO = ("define stream S1 (symbol string, price float, volume int);\n"
       "define stream S2 (symbol string, price double, volume long);\n")

SHAPES = {
    "c2_every_within": STOCK + "partition with (symbol of S) begin "
    "from every e1=S[price>20] -> e2=S[price>e1.price] within 1 sec select e1.price as a insert into O; end;",
    "no_every": STOCK + "partition with (symbol of S) begin "
    "from e1=S[price>30] -> e2=S[price<e1.price] select e1.price as a insert into O; end;",
    "every_both_within": STOCK + "partition with (symbol of S) begin "
    "from every (e1=S[price>25] -> e2=S[price>e1.price]) within 500 milliseconds select e1.price as a insert into O; end;",
    "every_no_within": STOCK + "partition with (symbol of S) begin "
    "from every e1=S[price>38] -> e2=S[price>e1.price] select e1.price as a insert into O; end;",
    "int_long_double": STOCK + "partition with (symbol of S) begin "
    "from every e1=S[volume > 1000 and price >= 12.5] -> e2=S[volume * 2L < e1.volume + 100 or "
    "e2.price - e1.price > 9.75] within 2 sec select e1.price as a insert into O; end;",
    "arith_null_div": STOCK + "partition with (symbol of S) begin "
    "from every e1=S[(volume % 7) != 3] -> e2=S[price / (volume - e1.volume) > 0.01f] within 1 sec "
    "select e1.price as a insert into O; end;",
    "two_streams": TWO + "partition with (symbol of S1, symbol of S2) begin "
    "from every e1=S1[price>20] -> e2=S2[price>e1.price and volume > e1.volume] within 1 sec "
    "select e1.price as a insert into O; end;",
}


def _push_both(gpu, ora, stream, seq_base, d, cols_names, ts=None):
    ts = d["ts"] if ts is None else ts
    cols = [d[c] for c in cols_names]
    for e in (gpu, ora):
        e.push(stream, seq_base, ts, cols, None, d["key"])


@pytest.mark.parametrize("reg_slots,stage", [(12, 0), (2, 0), (12, 64)])
@pytest.mark.parametrize("shape", sorted(SHAPES))
def test_gpu_random_streams_bit_exact(shape, reg_slots, stage, monkeypatch):
    """reg_slots=2: most keys outgrow the register window, so the HBM-slab path is exercised too;
    stage=64: the LDS staging region is too small for any wave, so every lane reads its run of the
    key-sorted batch from HBM directly"""
    monkeypatch.setenv("SGD_REG_SLOTS", str(reg_slots))
    if stage:
        monkeypatch.setenv("SGD_STAGE_CHUNKS", str(stage))
    n_keys, batch, nb = 2048, 40000, 4
    cq, gpu, ora = _engines(SHAPES[shape], n_keys, batch)
    seq = 0
    for b in range(nb):
        d = synth.stock_ticks(seq, batch, n_keys, seed=11 + b, rate_per_ms=16)
        if shape == "two_streams":
            half = batch // 2
            d1 = {k: v[:half] for k, v in d.items()}
            d2 = {k: v[half:] for k, v in d.items()}
            d2 = dict(d2, price=d2["price"].astype(np.float64), volume=d2["volume"].astype(np.int64))
            _push_both(gpu, ora, cq.stream_index("S1"), seq, d1, ["symbol", "price", "volume"])
            _push_both(gpu, ora, cq.stream_index("S2"), seq + half, d2, ["symbol", "price", "volume"])
        else:
            _push_both(gpu, ora, 0, seq, d, ["symbol", "price", "volume"])
        seq += batch
        _same(gpu.poll(), ora.poll())
    sg, so = gpu.stats(), ora.stats()
    assert sg["matches"] == so["matches"] and sg["matches"] > 0
    assert sg["partials_live"] == so["partials_live"]
    if reg_slots == 2 and shape not in ("no_every", "every_both_within"):  # at most one live partial
        assert sg["window_spills"] > 0


@pytest.mark.parametrize("reg_slots", [12, 3])
def test_gpu_non_monotonic_timestamps(reg_slots, monkeypatch):
    """prefix-only expiry and the stable ts sort of staged partials (StreamPreStateProcessor.java:331-342)"""
    monkeypatch.setenv("SGD_REG_SLOTS", str(reg_slots))
    n_keys, batch = 512, 30000
    cq, gpu, ora = _engines(SHAPES["two_streams"], n_keys, batch)
    rng = np.random.default_rng(5)
    seq = 0
    for b in range(3):
        d = synth.stock_ticks(seq, batch, n_keys, seed=3 + b, rate_per_ms=8)
        ts = d["ts"] + rng.integers(-900, 900, size=batch)
        half = batch // 2
        for s, lo, hi in ((0, 0, half), (1, half, batch)):
            dd = {k: v[lo:hi] for k, v in d.items()}
            if s == 1:
                dd = dict(dd, price=dd["price"].astype(np.float64), volume=dd["volume"].astype(np.int64))
            _push_both(gpu, ora, cq.stream_index("S1" if s == 0 else "S2"), seq + lo, dd,
                       ["symbol", "price", "volume"], ts=ts[lo:hi])
        seq += batch
        _same(gpu.poll(), ora.poll())


@pytest.mark.parametrize("within", ["1 sec", "20 days"])
def test_gpu_far_timestamps(within):
    """the staged pass holds timestamps / seqs as 32-bit offsets from a per-batch base: keys with a
    partial or an event more than 2^30 ms from the base, a ts of -1 (eventTimeComparator's unset) or
    a `within` of 2^30 ms or more must leave the staged pass for the 64-bit HBM pass, bit-exact"""
    q = (STOCK + "partition with (symbol of S) begin from every e1=S[price>20] -> e2=S[price>e1.price] "
         f"within {within} select e1.price as a insert into O; end;")
    n_keys, batch = 1024, 30000
    cq, gpu, ora = _engines(q, n_keys, batch)
    rng = np.random.default_rng(17)
    seq = 0
    for b in range(4):
        d = synth.stock_ticks(seq, batch, n_keys, seed=40 + b, rate_per_ms=16)
        ts = d["ts"].copy()
        pick = rng.random(batch)
        ts[pick < 0.01] += np.int64(1) << 33            # far future
        ts[(pick >= 0.01) & (pick < 0.015)] -= np.int64(1) << 40   # far past
        ts[(pick >= 0.015) & (pick < 0.018)] = -1
        ts[(pick >= 0.018) & (pick < 0.019)] = np.int64(2**62)     # near the long range's edge
        for e in (gpu, ora):
            e.push(0, seq, ts, [d["symbol"], d["price"], d["volume"]], None, d["key"])
        seq += batch
        _same(gpu.poll(), ora.poll())
    assert gpu.stats()["matches"] == ora.stats()["matches"] > 0


@pytest.mark.parametrize("first", ["unset", "far_past", "far_future"])
def test_gpu_batch_base_timestamp_far(first):
    """the payload's 32-bit timestamps are offsets from the batch's FIRST (arrival-order) timestamp: when
    that one is -1 or far from the rest, every other event of the batch is out of offset range and runs
    on the 64-bit path (the HBM pass reads the ts column), bit-exact"""
    q = (STOCK + "partition with (symbol of S) begin from every e1=S[price>20] -> e2=S[price>e1.price] "
         "within 1 sec select e1.price as a insert into O; end;")
    n_keys, batch = 512, 20000
    cq, gpu, ora = _engines(q, n_keys, batch)
    seq = 0
    for b in range(3):
        d = synth.stock_ticks(seq, batch, n_keys, seed=70 + b, rate_per_ms=16)
        ts = d["ts"].copy()
        ts[0] = {"unset": -1, "far_past": ts[1] - (np.int64(1) << 31), "far_future": ts[1] + (np.int64(1) << 35)}[first]
        for e in (gpu, ora):
            e.push(0, seq, ts, [d["symbol"], d["price"], d["volume"]], None, d["key"])
        seq += batch
        _same(gpu.poll(), ora.poll())
    assert gpu.stats()["matches"] == ora.stats()["matches"] > 0


def test_gpu_unpartitioned_single_key():
    q = STOCK + "from every e1=S[price>20] -> e2=S[price>e1.price] within 10 sec select e1.price as a insert into O;"
    cq, gpu, ora = _engines(q, 1, 20000)
    d = synth.stock_ticks(0, 20000, 1, rate_per_ms=2)
    for e in (gpu, ora):
        e.push(0, 0, d["ts"], [d["symbol"], d["price"], d["volume"]])
    _same(gpu.poll(), ora.poll())


def test_gpu_nulls_in_filters():
    """null attributes: compare -> false, != -> true, arithmetic -> null (CompareConditionExpressionExecutor)"""
    q = STOCK + ("partition with (symbol of S) begin from every e1=S[price != 15.0f] -> "
                 "e2=S[price > e1.price or volume != e1.volume] within 1 sec select e1.price as a insert into O; end;")
    n_keys, n = 256, 20000
    cq, gpu, ora = _engines(q, n_keys, n)
    d = synth.stock_ticks(0, n, n_keys, rate_per_ms=8)
    rng = np.random.default_rng(9)
    nulls = [None, (rng.random(n) < 0.1).astype(np.uint8), (rng.random(n) < 0.1).astype(np.uint8)]
    for e in (gpu, ora):
        e.push(0, 0, d["ts"], [d["symbol"], d["price"], d["volume"]], nulls, d["key"])
    _same(gpu.poll(), ora.poll())


def test_gpu_capacity_overflow_fails_loudly():
    q = STOCK + ("partition with (symbol of S) begin from every e1=S[price>0] -> e2=S[price>1000] "
                 "select e1.price as a insert into O; end;")
    cq, gpu, _ = _engines(q, 4, 4096, cap=8)
    d = synth.stock_ticks(0, 4096, 4)
    gpu.push(0, 0, d["ts"], [d["symbol"], d["price"], d["volume"]], None, d["key"])
    with pytest.raises(sa.EngineError, match="SG_ERR_CAPACITY"):
        gpu.poll()


@pytest.mark.slow
@pytest.mark.parametrize("n_keys,mod", [(1 << 20, 64), (1 << 23, 512)], ids=["C2", "C5_per_gpu"])
def test_gpu_baseline_size_key_subset_and_properties(n_keys, mod):
    """C2 at BASELINE size: 1,048,576 keys, two 2^24-event batches; and C5's per-GPU shape (2^23 keys:
    the three-pass 23-bit grouping).  Oracle on keys % mod == 0."""
    batch = 1 << 24
    cq, gpu, ora = _engines(synth.C2_QUERY, n_keys, batch, mcap=1 << 24)
    seq = 0
    for b in range(2):
        d = synth.stock_ticks(seq, batch, n_keys)
        gpu.push(0, seq, d["ts"], [d["symbol"], d["price"], d["volume"]], None, d["key"])
        mg = gpu.poll()
        sub = (d["key"] % mod) == 0
        idx = np.nonzero(sub)[0]
        # the oracle sees the subset with the same arrival seqs (runs of consecutive positions)
        starts = np.concatenate([[0], np.nonzero(np.diff(idx) != 1)[0] + 1])
        ends = np.concatenate([starts[1:], [len(idx)]])
        for s, t in zip(starts, ends):
            sl = idx[s:t]
            ora.push(0, seq + int(sl[0]), d["ts"][sl], [d["symbol"][sl], d["price"][sl], d["volume"][sl]],
                     None, d["key"][sl])
        mo = ora.poll()
        keep = (mg.key % mod) == 0
        assert int(keep.sum()) == len(mo) and len(mo) > 0
        assert np.array_equal(mg.trigger_seq[keep], mo.trigger_seq)
        assert np.array_equal(mg.slot_seq[keep], mo.slot_seq)
        # size-independent properties of every match
        trig = mg.trigger_seq.astype(np.int64) - seq
        e1 = mg.slot_seq[:, 0, 0].astype(np.int64)
        assert np.all(np.diff(mg.trigger_seq.astype(np.int64)) >= 0)      # global trigger order
        assert np.all(e1 < mg.trigger_seq.astype(np.int64))                 # e1 strictly before e2
        cur = (e1 >= seq)
        p1 = d["price"][e1[cur] - seq]
        p2 = d["price"][trig[cur]]
        assert np.all(p1 > 20) and np.all(p2 > p1)
        assert np.all(d["key"][trig] == mg.key)
        seq += batch
