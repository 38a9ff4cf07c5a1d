"""BASELINE configs[2] (C3) and configs[3] (C4) at their benchmarked sizes, on the general device engine.

Keys are independent (PartitionStateHolder.java:43-49), so each run is checked against the CPU oracle
on a key subset fed with the same arrival seqs (runs of consecutive positions), plus size-independent
properties of EVERY emitted match.  C4 runs the real C4 stream (burst_ticks: one key per millisecond)
with the real 30 s / 60 s windows and the playback clock advanced to each batch's last timestamp before
the batch (InputHandler.send(Event[]), InputHandler.java:86-90), exactly as bench.py does;
C4_deep adds bursts of 16 events per key-millisecond (16 live partials per key).

Timers: an advance with no due key must cost little (due-key compaction), and two keys sharing a due
time at one advance (the reference's Scheduler collapse quirk) must fail loudly.
"""
import importlib
import time

import numpy as np
import pytest

from oracle_backend import build_oracle
from test_gpu_parity import _same

sa = importlib.import_module("siddhi-1_amd")
synth = importlib.import_module("siddhi-1_amd.synth")

pytestmark = pytest.mark.gpu

TIMER = np.uint64(0xFFFFFFFFFFFFFFFF)


def _engines(query, n_keys, max_batch, cap, mcap):
    app = sa.parse_app(query)
    cq = sa.compile_query(app, app.queries[0], sa.StringDictionary())
    gpu = sa.NativeEngine(sa.load_hip_library(), "sg_", cq.ir, n_keys=n_keys, max_batch=max_batch,
                          partial_capacity=cap, match_capacity=mcap)
    ora = sa.NativeEngine(build_oracle(), "sgo_", cq.ir, n_keys=n_keys)
    return gpu, ora


def _push_subset(ora, seq, d, sub):
    idx = np.nonzero(sub)[0]
    if len(idx) == 0:
        return
    starts = np.concatenate([[0], np.nonzero(np.diff(idx) != 1)[0] + 1])
    ends = np.concatenate([starts[1:], [len(idx)]])
    for s, t in zip(starts, ends):
        sl = idx[s:t]
        ora.push(0, seq + int(sl[0]), d["ts"][sl], [d["symbol"][sl], d["price"][sl], d["volume"][sl]], None,
                 d["key"][sl])


def _check_subset(mg, mo, mod):
    keep = (mg.key % mod) == 0
    assert int(keep.sum()) == len(mo), (int(keep.sum()), len(mo))
    assert np.array_equal(mg.trigger_seq[keep], mo.trigger_seq)
    assert np.array_equal(mg.key[keep], mo.key)
    assert np.array_equal(mg.ts[keep], mo.ts)
    assert np.array_equal(mg.chain_len[keep], mo.chain_len)
    w = min(mg.slot_seq.shape[2], mo.slot_seq.shape[2])
    assert np.array_equal(mg.slot_seq[keep][:, :, :w], mo.slot_seq[:, :, :w])


def _run(query, make_batch, n_keys, batch, nb, cap, mod, playback, props):
    gpu, ora = _engines(query, n_keys, batch, cap, 4 * batch)
    seqs = []
    total = 0
    for b in range(nb):
        d = make_batch(b)
        seq = b * batch
        seqs.append((seq, d))
        if playback:
            t = int(d["ts"][-1])
            gpu.advance_time(t)
            ora.advance_time(t)
            mg, mo = gpu.poll(), ora.poll()
            _check_subset(mg, mo, mod)
            props(mg, seqs)
            total += len(mg)
        gpu.push(0, seq, d["ts"], [d["symbol"], d["price"], d["volume"]], None, d["key"])
        _push_subset(ora, seq, d, (d["key"] % mod) == 0)
        mg, mo = gpu.poll(), ora.poll()
        _check_subset(mg, mo, mod)
        props(mg, seqs)
        total += len(mg)
    return total, gpu, ora


def _lookup(seqs, s):
    """column values of the events with arrival seqs s (all from the batches seen so far)"""
    out = {k: np.empty(len(s), dtype=v.dtype) for k, v in seqs[0][1].items()}
    s = s.astype(np.int64)
    for base, d in seqs:
        m = (s >= base) & (s < base + len(d["ts"]))
        for k in out:
            out[k][m] = d[k][s[m] - base]
    return out


def _c3_props(mg, seqs):
    """every C3 match: e1 chain of 1..5 events with price > 20, then e2 (price > e1[last].price) or e3
    (volume > 1000) as the trigger, all of one key, strictly increasing seqs, within 10 s of e1[0]"""
    if len(mg) == 0:
        return
    trig = mg.trigger_seq
    assert np.all(np.diff(trig.astype(np.int64)) >= 0)
    n1 = mg.chain_len[:, 0].astype(np.int64)
    assert np.all((n1 >= 1) & (n1 <= 5))
    first = mg.slot_seq[:, 0, 0]
    last = mg.slot_seq[np.arange(len(mg)), 0, n1 - 1]
    ev_first, ev_last, ev_t = _lookup(seqs, first), _lookup(seqs, last), _lookup(seqs, trig)
    assert np.all(ev_first["key"] == mg.key) and np.all(ev_t["key"] == mg.key)
    assert np.all(ev_first["price"] > 20) and np.all(ev_last["price"] > 20)
    assert np.all(first <= last) and np.all(last < trig)
    e3 = mg.chain_len[:, 1] == 1   # slots in the reference's parse order: the `or`'s second element first
    e2 = mg.chain_len[:, 2] == 1
    assert np.all(e2 ^ e3)
    assert np.all(ev_t["price"][e2] > ev_last["price"][e2])
    assert np.all(ev_t["volume"][e3] > 1000)
    assert np.all(np.abs(ev_t["ts"] - ev_first["ts"]) <= 10_000)
    assert np.all(mg.ts == ev_t["ts"])


def _c4_props(mg, seqs):
    """every C4 match is a timer emission: e1 (price > 20) of the match's key, fired at e1.ts + 30 s
    (AbsentStreamPreStateProcessor: the partial's ts becomes the due time), no slot-1 event"""
    if len(mg) == 0:
        return
    assert np.all(mg.trigger_seq == TIMER)
    e1 = mg.slot_seq[:, 0, 0]
    ev = _lookup(seqs, e1)
    assert np.all(ev["key"] == mg.key)
    assert np.all(ev["price"] > 20)
    assert np.all(mg.ts == ev["ts"] + 30_000)
    assert np.all(mg.chain_len[:, 1] == 0)


C3_SHAPES = {"C3": synth.C3_QUERY, "C3_min1": synth.C3_MIN1_QUERY}


@pytest.mark.parametrize("name", sorted(C3_SHAPES))
def test_c3_at_baseline_size(name):
    """C3 / C3_min1 on 1,048,576 keys, two 2^22-event batches of the C2-rate stream (as bench.py)"""
    K, B = 1 << 20, 1 << 22
    total, gpu, ora = _run(C3_SHAPES[name], lambda b: synth.stock_ticks(b * B, B, K), K, B, 2, 8, 256, False,
                           _c3_props)
    if name == "C3":
        assert total == 0   # SEQUENCE reset before <2:5> reaches 2: in the oracle too
    else:
        assert total > 100_000
    sg, so = gpu.stats(), ora.stats()
    assert sg["events"] == 2 * B


def _ordered_props(mg, seqs):
    """every match: trigger seqs in order, the trigger and the first slot's e1 events of the match's key"""
    if len(mg) == 0:
        return
    trig = mg.trigger_seq
    assert np.all(np.diff(trig.astype(np.int64)) >= 0)
    ev_t, ev_1 = _lookup(seqs, trig), _lookup(seqs, mg.slot_seq[:, 0, 0])
    assert np.all(ev_t["key"] == mg.key) and np.all(ev_1["key"] == mg.key)
    assert np.all(ev_1["price"] > 20)
    assert np.all(mg.ts == ev_t["ts"])


@pytest.mark.parametrize("name", ["C3_and", "P3"])
def test_general_shapes_at_bench_size(name):
    """the shapes that stay on the general kernel, benchmarked beside C3 (bench.py
    other_configs C3_and, P3), at their bench size — 2^20 keys, 2^22-event batches — bit-exact with the oracle on
    the keys k % 256 == 0"""
    K, B = 1 << 20, 1 << 22
    q = synth.C3_AND_QUERY if name == "C3_and" else synth.P3_QUERY
    total, gpu, ora = _run(q, lambda b: synth.stock_ticks(b * B, B, K), K, B, 2, 32, 256, False, _ordered_props)
    assert total > 10_000
    assert gpu.stats()["events"] == 2 * B


C4_CASES = {
    # (keys, burst, batch events, partial capacity, subset modulus)
    "C4": (1 << 20, 1, 1 << 22, 16, 256),
    "C4_deep": (1 << 18, 16, 1 << 22, 64, 64),
}


@pytest.mark.parametrize("name", sorted(C4_CASES))
def test_c4_at_baseline_depth(name):
    """C4 with its BASELINE windows (not S[...] for 30 sec within 60 sec) on the C4 stream, the playback
    clock advanced per batch; three batches, so partials of each batch fire at the next advance"""
    K, burst, B, cap, mod = C4_CASES[name]
    ms = B // burst
    total, gpu, ora = _run(synth.C4_QUERY, lambda b: synth.burst_ticks(b * ms, ms, K, burst), K, B, 3, cap, mod,
                           True, _c4_props)
    assert total > 10_000
    assert gpu.stats()["partials_live"] >= 0


def test_advance_without_due_keys_is_cheap():
    """due-key compaction: an advance with no due key at 2^20 keys is one pass over the deadline array,
    not a sweep of every key's state"""
    K = 1 << 20
    gpu, ora = _engines(synth.C4_QUERY, K, 1 << 20, 16, 1 << 22)
    d = synth.burst_ticks(0, 1 << 20, K, 1)
    t_last = int(d["ts"][-1])
    gpu.advance_time(t_last)
    gpu.push(0, 0, d["ts"], [d["symbol"], d["price"], d["volume"]], None, d["key"])
    gpu.poll()
    gpu.advance_time(t_last + 40_000)   # every armed timer (ts + 30 s) fires; none is re-armed
    assert len(gpu.poll()) > 0
    times = []
    for i in range(20):
        t0 = time.perf_counter()
        gpu.advance_time(t_last + 40_001 + i)
        times.append(time.perf_counter() - t0)
        assert len(gpu.poll()) == 0
    med = float(np.median(times)) * 1e6
    print(f"advance without due keys at 2^20 keys: median {med:.1f} us")
    assert med < 500.0


def test_a10_same_due_time_fails_loudly():
    """two keys whose absent timers fall due at the same time at one advance: the reference fires only one
    of them (TreeMultimap with an always-0 value comparator, Scheduler.java:78-89, 364-367), chosen by
    HashMap order; the device engine and the oracle both refuse the input instead of guessing"""
    q = synth.C4_QUERY
    gpu, ora = _engines(q, 64, 1024, 16, 1 << 16)
    ts = np.array([1000, 1000], dtype=np.int64)
    d = {"key": np.array([3, 7], dtype=np.uint32), "ts": ts, "price": np.array([25.0, 26.0], dtype=np.float32),
         "volume": np.array([1, 1], dtype=np.int32)}
    d["symbol"] = d["key"].copy()
    for e in (gpu, ora):
        e.advance_time(1000)
        e.poll()
        e.push(0, 0, d["ts"], [d["symbol"], d["price"], d["volume"]], None, d["key"])
        e.poll()
    with pytest.raises(sa.EngineError, match="A.10"):
        ora.advance_time(1000 + 40_000)
    with pytest.raises(sa.EngineError, match="SG_ERR_UNSUPPORTED"):
        gpu.advance_time(1000 + 40_000)


def test_timers_distinct_due_times_across_many_keys_bit_exact():
    """many keys, advances that make only some keys due (due-key compaction picks exactly those), timers
    armed by batches and by earlier firings, checked against the oracle on every key"""
    q = ("@app:playback define stream S (symbol string, price float, volume int);\n"
         "partition with (symbol of S) begin from every e1=S[price>20] -> not S[price>e1.price] for 50 milliseconds "
         "within 400 milliseconds select e1.price as a insert into O; end;")
    K = 4096
    gpu, ora = _engines(q, K, 1 << 14, 48, 1 << 20)
    rng = np.random.default_rng(12)
    seq, t = 0, 1_000_000
    for e in (gpu, ora):
        e.advance_time(t)
    _same(gpu.poll(), ora.poll())
    for b in range(40):
        n = int(rng.integers(50, 400))
        ts = t + np.arange(n, dtype=np.int64)          # one event per ms: distinct due times
        key = rng.integers(0, K, n).astype(np.uint32)
        d = {"key": key, "symbol": key.copy(), "ts": ts, "price": (10 + 30 * rng.random(n)).astype(np.float32),
             "volume": rng.integers(1, 2000, n).astype(np.int32)}
        for e in (gpu, ora):
            e.advance_time(int(ts[-1]))
        _same(gpu.poll(), ora.poll())
        for e in (gpu, ora):
            e.push(0, seq, d["ts"], [d["symbol"], d["price"], d["volume"]], None, d["key"])
        _same(gpu.poll(), ora.poll())
        seq += n
        t = int(ts[-1]) + int(rng.integers(1, 120))
    for e in (gpu, ora):
        e.advance_time(t + 10_000)
    _same(gpu.poll(), ora.poll())
