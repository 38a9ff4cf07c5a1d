"""The register-window kernel of chained stream states (csrc/chn_kernels.hip; the bench's P3 leg) against the CPU
oracle and against the general kernel it shortcuts (SG_NO_CHN=1), bit-exact:

    [every] e1=S[f0] -> e2=S[f1] -> ... -> en=S[f(n-1)] [within W]          (PATTERN, partitioned, n = 2..4)

* match records (trigger seq, key, ts, every slot's event), every work counter (scanned, created — the clones
  `every` stages —, keys touched, live partials) and the exported state documents (the kernel writes the general
  engine's blocks in a canonical layout: the document must not notice), over several pushes with state carried;
* 3- and 4-state chains, with and without `every` and `within`, filters reading e1 and e2 (two kept words), double
  attributes, nulls, random streams with several keys; a five-word event stays on the general kernel;
* the hand-overs to the general kernel: more live partials than the window holds (from the event where the key
  stops), timestamps out of order, an imported oracle document (pool entries in the oracle's order), one-event
  pushes (the canonical layout after every event).
Reference: StreamPreStateProcessor.java:118-129 / :308-403, StreamPostStateProcessor.java:64-83,
PatternMultiProcessStreamReceiver.java:31-51.
"""
import importlib

import numpy as np
import pytest

from oracle_backend import build_oracle
from test_gpu_parity import _same

sa = importlib.import_module("siddhi-1_amd")
synth = importlib.import_module("siddhi-1_amd.synth")
sd = importlib.import_module("siddhi-1_amd.state_doc")

pytestmark = pytest.mark.gpu

STOCK = "define stream S (symbol string, price float, volume int);\n"
WIDE = "define stream S (symbol string, price double, volume int);\n"     # (4 attribute words: the kernel's limit)
WIDER = "define stream S (symbol string, price double, volume long);\n"   # (5: the general kernel)


def chain(filters, every=True, within="within 200 milliseconds", schema=STOCK):
    states = " -> ".join(f"e{i + 1}=S[{f}]" for i, f in enumerate(filters))
    return (schema + "partition with (symbol of S) begin "
            f"from {'every ' if every else ''}{states} {within} "
            "select e1.price as a insert into O; end;")


SHAPES = {
    "p3": chain(["price>20", "price>e1.price", "price>e2.price"]),
    "p3_no_every": chain(["price>20", "price>e1.price", "price>e2.price"], every=False),
    "p3_no_within": chain(["price>20", "price>e1.price", "price>e2.price"], within=""),
    "p3_short_within": chain(["price>20", "price>e1.price", "price>e2.price"], within="within 40 milliseconds"),
    "p4": chain(["price>20", "price>e1.price", "price>e2.price", "price>e3.price"]),
    "p3_two_words": chain(["price>10", "volume>e1.volume", "price>e1.price"]),
    "p3_wide": chain(["price>20", "price>e1.price", "price>e2.price"], schema=WIDE),
    "p3_no_ref": chain(["price>20", "volume>500", "price<30"]),
    "p2": chain(["price>20", "price>e1.price"]),
}

ALL = ("matches", "partials_created", "partials_scanned", "keys_touched", "partials_live")


def _compile(q):
    app = sa.parse_app(q)
    return sa.compile_query(app, app.queries[0], sa.StringDictionary())


def _engine(q, n_keys, batch, general, monkeypatch, mcap=1 << 20, cap=32):
    cq = _compile(q)
    if general:
        monkeypatch.setenv("SG_NO_CHN", "1")
    e = sa.NativeEngine(sa.load_hip_library(), "sg_", cq.ir, n_keys=n_keys, max_batch=batch, partial_capacity=cap,
                        match_capacity=mcap)
    monkeypatch.delenv("SG_NO_CHN", raising=False)
    return e


def _oracle(q, n_keys):
    return sa.NativeEngine(build_oracle(), "sgo_", _compile(q).ir, n_keys=n_keys)


def _stream(n, n_keys, seed, nulls=False, wide=False, rate=3):
    d = synth.stock_ticks(0, n, n_keys, seed=seed, rate_per_ms=rate)
    price = d["price"].astype(np.float64) if wide else d["price"]
    vol = d["volume"]
    nul = None
    if nulls:
        nul = [None, ((d["volume"] % 13) == 5).astype(np.uint8), ((d["volume"] % 11) == 3).astype(np.uint8)]
    return d, [d["symbol"], price, vol], nul


def _drive(engines, d, cols, nul, chunks):
    total = 0
    for lo, hi in chunks:
        sl = slice(lo, hi)
        for e in engines:
            e.push(0, lo, d["ts"][sl], [c[sl] for c in cols], None if nul is None else
                   [x[sl] if x is not None else None for x in nul], d["key"][sl])
        ms = [e.poll() for e in engines]
        for m in ms[1:]:
            _same(ms[0], m)
        total += len(ms[0])
    return total


def _chunks(n, size):
    return [(i, min(n, i + size)) for i in range(0, n, size)]


def _docs_equal(a, b):
    assert sd.logical(sd.parse(a.state_export())) == sd.logical(sd.parse(b.state_export()))


@pytest.mark.parametrize("shape", sorted(SHAPES))
def test_chain_window_equals_oracle_and_general(shape, monkeypatch):
    q = SHAPES[shape]
    if shape == "p2":   # (a two-state chain goes to the specialised two-state kernel unless the general engine is forced)
        monkeypatch.setenv("SG_FORCE_GENERAL", "1")
    n_keys = 48
    d, cols, nul = _stream(8000, n_keys, seed=11, wide="double" in q)
    fast = _engine(q, n_keys, 4096, False, monkeypatch)
    assert "k_chn_batch" in fast.describe(), fast.describe()
    gen = _engine(q, n_keys, 4096, True, monkeypatch)
    assert "k_chn_batch" not in gen.describe()
    ora = _oracle(q, n_keys)
    total = _drive([fast, gen, ora], d, cols, nul, _chunks(len(d["ts"]), 900))
    assert total > 0
    sf, sg, so = fast.stats(), gen.stats(), ora.stats()
    for k in ALL:
        assert sf[k] == sg[k], (k, sf[k], sg[k])
    for k in ("matches", "partials_live"):
        assert sf[k] == so[k], (k, sf[k], so[k])
    _docs_equal(fast, ora)
    _docs_equal(fast, gen)


def test_five_attribute_words_stay_on_the_general_kernel(monkeypatch):
    """an event of more attribute words than the chain kernel holds in registers (double + long: 5) is not this
    kernel's shape: the general kernel runs it, equal to the oracle"""
    q = chain(["price>20", "price>e1.price", "volume>e2.volume"], schema=WIDER)
    n_keys = 32
    d = synth.stock_ticks(0, 5000, n_keys, seed=13, rate_per_ms=3)
    cols = [d["symbol"], d["price"].astype(np.float64), d["volume"].astype(np.int64)]
    e = _engine(q, n_keys, 4096, False, monkeypatch)
    assert "k_chn_batch" not in e.describe(), e.describe()
    ora = _oracle(q, n_keys)
    assert _drive([e, ora], d, cols, None, _chunks(len(d["ts"]), 800)) > 0
    _docs_equal(e, ora)


def test_chain_window_nulls(monkeypatch):
    q = SHAPES["p3_two_words"]
    n_keys = 40
    d, cols, nul = _stream(6000, n_keys, seed=3, nulls=True)
    fast = _engine(q, n_keys, 4096, False, monkeypatch)
    gen = _engine(q, n_keys, 4096, True, monkeypatch)
    ora = _oracle(q, n_keys)
    assert _drive([fast, gen, ora], d, cols, nul, _chunks(len(d["ts"]), 700)) > 0
    sf, sg = fast.stats(), gen.stats()
    for k in ALL:
        assert sf[k] == sg[k], (k, sf[k], sg[k])
    _docs_equal(fast, ora)


@pytest.mark.parametrize("wide", [True, False])
def test_chain_window_overflow_hands_over(wide, monkeypatch):
    """a filter that rarely passes: state-1 partials pile up past the window (24 for three states), the key is stored
    and the wide-window kernel (32) continues from the event where it stopped, then the general kernel from where
    that one stopped (wide = False: the general kernel directly); later batches load it back"""
    q = chain(["price>10", "price>39.5", "price>e2.price"], within="within 300 milliseconds")
    n_keys = 16
    d, cols, nul = _stream(8000, n_keys, seed=19, rate=2)
    if not wide:
        monkeypatch.setenv("SG_NO_CHN_WIDE", "1")
    fast = _engine(q, n_keys, 4096, False, monkeypatch, cap=64)
    monkeypatch.delenv("SG_NO_CHN_WIDE", raising=False)
    assert ("k_chn_wide" in fast.describe()) == wide, fast.describe()
    gen = _engine(q, n_keys, 4096, True, monkeypatch, cap=64)
    ora = _oracle(q, n_keys)
    total = _drive([fast, gen, ora], d, cols, nul, _chunks(len(d["ts"]), 1000))
    sf, sg = fast.stats(), gen.stats()
    assert sf["window_spills"] > 0, "no key outgrew the window: the test does not test"
    for k in ALL:
        assert sf[k] == sg[k], (k, sf[k], sg[k])
    assert total == ora.stats()["matches"]
    _docs_equal(fast, ora)


@pytest.mark.parametrize("n", [2, 4])
def test_chain_window_overflow_other_lengths(n, monkeypatch):
    """the hand-overs of the 2- and 4-state kernels (narrow windows 24 / 12, wide 32 / 21): state-1 partials pile up
    behind a filter that rarely passes, through the wide window and on to the general kernel, equal to the oracle and
    to the general kernel alone"""
    filters = ["price>10", "price>39.5", "price>e2.price", "price>e3.price"][:n]
    q = chain(filters, within="within 300 milliseconds")
    n_keys = 16
    if n == 2:   # (a two-state chain goes to the specialised two-state kernel unless the general engine is forced)
        monkeypatch.setenv("SG_FORCE_GENERAL", "1")
    d, cols, nul = _stream(9000, n_keys, seed=31 + n, rate=2)
    fast = _engine(q, n_keys, 4096, False, monkeypatch, cap=64)
    assert "k_chn_wide" in fast.describe(), fast.describe()
    gen = _engine(q, n_keys, 4096, True, monkeypatch, cap=64)
    ora = _oracle(q, n_keys)
    total = _drive([fast, gen, ora], d, cols, nul, _chunks(len(d["ts"]), 1100))
    sf, sg = fast.stats(), gen.stats()
    assert sf["window_spills"] > 0, "no key outgrew the window: the test does not test"
    for k in ALL:
        assert sf[k] == sg[k], (k, sf[k], sg[k])
    assert total == ora.stats()["matches"]
    _docs_equal(fast, ora)


def test_chain_window_out_of_order_timestamps(monkeypatch):
    q = SHAPES["p3"]
    n_keys = 32
    d, cols, nul = _stream(6000, n_keys, seed=29)
    sw = np.arange(0, len(d["ts"]) - 1, 37)
    d["ts"][sw], d["ts"][sw + 1] = d["ts"][sw + 1].copy(), d["ts"][sw].copy()
    fast = _engine(q, n_keys, 4096, False, monkeypatch)
    gen = _engine(q, n_keys, 4096, True, monkeypatch)
    ora = _oracle(q, n_keys)
    assert _drive([fast, gen, ora], d, cols, nul, _chunks(len(d["ts"]), 800)) > 0
    sf, sg = fast.stats(), gen.stats()
    for k in ALL:
        assert sf[k] == sg[k], (k, sf[k], sg[k])
    _docs_equal(fast, ora)


def test_chain_window_single_event_pushes(monkeypatch):
    """one event per push: the key's state goes through the canonical layout (alternating pool regions) after
    every event"""
    q = SHAPES["p4"]
    n_keys = 6
    d, cols, nul = _stream(1200, n_keys, seed=5)
    fast = _engine(q, n_keys, 64, False, monkeypatch)
    ora = _oracle(q, n_keys)
    assert _drive([fast, ora], d, cols, nul, _chunks(len(d["ts"]), 1)) > 0
    _docs_equal(fast, ora)


@pytest.mark.parametrize("shape", ["p3", "p3_wide"])
def test_chain_window_after_foreign_import_and_exports(shape, monkeypatch):
    """state imported from an oracle document (the general layout, pool entries in the oracle's order) continues
    exactly as the oracle does; state exports between pushes leave it unchanged"""
    q = SHAPES[shape]
    n_keys = 48
    d, cols, nul = _stream(8000, n_keys, seed=23, wide="double" in q)
    n = len(d["ts"])
    half = 4000
    ora = _oracle(q, n_keys)
    _drive([ora], d, cols, nul, _chunks(half, 600))
    fast = _engine(q, n_keys, 4096, False, monkeypatch)
    fast.state_import(ora.state_export())
    for i, (lo, hi) in enumerate([c for c in _chunks(n, 500) if c[0] >= half]):
        _drive([fast, ora], d, cols, nul, [(lo, hi)])
        if i % 2 == 1:
            _docs_equal(fast, ora)
    assert fast.stats()["matches"] > 0
    _docs_equal(fast, ora)


def test_p3_at_bench_keys(monkeypatch):
    """the bench's P3 leg at its size (2^20 keys, 2^22-event pushes, partial capacity 32): chain kernel == general
    kernel, every match and counter, seven pushes with state carried — past the 10-second window's fill (with the
    24-slot window no key outgrows it here; the overflow tests above take the hand-overs)"""
    q = synth.P3_QUERY
    K, B = 1 << 20, 1 << 22
    fast = _engine(q, K, B, False, monkeypatch, mcap=B)
    assert "k_chn_wide" in fast.describe(), fast.describe()
    gen = _engine(q, K, B, True, monkeypatch, mcap=B)
    total = 0
    for s in range(7):
        d = synth.stock_ticks(s * B, B, K)
        for e in (fast, gen):
            e.push(0, s * B, d["ts"], [d["symbol"], d["price"], d["volume"]], None, d["key"])
        mf, mg = fast.poll(), gen.poll()
        _same(mf, mg)
        total += len(mf)
    assert total > 0
    sf, sg = fast.stats(), gen.stats()
    for k in ALL:
        assert sf[k] == sg[k], (k, sf[k], sg[k])
