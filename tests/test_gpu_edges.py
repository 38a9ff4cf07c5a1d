"""Edge cases of the device path against the oracle, bit-exact: empty and ragged batches (sizes that
are not multiples of a wave, a workgroup or an ordering tile), key counts that are not multiples of
the wave, events only on the first and last key ids, a batch of exactly max_batch events, and very
deep per-key state (hundreds of live partials per key: the HBM pass and its slab for every key),
on the two-state kernel and on the general engine."""
import importlib

import numpy as np
import pytest

from test_gpu_general import GENERAL
from test_gpu_parity import SHAPES, _engines, _same

sa = importlib.import_module("siddhi-1_amd")
synth = importlib.import_module("siddhi-1_amd.synth")

pytestmark = pytest.mark.gpu

COLS = ["symbol", "price", "volume"]
QUERIES = {"c2": SHAPES["c2_every_within"], "every_both": SHAPES["every_both_within"],
           "gen_count": GENERAL["count_pattern"], "gen_sequence": GENERAL["sequence"]}


def _push(engines, seq, d):
    for e in engines:
        e.push(0, seq, d["ts"], [d[c] for c in COLS], None, d["key"])


@pytest.mark.parametrize("q", sorted(QUERIES))
def test_ragged_and_empty_batches(q):
    n_keys, maxb = 1000, 12345          # 1000 keys: not a multiple of 64 / 128
    cq, gpu, ora = _engines(QUERIES[q], n_keys, maxb)
    seq = 0
    total = 0
    for i, n in enumerate([1, 0, 63, 65, 4095, 4097, 0, 12345, 777]):
        d = synth.stock_ticks(seq, n, n_keys, seed=60 + i, rate_per_ms=4)
        _push((gpu, ora), seq, d)
        mg, mo = gpu.poll(), ora.poll()
        _same(mg, mo)
        total += len(mg)
        seq += n
    assert total > 0
    assert gpu.stats()["partials_live"] == ora.stats()["partials_live"]


@pytest.mark.parametrize("q", ["c2", "gen_count"])
def test_first_and_last_key_only(q):
    n_keys, batch = 4099, 6000
    cq, gpu, ora = _engines(QUERIES[q], n_keys, batch)
    seq = 0
    for b in range(3):
        d = synth.stock_ticks(seq, batch, 2, seed=80 + b, rate_per_ms=8)
        d = dict(d, key=np.where(d["key"] == 0, 0, n_keys - 1).astype(np.uint32))
        d["symbol"] = d["key"].copy()
        _push((gpu, ora), seq, d)
        _same(gpu.poll(), ora.poll())
        seq += batch


def test_exactly_max_batch():
    n_keys, batch = 4096, 1 << 16
    cq, gpu, ora = _engines(QUERIES["c2"], n_keys, batch)
    d = synth.stock_ticks(0, batch, n_keys, seed=90, rate_per_ms=16)
    _push((gpu, ora), 0, d)
    _same(gpu.poll(), ora.poll())
    d = synth.stock_ticks(batch, batch + 1, n_keys, seed=91, rate_per_ms=16)
    with pytest.raises(sa.EngineError):
        gpu.push(0, batch, d["ts"], [d[c] for c in COLS], None, d["key"])


def test_deep_state_few_keys():
    """4 keys, 2000 events each inside one `within` window, prices falling through the first batch (every
    event opens a partial, none matches: 2000 live partials per key, far beyond the register window, so
    every key runs on the HBM pass with its slab) and rising through the second (mass matching)"""
    n_keys, batch = 4, 8000
    cq, gpu, ora = _engines(QUERIES["c2"], n_keys, batch, cap=4095, mcap=1 << 24)
    i = np.arange(2 * batch)
    key = (i % n_keys).astype(np.uint32)
    ts = (1_700_000_000_000 + i // 40).astype(np.int64)
    fall = 39.9 - (i[:batch] * (19.0 / batch))
    rise = 20.5 + ((i[batch:] - batch) * (19.0 / batch))
    price = np.concatenate([fall, rise]).astype(np.float32)
    volume = np.full(2 * batch, 7, dtype=np.int32)
    total = 0
    for b in range(2):
        sl = slice(b * batch, (b + 1) * batch)
        d = {"key": key[sl], "symbol": key[sl].copy(), "ts": ts[sl], "price": price[sl], "volume": volume[sl]}
        _push((gpu, ora), b * batch, d)
        mg, mo = gpu.poll(), ora.poll()
        _same(mg, mo)
        total += len(mg)
        if b == 0:
            assert len(mg) == 0 and gpu.stats()["partials_live"] == ora.stats()["partials_live"] >= 4 * 1900
    assert total > 0
    assert gpu.stats()["partials_live"] == ora.stats()["partials_live"]
