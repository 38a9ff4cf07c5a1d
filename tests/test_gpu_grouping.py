"""The tile grouping (grp_kernels.hip: bucket by 256-key tile, split by key in LDS) against the oracle and
against the rocPRIM radix grouping (the default; the tile grouping is opt-in, SG_GROUP_TILES=1), bit-exact: skewed key streams whose
tiles overflow the LDS region (ranked from HBM), one hot key, partial last tiles, many empty tiles,
ragged scatter blocks, wide payloads (double/long columns), null bits, out-of-range and dropped null
key ids on device batches."""
import importlib
import os
import zlib

import numpy as np
import pytest
import torch

from test_gpu_parity import SHAPES, _engines, _same

sa = importlib.import_module("siddhi-1_amd")
synth = importlib.import_module("siddhi-1_amd.synth")

pytestmark = pytest.mark.gpu

COLS = ["symbol", "price", "volume"]


def _radix_engine(query, n_keys, max_batch, flags=0):
    app = sa.parse_app(query)
    cq = sa.compile_query(app, app.queries[0], sa.StringDictionary())
    saved = os.environ.pop("SG_GROUP_TILES", None)
    try:
        return sa.NativeEngine(sa.load_hip_library(), "sg_", cq.ir, n_keys=n_keys, max_batch=max_batch,
                               partial_capacity=64, match_capacity=1 << 22, flags=flags)
    finally:
        if saved is not None:
            os.environ["SG_GROUP_TILES"] = saved


@pytest.fixture(autouse=True)
def _tiles(monkeypatch):
    """engines created by the tests (the `gpu` one) take the tile grouping; _radix_engine drops the
    variable for the comparison engine"""
    monkeypatch.setenv("SG_GROUP_TILES", "1")


def _keys(kind, n, n_keys, rng):
    if kind == "uniform":
        return rng.integers(0, n_keys, n).astype(np.uint32)
    if kind == "zipf":        # a few tiles hold far more events than the LDS region
        return (np.minimum(rng.zipf(1.3, n), n_keys) - 1).astype(np.uint32)
    if kind == "hot":         # half the events on one key
        k = rng.integers(0, n_keys, n).astype(np.uint32)
        k[rng.random(n) < 0.5] = n_keys // 2
        return k
    if kind == "sparse":      # a handful of keys in a large key space: most tiles empty
        return rng.choice(np.array([0, 255, 256, 77777, n_keys - 1], dtype=np.uint32), n)
    raise ValueError(kind)


CASES = [
    ("uniform", 1 << 16, 1 << 18),
    ("zipf", 1 << 16, 1 << 18),
    ("hot", 5000, 100003),
    ("sparse", 1 << 20, 70000),
    ("uniform", 1000, 65537),      # partial last tile, one event past a scatter block
    ("uniform", 1 << 20, 1 << 16),  # K at the tile grouping's limit
]


@pytest.mark.parametrize("kind,n_keys,n", CASES)
@pytest.mark.parametrize("shape", ["c2_every_within", "every_both_within"])
def test_tile_grouping_vs_oracle_and_radix(kind, n_keys, n, shape):
    cq, gpu, ora = _engines(SHAPES[shape], n_keys, n)
    rad = _radix_engine(SHAPES[shape], n_keys, n)
    rng = np.random.default_rng(zlib.crc32(f"{kind}{n_keys}{n}".encode()))
    seq = 0
    for b in range(3):
        d = synth.stock_ticks(seq, n, n_keys, seed=300 + b, rate_per_ms=64)
        d["key"] = _keys(kind, n, n_keys, rng)
        d["symbol"] = d["key"].copy()
        for e in (gpu, ora, rad):
            e.push(0, seq, d["ts"], [d[c] for c in COLS], None, d["key"])
        mg, mo, mr = gpu.poll(), ora.poll(), rad.poll()
        _same(mg, mo)
        _same(mg, mr)
        seq += n
    sg, so, sr = gpu.stats(), ora.stats(), rad.stats()
    for f in ("partials_live", "matches"):
        assert sg[f] == so[f], f
    for f in ("partials_live", "partials_created", "partials_scanned", "matches", "keys_touched",
              "live_at_batch_start", "window_spills"):
        assert sg.get(f) == sr.get(f), f
    for e in (gpu, ora, rad):
        e.close()


def test_tile_grouping_wide_and_null_payloads():
    """two streams: S1 (float/int, with null prices: payload + null word) and S2 (double/long: 4 payload
    words), each pushed through the tile grouping, equal to the radix grouping and the oracle"""
    n_keys, n = 3000, 50000
    cq, gpu, ora = _engines(SHAPES["two_streams"], n_keys, n)
    rad = _radix_engine(SHAPES["two_streams"], n_keys, n)
    rng = np.random.default_rng(7)
    seq = 0
    for b in range(4):
        d = synth.stock_ticks(seq, n, n_keys, seed=400 + b, rate_per_ms=16)
        if b % 2 == 0:
            st, cols = cq.stream_index("S1"), [d["symbol"], d["price"], d["volume"]]
            nulls = [None, (rng.random(n) < 0.1).astype(np.uint8), None]
        else:
            st, cols = cq.stream_index("S2"), [d["symbol"], d["price"].astype(np.float64),
                                              d["volume"].astype(np.int64)]
            nulls = None
        for e in (gpu, ora, rad):
            e.push(st, seq, d["ts"], cols, nulls, d["key"])
        mg = gpu.poll()
        _same(mg, ora.poll())
        _same(mg, rad.poll())
        seq += n
    for e in (gpu, ora, rad):
        e.close()


def test_tile_grouping_device_keys_out_of_range_and_null():
    """device batches: SG_KEY_NULL ids dropped (SG_CFG_NULL_KEYS), an id == n_keys reported at the next poll
    with the valid keys' events processed, as the radix grouping does"""
    dev = torch.device("cuda", 0)
    n_keys, n = 2048, 40000
    flags = sa.native.SG_CFG_NULL_KEYS
    app = sa.parse_app(SHAPES["c2_every_within"])
    cq = sa.compile_query(app, app.queries[0], sa.StringDictionary())
    gpu = sa.NativeEngine(sa.load_hip_library(), "sg_", cq.ir, n_keys=n_keys, max_batch=n, partial_capacity=64,
                          match_capacity=1 << 22, flags=flags)
    rad = _radix_engine(SHAPES["c2_every_within"], n_keys, n, flags=flags)
    rng = np.random.default_rng(11)
    seq = 0
    for b in range(3):
        d = synth.stock_ticks(seq, n, n_keys, seed=500 + b, rate_per_ms=16)
        d["key"][rng.random(n) < 0.05] = sa.native.SG_KEY_NULL
        if b == 1:
            d["key"][123] = n_keys
        t = {k: torch.from_numpy(v.view(np.int32) if v.dtype == np.uint32 else v).to(dev) for k, v in d.items()}
        torch.cuda.synchronize()
        res = []
        for e in (gpu, rad):
            e.push(0, seq, (n, t["ts"].data_ptr(), [t["symbol"].data_ptr(), t["price"].data_ptr(),
                                                    t["volume"].data_ptr()], t["key"].data_ptr()),
                   [0, 1, 2], mem=sa.native.SG_MEM_DEVICE)
            e.synchronize()
            if b == 1:
                with pytest.raises(sa.EngineError, match="n_keys"):
                    e.poll()
                res.append(None)
            else:
                res.append(e.poll())
        if b != 1:
            _same(res[0], res[1])
        seq += n
    assert gpu.stats()["partials_live"] == rad.stats()["partials_live"]
    gpu.close()
    rad.close()


def _engine_env(query, n_keys, max_batch, env, flags=0):
    app = sa.parse_app(query)
    cq = sa.compile_query(app, app.queries[0], sa.StringDictionary())
    saved = {k: os.environ.pop(k, None) for k in ("SG_GROUP_TILES", "SG_BUCKET_GROUP")}
    os.environ.update(env)
    try:
        return sa.NativeEngine(sa.load_hip_library(), "sg_", cq.ir, n_keys=n_keys, max_batch=max_batch,
                               partial_capacity=64, match_capacity=1 << 22, flags=flags)
    finally:
        for k in env:
            os.environ.pop(k, None)
        for k, v in saved.items():
            if v is not None:
                os.environ[k] = v


BUCKET_CASES = CASES + [
    ("hot", 1 << 20, 200000),      # one key's run far beyond the LDS stage (placed directly)
    ("uniform", 3000, 70001),      # three buckets, the last one partial
    ("zipf", 1 << 20, 1 << 18),
]


@pytest.mark.parametrize("kind,n_keys,n", BUCKET_CASES)
@pytest.mark.parametrize("shape", ["c2_every_within", "every_both_within"])
def test_bucket_grouping_vs_oracle_and_radix(kind, n_keys, n, shape):
    """the opt-in bucket grouping (SG_BUCKET_GROUP=1: one radix pass on the bucket bits + the per-bucket split,
    grp_kernels.hip sgd_bucket_split) against the default two-pass radix sort + k_seg_bounds and the oracle"""
    cq, _, ora = _engines(SHAPES[shape], n_keys, n)
    bk = _engine_env(SHAPES[shape], n_keys, n, {"SG_BUCKET_GROUP": "1"})
    rad = _engine_env(SHAPES[shape], n_keys, n, {})
    rng = np.random.default_rng(zlib.crc32(f"b{kind}{n_keys}{n}".encode()))
    seq = 0
    for b in range(3):
        d = synth.stock_ticks(seq, n, n_keys, seed=600 + b, rate_per_ms=64)
        d["key"] = _keys(kind, n, n_keys, rng)
        d["symbol"] = d["key"].copy()
        for e in (bk, ora, rad):
            e.push(0, seq, d["ts"], [d[c] for c in COLS], None, d["key"])
        mb, mo, mr = bk.poll(), ora.poll(), rad.poll()
        _same(mb, mo)
        _same(mb, mr)
        seq += n
    sb, so, sr = bk.stats(), ora.stats(), rad.stats()
    for f in ("partials_live", "matches"):
        assert sb[f] == so[f], f
    for f in ("partials_live", "partials_created", "partials_scanned", "matches", "keys_touched",
              "live_at_batch_start", "window_spills"):
        assert sb.get(f) == sr.get(f), f
    for e in (bk, ora, rad):
        e.close()


def test_bucket_grouping_wide_null_and_device_keys():
    """wide payloads (double/long: 4 words) and null bits through the bucket split, and device batches with
    dropped SG_KEY_NULL ids and one out-of-range id (reported), equal to the two-pass radix grouping"""
    n_keys, n = 5000, 60000
    cq, _, ora = _engines(SHAPES["two_streams"], n_keys, n)
    bk = _engine_env(SHAPES["two_streams"], n_keys, n, {"SG_BUCKET_GROUP": "1"})
    rad = _engine_env(SHAPES["two_streams"], n_keys, n, {})
    rng = np.random.default_rng(8)
    seq = 0
    for b in range(4):
        d = synth.stock_ticks(seq, n, n_keys, seed=700 + b, rate_per_ms=16)
        if b % 2 == 0:
            st, cols = cq.stream_index("S1"), [d["symbol"], d["price"], d["volume"]]
            nulls = [None, (rng.random(n) < 0.1).astype(np.uint8), None]
        else:
            st, cols = cq.stream_index("S2"), [d["symbol"], d["price"].astype(np.float64),
                                              d["volume"].astype(np.int64)]
            nulls = None
        for e in (bk, ora, rad):
            e.push(st, seq, d["ts"], cols, nulls, d["key"])
        mb = bk.poll()
        _same(mb, ora.poll())
        _same(mb, rad.poll())
        seq += n
    for e in (bk, ora, rad):
        e.close()
    dev = torch.device("cuda", 0)
    n_keys, n = 4097, 40000
    flags = sa.native.SG_CFG_NULL_KEYS
    bk = _engine_env(SHAPES["c2_every_within"], n_keys, n, {"SG_BUCKET_GROUP": "1"}, flags)
    rad = _engine_env(SHAPES["c2_every_within"], n_keys, n, {}, flags)
    seq = 0
    for b in range(3):
        d = synth.stock_ticks(seq, n, n_keys, seed=800 + b, rate_per_ms=16)
        d["key"][rng.random(n) < 0.05] = sa.native.SG_KEY_NULL
        if b == 1:
            d["key"][321] = n_keys
        t = {k: torch.from_numpy(v.view(np.int32) if v.dtype == np.uint32 else v).to(dev) for k, v in d.items()}
        torch.cuda.synchronize()
        res = []
        for e in (bk, rad):
            e.push(0, seq, (n, t["ts"].data_ptr(), [t["symbol"].data_ptr(), t["price"].data_ptr(),
                                                    t["volume"].data_ptr()], t["key"].data_ptr()),
                   [0, 1, 2], mem=sa.native.SG_MEM_DEVICE)
            e.synchronize()
            if b == 1:
                with pytest.raises(sa.EngineError, match="n_keys"):
                    e.poll()
                res.append(None)
            else:
                res.append(e.poll())
        if b != 1:
            _same(res[0], res[1])
        seq += n
    assert bk.stats()["partials_live"] == rad.stats()["partials_live"]
    bk.close()
    rad.close()
