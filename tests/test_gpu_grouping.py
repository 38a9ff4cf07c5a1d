"""The hand-written key grouping (part_kernels.hip) against the oracle, bit-exact, both ways the two-state engine
takes it:

- fused (the default where the batch density allows it): two stable 6-bit passes group the batch by key tile
  (the 256 keys of one advance workgroup) and the advance kernel splits its tile by key in LDS
  (p2_jit.hip tile_split_lds); tiles too large for LDS are split into HBM by the same workgroup and walked by
  the HBM pass (tile_split_glb), keys that stop early write their runs for the HBM pass to resume;
- sorted (SG_NO_FUSED=1, and every batch too dense per tile): LSD passes of <= 8 bits to a key-sorted payload
  + per-key bounds.

Skewed streams (Zipf, one hot key: tiles far beyond the LDS region), sparse keys (most tiles empty), partial
last tiles, a single-pass tile grouping (<= 256 tiles), the register window forced small (stops and resumes),
the LDS region forced small (every tile split in HBM), wide and null payloads, dropped SG_KEY_NULL and
out-of-range ids on device batches.  Reference: PartitionStreamReceiver.java:175-260 (the key-run grouping)."""
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
STATS = ("partials_live", "partials_created", "partials_scanned", "matches", "keys_touched", "live_at_batch_start")


def _engine_env(query, n_keys, max_batch, env, flags=0):
    app = sa.parse_app(query)
    cq = sa.compile_query(app, app.queries[0], sa.StringDictionary())
    saved = {k: os.environ.pop(k, None) for k in env}
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
    ("uniform", 1 << 16, 1 << 18),    # fused, 256 tiles: the one-pass tile grouping
    ("uniform", 1 << 14, 1 << 18),    # fused at the C2 density (16 events per key, ~4096 per tile)
    ("zipf", 1 << 16, 1 << 18),       # fused, the head tiles split in HBM
    ("hot", 50000, 100003),           # fused, one tile of ~50K events split in HBM
    ("sparse", 1 << 20, 70000),       # fused, 4096 tiles (two passes), most empty
    ("uniform", 1000, 2000),          # fused, 4 tiles, the last one partial
    ("uniform", 1000, 65537),         # too dense per tile: the sorted grouping
    ("uniform", 1 << 20, 1 << 16),    # K at the fused grouping's limit
]


@pytest.mark.parametrize("kind,n_keys,n", CASES)
@pytest.mark.parametrize("shape", ["c2_every_within", "every_both_within"])
def test_grouping_fused_vs_sorted_vs_oracle(kind, n_keys, n, shape):
    cq, gpu, ora = _engines(SHAPES[shape], n_keys, n)
    srt = _engine_env(SHAPES[shape], n_keys, n, {"SG_NO_FUSED": "1"})
    rng = np.random.default_rng(zlib.crc32(f"{kind}{n_keys}{n}".encode()))
    seq = 0
    for b in range(3):
        d = synth.stock_ticks(seq, n, n_keys, seed=300 + b, rate_per_ms=64)
        d["key"] = _keys(kind, n, n_keys, rng)
        d["symbol"] = d["key"].copy()
        for e in (gpu, ora, srt):
            e.push(0, seq, d["ts"], [d[c] for c in COLS], None, d["key"])
        mg, mo, ms = gpu.poll(), ora.poll(), srt.poll()
        _same(mg, mo)
        _same(mg, ms)
        seq += n
    sg, so, ss = gpu.stats(), ora.stats(), srt.stats()
    for f in ("partials_live", "matches"):
        assert sg[f] == so[f], f
    for f in STATS:
        assert sg.get(f) == ss.get(f), f
    for e in (gpu, ora, srt):
        e.close()


@pytest.mark.parametrize("env", [{"SGD_REG_SLOTS": "2"}, {"SGD_STAGE_CHUNKS": "64"}, {"SGD_REG_SLOTS": "3",
                                                                                       "SGD_STAGE_CHUNKS": "64"}])
@pytest.mark.parametrize("shape", ["c2_every_within", "every_both_within", "no_every"])
def test_fused_grouping_hbm_paths(env, shape, monkeypatch):
    """the fused grouping's hand-offs to the HBM pass: a register window of 2-3 slots stops most keys (their runs,
    split in LDS, written to the key-sorted payload for the HBM pass to resume), an LDS region of 64 chunks makes
    every tile go through the split in HBM; both equal the sorted grouping and the oracle"""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    n_keys, n = 1 << 14, 1 << 17
    cq, gpu, ora = _engines(SHAPES[shape], n_keys, n)
    srt = _engine_env(SHAPES[shape], n_keys, n, {"SG_NO_FUSED": "1"})
    seq = 0
    for b in range(3):
        d = synth.stock_ticks(seq, n, n_keys, seed=900 + b, rate_per_ms=32)
        for e in (gpu, ora, srt):
            e.push(0, seq, d["ts"], [d[c] for c in COLS], None, d["key"])
        mg = gpu.poll()
        _same(mg, ora.poll())
        _same(mg, srt.poll())
        seq += n
    sg, ss = gpu.stats(), srt.stats()
    # (window_spills counts the keys each path stops or spills: with the LDS region forced small the fused tiles are
    # walked by the staged pass from HBM, the sorted ones by the HBM pass, so it differs there by design)
    for f in STATS + (() if "SGD_STAGE_CHUNKS" in env else ("window_spills",)):
        assert sg.get(f) == ss.get(f), f
    assert sg["matches"] > 0
    for e in (gpu, ora, srt):
        e.close()


def test_grouping_wide_and_null_payloads():
    """two streams: S1 (float/int, with null prices: payload + null word) and S2 (double/long: 4 payload
    words), fused and sorted, equal to the oracle"""
    n_keys, n = 1 << 14, 1 << 16
    cq, gpu, ora = _engines(SHAPES["two_streams"], n_keys, n)
    srt = _engine_env(SHAPES["two_streams"], n_keys, n, {"SG_NO_FUSED": "1"})
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
        for e in (gpu, ora, srt):
            e.push(st, seq, d["ts"], cols, nulls, d["key"])
        mg = gpu.poll()
        _same(mg, ora.poll())
        _same(mg, srt.poll())
        seq += n
    for e in (gpu, ora, srt):
        e.close()


@pytest.mark.parametrize("fused", [True, False])
def test_grouping_device_keys_out_of_range_and_null(fused):
    """device batches: SG_KEY_NULL ids dropped (SG_CFG_NULL_KEYS), an id == n_keys reported at the next poll
    with the valid keys' events processed; fused and sorted groupings agree"""
    dev = torch.device("cuda", 0)
    n_keys, n = 1 << 14, 1 << 16
    flags = sa.native.SG_CFG_NULL_KEYS
    gpu = _engine_env(SHAPES["c2_every_within"], n_keys, n, {} if fused else {"SG_NO_FUSED": "1"}, flags)
    ref = _engine_env(SHAPES["c2_every_within"], n_keys, n, {"SG_NO_FUSED": "1"} if fused else {}, flags)
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
        for e in (gpu, ref):
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
    assert gpu.stats()["partials_live"] == ref.stats()["partials_live"]
    gpu.close()
    ref.close()


def test_fused_grouping_is_the_c2_path():
    """at the C2 density the engine reports the fused grouping (no library sort on the path)"""
    n_keys, n = 1 << 14, 1 << 18
    gpu = _engine_env(SHAPES["c2_every_within"], n_keys, n, {})
    d = synth.stock_ticks(0, n, n_keys, seed=1, rate_per_ms=64)
    gpu.push(0, 0, d["ts"], [d[c] for c in COLS], None, d["key"])
    gpu.poll()
    desc = gpu.describe()
    assert "k_tile_bounds" in desc and "key split in LDS" in desc, desc
    assert "rocPRIM" not in desc
    gpu.close()
