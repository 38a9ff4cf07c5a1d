"""Synthetic stock-tick streams, stateless per event so any slice can be regenerated.

Schema `StockStream (symbol string, price float, volume int)` (siddhi-samples PartitionSample.java:41)
plus the event timestamp.  Every field of event i is a function of (seed, i) through splitmix64:

    key    = h0 % n_keys                      (uniform; symbol id == key id)
    price  = float32(10 + 30 * u),  u = (h1 >> 40) / 2^24      (price > 20 for ~2/3 of events)
    volume = 1 + h2 % 2000
    ts     = t0 + i // rate_per_ms            (global, non-decreasing)

(The survey's per-key random walk is replaced by i.i.d. prices so that generation is stateless and
identical for the host baseline and the device run; documented in DESIGN.md.)
"""
from __future__ import annotations

import numpy as np

C2_QUERY = """
define stream StockStream (symbol string, price float, volume int);
partition with (symbol of StockStream)
begin
  @info(name = 'query1')
  from every e1=StockStream[price > 20] -> e2=StockStream[price > e1.price]
       within 10 sec
  select e1.symbol as symbol, e1.price as price1, e2.price as price2, e2.price - e1.price as d
  insert into OutputStream;
end;
"""

C1_QUERY = """
define stream StockStream (symbol string, price float, volume int);
@info(name = 'query1')
from every e1=StockStream[price > 20] -> e2=StockStream[price > e1.price]
     within 10 sec
select e1.symbol as symbol, e1.price as price1, e2.price as price2, e2.price - e1.price as d
insert into OutputStream;
"""

# BASELINE configs[2] (C3): strict sequence with counting plus logical or (SiddhiQL counting syntax <m:n>)
C3_QUERY = """
define stream StockStream (symbol string, price float, volume int);
partition with (symbol of StockStream)
begin
  @info(name = 'query1')
  from every e1=StockStream[price > 20]<2:5>, e2=StockStream[price > e1[last].price] or e3=StockStream[volume > 1000]
       within 10 sec
  select e1[0].price as p0, e1[last].price as plast, e2.price as p2, e3.volume as v3
  insert into OutputStream;
end;
"""

# C3 with <1:5>: under the reference's SEQUENCE semantics a start count state with min 2 is cleared by
# StateStreamRuntime.resetAndUpdate (StateStreamRuntime.java:81-88 -> StreamPreStateProcessor.resetState,
# StreamPreStateProcessor.java:288-305) before every event, and CountPostStateProcessor only re-adds the
# partial once it holds min events (CountPostStateProcessor.java:39-66), so C3 as written never matches;
# this variant is the same shape with matches, benchmarked beside it
C3_MIN1_QUERY = C3_QUERY.replace("<2:5>", "<1:5>")

# BASELINE configs[2] names "logical and/or": the C3 shape with the logical AND (e2 and e3 both arrive, in
# either order, before the sequence moves on; LogicalPreStateProcessor.java:43-202); under SEQUENCE semantics a
# match needs both filters on one event (cnt_kernels.hip runs it)
C3_AND_QUERY = C3_MIN1_QUERY.replace(" or e3=", " and e3=")

# a 3-state pattern (a chain past the two-state kernel's shape, StreamPreStateProcessor.java:364-403 per state),
# on the general kernel
P3_QUERY = """
define stream StockStream (symbol string, price float, volume int);
partition with (symbol of StockStream)
begin
  @info(name = 'query1')
  from every e1=StockStream[price > 20] -> e2=StockStream[price > e1.price] -> e3=StockStream[price > e2.price]
       within 10 sec
  select e1.price as p1, e2.price as p2, e3.price as p3
  insert into OutputStream;
end;
"""

# BASELINE configs[3] (C4): absent state with a long within, playback clock
C4_QUERY = """
@app:playback
define stream StockStream (symbol string, price float, volume int);
partition with (symbol of StockStream)
begin
  @info(name = 'query1')
  from every e1=StockStream[price > 20] -> not StockStream[price > e1.price] for 30 sec
       within 60 sec
  select e1.symbol as symbol, e1.price as price
  insert into OutputStream;
end;
"""

T0 = 1_700_000_000_000
SEED = 0x5EED5EED

_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)
_G = np.uint64(0x9E3779B97F4A7C15)


def splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x + _G
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def stock_ticks(start: int, n: int, n_keys: int, seed: int = SEED, rate_per_ms: int = 2000, t0: int = T0):
    """Events [start, start + n) of the stream: dict of numpy arrays (key, ts, symbol, price, volume)."""
    i = np.arange(start, start + n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        base = np.uint64(seed) * np.uint64(0x100000001B3) if seed else np.uint64(0)
    with np.errstate(over="ignore"):
        s = (i * np.uint64(3) + base)
        h0 = splitmix64(s)
        h1 = splitmix64(s + np.uint64(1))
        h2 = splitmix64(s + np.uint64(2))
    key = (h0 % np.uint64(n_keys)).astype(np.uint32)
    u = (h1 >> np.uint64(40)).astype(np.float64) / float(1 << 24)
    price = (10.0 + 30.0 * u).astype(np.float32)
    volume = (np.uint64(1) + h2 % np.uint64(2000)).astype(np.int32)
    ts = (np.int64(t0) + (i // np.uint64(rate_per_ms)).astype(np.int64)).astype(np.int64)
    return {"key": key, "ts": ts, "symbol": key.copy(), "price": price, "volume": volume}


def _i64(u: int) -> int:
    """a uint64 constant as the int64 with the same bits (torch has no uint64 arithmetic)"""
    return u - (1 << 64) if u >= (1 << 63) else u


def _srl(torch, x, n: int):
    """logical right shift of int64 bit patterns"""
    return (x >> n) & ((1 << (64 - n)) - 1)


def splitmix64_torch(torch, x):
    """splitmix64 over int64 tensors holding uint64 bit patterns (wrapping multiplication)"""
    z = x + _i64(0x9E3779B97F4A7C15)
    z = (z ^ _srl(torch, z, 30)) * _i64(0xBF58476D1CE4E5B9)
    z = (z ^ _srl(torch, z, 27)) * _i64(0x94D049BB133111EB)
    return z ^ _srl(torch, z, 31)


def stock_ticks_torch(torch, start: int, n: int, n_keys: int, device, seed: int = SEED, rate_per_ms: int = 2000,
                      t0: int = T0):
    """stock_ticks generated on `device` (bit-identical values; n_keys a power of two): dict of tensors key,
    symbol (int32 bit patterns of the uint32 ids), ts (int64), price (float32), volume (int32).  The bench
    builds its HBM-resident batches with it (the numpy generator takes seconds per 2^24-event batch)."""
    if n_keys & (n_keys - 1):
        raise ValueError("stock_ticks_torch: n_keys must be a power of two")
    i = torch.arange(start, start + n, dtype=torch.int64, device=device)
    base = _i64((seed * 0x100000001B3) & ((1 << 64) - 1)) if seed else 0
    s = i * 3 + base
    h0 = splitmix64_torch(torch, s)
    h1 = splitmix64_torch(torch, s + 1)
    h2 = splitmix64_torch(torch, s + 2)
    key = (h0 & (n_keys - 1)).to(torch.int32)
    u = _srl(torch, h1, 40).to(torch.float64) / float(1 << 24)
    price = (10.0 + 30.0 * u).to(torch.float32)
    # h2 mod 2000 of the unsigned value: 2 * ((h2 >>> 1) mod 1000) + (h2 & 1)
    volume = (1 + 2 * (_srl(torch, h2, 1) % 1000) + (h2 & 1)).to(torch.int32)
    ts = t0 + torch.div(i, rate_per_ms, rounding_mode="floor")
    return {"key": key, "ts": ts, "symbol": key.clone(), "price": price, "volume": volume}


def burst_ticks(start_ms: int, n_ms: int, n_keys: int, burst: int, seed: int = SEED, t0: int = T0):
    """C4 input: millisecond t carries `burst` events of ONE key (key = h(t) % n_keys), timestamp
    t0 + t.  Timer due times of different keys then never coincide, which keeps the reference's
    Scheduler collapse quirk out of the input.  Stateless per event index."""
    t = np.repeat(np.arange(start_ms, start_ms + n_ms, dtype=np.uint64), burst)
    i = np.arange(start_ms * burst, (start_ms + n_ms) * burst, dtype=np.uint64)
    with np.errstate(over="ignore"):
        base = np.uint64(seed) * np.uint64(0x100000001B3) if seed else np.uint64(0)
        hk = splitmix64(t * np.uint64(7) + base)
        s = i * np.uint64(3) + base + np.uint64(0x51)
        h1 = splitmix64(s + np.uint64(1))
        h2 = splitmix64(s + np.uint64(2))
    key = (hk % np.uint64(n_keys)).astype(np.uint32)
    u = (h1 >> np.uint64(40)).astype(np.float64) / float(1 << 24)
    price = (10.0 + 30.0 * u).astype(np.float32)
    volume = (np.uint64(1) + h2 % np.uint64(2000)).astype(np.int32)
    ts = (np.int64(t0) + t.astype(np.int64)).astype(np.int64)
    return {"key": key, "ts": ts, "symbol": key.copy(), "price": price, "volume": volume}


def absent_deep_ticks(start_ms: int, n_ms: int, n_keys: int, burst: int, seed: int = SEED, t0: int = T0,
                      period_ms: int = 600_000):
    """Deep absent state (C4 with hundreds of live partials per key): as burst_ticks, millisecond t carries
    `burst` events of ONE key (distinct timer due times across keys), but each key's
    price falls steadily along a sawtooth of `period_ms` (key-specific phase) and, inside a burst, with the
    event index: `not S[price > e1.price]` then almost never fires on an event, so every partial lives until
    its `for` timer (or `within` expiry), and each key's sawtooth jump kills its whole list at once."""
    t = np.repeat(np.arange(start_ms, start_ms + n_ms, dtype=np.uint64), burst)
    j = np.tile(np.arange(burst, dtype=np.float64), n_ms)
    i = np.arange(start_ms * burst, (start_ms + n_ms) * burst, dtype=np.uint64)
    with np.errstate(over="ignore"):
        base = np.uint64(seed) * np.uint64(0x100000001B3) if seed else np.uint64(0)
        hk = splitmix64(t * np.uint64(7) + base)
        h2 = splitmix64(i * np.uint64(3) + base + np.uint64(0x53))
    key = (hk % np.uint64(n_keys)).astype(np.uint32)
    phase = (splitmix64(key.astype(np.uint64) + base) % np.uint64(period_ms)).astype(np.float64)
    frac = ((t.astype(np.float64) + phase) % period_ms) / period_ms
    price = (21.0 + 60.0 * (1.0 - frac) - 1e-3 * j).astype(np.float32)
    volume = (np.uint64(1) + h2 % np.uint64(2000)).astype(np.int32)
    ts = (np.int64(t0) + t.astype(np.int64)).astype(np.int64)
    return {"key": key, "ts": ts, "symbol": key.copy(), "price": price, "volume": volume}


# ---- SURVEY §8(d) workload variants: Zipf s=1.1 keys ("reported separately") and the per-key random-walk price ----
ZIPF_S = 1.1
_ZIPF_CDF = {}
_KEY_MIX = 0x9E3779B1  # odd: rank -> key id is a bijection of [0, 2^b) (hot keys spread over tiles and waves)


def zipf_cdf(n_keys: int, s: float = ZIPF_S) -> np.ndarray:
    """cumulative probabilities of Zipf ranks 1..n_keys (float64)"""
    k = (n_keys, s)
    if k not in _ZIPF_CDF:
        w = 1.0 / np.power(np.arange(1, n_keys + 1, dtype=np.float64), s)
        c = np.cumsum(w)
        _ZIPF_CDF[k] = c / c[-1]
    return _ZIPF_CDF[k]


def _rank_to_key(rank, n_keys: int):
    """rank r (0 = hottest) -> key id: (r * odd) mod n_keys for a power-of-two n_keys, else r"""
    if n_keys & (n_keys - 1):
        return rank
    return (rank * _KEY_MIX) & (n_keys - 1)


def zipf_ticks(start: int, n: int, n_keys: int, seed: int = SEED, rate_per_ms: int = 2000, t0: int = T0, s: float = ZIPF_S):
    """stock_ticks with Zipf(s) partition keys: key = bijection(rank), rank ~ Zipf over n_keys ranks (the hottest key
    ~12 % of the events at s = 1.1, 2^20 keys); the other fields as stock_ticks"""
    d = stock_ticks(start, n, n_keys, seed, rate_per_ms, t0)
    i = np.arange(start, start + n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        base = np.uint64(seed) * np.uint64(0x100000001B3) if seed else np.uint64(0)
        h = splitmix64(i * np.uint64(3) + base + np.uint64(0x7A))
    u = (h >> np.uint64(11)).astype(np.float64) / float(1 << 53)
    rank = np.minimum(np.searchsorted(zipf_cdf(n_keys, s), u, side="right"), n_keys - 1).astype(np.uint64)
    key = _rank_to_key(rank, n_keys).astype(np.uint32)
    d["key"] = key
    d["symbol"] = key.copy()
    return d


def zipf_ticks_torch(torch, start: int, n: int, n_keys: int, device, seed: int = SEED, rate_per_ms: int = 2000,
                     t0: int = T0, s: float = ZIPF_S):
    """zipf_ticks on the device (bit-identical keys: the same splitmix draws and CDF table)"""
    d = stock_ticks_torch(torch, start, n, n_keys, device, seed, rate_per_ms, t0)
    i = torch.arange(start, start + n, dtype=torch.int64, device=device)
    base = _i64((seed * 0x100000001B3) & ((1 << 64) - 1)) if seed else 0
    h = splitmix64_torch(torch, i * 3 + base + 0x7A)
    u = _srl(torch, h, 11).to(torch.float64) / float(1 << 53)
    cdf = torch.from_numpy(zipf_cdf(n_keys, s)).to(device)
    rank = torch.clamp(torch.searchsorted(cdf, u, right=True), max=n_keys - 1)
    key = ((rank * _KEY_MIX) & (n_keys - 1)).to(torch.int32)
    d["key"] = key
    d["symbol"] = key.clone()
    return d


class RandomWalk:
    """SURVEY §8(d) price model: per key p <- clamp(p + 0.25 N(0,1), 1, 100) rounded to f32 at each of the key's
    events, initial U[10, 40] per key.  Stateful across batches (call step() on consecutive batches in order);
    deterministic: the increments are Box-Muller normals of splitmix64 draws of the global event index.  Works on
    numpy arrays or (with `torch`) on device tensors."""

    def __init__(self, n_keys: int, seed: int = SEED, torch=None, device=None):
        self.torch, self.device = torch, device
        k = np.arange(n_keys, dtype=np.uint64)
        with np.errstate(over="ignore"):
            base = np.uint64(seed) * np.uint64(0x100000001B3) if seed else np.uint64(0)
            h = splitmix64(k * np.uint64(5) + base + np.uint64(0x3F))
        p = (10.0 + 30.0 * ((h >> np.uint64(40)).astype(np.float64) / float(1 << 24))).astype(np.float32)
        self.seed = seed
        self.p = torch.from_numpy(p).to(device) if torch is not None else p

    def _inc(self, start: int, n: int):
        i = np.arange(start, start + n, dtype=np.uint64)
        with np.errstate(over="ignore"):
            base = np.uint64(self.seed) * np.uint64(0x100000001B3) if self.seed else np.uint64(0)
            h1 = splitmix64(i * np.uint64(3) + base + np.uint64(0x91))
            h2 = splitmix64(i * np.uint64(3) + base + np.uint64(0x92))
        u1 = ((h1 >> np.uint64(11)).astype(np.float64) + 1.0) / float(1 << 53)   # (0, 1]
        u2 = (h2 >> np.uint64(11)).astype(np.float64) / float(1 << 53)
        return 0.25 * np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * np.pi * u2)

    def step(self, key, start: int):
        """the prices of events [start, start + n) whose keys are `key` (arrival order); advances the walk"""
        t = self.torch
        n = int(key.shape[0])
        inc = self._inc(start, n)
        if t is not None:
            inc = t.from_numpy(inc).to(self.device)
            k = key.to(t.int64)
            order = t.argsort(k, stable=True)
            ks = k[order]
            first = t.ones(n, dtype=t.bool, device=self.device)
            first[1:] = ks[1:] != ks[:-1]
            pos = t.arange(n, device=self.device)
            seg0 = t.cummax(t.where(first, pos, t.zeros_like(pos)), 0).values
            rank = t.empty_like(pos)
            rank[order] = pos - seg0
            price = t.empty(n, dtype=t.float32, device=self.device)
            for r in range(int(rank.max().item()) + 1 if n else 0):
                idx = t.nonzero(rank == r).flatten()
                kk = k[idx]
                v = t.clamp(self.p[kk].to(t.float64) + inc[idx], 1.0, 100.0).to(t.float32)
                self.p[kk] = v
                price[idx] = v
            return price
        k = np.asarray(key).astype(np.int64)
        order = np.argsort(k, kind="stable")
        ks = k[order]
        first = np.ones(n, dtype=bool)
        first[1:] = ks[1:] != ks[:-1]
        pos = np.arange(n)
        seg0 = np.maximum.accumulate(np.where(first, pos, 0))
        rank = np.empty(n, dtype=np.int64)
        rank[order] = pos - seg0
        price = np.empty(n, dtype=np.float32)
        for r in range(int(rank.max()) + 1 if n else 0):
            idx = np.nonzero(rank == r)[0]
            kk = k[idx]
            v = np.clip(self.p[kk].astype(np.float64) + inc[idx], 1.0, 100.0).astype(np.float32)
            self.p[kk] = v
            price[idx] = v
        return price
