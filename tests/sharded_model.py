"""Test model: the multi-device fan-out over N engines of any backend, in Python.

The product's multi-device path is the C-ABI's own fan-out (sg_config.n_devices, csrc/sg_sharded.cpp: one
sg_engine handle over one engine per device, what a JNI shim bound to siddhi_gpu.h gets; SiddhiManager(devices=..)
uses it).  This module restates the same splitting / seq mapping / merge over NativeEngine objects so that
the CPU tests can run it over the oracle (tests/test_sharded.py) and the GPU tests can compare both.

`ShardedEngine` has the interface of `NativeEngine` (push / poll / advance_time / reset_keys / snapshot /
restore / stats) and drives one engine per device.  Partition key ids are dense (first-seen order of the
key dictionary, so consecutive ids are unrelated keys): shard = key % N owns the key and sees it as local
id key // N, dense in [0, ceil(n_keys / N)).  No processor reads another key's state
(PartitionStateHolder.java:43-49), so each shard runs its keys exactly as one engine would.

Each host batch is split stably by owner (per key the arrival order is kept); a shard numbers the events
it receives with its own arrival seqs and keeps the map back to the global seqs, so matches leave poll()
with the global trigger / slot seqs and global key ids, merged into the single engine's order: batch
matches by (trigger seq, emission order) — per trigger all matches come from the one shard that owns the
trigger's key — and timer matches by (fire time, key) (the reference's listener order for one absent
state; two keys due at the same time are refused by every shard).  The playback / wall clock
is global: every shard gets the same advance_time sequence.  Unpartitioned queries do not shard (one
key's NFA is sequential): they run on the first device (replicas only).

Pushes and polls of the shards run concurrently, one host thread per device (the C-ABI allows one
caller thread per engine; ctypes releases the GIL during the calls).
"""
from __future__ import annotations

import struct
from concurrent.futures import ThreadPoolExecutor

import numpy as np

import importlib

_native = importlib.import_module("siddhi-1_amd.native")
SG_MEM_HOST, SG_NULL_SEQ, Matches, NativeEngine = (_native.SG_MEM_HOST, _native.SG_NULL_SEQ, _native.Matches,
                                                   _native.NativeEngine)

TIMER_SEQ = np.uint64(0xFFFFFFFFFFFFFFFF)
BLANK_SEQ = np.uint64(0xFFFFFFFFFFFFFFFE)
_SNAP = b"SGSH\x01\x00\x00\x00"


class ShardedEngine:
    def __init__(self, lib, prefix, ir: bytes, n_keys=1, devices=(0,), max_batch=1 << 16, partial_capacity=64,
                 match_capacity=1 << 20, flags=0):
        self.n_keys = n_keys
        self.N = len(devices) if n_keys > 1 else 1
        local = (n_keys + self.N - 1) // self.N
        self.shards = [NativeEngine(lib, prefix, ir, n_keys=local if n_keys > 1 else 1, max_batch=max_batch,
                                    partial_capacity=partial_capacity, match_capacity=match_capacity, device=d,
                                    flags=flags)
                       for d in list(devices)[:self.N]]
        # per shard: global arrival seq of each local arrival seq (local seqs are dense: 0, 1, 2, ...)
        self.gmap = [np.zeros(1024, dtype=np.uint64) for _ in range(self.N)]
        self.next_local = [0] * self.N
        self.pool = ThreadPoolExecutor(max_workers=self.N) if self.N > 1 else None

    # -- helpers -------------------------------------------------------------------------------------
    def _append(self, r, g):
        """record the global seqs g of the next len(g) local seqs of shard r"""
        n0 = self.next_local[r]
        need = n0 + len(g)
        if need > len(self.gmap[r]):
            grown = np.zeros(max(need, 2 * len(self.gmap[r])), dtype=np.uint64)
            grown[:n0] = self.gmap[r][:n0]
            self.gmap[r] = grown
        self.gmap[r][n0:need] = g
        self.next_local[r] = need
        return n0

    def _map(self, r, local):
        """global seqs of shard r's local arrival seqs (null / blank / timer markers pass through)"""
        local = np.asarray(local, dtype=np.uint64)
        out = local.copy()
        sel = local < BLANK_SEQ
        out[sel] = self.gmap[r][local[sel].astype(np.int64)]
        return out

    def _each(self, fn):
        if self.pool is None:
            return [fn(0)]
        return list(self.pool.map(fn, range(self.N)))

    # -- NativeEngine interface ------------------------------------------------------------------------
    def set_projection(self, *prog):
        for s in self.shards:
            s.set_projection(*prog)
    def push(self, stream, seq_base, ts, cols, nulls=None, key=None, mem=SG_MEM_HOST):
        if mem != SG_MEM_HOST:
            raise ValueError("ShardedEngine takes host batches (the device path is bench.py's RCCL reshard)")
        ts = np.ascontiguousarray(ts, dtype=np.int64)
        n = len(ts)
        if self.N == 1:
            base = self._append(0, np.arange(seq_base, seq_base + n, dtype=np.uint64))
            self.shards[0].push(stream, base, ts, cols, nulls, key)
            return
        key = np.ascontiguousarray(key, dtype=np.uint32)
        if len(key) and int(key.max()) >= self.n_keys:
            raise ValueError("key id outside [0, n_keys)")
        owner = key % np.uint32(self.N)
        parts = []
        for r in range(self.N):
            idx = np.nonzero(owner == r)[0]          # stable: arrival order within the shard
            if len(idx) == 0:
                parts.append(None)
                continue
            parts.append((self._append(r, np.uint64(seq_base) + idx.astype(np.uint64)), idx))

        def run(r):
            if parts[r] is None:
                return
            base, idx = parts[r]
            sub = [np.ascontiguousarray(c[idx]) for c in cols]
            subn = [np.ascontiguousarray(x[idx]) if x is not None else None for x in nulls] if nulls else None
            self.shards[r].push(stream, base, ts[idx], sub, subn, key[idx] // np.uint32(self.N))
        self._each(run)

    def poll(self) -> Matches:
        got = self._each(lambda r: self.shards[r].poll())
        parts = []
        for r, m in enumerate(got):
            if len(m) == 0:
                continue
            trig = m.trigger_seq.copy()
            timer = trig == TIMER_SEQ
            trig[~timer] = self._map(r, trig[~timer])
            slot = m.slot_seq.copy()
            live = slot != SG_NULL_SEQ
            slot[live] = self._map(r, slot[live])
            key = (m.key.astype(np.uint64) * np.uint64(self.N) + np.uint64(r)).astype(np.uint32) \
                if self.N > 1 else m.key
            parts.append(Matches(trig, key, m.ts.copy(), slot, m.chain_len.copy(), m.proj_value, m.proj_null))
        if not parts:
            return got[0] if got else Matches(np.zeros(0, np.uint64), np.zeros(0, np.uint32), np.zeros(0, np.int64),
                                             np.zeros((0, 1, 1), np.uint64), np.zeros((0, 1), np.uint32))
        w = max(p.slot_seq.shape[2] for p in parts)
        for i, p in enumerate(parts):      # the chain dimension padded to the widest shard's
            if p.slot_seq.shape[2] < w:
                pad = np.full(p.slot_seq.shape[:2] + (w - p.slot_seq.shape[2],), SG_NULL_SEQ, dtype=np.uint64)
                parts[i] = Matches(p.trigger_seq, p.key, p.ts, np.concatenate([p.slot_seq, pad], axis=2), p.chain_len,
                                   p.proj_value, p.proj_null)
        cat = Matches(*[np.concatenate([getattr(p, f) for p in parts]) for f in
                        ("trigger_seq", "key", "ts", "slot_seq", "chain_len")])
        if parts[0].proj_value is not None:
            cat.proj_value = np.concatenate([p.proj_value for p in parts], axis=1)
            cat.proj_null = np.concatenate([p.proj_null for p in parts], axis=1)
        pos = np.arange(len(cat.trigger_seq))
        timer = cat.trigger_seq == TIMER_SEQ
        # timer matches first (a poll after advance_time holds only those), by (fire time, key); batch
        # matches by trigger seq; each stable in the shards' own emission order
        primary = np.where(timer, np.int64(-1), 0)
        k1 = np.where(timer, cat.ts, cat.trigger_seq.astype(np.int64))
        k2 = np.where(timer, cat.key.astype(np.int64), 0)
        order = np.lexsort((pos, k2, k1, primary))
        return Matches(cat.trigger_seq[order], cat.key[order], cat.ts[order], cat.slot_seq[order],
                       cat.chain_len[order], None if cat.proj_value is None else cat.proj_value[:, order],
                       None if cat.proj_null is None else cat.proj_null[:, order])

    def advance_time(self, now):
        self._each(lambda r: self.shards[r].advance_time(now))

    def synchronize(self):
        self._each(lambda r: self.shards[r].synchronize())

    def reset_keys(self, keys):
        k = np.ascontiguousarray(keys, dtype=np.uint32)
        if self.N == 1:
            self.shards[0].reset_keys(k)
            return
        if len(k) and int(k.max()) >= self.n_keys:
            raise ValueError("key id outside [0, n_keys)")
        self._each(lambda r: self.shards[r].reset_keys(k[k % np.uint32(self.N) == r] // np.uint32(self.N)))

    def stats(self):
        out = {}
        for s in self._each(lambda r: self.shards[r].stats()):
            for k, v in s.items():
                out[k] = out.get(k, 0) + v
        return out

    def snapshot(self) -> bytes:
        imgs = self._each(lambda r: self.shards[r].snapshot())
        parts = [_SNAP, struct.pack("<I", self.N)]
        for r, img in enumerate(imgs):
            parts.append(struct.pack("<QQ", len(img), self.next_local[r]))
            parts.append(img)
            parts.append(self.gmap[r][:self.next_local[r]].tobytes())
        return b"".join(parts)

    def restore(self, image: bytes):
        if image[:8] != _SNAP:
            raise ValueError("not a snapshot of a sharded engine")
        (n,) = struct.unpack_from("<I", image, 8)
        if n != self.N:
            raise ValueError("snapshot of a different shard count")
        off, imgs, maps, nxt = 12, [], [], []
        for _ in range(n):
            ln, nl = struct.unpack_from("<QQ", image, off)
            off += 16
            imgs.append(image[off:off + ln])
            off += ln
            maps.append(np.frombuffer(image, dtype=np.uint64, count=nl, offset=off).copy())
            off += 8 * nl
            nxt.append(nl)
        self._each(lambda r: self.shards[r].restore(imgs[r]))
        self.gmap = [np.concatenate([m, np.zeros(1024, np.uint64)]) for m in maps]
        self.next_local = nxt

    def state_export(self) -> bytes:
        """one state document over every shard (state_doc.py): keys and event seqs mapped to global ids"""
        sd = importlib.import_module("siddhi-1_amd.state_doc")
        docs = [sd.parse(b) for b in self._each(lambda r: self.shards[r].state_export())]
        out = sd.StateDoc(docs[0].n_procs, docs[0].n_slots, docs[0].desc, docs[0].now, docs[0].last_event_ts,
                          max(d.clock_flags for d in docs))
        for r, d in enumerate(docs):
            for k in d.keys:
                if self.N > 1:
                    k.key = k.key * self.N + r
                for ev in k.streams:
                    if ev.seq < int(BLANK_SEQ):
                        ev.seq = int(self.gmap[r][ev.seq])
                out.keys.append(k)
        out.keys.sort(key=lambda k: k.key)
        return sd.write(out)

    def state_import(self, doc: bytes):
        """split a state document by owner shard; its events get fresh local seqs mapped to their global ones"""
        sd = importlib.import_module("siddhi-1_amd.state_doc")
        d = sd.parse(doc)
        parts = [sd.StateDoc(d.n_procs, d.n_slots, d.desc, d.now, d.last_event_ts, d.clock_flags) for _ in range(self.N)]
        for k in d.keys:
            if k.key >= self.n_keys:
                raise ValueError("state document key id outside [0, n_keys)")
            r = k.key % self.N
            k.key //= self.N
            parts[r].keys.append(k)
        for r, p in enumerate(parts):
            glob = sorted({ev.seq for k in p.keys for ev in k.streams if ev.seq < int(BLANK_SEQ)})
            base = self._append(r, np.array(glob, dtype=np.uint64))
            local = {g: base + i for i, g in enumerate(glob)}
            for k in p.keys:
                for ev in k.streams:
                    if ev.seq < int(BLANK_SEQ):
                        ev.seq = local[ev.seq]
        self._each(lambda r: self.shards[r].state_import(sd.write(parts[r])))

    def close(self):
        for s in self.shards:
            s.close()
        if self.pool is not None:
            self.pool.shutdown()
            self.pool = None
