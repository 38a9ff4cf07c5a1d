"""ctypes binding of the engine C-ABI (include/siddhi_gpu.h).

`NativeEngine` drives any library that exports the `sg_*` entry points under a given symbol
prefix.  The product loads the HIP engine `libsiddhi_gpu.so` built next to this file
(`load_hip_library`); there is no fallback: if the library is missing the call raises.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass
from typing import Optional

import numpy as np

SG_OK = 0
SG_MEM_HOST = 0
SG_MEM_DEVICE = 1
SG_POLL_READY = 0x10
SG_CFG_ASYNC_HOST = 8
SG_NULL_SEQ = np.uint64(0xFFFFFFFFFFFFFFFF)
SG_CFG_NO_ORDER = 1
SG_CFG_TIMING = 2
SG_CFG_NULL_KEYS = 4

ERRORS = {-1: "SG_ERR_INVALID", -2: "SG_ERR_UNSUPPORTED", -3: "SG_ERR_DEVICE",
          -4: "SG_ERR_CAPACITY", -5: "SG_ERR_STATE"}

HERE = os.path.dirname(os.path.abspath(__file__))
HIP_LIBRARY = os.path.join(HERE, "lib", "libsiddhi_gpu.so")
# experiments only (tools/): an alternative build of the same library (e.g. another state layout)
if os.environ.get("SG_HIP_LIBRARY"):
    HIP_LIBRARY = os.path.abspath(os.environ["SG_HIP_LIBRARY"])


class EngineError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code


class sg_config(C.Structure):
    _fields_ = [("struct_size", C.c_uint32), ("device", C.c_int32), ("n_keys", C.c_uint32),
                ("max_batch", C.c_uint32), ("partial_capacity", C.c_uint32), ("flags", C.c_uint32),
                ("match_capacity", C.c_uint64), ("n_devices", C.c_uint32), ("reserved", C.c_uint32),
                ("devices", C.POINTER(C.c_int32))]


class sg_batch(C.Structure):
    _fields_ = [("struct_size", C.c_uint32), ("stream", C.c_uint32), ("n", C.c_uint64),
                ("seq_base", C.c_uint64), ("key", C.c_void_p), ("ts", C.c_void_p),
                ("cols", C.POINTER(C.c_void_p)), ("nulls", C.POINTER(C.c_void_p)),
                ("n_cols", C.c_uint32), ("mem", C.c_uint32)]


class sg_match_batch(C.Structure):
    _fields_ = [("n", C.c_uint64), ("n_slots", C.c_uint32), ("max_chain", C.c_uint32),
                ("trigger_seq", C.c_void_p), ("key", C.c_void_p), ("ts", C.c_void_p),
                ("slot_seq", C.c_void_p), ("chain_len", C.c_void_p), ("mem", C.c_uint32),
                ("reserved", C.c_uint32)]


class sg_stats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("events", "batches", "partials_scanned", "partials_created",
                                          "partials_live", "matches", "keys_touched",
                                          "live_at_batch_start", "group_ns", "advance_ns", "order_ns",
                                          "advance_launches", "window_spills", "advance_hbm_ns",
                                          "host_staged_bytes", "seq_map_entries", "hot_keys", "hot_events",
                                          "seq_map_trims", "host_syncs")]


class sg_projection(C.Structure):
    _fields_ = [("n", C.c_uint64), ("n_items", C.c_uint32), ("mem", C.c_uint32), ("value", C.c_void_p),
                ("null", C.c_void_p)]


@dataclass
class Matches:
    """Host copy of one sg_match_batch (+ the on-device projection of the select list, when set)."""
    trigger_seq: np.ndarray   # [n] uint64
    key: np.ndarray           # [n] uint32
    ts: np.ndarray            # [n] int64
    slot_seq: np.ndarray      # [n, n_slots, max_chain] uint64
    chain_len: np.ndarray     # [n, n_slots] uint32
    proj_value: Optional[np.ndarray] = None   # [n_items, n] uint64 value bits
    proj_null: Optional[np.ndarray] = None    # [n_items, n] uint8

    def __len__(self):
        return int(self.trigger_seq.shape[0])


_LIBS = {}


def load_library(path):
    path = os.path.abspath(path)
    if path not in _LIBS:
        if not os.path.exists(path):
            raise FileNotFoundError(f"engine library {path} is missing: build it with "
                                    f"`python __graft_entry__.py build` (no CPU fallback exists)")
        _LIBS[path] = C.CDLL(path)
    return _LIBS[path]


def load_hip_library():
    return load_library(HIP_LIBRARY)


def jit_check(ir: bytes, variant_flags=0, lib=None):
    """Generate and compile (hipRTC, gfx950, no device needed) the query-specialised advance kernel
    of an IR blob.  Returns the generated query header; raises EngineError with the log on failure."""
    lib = lib or load_hip_library()
    f = lib.sg_jit_check
    f.argtypes = [C.c_void_p, C.c_size_t, C.c_uint32, C.c_char_p, C.c_size_t]
    buf = C.create_string_buffer(1 << 20)
    irb = C.create_string_buffer(ir, len(ir))
    rc = f(irb, len(ir), variant_flags, buf, len(buf))
    if rc != SG_OK:
        lib.sg_last_error.restype = C.c_char_p
        raise EngineError(rc, lib.sg_last_error().decode(errors="replace"))
    return buf.value.decode()


def _np_ptr(a):
    return C.c_void_p(a.ctypes.data) if a is not None else None


SG_KEY_NULL = 0xFFFFFFFF


def pack_strings(strings):
    """Arrow-style (bytes, offsets[n+1], valid) of a sequence of str/None (UTF-8, as Java's String
    bytes for the dictionary's equality).  A numpy bytes array ('S', UTF-8, no nulls) packs without a
    per-value Python loop (numpy drops trailing NUL characters of fixed-width strings)."""
    if isinstance(strings, np.ndarray) and strings.dtype.kind == "U":
        strings = strings.tolist()   # (one encode per value below: faster than np.char.encode)
    if isinstance(strings, np.ndarray) and strings.dtype.kind == "S":
        enc = strings
        n, w = len(enc), enc.dtype.itemsize
        lens = np.char.str_len(enc).astype(np.uint64) if n else np.zeros(0, dtype=np.uint64)
        offsets = np.zeros(n + 1, dtype=np.uint64)
        np.cumsum(lens, out=offsets[1:])
        if n and w:
            mat = np.ascontiguousarray(enc).view(np.uint8).reshape(n, w)
            data = mat[np.arange(w, dtype=np.uint64)[None, :] < lens[:, None]]
        else:
            data = np.zeros(0, dtype=np.uint8)
        if data.size == 0:
            data = np.zeros(1, dtype=np.uint8)
        return np.ascontiguousarray(data), offsets, np.ones(n, dtype=np.uint8)
    enc = [s.encode("utf-8") if s is not None else b"" for s in strings]
    offsets = np.zeros(len(enc) + 1, dtype=np.uint64)
    if enc:
        np.cumsum([len(b) for b in enc], out=offsets[1:])
    data = np.frombuffer(b"".join(enc) or b"\0", dtype=np.uint8)
    valid = np.array([s is not None for s in strings], dtype=np.uint8)
    return data, offsets, valid


class KeyDictionary:
    """Partition-key dictionary over sg_dict (include/siddhi_gpu.h): key String -> dense key_id in
    first-seen order, the map PartitionStreamReceiver keeps per partition
    (partition/PartitionStreamReceiver.java:175-260).  Behaves as the dict the host runtime used
    (get / [] / in / len / keys / clear / update with first-seen ids) and adds the batched
    `intern`, which is what ingest calls."""

    def __init__(self, max_ids=(1 << 32) - 2, capacity_hint=0, lib=None):
        self._lib = lib or load_hip_library()
        L = self._lib
        L.sg_dict_create.argtypes = [C.c_uint32, C.c_uint64, C.POINTER(C.c_void_p)]
        L.sg_dict_intern.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p,
                                     C.POINTER(C.c_uint64)]
        L.sg_dict_lookup.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p]
        L.sg_dict_size.argtypes = [C.c_void_p]
        L.sg_dict_size.restype = C.c_uint32
        L.sg_dict_key.argtypes = [C.c_void_p, C.c_uint32, C.POINTER(C.c_void_p), C.POINTER(C.c_uint64)]
        L.sg_dict_remove.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64]
        L.sg_dict_put.argtypes = [C.c_void_p, C.c_uint32, C.c_char_p, C.c_uint64]
        L.sg_dict_clear.argtypes = [C.c_void_p]
        L.sg_dict_destroy.argtypes = [C.c_void_p]
        L.sg_dict_destroy.restype = None
        L.sg_last_error.restype = C.c_char_p
        h = C.c_void_p()
        self._check(L.sg_dict_create(max_ids, capacity_hint, C.byref(h)))
        self._h = h

    def _check(self, rc):
        if rc != SG_OK:
            raise EngineError(rc, self._lib.sg_last_error().decode(errors="replace"))

    def intern(self, strings):
        """uint32 ids of a batch of key strings (None -> SG_KEY_NULL), new keys numbered in order of
        first appearance; all-or-nothing (EngineError SG_ERR_CAPACITY past max_ids)."""
        data, offsets, valid = pack_strings(strings)
        ids = np.empty(len(offsets) - 1, dtype=np.uint32)
        n_new = C.c_uint64()
        self._check(self._lib.sg_dict_intern(self._h, _np_ptr(data), _np_ptr(offsets), _np_ptr(valid),
                                             len(ids), _np_ptr(ids), C.byref(n_new)))
        return ids

    def intern_string_ids(self, sids, isnull, strings):
        """intern over a STRING column given as the host string dictionary's ids (`strings`, a runtime
        StringDictionary; isnull: the null bytes or None): ids seen before map through a cache (string id ->
        key id, one gather per batch), the others are interned in order of first appearance.  The cache
        follows this dictionary: remove / clear / put / update drop it, and so must a caller that replaces
        `strings`' ids (drop_string_cache)."""
        sids = np.asarray(sids, dtype=np.uint32)
        c = self.__dict__.get("_scache")
        if c is None or c[0] is not strings:
            c = self._scache = (strings, np.full(max(1024, 2 * len(strings.strs)), 0xFFFFFFFE, dtype=np.uint32))
        tab = c[1]
        if len(tab) < len(strings.strs):
            grown = np.full(2 * len(strings.strs), 0xFFFFFFFE, dtype=np.uint32)
            grown[:len(tab)] = tab
            tab = grown
            self._scache = (strings, tab)
        kids = tab[sids]
        miss = kids == 0xFFFFFFFE
        if isnull is not None:
            miss &= isnull == 0
        if miss.any():
            u, first = np.unique(sids[miss], return_index=True)
            u = u[np.argsort(first, kind="stable")]   # first-seen order within the batch
            strs = strings.strs
            tab[u] = self.intern([strs[i] for i in u.tolist()])
            kids = tab[sids]
        if isnull is not None and isnull.any():
            kids = np.where(isnull != 0, np.uint32(SG_KEY_NULL), kids).astype(np.uint32)
        return kids

    def drop_string_cache(self):
        self.__dict__.pop("_scache", None)

    def lookup(self, strings):
        data, offsets, valid = pack_strings(strings)
        ids = np.empty(len(offsets) - 1, dtype=np.uint32)
        self._check(self._lib.sg_dict_lookup(self._h, _np_ptr(data), _np_ptr(offsets), _np_ptr(valid),
                                             len(ids), _np_ptr(ids)))
        return ids

    def key(self, i):
        p, n = C.c_void_p(), C.c_uint64()
        self._check(self._lib.sg_dict_key(self._h, i, C.byref(p), C.byref(n)))
        return C.string_at(p, n.value).decode("utf-8") if n.value else ""

    def remove(self, ids):
        """Partition purge: the ids leave the dictionary; later new keys reuse them, smallest first
        (all-or-nothing; an id not in use raises EngineError SG_ERR_INVALID)."""
        a = np.ascontiguousarray(ids, dtype=np.uint32)
        self.drop_string_cache()
        self._check(self._lib.sg_dict_remove(self._h, _np_ptr(a) if len(a) else None, len(a)))

    def put(self, i, k):
        """Bind key string k to the free id i (snapshot restore)."""
        b = k.encode("utf-8")
        self.drop_string_cache()
        self._check(self._lib.sg_dict_put(self._h, i, b, len(b)))

    def _live(self, i):
        p, n = C.c_void_p(), C.c_uint64()
        return self._lib.sg_dict_key(self._h, i, C.byref(p), C.byref(n)) == SG_OK

    # the dict protocol of the host runtime --------------------------------------------------------
    def __len__(self):
        return int(self._lib.sg_dict_size(self._h))

    def get(self, k, default=None):
        i = int(self.lookup([k])[0])
        return default if i == SG_KEY_NULL else i

    def __getitem__(self, k):
        i = self.get(k)
        if i is None:
            raise KeyError(k)
        return i

    def __contains__(self, k):
        return self.get(k) is not None

    def __setitem__(self, k, v):
        if int(self.intern([k])[0]) != v:
            raise ValueError("key ids are assigned in first-seen order")

    def keys(self):
        """key string per id below the id bound, None for a removed (free) id"""
        return [self.key(i) if self._live(i) else None for i in range(len(self))]

    def clear(self):
        self.drop_string_cache()
        self._check(self._lib.sg_dict_clear(self._h))

    def update(self, mapping):
        """bind every key -> id of mapping (ids in between stay free)"""
        for k, v in sorted(mapping.items(), key=lambda kv: kv[1]):
            self.put(int(v), k)

    def close(self):
        if getattr(self, "_h", None):
            self._lib.sg_dict_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class NativeEngine:
    """One sg_engine (one compiled query on one device)."""

    def __init__(self, lib, prefix, ir: bytes, n_keys=1, max_batch=1 << 16, partial_capacity=64,
                 match_capacity=1 << 20, device=0, flags=0, devices=None):
        """devices: several HIP device ordinals -> the engine's own multi-device fan-out (sg_config.n_devices,
        sg_sharded.cpp): keys sharded key % len(devices), one engine per device behind this one handle"""
        self.lib = lib
        self.p = prefix
        f = lambda n: getattr(lib, prefix + n)
        self._create = f("engine_create")
        self._create.argtypes = [C.c_void_p, C.c_size_t, C.POINTER(sg_config), C.POINTER(C.c_void_p)]
        self._push = f("push_batch")
        self._push.argtypes = [C.c_void_p, C.POINTER(sg_batch)]
        self._poll = f("poll_matches")
        self._poll.argtypes = [C.c_void_p, C.c_uint32, C.POINTER(sg_match_batch)]
        self._release = f("release_matches")
        self._release.argtypes = [C.c_void_p, C.POINTER(sg_match_batch)]
        self._stats = f("get_stats")
        self._stats.argtypes = [C.c_void_p, C.POINTER(sg_stats)]
        self._destroy = f("engine_destroy")
        self._destroy.argtypes = [C.c_void_p]
        self._destroy.restype = None
        self._err = f("last_error")
        self._err.restype = C.c_char_p
        self._advance = f("advance_time")
        self._advance.argtypes = [C.c_void_p, C.c_int64]
        self._sync = getattr(lib, prefix + "synchronize", None)
        if self._sync is not None:
            self._sync.argtypes = [C.c_void_p]
        devs = list(devices) if devices is not None else [device]
        self._devs = (C.c_int32 * len(devs))(*devs)
        cfg = sg_config(C.sizeof(sg_config), devs[0], n_keys, max_batch, partial_capacity, flags,
                        match_capacity, len(devs), 0, self._devs)
        self._ir = C.create_string_buffer(ir, len(ir))
        h = C.c_void_p()
        self._check(self._create(self._ir, len(ir), C.byref(cfg), C.byref(h)))
        self.h = h
        self.n_keys = n_keys
        self.proj_items = 0

    def set_projection(self, code, item_pc, item_len, item_type, part_attr):
        """On-device projection of the select list (sg_set_projection); raises EngineError when the
        engine cannot evaluate it (SG_ERR_UNSUPPORTED: keep projecting on the host)."""
        f = getattr(self.lib, self.p + "set_projection", None)
        if f is None:   # (the CPU oracle projects on the host)
            raise EngineError(-2, "this engine library has no on-device projection")
        f.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                      C.c_void_p, C.c_uint32]
        arr = lambda x, dt: np.ascontiguousarray(np.array(x, dtype=dt))
        code, pc, ln, ty, pa = (arr(code, np.uint32), arr(item_pc, np.uint32), arr(item_len, np.uint32),
                                arr(item_type, np.uint32), arr(part_attr, np.int32))
        self._check(f(self.h, _np_ptr(code), len(code), _np_ptr(pc), _np_ptr(ln), _np_ptr(ty), len(pc), _np_ptr(pa),
                      len(pa)))
        # output items: the select list and `having` (the aggregator-argument items feed them)
        self.proj_items = int(np.sum((ty & 0x10000) == 0))

    def _check(self, rc):
        if rc != SG_OK:
            raise EngineError(rc, self._err().decode(errors="replace"))

    def push(self, stream, seq_base, ts, cols, nulls=None, key=None, mem=SG_MEM_HOST):
        """Push one batch.  cols/nulls/key/ts: numpy arrays (host) or raw pointers (device)."""
        n_cols = len(cols)
        if mem == SG_MEM_HOST:
            ts = np.ascontiguousarray(ts, dtype=np.int64)
            n = ts.shape[0]
            keep = [ts]
            colp = (C.c_void_p * max(1, n_cols))(*[c.ctypes.data for c in cols])
            keep += list(cols)
            nullp = None
            if nulls is not None and any(x is not None for x in nulls):
                nullp = (C.c_void_p * max(1, n_cols))(*[(x.ctypes.data if x is not None else None)
                                                        for x in nulls])
                keep += [x for x in nulls if x is not None]
            kp = None
            if key is not None:
                key = np.ascontiguousarray(key, dtype=np.uint32)
                keep.append(key)
                kp = key.ctypes.data
            b = sg_batch(C.sizeof(sg_batch), stream, n, seq_base, kp, ts.ctypes.data,
                         C.cast(colp, C.POINTER(C.c_void_p)),
                         C.cast(nullp, C.POINTER(C.c_void_p)) if nullp is not None else None,
                         n_cols, SG_MEM_HOST)
            self._check(self._push(self.h, C.byref(b)))
            del keep
        else:
            n, ts_ptr, col_ptrs, key_ptr = ts
            colp = (C.c_void_p * max(1, n_cols))(*col_ptrs)
            b = sg_batch(C.sizeof(sg_batch), stream, n, seq_base, key_ptr, ts_ptr,
                         C.cast(colp, C.POINTER(C.c_void_p)), None, n_cols, SG_MEM_DEVICE)
            self._check(self._push(self.h, C.byref(b)))

    def poll(self, copy=True, ready=False) -> Matches:
        """Matches emitted since the previous poll, in host memory.  copy=False returns views of the
        engine's pinned staging, valid until the next poll of this engine (no host-side copy).
        ready=True: only the matches of batches already complete (SG_POLL_READY, no wait)."""
        m = sg_match_batch()
        self._check(self._poll(self.h, SG_MEM_HOST | (SG_POLL_READY if ready else 0), C.byref(m)))
        n, ns, mc = int(m.n), int(m.n_slots), int(m.max_chain)

        def arr(ptr, dtype, shape):
            cnt = int(np.prod(shape))
            if cnt == 0 or not ptr:
                return np.zeros(shape, dtype=dtype)
            buf = (C.c_char * (cnt * np.dtype(dtype).itemsize)).from_address(ptr)
            a = np.frombuffer(buf, dtype=dtype).reshape(shape)
            return a.copy() if copy else a

        out = Matches(arr(m.trigger_seq, np.uint64, (n,)), arr(m.key, np.uint32, (n,)),
                      arr(m.ts, np.int64, (n,)), arr(m.slot_seq, np.uint64, (n, ns, mc)),
                      arr(m.chain_len, np.uint32, (n, ns)))
        if self.proj_items:
            pr = sg_projection()
            g = getattr(self.lib, self.p + "get_projection")
            g.argtypes = [C.c_void_p, C.c_uint32, C.POINTER(sg_projection)]
            self._check(g(self.h, SG_MEM_HOST, C.byref(pr)))
            out.proj_value = arr(pr.value, np.uint64, (self.proj_items, n))
            out.proj_null = arr(pr.null, np.uint8, (self.proj_items, n))
        self._check(self._release(self.h, C.byref(m)))
        return out

    def poll_device(self, ready=False):
        """Matches stay in HBM; returns the raw sg_match_batch (caller must release()).
        ready=True: only the batches already complete (SG_POLL_READY)."""
        m = sg_match_batch()
        self._check(self._poll(self.h, SG_MEM_DEVICE | (SG_POLL_READY if ready else 0), C.byref(m)))
        return m

    def discard(self):
        """poll to host memory and release at once, without building arrays (a caller that only needs the
        engine to hand its matches out, e.g. a throughput loop)"""
        m = sg_match_batch()
        self._check(self._poll(self.h, SG_MEM_HOST, C.byref(m)))
        n = int(m.n)
        self._check(self._release(self.h, C.byref(m)))
        return n

    def release(self, m):
        self._check(self._release(self.h, C.byref(m)))

    def advance_time(self, now):
        self._check(self._advance(self.h, int(now)))

    def synchronize(self):
        if self._sync is not None:
            self._check(self._sync(self.h))

    def wait_stream(self, stream_handle):
        """sg_wait_stream: the engine's later work (a fan-out's later device splits) waits for what is queued on
        the HIP stream `stream_handle` (an int handle, e.g. torch.cuda.Stream().cuda_stream; 0 = legacy default)"""
        f = getattr(self.lib, self.p + "wait_stream")
        f.argtypes = [C.c_void_p, C.c_void_p]
        self._check(f(self.h, C.c_void_p(int(stream_handle) or None)))

    def reset_keys(self, keys):
        """Partition purge: the listed keys' NFA state back to never-seen (sg_reset_keys)."""
        f = getattr(self.lib, self.p + "reset_keys")
        f.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32]
        k = np.ascontiguousarray(keys, dtype=np.uint32)
        self._check(f(self.h, C.c_void_p(k.ctypes.data) if len(k) else None, len(k), SG_MEM_HOST))

    def snapshot(self) -> bytes:
        """Image of the device NFA state (sg_snapshot; poll the matches first)."""
        f, free = getattr(self.lib, self.p + "snapshot"), self.lib.sg_free_buffer
        f.argtypes = [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]
        free.argtypes = [C.c_void_p]
        buf, n = C.c_void_p(), C.c_size_t()
        self._check(f(self.h, C.byref(buf), C.byref(n)))
        try:
            return C.string_at(buf, n.value)
        finally:
            free(buf)

    def restore(self, image: bytes):
        """Replace the engine's NFA state with a snapshot of an engine of the same query (sg_restore)."""
        f = getattr(self.lib, self.p + "restore")
        f.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t]
        self._check(f(self.h, image, len(image)))

    def state_export(self) -> bytes:
        """The NFA state in the reference's per-state-processor form (sg_state_export, state_doc.py)."""
        f, free = getattr(self.lib, self.p + "state_export"), getattr(self.lib, self.p + "free_buffer")
        f.argtypes = [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]
        free.argtypes = [C.c_void_p]
        buf, n = C.c_void_p(), C.c_size_t()
        self._check(f(self.h, C.byref(buf), C.byref(n)))
        try:
            return C.string_at(buf, n.value)
        finally:
            free(buf)

    def state_import(self, doc: bytes):
        """Replace the NFA state with a state document of any engine of the same query (sg_state_import)."""
        f = getattr(self.lib, self.p + "state_import")
        f.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t]
        self._check(f(self.h, doc, len(doc)))

    def stats(self):
        s = sg_stats()
        self._check(self._stats(self.h, C.byref(s)))
        return {n: int(getattr(s, n)) for n, _ in sg_stats._fields_}

    def describe(self):
        """the kernels this engine dispatches per push / advance (sg_engine_describe); None when the library
        has no such entry (the CPU oracle)"""
        fn = getattr(self.lib, self.p + "engine_describe", None)
        if fn is None:
            return None
        fn.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t]
        buf = C.create_string_buffer(1024)
        self._check(fn(self.h, buf, 1024))
        return buf.value.decode()

    def close(self):
        if getattr(self, "h", None):
            self._destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
