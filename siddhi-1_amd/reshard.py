"""Key reshard of arrival-ordered ingest across GPUs.

Partition keys shard: no processor reads another key's state (PartitionStateHolder.java:43-49,
PartitionStreamReceiver.send :262-272), so each GPU owns the keys with ``key % world == rank`` and
runs its own engine on them (local key id ``key // world``, dense in [0, keys_per_rank)).

Each rank ingests a contiguous slice of the global arrival order (rank r holds events
[r*n, (r+1)*n) of a step).  One exchange per micro-batch moves every event to the rank that owns its
key: a stable bucket by destination, one ``all_to_all_single`` of the counts and one of the packed
payload (RCCL over xGMI with the nccl backend; gloo on CPU).  Chunks arrive in source-rank order and
each chunk is in arrival order, so the received events are in global arrival order — per key that is
exactly the order the reference processes them in.
"""
from __future__ import annotations

from typing import Dict, List, Tuple

import torch
import torch.distributed as dist


def owner(key: torch.Tensor, world: int) -> torch.Tensor:
    return torch.remainder(key.to(torch.int64), world)


def local_key(key: torch.Tensor, world: int) -> torch.Tensor:
    return torch.div(key.to(torch.int64), world, rounding_mode="floor")


def _as_words(t: torch.Tensor) -> torch.Tensor:
    """1-D tensor -> [n, w] int32 words (bit-exact reinterpretation)."""
    if t.element_size() == 8:
        return t.contiguous().view(torch.int32).view(-1, 2)
    if t.element_size() == 4:
        return t.contiguous().view(torch.int32).view(-1, 1)
    return t.to(torch.int32).view(-1, 1)


def _from_words(w: torch.Tensor, like: torch.Tensor) -> torch.Tensor:
    if like.element_size() == 8:
        return w.contiguous().view(like.dtype).view(-1)
    if like.element_size() == 4:
        return w.contiguous().view(like.dtype).view(-1)
    return w.view(-1).to(like.dtype)


def reshard(cols: Dict[str, torch.Tensor], key_col: str, world: int, group=None) -> Dict[str, torch.Tensor]:
    """Exchange this rank's slice of the arrival-ordered stream so that every rank receives the
    events of the keys it owns, in global arrival order.  ``cols`` are 1-D tensors of equal length
    on the collective's device; the result has the same columns (``key_col`` keeps the GLOBAL key)."""
    if world == 1:
        return dict(cols)
    names = list(cols)
    key = cols[key_col]
    dest = owner(key, world)
    order = torch.sort(dest, stable=True).indices           # stable: arrival order within a bucket
    send_counts = torch.bincount(dest, minlength=world)
    recv_counts = torch.empty_like(send_counts)
    dist.all_to_all_single(recv_counts, send_counts, group=group)
    parts: List[torch.Tensor] = [_as_words(cols[n])[order] for n in names]
    widths = [p.shape[1] for p in parts]
    packed = torch.cat(parts, dim=1).contiguous()            # [n, W] int32
    W = packed.shape[1]
    sc = send_counts.tolist()
    rc = recv_counts.tolist()
    out = torch.empty((sum(rc), W), dtype=torch.int32, device=packed.device)
    dist.all_to_all_single(out.view(-1), packed.view(-1), [c * W for c in rc], [c * W for c in sc], group=group)
    res, off = {}, 0
    for n, w in zip(names, widths):
        res[n] = _from_words(out[:, off:off + w], cols[n])
        off += w
    return res


def reshard_device(lib, cols: Dict[str, torch.Tensor], world: int, group=None,
                   exchange: bool = True) -> Dict[str, torch.Tensor]:
    """The GPU path of `reshard` (RCCL): the HIP stable pack by owning rank (``sg_shard_pack``), one
    all_to_all of the counts and one of the packed rows, and the unpack into SoA columns
    (``sg_shard_unpack``).  ``cols``: "key" (global key id, int32/uint32), "ts" (int64) and 32-bit
    attribute columns, all CUDA tensors of this rank's slice.  Returns "key" as the LOCAL key id
    (key // world, int32), "ts" and the attribute columns, in global arrival order."""
    import ctypes as C
    key, ts = cols["key"].to(torch.int32).contiguous(), cols["ts"].contiguous()
    names = [n for n in cols if n not in ("key", "ts")]
    attrs = [cols[n].contiguous() for n in names]
    if any(a.element_size() != 4 for a in attrs):
        raise ValueError("reshard_device packs 32-bit attribute columns")
    n, dev = key.numel(), key.device
    W = 3 + len(attrs)
    stream = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    lib.sg_shard_scratch_bytes.restype = C.c_size_t
    lib.sg_shard_scratch_bytes.argtypes = [C.c_uint64, C.c_uint32]
    scratch = torch.empty(int(lib.sg_shard_scratch_bytes(n, world)), dtype=torch.uint8, device=dev)
    rows = torch.empty((max(n, 1), W), dtype=torch.int32, device=dev)
    send = torch.empty(world, dtype=torch.int64, device=dev)
    colp = (C.c_void_p * max(1, len(attrs)))(*[a.data_ptr() for a in attrs])
    f = lib.sg_shard_pack
    f.argtypes = [C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p,
                  C.c_void_p, C.c_size_t, C.c_void_p]
    rc = f(n, key.data_ptr(), ts.data_ptr(), colp, len(attrs), world, rows.data_ptr(), send.data_ptr(),
           scratch.data_ptr(), scratch.numel(), stream)
    if rc != 0:
        raise RuntimeError(f"sg_shard_pack failed ({rc})")
    if world == 1 or not exchange:
        got = rows[:n]
    else:
        host = dist.get_backend(group) == "gloo"  # rehearsal on one GPU: exchange through host memory
        sd = send.cpu() if host else send
        recv = torch.empty_like(sd)
        dist.all_to_all_single(recv, sd, group=group)
        sc, rc_ = send.tolist(), recv.tolist()
        src = rows[:n].reshape(-1)
        src = src.cpu() if host else src
        got = torch.empty((sum(rc_), W), dtype=torch.int32, device=src.device)
        dist.all_to_all_single(got.view(-1), src, [c * W for c in rc_], [c * W for c in sc], group=group)
        got = got.to(dev)
    m = got.shape[0]
    out = {"key": torch.empty(m, dtype=torch.int32, device=dev), "ts": torch.empty(m, dtype=torch.int64, device=dev)}
    for nm, a in zip(names, attrs):
        out[nm] = torch.empty(m, dtype=a.dtype, device=dev)
    ptrs = torch.tensor([out[nm].data_ptr() for nm in names] or [0], dtype=torch.int64, device=dev)
    g = lib.sg_shard_unpack
    g.argtypes = [C.c_uint64, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    rc = g(m, got.data_ptr(), len(attrs), out["key"].data_ptr(), out["ts"].data_ptr(), ptrs.data_ptr(), stream)
    if rc != 0:
        raise RuntimeError(f"sg_shard_unpack failed ({rc})")
    return out


def block_capacity(n: int, world: int) -> int:
    """Rows per destination block of `reshard_device_blocks` for a slice of n uniformly keyed events: the
    mean n / world plus 8 standard deviations of its binomial count (overflow is detected, never silent)."""
    m = n / world
    return int(m + 8.0 * (m * (1.0 - 1.0 / world)) ** 0.5 + 256)


class BlockResharder:
    """`reshard_device` without any device->host synchronisation, for the per-step exchange of a
    multi-GPU run: the pack fills fixed-size destination blocks of `cap` rows (``sg_shard_pack_blocks``;
    the unused rows of a block are padding whose local key is SG_KEY_NULL), one equal-split all_to_all
    moves them, and the received world * cap rows unpack into a padded batch in global arrival order.
    The engine (created with SG_CFG_NULL_KEYS) drops the padding as the reference drops null-key events.
    Buffers are allocated once (`slots` output sets, reused round-robin: the engine reads set s while
    the next step is resharded into set s + 1).  A destination with more than cap rows raises the
    device flag `overflow`; `check()` reads it once (the run is then invalid)."""

    def __init__(self, lib, n: int, world: int, names, dtypes, device, cap=None, slots=2, group=None):
        import ctypes as C
        self.C, self.lib, self.n, self.world, self.group = C, lib, n, world, group
        self.cap = cap or block_capacity(n, world)
        self.names = list(names)
        self.W = 3 + len(self.names)
        self.dev = device
        m = world * self.cap
        lib.sg_shard_scratch_bytes.restype = C.c_size_t
        lib.sg_shard_scratch_bytes.argtypes = [C.c_uint64, C.c_uint32]
        self.scratch = torch.empty(int(lib.sg_shard_scratch_bytes(n, world)), dtype=torch.uint8, device=device)
        self.send = torch.empty((m, self.W), dtype=torch.int32, device=device)
        self.recv = torch.empty_like(self.send)
        self.counts = torch.empty(world, dtype=torch.int64, device=device)
        self.flag = torch.zeros(1, dtype=torch.int32, device=device)
        self.overflow = torch.zeros(1, dtype=torch.int32, device=device)
        self.host = world > 1 and dist.get_backend(group) == "gloo"  # one-GPU rehearsal through host memory
        self.sets, self.ptrs = [], []
        for _ in range(slots):
            o = {"key": torch.empty(m, dtype=torch.int32, device=device),
                 "ts": torch.empty(m, dtype=torch.int64, device=device)}
            for nm, dt in zip(self.names, dtypes):
                o[nm] = torch.empty(m, dtype=dt, device=device)
            self.sets.append(o)
            self.ptrs.append(torch.tensor([o[nm].data_ptr() for nm in self.names] or [0], dtype=torch.int64,
                                          device=device))
        self.next = 0
        f = lib.sg_shard_pack_blocks
        f.argtypes = [C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p,
                      C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]
        g = lib.sg_shard_unpack
        g.argtypes = [C.c_uint64, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]

    def __call__(self, cols: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
        """this rank's slice ("key": global key id, "ts", the attribute columns) -> the padded batch of the
        keys this rank owns (local key ids), queued on the current stream"""
        C = self.C
        key, ts = cols["key"], cols["ts"]
        attrs = [cols[nm] for nm in self.names]
        stream = C.c_void_p(torch.cuda.current_stream(self.dev).cuda_stream)
        colp = (C.c_void_p * max(1, len(attrs)))(*[a.data_ptr() for a in attrs])
        rc = self.lib.sg_shard_pack_blocks(key.numel(), key.data_ptr(), ts.data_ptr(), colp, len(attrs), self.world,
                                           self.cap, self.send.data_ptr(), self.counts.data_ptr(), self.flag.data_ptr(),
                                           self.scratch.data_ptr(), self.scratch.numel(), stream)
        if rc != 0:
            raise RuntimeError(f"sg_shard_pack_blocks failed ({rc})")
        self.overflow.bitwise_or_(self.flag)
        rows = self.send
        if self.world > 1:
            if self.host:
                got = torch.empty(self.send.numel(), dtype=torch.int32)
                dist.all_to_all_single(got, self.send.view(-1).cpu(), group=self.group)
                self.recv.view(-1).copy_(got)
            else:
                dist.all_to_all_single(self.recv.view(-1), self.send.view(-1), group=self.group)
            rows = self.recv
        o, p = self.sets[self.next], self.ptrs[self.next]
        self.next = (self.next + 1) % len(self.sets)
        m = self.world * self.cap
        rc = self.lib.sg_shard_unpack(m, rows.data_ptr(), len(attrs), o["key"].data_ptr(), o["ts"].data_ptr(),
                                      p.data_ptr(), stream)
        if rc != 0:
            raise RuntimeError(f"sg_shard_unpack failed ({rc})")
        return o

    def check(self):
        if int(self.overflow.item()):
            raise RuntimeError(f"a destination block overflowed its {self.cap} rows: the key distribution is "
                               f"too skewed for this block size")


def merge_by_trigger(parts: List[Tuple[torch.Tensor, ...]]) -> torch.Tensor:
    """Host-side k-way merge order of per-rank match streams (each sorted by global trigger seq):
    returns the permutation of the concatenation that orders it by (trigger seq, rank, position) —
    the reference's global callback order for per-event sends."""
    trig = torch.cat([p[0] for p in parts])
    rank = torch.cat([torch.full_like(p[0], i) for i, p in enumerate(parts)])
    pos = torch.cat([torch.arange(p[0].numel(), dtype=torch.int64) for p in parts])
    # lexicographic (trig, rank, pos) via stable sorts from the least significant key
    o = torch.sort(pos, stable=True).indices
    o = o[torch.sort(rank[o], stable=True).indices]
    o = o[torch.sort(trig[o], stable=True).indices]
    return o
