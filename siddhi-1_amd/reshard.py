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
