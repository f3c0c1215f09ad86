"""Vectorised relational primitives on tuple-set columns (GPU or CPU tensors).

Reference: src/queryExecution + src/lambdas/headers (HashSink, JoinTuple, JoinMap/PairArray,
AggregationMap, FilterExecutor, FlattenExecutor, HashPartitionSink).  netsDB uses per-record
C++ hash maps; here hashing, join matching and group-by run as whole-column tensor ops
(sort + searchsorted joins, unique/inverse group ids, index_add segment sums) so they execute
on the GPU for device-resident columns.
"""
from __future__ import annotations

from typing import Any, List, Tuple

import torch
import xxhash

from .. import _ext
from ..objects.record import RecordBatch, RecordView
from ..objects.strings import StringColumn, hash_str, is_string_list

_M1 = -0x40A7B892E31B1A47   # 0xBF58476D1CE4E5B9 as signed int64
_M2 = -0x6B2FB644ECCEEE15   # 0x94D049BB133111EB as signed int64
_GOLD = -0x61C8864680B583EB  # 0x9E3779B97F4A7C15


def _lsr(x: torch.Tensor, k: int) -> torch.Tensor:
    """Logical right shift on int64."""
    return (x >> k) & ((1 << (64 - k)) - 1)


def mix64(x: torch.Tensor) -> torch.Tensor:
    """splitmix64 finaliser in wrapping int64 arithmetic (matches netsdb_amd._native.hash64)."""
    x = x + _GOLD
    x = (x ^ _lsr(x, 30)) * _M1
    x = (x ^ _lsr(x, 27)) * _M2
    return x ^ _lsr(x, 31)


def _obj_key(v) -> int:
    if isinstance(v, RecordView):
        v = v.as_tuple()
    if isinstance(v, str):
        return hash_str(v)               # same key as a StringColumn row (device hash kernel)
    if isinstance(v, torch.Tensor):
        v = v.tolist()
    h = xxhash.xxh64_intdigest(repr(v).encode())
    return h - (1 << 64) if h >= (1 << 63) else h


def column_to_int64(c, device=None) -> torch.Tensor:
    """Map a key column (int/float/bool tensor, list of hashables, tuple of columns) to int64."""
    if isinstance(c, tuple):
        out = None
        for x in c:
            h = column_to_int64(x, device)
            out = h if out is None else mix64(out ^ h)
        return out
    if isinstance(c, torch.Tensor):
        if c.dim() > 1:
            c = c.reshape(c.shape[0], -1)
            out = torch.zeros(c.shape[0], dtype=torch.int64, device=c.device)
            for j in range(c.shape[1]):
                out = mix64(out ^ column_to_int64(c[:, j]))
            return out
        if c.dtype == torch.int64:
            return c
        if c.is_floating_point():
            return c.double().view(torch.int64) if c.dtype == torch.float64 else c.float().double().view(torch.int64)
        return c.long()
    if isinstance(c, RecordBatch):
        cols = tuple(v for v in c.columns.values())
        return column_to_int64(cols, device)
    if isinstance(c, StringColumn):
        return c.hash64()
    if is_string_list(c):               # vectorised: pack once, hash on the device (or numpy on CPU)
        return StringColumn.from_list(c, device).hash64()
    vals = [_obj_key(v) for v in c]
    return torch.tensor(vals, dtype=torch.int64, device=device)


def hash_keys(c, device=None) -> torch.Tensor:
    return mix64(column_to_int64(c, device))


def join_match(build_h: torch.Tensor, probe_h: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """All (build_idx, probe_idx) pairs with equal hashes: sort build side, binary-search probes."""
    dev = probe_h.device
    build_h = build_h.to(dev)
    if build_h.numel() == 0 or probe_h.numel() == 0:
        e = torch.empty(0, dtype=torch.int64, device=dev)
        return e, e
    sh, order = torch.sort(build_h)
    lo = torch.searchsorted(sh, probe_h, right=False)
    hi = torch.searchsorted(sh, probe_h, right=True)
    cnt = hi - lo
    probe_idx = torch.repeat_interleave(torch.arange(probe_h.numel(), device=dev), cnt)
    if probe_idx.numel() == 0:
        e = torch.empty(0, dtype=torch.int64, device=dev)
        return e, e
    starts = torch.repeat_interleave(lo, cnt)
    csum = torch.cumsum(cnt, 0)
    offs = torch.arange(probe_idx.numel(), device=dev) - torch.repeat_interleave(csum - cnt, cnt)
    build_idx = order[starts + offs]
    return build_idx, probe_idx


def group_ids(keys) -> Tuple[torch.Tensor, Any, int]:
    """Exact group-by: returns (inverse index per row, representative key column, #groups)."""
    if isinstance(keys, StringColumn):
        inv, first, n = _unique_first(keys.hash64())
        return inv, keys.take(first), n
    if isinstance(keys, tuple) and any(isinstance(k, StringColumn) for k in keys) and all(
            isinstance(k, StringColumn) or (isinstance(k, torch.Tensor) and k.dim() == 1) for k in keys):
        dev = keys[0].device
        cols = [k.hash64() if isinstance(k, StringColumn) else
                (k.to(dev).long() if not k.is_floating_point() else k.double().view(torch.int64).to(dev)) for k in keys]
        uniq, inv = torch.unique(torch.stack([c.to(dev) for c in cols], 1), dim=0, return_inverse=True)
        first = torch.full((uniq.shape[0],), inv.numel(), dtype=torch.long, device=dev)
        first.scatter_reduce_(0, inv, torch.arange(inv.numel(), device=dev), "amin")
        reps = tuple(k.take(first) if isinstance(k, StringColumn) else k.index_select(0, first.to(k.device))
                     for k in keys)
        return inv, reps, uniq.shape[0]
    if isinstance(keys, tuple) and all(isinstance(k, torch.Tensor) and k.dim() == 1 for k in keys):
        dev = keys[0].device
        stacked = torch.stack([k.to(dev).long() if not k.is_floating_point() else k.double().view(torch.int64).to(dev)
                               for k in keys], 1)
        uniq, inv = torch.unique(stacked, dim=0, return_inverse=True)
        reps = tuple(uniq[:, j].to(k.dtype) if not k.is_floating_point() else uniq[:, j].view(torch.float64).to(k.dtype)
                     for j, k in enumerate(keys))
        return inv, reps, uniq.shape[0]
    if isinstance(keys, torch.Tensor) and keys.dim() == 1:
        if keys.is_cuda and not keys.is_floating_point() and keys.dtype != torch.bool and _hash_groupby():
            # device hash table (hashagg.hip): O(n) insert, only the distinct keys are sorted
            inv, uniq = _ext.hip().hash_group_ids(keys.long())
            return inv, uniq.to(keys.dtype), uniq.numel()
        uniq, inv = torch.unique(keys, return_inverse=True)
        return inv, uniq, uniq.numel()
    # host objects: dict grouping preserving first-seen order
    seen = {}
    inv = []
    reps = []
    vals = keys if not isinstance(keys, tuple) else list(zip(*[k.tolist() if isinstance(k, torch.Tensor) else k for k in keys]))
    for v in vals:
        hk = _hashable(v)
        g = seen.get(hk)
        if g is None:
            g = len(reps)
            seen[hk] = g
            reps.append(v)
        inv.append(g)
    return torch.tensor(inv, dtype=torch.int64), reps, len(reps)


def _hash_groupby() -> bool:
    """Device hash-table group ids (hashagg.hip) instead of torch.unique; ops.kernel_options(hash_groupby=...)."""
    from .. import ops
    return bool(ops._kopt("hash_groupby", HASH_GROUPBY_DEFAULT))


HASH_GROUPBY_DEFAULT = False


def _unique_first(h: torch.Tensor):
    """(inverse, first row of each group, #groups) for a 1-D key tensor."""
    if h.is_cuda and _hash_groupby():
        inv, uniq = _ext.hip().hash_group_ids(h)
    else:
        uniq, inv = torch.unique(h, return_inverse=True)
    first = torch.full((uniq.numel(),), h.numel(), dtype=torch.long, device=h.device)
    first.scatter_reduce_(0, inv, torch.arange(h.numel(), device=h.device), "amin")
    return inv, first, uniq.numel()


def _hashable(v):
    if isinstance(v, RecordView):
        v = v.materialize()
    if isinstance(v, torch.Tensor):
        return tuple(v.flatten().tolist())
    if isinstance(v, list):
        return tuple(_hashable(x) for x in v)
    try:
        hash(v)
        return v
    except TypeError:
        return repr(v)


def segment_reduce(values, inv: torch.Tensor, ngroups: int, op: str = "sum", combine=None):
    """Combine values of rows sharing a group id."""
    from ..objects.nested import MapColumn, NestedColumn

    if isinstance(values, MapColumn):       # PDBMap merge per group, on the device
        return MapColumn.merge(values, inv, ngroups)
    if isinstance(values, NestedColumn):    # Vector concatenation per group (stable order)
        order = torch.argsort(inv.to(values.device), stable=True)
        ent = values.take(order)
        glens = torch.zeros(ngroups, dtype=torch.int64, device=values.device).index_add_(
            0, inv.to(values.device), values.lengths())
        off = torch.zeros(ngroups + 1, dtype=torch.int64, device=values.device)
        torch.cumsum(glens, 0, out=off[1:])
        return NestedColumn(off, ent.values)
    if isinstance(values, torch.Tensor):
        inv = inv.to(values.device)
        shape = (ngroups,) + tuple(values.shape[1:])
        if op == "sum":
            acc_dtype = torch.float32 if values.dtype in (torch.bfloat16, torch.float16) else values.dtype
            out = torch.zeros(shape, dtype=acc_dtype, device=values.device)
            out.index_add_(0, inv, values.to(acc_dtype))
            return out.to(values.dtype) if acc_dtype != values.dtype else out
        if op in ("max", "min", "mean", "prod"):
            red = {"max": "amax", "min": "amin", "mean": "mean", "prod": "prod"}[op]
            flat = values.reshape(values.shape[0], -1)
            out = torch.zeros((ngroups, flat.shape[1]), dtype=values.dtype, device=values.device)
            idx = inv.view(-1, 1).expand_as(flat)
            out = out.scatter_reduce(0, idx, flat, reduce=red, include_self=False)
            return out.reshape(shape)
        if op == "count":
            out = torch.zeros(ngroups, dtype=torch.int64, device=values.device)
            out.index_add_(0, inv, torch.ones_like(inv))
            return out
    # generic objects: fold with combine()
    fold = combine or (lambda a, b: a + b)
    acc: List[Any] = [None] * ngroups
    have = [False] * ngroups
    items = values if not isinstance(values, RecordBatch) else [RecordView(values, i).materialize() for i in range(values.n)]
    for g, v in zip(inv.tolist(), items):
        if isinstance(v, RecordView):
            v = v.materialize()
        if not have[g]:
            acc[g] = v
            have[g] = True
        else:
            acc[g] = fold(acc[g], v)
    return acc


def take_reps(reps, idx: torch.Tensor):
    if isinstance(reps, tuple):
        return tuple(take_reps(r, idx) for r in reps)
    if isinstance(reps, torch.Tensor):
        return reps.index_select(0, idx.to(reps.device))
    return [reps[i] for i in idx.tolist()]


def partition_of(h: torch.Tensor, nparts: int) -> torch.Tensor:
    """Destination rank per row from a hash column (non-negative modulo)."""
    return torch.remainder(h, nparts)


def split_by_dest(batch: RecordBatch, dest: torch.Tensor, nparts: int) -> List[RecordBatch]:
    order = torch.argsort(dest, stable=True)
    counts = torch.bincount(dest, minlength=nparts).tolist()
    sorted_b = batch.take(order)
    out, s = [], 0
    for c in counts:
        out.append(sorted_b.slice(s, s + c))
        s += c
    return out


__all__ = ["mix64", "hash_keys", "column_to_int64", "join_match", "group_ids", "segment_reduce", "take_reps",
           "partition_of", "split_by_dest"]
