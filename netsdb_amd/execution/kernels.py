"""Vectorised relational primitives on tuple-set columns (GPU or CPU tensors).

Reference: src/queryExecution + src/lambdas/headers (HashSink, JoinTuple, JoinMap/PairArray,
AggregationMap, FilterExecutor, FlattenExecutor, HashPartitionSink).  netsDB uses per-record
C++ hash maps; here every operator runs over whole columns. On the GPU the hot ones are device hash
tables (csrc/kernels/relops.hip): the join build/probe (JoinTable), the fused group-by + aggregate
(group_reduce; group_ids for the inverse) and the partition permutation of the shuffle sink
(partition_order). Keys are value-exact: several int columns pack into one int64 when their ranges allow,
otherwise (and for strings) a 64-bit hash groups and every row is then compared with its group's
representative row (strings byte by byte), so colliding keys are never merged. On the CPU the same
operators are sort / unique / searchsorted tensor ops.
"""
from __future__ import annotations

import os
import weakref
from typing import Any, List, Optional, Tuple

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


def mix64(x: torch.Tensor, y: Optional[torch.Tensor] = None) -> torch.Tensor:
    """splitmix64 finaliser of (x ^ y) + GOLD in wrapping int64 arithmetic (matches netsdb_amd._native.hash64). On the
    GPU one pass of relops.hip mix64_kernel; the torch expression below is the CPU path and the reference."""
    if x.is_cuda and x.dim() == 1 and x.dtype == torch.int64 and x.numel() >= _MIX_MIN_ROWS and \
            (y is None or (y.is_cuda and y.dtype == torch.int64 and y.shape == x.shape)):
        return _ext.hip().mix64(x, y)
    if y is not None:
        x = x ^ y
    x = x + _GOLD
    x = (x ^ _lsr(x, 30)) * _M1
    x = (x ^ _lsr(x, 27)) * _M2
    return x ^ _lsr(x, 31)


_MIX_MIN_ROWS = 1           # every device column: one launch instead of the torch expression's eleven


def selected_rows(mask: torch.Tensor) -> torch.Tensor:
    """The row ids of a filter's kept rows, in order (torch.nonzero(mask).flatten()). On the GPU the relops.hip
    stable compaction for large masks (per-tile counts, one scan, ordered id runs: a third of rocprim's partition
    time on a 60 M-row mask)."""
    if mask.is_cuda and mask.dim() == 1 and mask.numel() >= _COMPACT_MIN_ROWS and \
            mask.dtype in (torch.bool, torch.uint8):
        return _ext.hip().compact(mask)
    return torch.nonzero(mask, as_tuple=False).flatten()


_COMPACT_MIN_ROWS = 1 << 16


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
            out = h if out is None else mix64(out, h)
        return out
    if isinstance(c, torch.Tensor):
        if c.dim() > 1:
            c = c.reshape(c.shape[0], -1)
            out = torch.zeros(c.shape[0], dtype=torch.int64, device=c.device)
            for j in range(c.shape[1]):
                out = mix64(out, column_to_int64(c[:, j]))
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


class JoinTable:
    """A join build side keyed by its int64 join-hash column, built ONCE and probed by every probe batch
    (reference JoinMap / JoinProbe, src/lambdas/headers/JoinTuple.h:434, HashSink.h:14).

    On the GPU: a device open-addressing table of 16-byte slots {key, count, payload} (relops.hip join_insert /
    join_perm; payload = the build row for a unique key, else the start of its CSR run), probed by ONE 16-byte
    lookup per probe row (join_probe) and expanded into the (build, probe) pairs probe-major (join_expand).
    On the CPU: the build hashes sorted once, probes binary-searched."""

    def __init__(self, build_h: torch.Tensor):
        self.h = build_h
        self.n = int(build_h.numel())
        self._dev = None
        self._sorted = None
        if self.n and build_h.is_cuda and self.n < JOIN_TABLE_MAX_ROWS:
            self._dev = _ext.hip().join_build(build_h.long().contiguous())
            st = self._dev[3] if len(self._dev) > 3 else None
            if st is not None and st.numel():                 # the build's own host read carried the max count
                self._max_mult = int(st[1]) + 1
        elif self.n:
            # builds past the device table's 2^29-row bound (32-bit payloads): sorted keys + binary search, on the device
            self._sorted = torch.sort(build_h)

    _max_mult = None

    def max_multiplicity(self) -> int:
        """The most build rows any one key has (the fused probe kernels size their output regions by it): one device
        reduction over the table's counts and one host read, once per table."""
        if self._max_mult is None:
            if self._dev is not None:
                cnt = self._dev[0][:, 1] & 0xFFFFFFFF            # extra rows beyond the first, per slot
                self._max_mult = int(cnt.max().item()) + 1 if self.n else 0
            elif self.n:
                _, c = torch.unique(self.h, return_counts=True)
                self._max_mult = int(c.max().item())
            else:
                self._max_mult = 0
        return self._max_mult

    def probe(self, probe_h: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """All (build_idx, probe_idx) pairs with equal keys, probe-major."""
        dev = probe_h.device
        if self.n == 0 or probe_h.numel() == 0:
            e = torch.empty(0, dtype=torch.int64, device=dev)
            return e, e
        if self._dev is not None:
            tab, perm = self._dev[0], self._dev[1]
            bloom = self._dev[2] if len(self._dev) > 2 else None
            return tuple(_ext.hip().join_probe(tab, perm, probe_h.to(tab.device).long().contiguous(), bloom))
        sh, order = self._sorted
        sh, order = sh.to(dev), order.to(dev)
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


JOIN_TABLE_MAX_ROWS = 1 << 29


def join_match(build_h: torch.Tensor, probe_h: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """All (build_idx, probe_idx) pairs with equal hashes (one-shot JoinTable)."""
    return JoinTable(build_h.to(probe_h.device)).probe(probe_h)


# ------------------------------------------------------------------------------ exact grouping on the device
_MAG = 0x7FFFFFFFFFFFFFFF


def _float_word(bits: torch.Tensor) -> torch.Tensor:
    """IEEE-754 double bits -> an int64 with the same ORDER as the values (negative magnitudes flipped); an
    involution, so it also maps such a word back to the bits."""
    return bits ^ ((bits >> 63) & _MAG)


def _norm_col(c: torch.Tensor) -> torch.Tensor:
    """1-D key column -> int64 words with value equality AND value order (floats by an order-preserving transform
    of their bits, -0.0 folded into +0.0), so groups sort like torch.unique(sorted=True)."""
    if c.dtype == torch.int64:
        return c.contiguous()
    if c.is_floating_point():
        return _float_word((c.double() + 0.0).view(torch.int64))
    return c.long()


def _pack_exact(words: List[torch.Tensor]):
    """Several int64 key columns -> ONE int64 with the same equality and lexicographic order, when their value
    ranges fit in 62 bits together (one host read of the column minima / maxima): (packed, layout) or None."""
    if len(words) == 1:
        return words[0], None
    mm = torch.stack([torch.stack(list(torch.aminmax(w))) for w in words]).cpu().tolist()
    bits = [int(hi - lo).bit_length() for lo, hi in mm]
    if sum(bits) > 62:
        return None
    shifts, sh = [], sum(bits)
    for b in bits:
        sh -= b
        shifts.append(sh)
    packed = None
    for w, (lo, _), s in zip(words, mm, shifts):
        t = (w - lo) << s if s else (w - lo)
        packed = t if packed is None else packed | t
    return packed, [(lo, s, b) for (lo, _), s, b in zip(mm, shifts, bits)]


def _unpack(packed: torch.Tensor, layout) -> List[torch.Tensor]:
    out = []
    for lo, s, b in layout:
        v = _lsr(packed, s) if s else packed
        out.append((v & ((1 << b) - 1) if b < 63 else v) + lo)
    return out


def _combine_words(words: List[torch.Tensor]) -> torch.Tensor:
    out = None
    for h in words:
        out = h if out is None else mix64(out, h)
    return out


def _device_cols(keys):
    """The key as a list of device columns (StringColumn or 1-D tensor), or None if it is not device-groupable."""
    cols = list(keys) if isinstance(keys, tuple) else [keys]
    if not cols:
        return None
    for c in cols:
        if isinstance(c, StringColumn):
            if c.device.type != "cuda":
                return None
        elif not (isinstance(c, torch.Tensor) and c.is_cuda and c.dim() == 1 and c.dtype != torch.bool
                  or isinstance(c, torch.Tensor) and c.is_cuda and c.dim() == 1 and c.dtype == torch.bool):
            return None
    n = len(cols[0])
    if any(len(c) != n for c in cols):
        return None
    return cols


def _exact_words(cols):
    """Value-exact int64 words of key columns (numbers by value, strings of <= 7 bytes by their order-preserving
    short codes, StringColumn.short_codes), or None when a string column holds longer rows (hash + re-check)."""
    out = []
    for c in cols:
        if isinstance(c, StringColumn):
            w = c.short_codes()
            if w is None:
                return None
            out.append(w)
        else:
            out.append(_norm_col(c))
    return out


def _key_words(cols):
    """(words, packed): exact words packed into one int64 when they fit, else hash words (packed None)."""
    exact = _exact_words(cols)
    if exact is not None:
        packed = _pack_exact(exact)
        if packed is not None:
            return exact, packed
        return exact, None
    return [c.hash64() if isinstance(c, StringColumn) else _norm_col(c) for c in cols], None


def _rep_from_word(u: torch.Tensor, c):
    """A group's key column from its exact int64 word (inverse of _exact_words for one column)."""
    if isinstance(c, StringColumn):
        return StringColumn.from_short_codes(u, c.max_len())
    return u.to(c.dtype) if not c.is_floating_point() else _float_word(u).view(torch.float64).to(c.dtype)


def _rows_match_rep(cols, words, ref: torch.Tensor) -> bool:
    """Every row's key equals the key of its group's representative row ``ref`` (exactness check of a
    hash-decided grouping)."""
    ok = None
    for c, w in zip(cols, words):
        eq = c.eq_rows(None, c, ref) if isinstance(c, StringColumn) else (w == w.index_select(0, ref))
        ok = eq if ok is None else ok & eq
    return bool(ok.all())


# ------------------------------------------------------------------------ relational scratch accounting
# The device relational kernels' scratch (the PART path's partitioned rows and n-group output) is charged to the
# storage manager that owns the device's HBM budget while it is allocated, so out-of-core accounting sees it (it may
# evict pages to make room). One manager per device (the client's), registered by the StorageManager.
_SCRATCH = {}
SCRATCH_STATS = {"charged_bytes": 0, "peak_bytes": 0, "calls": 0}


def register_scratch_accounting(manager) -> None:
    dev = getattr(manager, "home", None)
    if dev is not None and torch.device(dev).type == "cuda":
        _SCRATCH[str(torch.device(dev))] = weakref.ref(manager)


def _scratch_cb(dev):
    ref = _SCRATCH.get(str(dev))
    m = ref() if ref is not None else None

    def cb(nbytes: int):
        nbytes = int(nbytes)
        if nbytes > 0:
            SCRATCH_STATS["calls"] += 1
            SCRATCH_STATS["charged_bytes"] += nbytes
            SCRATCH_STATS["peak_bytes"] = max(SCRATCH_STATS["peak_bytes"], SCRATCH_STATS["charged_bytes"])
            if m is not None:
                m.account_bytes(nbytes, m.home)
        else:
            SCRATCH_STATS["charged_bytes"] += nbytes
            if m is not None:
                m.release_bytes(-nbytes, m.home)
    return cb


# rows per device aggregation call (the kernels index rows with 32-bit offsets): larger inputs are chunked and the
# per-chunk groups merged
AGG_CHUNK_ROWS = (1 << 31) - (1 << 20)
LAST_AGG_STATUS = {}


def _hash_aggregate(key64: torch.Tensor, vals, op: str, want_inv: bool, want_first: bool = True):
    n = key64.numel()
    if n > AGG_CHUNK_ROWS:
        return _hash_aggregate_chunked(key64, vals, op, want_inv, want_first)
    r = _ext.hip().hash_aggregate(key64.contiguous(), vals, op, want_inv, 0, want_first, _scratch_cb(key64.device))
    status = r[5].tolist()
    LAST_AGG_STATUS.update(groups=status[0], path=("LOW", "PART")[status[1]], ok=status[2],
                           sample_distinct=status[3], scratch_bytes=status[4] if len(status) > 4 else None)
    if status[2] != 1:
        return None
    return r[0], r[1], r[2], r[3], r[4]


RUN_AGG_MIN_ROWS = 1 << 18     # group_reduce tries the clustered-key path from this many rows
RUN_AGG = os.environ.get("NSDB_RUN_AGG", "1") != "0"
LAST_RUN_AGG = {"tried": 0, "used": 0}


def _run_aggregate(key64: torch.Tensor, vals, op: str):
    """Group-by of packed keys that arrive in runs of equal keys (relops.hip run_*_kernel: a scan of a table stored in
    key order, e.g. TPC-H lineitem by l_orderkey): every run is one group, no hash table. None when the keys are not
    ordered (checked on the device in the same pass that counts the runs), or too few rows to be worth the check."""
    n = key64.numel()
    h = _ext.hip()
    if not RUN_AGG or n < RUN_AGG_MIN_ROWS or not hasattr(h, "run_aggregate"):
        return None
    LAST_RUN_AGG["tried"] += 1
    r = h.run_aggregate(key64, vals, op)
    if not r:
        return None
    LAST_RUN_AGG["used"] += 1
    return r[0], r[1], r[2], r[3], None


def _hash_aggregate_chunked(key64, vals, op, want_inv, want_first):
    """> AGG_CHUNK_ROWS rows: aggregate each chunk, then merge the chunks' groups (sum of sums / counts, min of mins,
    max of maxes); first rows and the per-row inverse are mapped through the merge."""
    n = key64.numel()
    parts = []
    for s in range(0, n, AGG_CHUNK_ROWS):
        e = min(n, s + AGG_CHUNK_ROWS)
        r = _hash_aggregate(key64[s:e], None if vals is None else vals[s:e], op, want_inv, want_first)
        if r is None:
            return None
        parts.append((s, r))
    reps = torch.cat([r[0] for _, r in parts])
    has_v = vals is not None and parts[0][1][1] is not None and parts[0][1][1].numel()
    aggs = torch.cat([r[1] for _, r in parts]) if has_v else None
    cnts = torch.cat([r[2] for _, r in parts])
    firsts = torch.cat([r[3] + s for s, r in parts])
    m = _hash_aggregate(reps, aggs, op, True, False)   # merge: the chunks' groups are few
    if m is None:
        return None
    g_reps, g_aggs, _, _, ginv, = m
    g = g_reps.numel()
    g_cnt = torch.zeros(g, dtype=torch.int64, device=reps.device).index_add_(0, ginv, cnts)
    g_first = torch.full((g,), n, dtype=torch.int64, device=reps.device).scatter_reduce_(0, ginv, firsts, "amin")
    inv = None
    if want_inv:
        off, invs = 0, []
        for s, r in parts:
            k = r[0].numel()
            invs.append(ginv[off: off + k].index_select(0, r[4]))
            off += k
        inv = torch.cat(invs)
    return g_reps, g_aggs, g_cnt, g_first, inv


def _sort_groups(key_reps: torch.Tensor):
    """Order of the groups by key value (the order torch.unique(sorted=True) gives) and its inverse rank."""
    order = torch.argsort(key_reps)
    rank = torch.empty_like(order)
    rank[order] = torch.arange(order.numel(), device=order.device)
    return order, rank


def _take_col(c, idx):
    return c.take(idx) if isinstance(c, StringColumn) else c.index_select(0, idx)


def _group_ids_device(keys):
    """Exact group ids of device key columns: packed ints, or a 64-bit hash + a check of every row against its
    group's representative (strings byte-compared). None when the caller must take the generic path."""
    cols = _device_cols(keys)
    if cols is None or len(cols[0]) == 0:
        return None
    words, packed = _key_words(cols)
    key = packed[0] if packed is not None else _combine_words(words)
    r = _hash_aggregate(key, None, "sum", True)
    if r is None:
        return None
    reps_k, _, _, first, inv = r
    if packed is None and not _rows_match_rep(cols, words, first.index_select(0, inv)):
        return None          # two different keys share a hash: the exact generic path decides
    order, rank = _sort_groups(reps_k)
    first = first.index_select(0, order)
    inv = rank.index_select(0, inv)
    reps = tuple(_take_col(c, first) for c in cols)
    return inv, (reps if isinstance(keys, tuple) else reps[0]), int(first.numel())


def group_reduce(keys, values, op: str = "sum"):
    """Fused device group-by + aggregation (relops.hip hash_aggregate: LDS pre-aggregation for few groups, radix
    partitioning for many): ``(representative keys, aggregates)`` ordered like :func:`group_ids` up to
    SORTED_GROUPS_MAX groups (larger results in the table's order), or None when
    the inputs need the generic path (host objects, non-numeric values, unsupported op).
    Reference: AggregationProcessor.h:16 / CombinerProcessor over PDBMap hash tables."""
    if op not in ("sum", "count", "min", "max", "mean") or not isinstance(values, torch.Tensor) or not values.is_cuda:
        return None
    cols = _device_cols(keys)
    if cols is None or len(cols[0]) != values.shape[0] or values.shape[0] == 0:
        return None
    if values.dtype == torch.bool or values.is_complex():
        return None
    n = values.shape[0]
    flat = values.reshape(n, -1)
    if flat.shape[1] > 16:
        return None
    is_float = values.is_floating_point()
    vals = None
    if op != "count":
        vals = flat.double() if is_float else flat.long()
    kop = {"sum": "sum", "mean": "sum", "count": "sum", "min": "min", "max": "max"}[op]
    words, packed = _key_words(cols)
    key = packed[0] if packed is not None else _combine_words(words)
    # packed keys are the values themselves: no representative row (first / inverse) is needed, so the
    # partition passes carry no row ids
    r = _run_aggregate(key, vals, kop) if packed is not None else None
    if r is None:
        r = _hash_aggregate(key, vals, kop, packed is None, packed is None)
    if r is None:
        return None
    reps_k, aggs, cnt, first, inv = r
    if packed is None and not _rows_match_rep(cols, words, first.index_select(0, inv)):
        return None
    g = int(reps_k.numel())
    if g > SORTED_GROUPS_MAX:
        # an aggregation's output is a set: past this many groups they stay in the table's emit order (sorting 15 M
        # group keys and gathering every output column by the permutation cost ~2 ms of TPC-H Q04's 8.6 at SF 10)
        order = None
    else:
        order, _ = _sort_groups(reps_k)

    def sel(t):
        return t if order is None else t.index_select(0, order)

    cnt = sel(cnt)
    if op == "count":
        agg = cnt
    else:
        agg = sel(aggs)
        if op == "mean":
            agg = agg / cnt.unsqueeze(1).to(agg.dtype)
        out_dtype = values.dtype if (is_float or op != "mean") else torch.float64
        agg = agg.to(out_dtype).reshape((g,) + tuple(values.shape[1:]))
    if packed is not None and packed[1] is not None:
        unp = _unpack(sel(reps_k), packed[1])
        reps = tuple(_rep_from_word(u, c) for u, c in zip(unp, cols))
    elif packed is not None:
        reps = (_rep_from_word(sel(reps_k), cols[0]),)
    else:
        fo = sel(first)
        reps = tuple(_take_col(c, fo) for c in cols)
    return (reps if isinstance(keys, tuple) else reps[0]), agg


SORTED_GROUPS_MAX = 1 << 16     # group_reduce: results with more groups are not sorted by key (Q13 SF 10: a 1 M-group
# intermediate sorted by a 193 us merge sort nobody needed)


def group_ids(keys) -> Tuple[torch.Tensor, Any, int]:
    """Exact group-by: returns (inverse index per row, representative key column, #groups), groups in key order
    (hash order for string keys). Device columns group on the device hash tables (values compared exactly);
    host data groups with torch.unique / a dict."""
    if _device_cols(keys) is not None and _hip_groupby():
        r = _group_ids_device(keys)
        if r is not None:
            return r
    if isinstance(keys, StringColumn):
        return _group_strings_exact(keys)
    if isinstance(keys, tuple) and any(isinstance(k, StringColumn) for k in keys) and all(
            isinstance(k, StringColumn) or (isinstance(k, torch.Tensor) and k.dim() == 1) for k in keys):
        dev = keys[0].device
        strs = [k for k in keys if isinstance(k, StringColumn)]
        # exact: string columns by their dictionary codes (hash + byte re-check), then a lexicographic unique
        cols = [_group_strings_exact(k)[0] if isinstance(k, StringColumn) else _norm_col(k.to(dev)) for k in keys]
        del strs
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


def _group_strings_exact(col: StringColumn):
    """(inverse, representative strings, #groups) of a string column: group by 64-bit hash, then byte-compare
    every row with its group's first row; rows of a hash shared by different strings are regrouped by value."""
    h = col.hash64()
    inv, first, g = _unique_first(h)
    ok = col.eq_rows(None, col, first.index_select(0, inv))
    if bool(ok.all()):
        return inv, col.take(first), g
    # hash collision(s): split exactly by value (host dict over the distinct strings of the colliding groups)
    strs = col.tolist()
    seen, inv_l, firsts = {}, [], []
    for i, s in enumerate(strs):
        gi = seen.get(s)
        if gi is None:
            gi = len(firsts)
            seen[s] = gi
            firsts.append(i)
        inv_l.append(gi)
    dev = col.device
    return (torch.tensor(inv_l, dtype=torch.int64, device=dev),
            col.take(torch.tensor(firsts, dtype=torch.int64, device=dev)), len(firsts))


def _hip_groupby() -> bool:
    """Device hash tables for group-by (relops.hip) instead of torch.unique; ops.kernel_options(hash_groupby=...)."""
    from .. import ops
    return bool(ops._kopt("hash_groupby", HASH_GROUPBY_DEFAULT))


_hash_groupby = _hip_groupby
HASH_GROUPBY_DEFAULT = True


def _unique_first(h: torch.Tensor):
    """(inverse, first row of each group, #groups) for a 1-D int64 key tensor."""
    if h.is_cuda and _hip_groupby() and h.numel():
        r = _hash_aggregate(h.long(), None, "sum", True)
        if r is not None:
            reps_k, _, _, first, inv = r
            order, rank = _sort_groups(reps_k)
            return rank.index_select(0, inv), first.index_select(0, order), int(order.numel())
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


def partition_perm(dest: torch.Tensor, nparts: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """Stable permutation grouping rows by destination + per-destination counts as a tensor (no host read):
    on the GPU one pass of per-workgroup histograms + a ballot-ranked scatter (relops.hip partition_perm)."""
    if dest.is_cuda and 0 < nparts <= 2048 and dest.numel():
        perm, counts = _ext.hip().partition_perm(dest.long().contiguous(), nparts)
        return perm, counts
    return torch.argsort(dest, stable=True), torch.bincount(dest, minlength=nparts)


def partition_order(dest: torch.Tensor, nparts: int) -> Tuple[torch.Tensor, List[int]]:
    """:func:`partition_perm` with the counts read back as a list (HashPartitionSink)."""
    perm, counts = partition_perm(dest, nparts)
    return perm, counts.tolist()


def split_by_dest(batch: RecordBatch, dest: torch.Tensor, nparts: int) -> List[RecordBatch]:
    order, counts = partition_order(dest, nparts)
    sorted_b = batch.take(order)
    out, s = [], 0
    for c in counts:
        out.append(sorted_b.slice(s, s + c))
        s += c
    return out


__all__ = ["mix64", "hash_keys", "column_to_int64", "JoinTable", "join_match", "group_ids", "group_reduce",
           "segment_reduce", "take_reps", "partition_of", "partition_perm", "partition_order", "split_by_dest"]
