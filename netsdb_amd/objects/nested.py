"""Device-resident nested columns: ``pdb::Vector<T>`` and ``pdb::Map<K, V>`` fields as offsets + values.

Reference: src/objectModel/headers/PDBVector.h (a Vector is an offset pointer to a contiguous array of T
inside the page) and src/builtInPDBObjects/headers/PDBMap.h:16 (an open-addressing map stored in the
page); nested types such as tpchBench's Customer{Vector<Order{Vector<LineItem{Handle<Supplier>,
Handle<Part>}>}>}.

Here a nested field of a RecordBatch is a ragged column: ``offsets`` [n + 1] int64 plus a child column
``values`` holding every element of every row back to back — a tensor for ``Vector(int|float)``, a
:class:`~netsdb_amd.objects.record.RecordBatch` (struct of columns, recursively nested) for
``Vector(SomePDBObject)``, a StringColumn for ``Vector(str)``.  A :class:`MapColumn` adds a parallel
``keys`` child.  Every structural operation — row gather, slice, concat, FLATTEN (rows -> elements with
the parent index), map merge (group entries by (group, key) and concatenate their values) — is a
handful of whole-column tensor ops, so on a GPU-resident set they run on the device with no per-record
host loop.  Python lambdas that walk records still work: a row reads back as a list / dict view.
"""
from __future__ import annotations

from typing import Any, List, Optional, Sequence

import torch

from .strings import StringColumn


def _lengths(offsets: torch.Tensor) -> torch.Tensor:
    return offsets[1:] - offsets[:-1]


def _offsets_from_lengths(lens: torch.Tensor) -> torch.Tensor:
    out = torch.zeros(lens.numel() + 1, dtype=torch.int64, device=lens.device)
    if lens.numel():
        torch.cumsum(lens, 0, out=out[1:])
    return out


def ragged_positions(offsets: torch.Tensor, idx: torch.Tensor):
    """Element positions of rows ``idx`` (concatenated) and the new offsets: the ragged gather index."""
    idx = idx.to(offsets.device).long()
    starts = offsets[idx]
    lens = offsets[idx + 1] - starts
    new_off = _offsets_from_lengths(lens)
    total = int(new_off[-1]) if new_off.numel() else 0
    if total == 0:
        return torch.empty(0, dtype=torch.int64, device=offsets.device), new_off
    rep_start = torch.repeat_interleave(starts - new_off[:-1], lens)
    pos = torch.arange(total, device=offsets.device) + rep_start
    return pos, new_off


class NestedColumn:
    """A ragged column: row i holds ``values[offsets[i]:offsets[i+1]]``."""

    __slots__ = ("offsets", "values")

    def __init__(self, offsets: torch.Tensor, values):
        self.offsets = offsets
        self.values = values

    # ------------------------------------------------------------------ construction
    @staticmethod
    def from_lists(rows: Sequence[Sequence[Any]], elem=None, device=None) -> "NestedColumn":
        from .record import make_column

        lens = torch.tensor([len(r) for r in rows], dtype=torch.int64)
        flat = [x for r in rows for x in r]
        if elem is None and flat:
            elem = type(flat[0])
        values = make_column(flat, elem if elem is not None else object, device)
        off = _offsets_from_lengths(lens)
        return NestedColumn(off.to(device) if device is not None else off, values)

    # ------------------------------------------------------------------ column protocol
    def __len__(self) -> int:
        return self.offsets.numel() - 1

    @property
    def device(self) -> torch.device:
        return self.offsets.device

    def lengths(self) -> torch.Tensor:
        return _lengths(self.offsets)

    def take(self, idx) -> "NestedColumn":
        from .record import column_take

        if not isinstance(idx, torch.Tensor):
            idx = torch.as_tensor(idx, dtype=torch.long)
        pos, off = ragged_positions(self.offsets, idx)
        return NestedColumn(off, column_take(self.values, pos))

    def slice(self, s: int, e: int) -> "NestedColumn":
        from .record import column_slice

        e = min(e, len(self))
        off = self.offsets[s: e + 1]
        a, b = (int(off[0]), int(off[-1])) if off.numel() else (0, 0)
        return NestedColumn(off - a, column_slice(self.values, a, b))

    def __getitem__(self, i):
        if isinstance(i, slice):
            s, e, _ = i.indices(len(self))
            return self.slice(s, e)
        return self.item(i)

    def to(self, device) -> "NestedColumn":
        from .record import _col_to

        return NestedColumn(self.offsets.to(device), _col_to(self.values, device))

    @property
    def nbytes(self) -> int:
        from .record import RecordBatch

        v = self.values
        if isinstance(v, torch.Tensor):
            vb = v.numel() * v.element_size()
        elif isinstance(v, RecordBatch):
            vb = v.nbytes()
        elif isinstance(v, (StringColumn, NestedColumn)):
            vb = v.nbytes
        else:
            vb = 16 * len(v)
        return self.offsets.numel() * 8 + vb

    @staticmethod
    def concat(parts: Sequence["NestedColumn"]) -> "NestedColumn":
        from .record import column_concat

        parts = list(parts)
        dev = parts[0].offsets.device
        lens = torch.cat([p.lengths().to(dev) for p in parts])
        return NestedColumn(_offsets_from_lengths(lens), column_concat([p.values for p in parts]))

    def item(self, i: int):
        """Row i as a Python list (elements: scalars, RecordViews or nested lists)."""
        from .record import column_item

        a, b = int(self.offsets[i]), int(self.offsets[i + 1])
        return [column_item(self.values, j) for j in range(a, b)]

    def tolist(self) -> List[list]:
        return [self.item(i) for i in range(len(self))]

    def __iter__(self):
        for i in range(len(self)):
            yield self.item(i)

    # ------------------------------------------------------------------ relational operators
    def flatten(self):
        """FLATTEN: (element column, parent row of every element) — both on the column's device."""
        lens = self.lengths()
        parent = torch.repeat_interleave(torch.arange(len(self), device=lens.device), lens)
        return self.values, parent

    def segment_sum(self, x: torch.Tensor) -> torch.Tensor:
        """Sum an element-aligned tensor per row."""
        out = torch.zeros((len(self),) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        _, parent = self.flatten()
        return out.index_add_(0, parent.to(x.device), x)


class MapColumn(NestedColumn):
    """A ragged column of maps: row i holds ``keys[o_i:o_{i+1}] -> values[o_i:o_{i+1}]`` (PDBMap)."""

    __slots__ = ("keys",)

    def __init__(self, offsets: torch.Tensor, keys, values):
        super().__init__(offsets, values)
        self.keys = keys

    @staticmethod
    def from_dicts(rows: Sequence[dict], device=None) -> "MapColumn":
        from .record import make_column

        lens = torch.tensor([len(r) for r in rows], dtype=torch.int64)
        ks = [k for r in rows for k in r.keys()]
        vs = [v for r in rows for v in r.values()]
        kcol = make_column(ks, type(ks[0]) if ks else str, device)
        if vs and isinstance(vs[0], (list, tuple)):
            vcol = NestedColumn.from_lists(vs, device=device)
        else:
            vcol = make_column(vs, type(vs[0]) if vs else float, device)
        off = _offsets_from_lengths(lens)
        return MapColumn(off.to(device) if device is not None else off, kcol, vcol)

    def take(self, idx) -> "MapColumn":
        from .record import column_take

        if not isinstance(idx, torch.Tensor):
            idx = torch.as_tensor(idx, dtype=torch.long)
        pos, off = ragged_positions(self.offsets, idx)
        return MapColumn(off, column_take(self.keys, pos), column_take(self.values, pos))

    def slice(self, s: int, e: int) -> "MapColumn":
        from .record import column_slice

        e = min(e, len(self))
        off = self.offsets[s: e + 1]
        a, b = (int(off[0]), int(off[-1])) if off.numel() else (0, 0)
        return MapColumn(off - a, column_slice(self.keys, a, b), column_slice(self.values, a, b))

    def to(self, device) -> "MapColumn":
        from .record import _col_to

        return MapColumn(self.offsets.to(device), _col_to(self.keys, device), _col_to(self.values, device))

    @property
    def nbytes(self) -> int:
        kb = self.keys.nbytes if isinstance(self.keys, (StringColumn, NestedColumn)) else \
            (self.keys.numel() * self.keys.element_size() if isinstance(self.keys, torch.Tensor) else 16 * len(self.keys))
        return NestedColumn.nbytes.fget(self) + kb

    @staticmethod
    def concat(parts: Sequence["MapColumn"]) -> "MapColumn":
        from .record import column_concat

        parts = list(parts)
        dev = parts[0].offsets.device
        lens = torch.cat([p.lengths().to(dev) for p in parts])
        return MapColumn(_offsets_from_lengths(lens), column_concat([p.keys for p in parts]),
                         column_concat([p.values for p in parts]))

    def item(self, i: int) -> dict:
        from .record import column_item

        a, b = int(self.offsets[i]), int(self.offsets[i + 1])
        out = {}
        for j in range(a, b):
            k = column_item(self.keys, j)
            out[k.item() if isinstance(k, torch.Tensor) and k.dim() == 0 else k] = column_item(self.values, j)
        return out

    @staticmethod
    def merge(maps: "MapColumn", group: torch.Tensor, ngroups: int) -> "MapColumn":
        """Map-merge aggregation (PDBMap operator+ folded per group): entries of all rows in one group,
        grouped by key; values with equal (group, key) are concatenated (ragged values) or summed
        (scalar values).  Sort + unique over (group, key hash) — whole-column ops, device-resident."""
        from ..execution.kernels import column_to_int64
        from .record import column_take

        dev = maps.offsets.device
        lens = maps.lengths()
        egroup = torch.repeat_interleave(group.to(dev).long(), lens)          # group of every entry
        kh = column_to_int64(maps.keys, dev).to(dev)
        if egroup.numel() == 0:
            return MapColumn(torch.zeros(ngroups + 1, dtype=torch.int64, device=dev), maps.keys, maps.values)
        # stable order by (group, key hash); entries keep their arrival order inside an equal pair
        order = torch.argsort(kh, stable=True)
        order = order[torch.argsort(egroup[order], stable=True)]
        g_s, k_s = egroup[order], kh[order]
        new_pair = torch.ones(order.numel(), dtype=torch.bool, device=dev)
        new_pair[1:] = (g_s[1:] != g_s[:-1]) | (k_s[1:] != k_s[:-1])
        pair_id = torch.cumsum(new_pair.long(), 0) - 1
        npairs = int(pair_id[-1]) + 1
        first = torch.nonzero(new_pair).flatten()
        keys = column_take(maps.keys, order[first])
        vals = maps.values
        if isinstance(vals, NestedColumn):
            # concatenate the ragged values of every pair: gather the entries' values in pair order
            ent = vals.take(order)
            plens = torch.zeros(npairs, dtype=torch.int64, device=dev).index_add_(0, pair_id, ent.lengths())
            merged_vals = NestedColumn(_offsets_from_lengths(plens), ent.values)
        else:
            v = column_take(vals, order)
            merged_vals = torch.zeros((npairs,) + tuple(v.shape[1:]), dtype=v.dtype, device=dev).index_add_(
                0, pair_id, v)
        pgroup = g_s[first]
        glens = torch.zeros(ngroups, dtype=torch.int64, device=dev).index_add_(0, pgroup, torch.ones_like(pgroup))
        return MapColumn(_offsets_from_lengths(glens), keys, merged_vals)


def is_nested(c) -> bool:
    return isinstance(c, NestedColumn)


__all__ = ["NestedColumn", "MapColumn", "ragged_positions", "is_nested"]
