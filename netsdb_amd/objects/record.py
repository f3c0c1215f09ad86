"""PDB object model, re-designed columnar for MI355X.

The reference stores C++ objects (``pdb::Object`` + ``Handle`` offset pointers, vtable-fixed
shared-library types; src/objectModel/headers/Object.h, Handle.h, PDBVector.h, PDBMap.h) in
pages and runs UDFs object-at-a-time.  Here a *type* is a Python class deriving from
:class:`PDBObject` whose annotated fields form a schema; a page holds a :class:`RecordBatch` —
one column per field:

* ``int``/``float``/``bool`` -> 1-D torch tensor (int64 / float64 / bool)
* ``Tensor(shape, dtype)``  -> one stacked tensor ``[n, *shape]`` (lives in HBM when the set is
  device-resident: the MatrixBlock payloads of the linear-algebra sets)
* ``Vector(int|float|str|SomePDBObject)`` -> :class:`~netsdb_amd.objects.nested.NestedColumn` (offsets +
  element column, device-resident, recursively nested); ``Map(K, V)`` -> ``MapColumn``
* a field annotated with a PDBObject subclass (a ``Handle<T>``) -> a nested RecordBatch (struct column)
* ``str`` / ``object`` / ``Vector(object)`` -> Python list (host)

UDF lambdas operate on whole columns (vectorised, GPU) or, for opaque Python lambdas, on
:class:`RecordView` objects (the analogue of dereferencing a ``Handle<T>``).
"""
from __future__ import annotations

from typing import Any, Dict, Iterable, List, Optional, Sequence

import os

import torch

from .strings import StringColumn, is_string_list, use_device_strings


class Tensor:
    """Field type for fixed-shape tensor payloads (e.g. a MatrixBlock's rawData)."""

    def __init__(self, shape: Optional[Sequence[int]] = None, dtype: torch.dtype = torch.float32):
        self.shape = tuple(shape) if shape is not None else None
        self.dtype = dtype

    def __repr__(self):
        return f"Tensor({self.shape}, {self.dtype})"


class Vector:
    """Variable-length vector field (pdb::Vector<T>): a device NestedColumn when the element type is a
    scalar, ``str`` or a PDBObject type; ``Vector(object)`` stays a host list column."""

    def __init__(self, elem=float):
        self.elem = elem

    def nested(self) -> bool:
        return self.elem in (int, float, bool, str) or (isinstance(self.elem, type) and issubclass(self.elem, PDBObject))

    def __repr__(self):
        return f"Vector({getattr(self.elem, '__name__', self.elem)})"


class Map:
    """Map field (pdb::Map<K, V>): a device MapColumn (keys + values children)."""

    def __init__(self, key=str, value=float):
        self.key, self.value = key, value

    def __repr__(self):
        return f"Map({getattr(self.key, '__name__', self.key)}, {getattr(self.value, '__name__', self.value)})"


SCALAR_TYPES = {int: torch.int64, float: torch.float64, bool: torch.bool}

_REGISTRY: Dict[str, type] = {}


def register_type(cls: type) -> type:
    _REGISTRY[cls.type_name()] = cls
    return cls


def lookup_type(name: str) -> type:
    if name not in _REGISTRY:
        raise KeyError(f"type '{name}' is not registered (PDBClient.register_type)")
    return _REGISTRY[name]


def registered_types() -> Dict[str, type]:
    return dict(_REGISTRY)


_BUILTIN_ANN = {"int": int, "float": float, "str": str, "bool": bool, "bytes": bytes, "object": object}


def _resolve_annotation(ann: str, cls):
    if ann in _BUILTIN_ANN:
        return _BUILTIN_ANN[ann]
    import sys

    scope = dict(vars(sys.modules.get(cls.__module__, object())))
    scope.update(vars(cls))
    try:
        return eval(ann, scope)  # noqa: S307 - class annotations of in-process types only
    except Exception:
        return object


class PDBObject:
    """Base class of every storable type. Subclasses declare fields via annotations."""

    __fields__: Dict[str, Any] = {}

    def __init_subclass__(cls, **kw):
        super().__init_subclass__(**kw)
        fields: Dict[str, Any] = {}
        for base in reversed(cls.__mro__[1:]):
            fields.update(getattr(base, "__fields__", {}))
        for name, ann in cls.__dict__.get("__annotations__", {}).items():
            if name.startswith("_"):
                continue
            if isinstance(ann, str):           # postponed annotations (from __future__ import annotations)
                ann = _resolve_annotation(ann, cls)
            fields[name] = cls.__dict__.get(name, None) if isinstance(cls.__dict__.get(name), (Tensor, Vector, Map)) \
                else ann
        cls.__fields__ = fields
        register_type(cls)

    def __init__(self, *args, **kw):
        names = list(self.__fields__)
        if len(args) > len(names):
            raise TypeError(f"{type(self).__name__} takes {len(names)} fields")
        for n, v in zip(names, args):
            setattr(self, n, v)
        for n, v in kw.items():
            if n not in self.__fields__:
                raise TypeError(f"unknown field {n} for {type(self).__name__}")
            setattr(self, n, v)
        for n in names:
            if not hasattr(self, n) or isinstance(getattr(self, n), (Tensor, Vector, Map)):
                setattr(self, n, _default_for(self.__fields__[n]))

    @classmethod
    def type_name(cls) -> str:
        return cls.__name__

    @classmethod
    def fields(cls) -> Dict[str, Any]:
        return dict(cls.__fields__)

    def to_dict(self) -> Dict[str, Any]:
        return {n: getattr(self, n) for n in self.__fields__}

    def __eq__(self, other):
        if type(other) is not type(self):
            return NotImplemented
        for n in self.__fields__:
            a, b = getattr(self, n), getattr(other, n)
            if isinstance(a, torch.Tensor) or isinstance(b, torch.Tensor):
                if not (isinstance(a, torch.Tensor) and isinstance(b, torch.Tensor) and torch.equal(a.cpu(), b.cpu())):
                    return False
            elif a != b:
                return False
        return True

    def __hash__(self):
        return hash(tuple(getattr(self, n) for n in self.__fields__ if not isinstance(getattr(self, n), torch.Tensor)))

    def __repr__(self):
        parts = []
        for n in self.__fields__:
            v = getattr(self, n)
            if isinstance(v, torch.Tensor):
                v = f"tensor{tuple(v.shape)}"
            parts.append(f"{n}={v!r}")
        return f"{type(self).__name__}({', '.join(parts)})"


def _default_for(ft):
    if ft is int or (isinstance(ft, type) and issubclass(ft, int) and ft is not bool):
        return 0
    if ft is float:
        return 0.0
    if ft is bool:
        return False
    if ft is str:
        return ""
    if isinstance(ft, Vector):
        return []
    if isinstance(ft, Map):
        return {}
    return None


def column_kind(ft) -> str:
    if isinstance(ft, Vector):
        return "nested" if ft.nested() else "object"
    if isinstance(ft, Map):
        return "map"
    if isinstance(ft, type) and issubclass(ft, PDBObject):
        return "struct"
    if ft in SCALAR_TYPES:
        return "scalar"
    if isinstance(ft, Tensor) or ft is torch.Tensor:
        return "tensor"
    return "object"


LAZY_TAKE_MIN_COLS = 4
LAZY_TAKE_ANY_DEVICE = os.environ.get("NSDB_LAZY_TAKE") == "1"   # tests: the lazy path on CPU batches too
# a lazy selection of at most this many rows gathers all of its pending device columns at once on its first read
GROUP_TAKE_MAX_ROWS = int(os.environ.get("NSDB_GROUP_TAKE_ROWS", str(1 << 18)))

_TAKE_BAD: Dict[Any, torch.Tensor] = {}     # device -> int32 word take_many sets on an out-of-range row id


def take_many(cols: List[torch.Tensor], idx: torch.Tensor) -> List[torch.Tensor]:
    """Rows ``idx`` of several device tensors (dim 0) in ONE kernel launch (relops.hip take_many_kernel)."""
    from .. import _ext

    bad = _TAKE_BAD.get(idx.device)
    if bad is None:
        bad = _TAKE_BAD[idx.device] = torch.zeros(1, dtype=torch.int32, device=idx.device)
    return list(_ext.hip().take_many(cols, idx.long().contiguous(), bad))


def take_many_check() -> bool:
    """True when no take_many launch so far met an out-of-range row id (reads and clears the per-device words)."""
    ok = True
    for b in _TAKE_BAD.values():
        if int(b.item()) != 0:
            ok = False
            b.zero_()
    return ok


def _group_take_ok(v, idx) -> bool:
    return (isinstance(idx, torch.Tensor) and idx.is_cuda and idx.dtype == torch.int64 and idx.dim() == 1
            and idx.numel() <= GROUP_TAKE_MAX_ROWS and GROUP_TAKE_MAX_ROWS > 0
            and isinstance(v, (torch.Tensor, StringColumn)))


class _LazyView:
    """values() / items() of LazyTakeColumns: re-iterable, each column gathered when the iteration reaches it."""

    __slots__ = ("_d", "_items")

    def __init__(self, d, items: bool):
        self._d, self._items = d, items

    def __iter__(self):
        d = self._d
        return ((k, d[k]) for k in d.keys()) if self._items else (d[k] for k in d.keys())

    def __len__(self):
        return len(self._d.keys())


class LazyTakeColumns(dict):
    """The columns of a row selection, gathered from ``src`` on first access and cached. Behaves as the dict of
    every column (iteration, items(), values(), dict(...) and ** materialise what they touch); columns set or
    deleted on it shadow the source."""

    __slots__ = ("_src", "_idx", "_gone", "_idxs")

    def __init__(self, src: Dict[str, Any], idx: Optional[torch.Tensor], idxs: Optional[Dict[str, Any]] = None):
        super().__init__()
        self._src, self._idx, self._gone, self._idxs = src, idx, set(), idxs

    def _fetch(self, k):
        idx = self._idx if self._idxs is None else self._idxs[k]
        if idx is not None and _group_take_ok(self._src[k], idx):
            self._fetch_group(idx)
            if dict.__contains__(self, k):
                return dict.__getitem__(self, k)
        v = self._src[k] if idx is None else column_take(self._src[k], idx)
        dict.__setitem__(self, k, v)
        return v

    def _fetch_group(self, idx):
        """A small selection's first read gathers EVERY pending device column at the same row ids in one launch
        (relops take_many: plain tensors and the start / end offsets of string columns), instead of one or two
        index_select launches per column as each is read: a few bytes per row of over-gathering against ~6 us of
        host time per launch (Q02's join outputs: ~170 gathers per query)."""
        names, srcs, parts = [], [], []
        for c in self._src:
            if dict.__contains__(self, c) or c in self._gone:
                continue
            ci = self._idx if self._idxs is None else self._idxs[c]
            if ci is not idx:
                continue
            v = self._src[c]
            # contiguous sources only: a strided view (a column of a stacked value matrix) would be copied whole by
            # .contiguous() for a small gather; it keeps its own index_select
            if isinstance(v, StringColumn):
                if v.data.device != idx.device or not (v.starts.is_contiguous() and v.ends.is_contiguous()):
                    continue
                names.append((c, v))
                parts.append(2)
                srcs += [v.starts, v.ends]
            elif (isinstance(v, torch.Tensor) and v.device == idx.device and v.dim() >= 1 and v.dtype != torch.bool
                  and v.is_contiguous()):
                names.append((c, v))
                parts.append(1)
                srcs.append(v)
        if len(srcs) < 2:
            return
        out = take_many(srcs, idx)
        j = 0
        for (c, v), p in zip(names, parts):
            if p == 2:
                r = StringColumn.view(v.data, out[j], out[j + 1], v.payload, v.buf_rows, v._maxlen)
            else:
                r = out[j]
            j += p
            dict.__setitem__(self, c, r)

    def _source(self, k):
        """(source column, row ids or None) of a column not gathered yet."""
        return self._src[k], (self._idx if self._idxs is None else self._idxs[k])

    @staticmethod
    def merged(parts) -> "LazyTakeColumns":
        """The columns of several row selections side by side (a join's output: the probe side's columns at the probe
        rows next to the build side's at the build rows), each still gathered only when first read. ``parts``: (batch,
        column names) in output order; a later part's column of the same name wins, as in a dict."""
        src, idxs = {}, {}
        for b, names in parts:
            cols = b.columns
            lazy = isinstance(cols, LazyTakeColumns)
            for c in names:
                if lazy and not dict.__contains__(cols, c) and c not in cols._gone and c in cols._src:
                    src[c], idxs[c] = cols._source(c)
                else:
                    src[c], idxs[c] = cols[c], None
        return LazyTakeColumns(src, None, idxs)

    def __getitem__(self, k):
        if dict.__contains__(self, k):
            return dict.__getitem__(self, k)
        if k in self._src and k not in self._gone:
            return self._fetch(k)
        raise KeyError(k)

    def __setitem__(self, k, v):
        self._gone.discard(k)
        dict.__setitem__(self, k, v)

    def __delitem__(self, k):
        if k not in self:
            raise KeyError(k)
        if dict.__contains__(self, k):
            dict.__delitem__(self, k)
        if k in self._src:
            self._gone.add(k)

    def __contains__(self, k):
        return dict.__contains__(self, k) or (k in self._src and k not in self._gone)

    def keys(self):
        ks = [k for k in self._src if k not in self._gone]
        ks += [k for k in dict.keys(self) if k not in self._src]
        return ks

    def __iter__(self):
        return iter(self.keys())

    def __len__(self):
        return len(self.keys())

    def values(self):
        return _LazyView(self, False)     # gathers as it iterates (a loop that stops early gathers no more)

    def items(self):
        return _LazyView(self, True)

    def get(self, k, default=None):
        return self[k] if k in self else default

    def pop(self, k, *default):
        if k in self:
            v = self[k]
            del self[k]
            return v
        if default:
            return default[0]
        raise KeyError(k)

    def copy(self):
        return dict(self.items())

    def update(self, other=(), **kw):
        for k, v in (other.items() if hasattr(other, "items") else other):
            self[k] = v
        for k, v in kw.items():
            self[k] = v

    def setdefault(self, k, default=None):
        if k not in self:
            self[k] = default
        return self[k]

    def __repr__(self):
        return repr(dict(self.items()))


class RecordBatch:
    """Columnar batch of records of one type (or an anonymous tuple set when type is None)."""

    __slots__ = ("type", "columns", "n")

    def __init__(self, columns: Dict[str, Any], n: Optional[int] = None, type_: Optional[type] = None):
        self.columns = columns
        self.type = type_
        if n is None:
            n = 0
            for c in columns.values():
                n = column_len(c)
                break
        self.n = n

    def __len__(self):
        return self.n

    def __getitem__(self, name):
        return self.columns[name]

    def names(self) -> List[str]:
        return list(self.columns)

    @property
    def device(self) -> torch.device:
        cols = self.columns
        if isinstance(cols, LazyTakeColumns):
            cols = cols._src                 # a row selection lives where its source does: nothing gathered to answer
        if type(cols) is dict:
            for c in cols.values():              # fast path: the first column is a tensor (asked per batch and atom)
                if isinstance(c, torch.Tensor):
                    return c.device
                break
        from .nested import NestedColumn

        for c in cols.values():
            if isinstance(c, (torch.Tensor, StringColumn, NestedColumn)):
                return c.device
        for c in cols.values():             # only object columns: where their records live (a scan's tuple set)
            if isinstance(c, RecordBatch):
                return c.device
        return torch.device("cpu")

    @staticmethod
    def from_objects(objs: Sequence[PDBObject], type_: Optional[type] = None,
                     device: Optional[torch.device] = None) -> "RecordBatch":
        objs = list(objs)
        if type_ is None:
            if not objs:
                raise ValueError("empty object list needs an explicit type")
            type_ = type(objs[0])
        cols: Dict[str, Any] = {}
        for name, ft in type_.__fields__.items():
            vals = [getattr(o, name) for o in objs]
            cols[name] = make_column(vals, ft, device)
        return RecordBatch(cols, len(objs), type_)

    @staticmethod
    def empty(type_: type, device=None) -> "RecordBatch":
        return RecordBatch.from_objects([], type_, device)

    def to_objects(self) -> List[PDBObject]:
        if self.type is None:
            return [RecordView(self, i).as_tuple() for i in range(self.n)]
        out = []
        for i in range(self.n):
            o = self.type.__new__(self.type)
            for name in self.type.__fields__:
                setattr(o, name, column_item(self.columns[name], i))
            out.append(o)
        return out

    def take(self, idx) -> "RecordBatch":
        """Gather rows (idx: int64 tensor or list). A wide batch on the GPU gathers lazily: each column on its first
        access (a filter feeding a UDF that reads a few fields of a wide record gathers only those)."""
        n = len(idx) if not isinstance(idx, torch.Tensor) else int(idx.numel())
        if isinstance(idx, torch.Tensor) and len(self.columns) > LAZY_TAKE_MIN_COLS and \
                (idx.is_cuda or LAZY_TAKE_ANY_DEVICE):
            return RecordBatch(LazyTakeColumns(self.columns, idx), n, self.type)
        cols = {}
        for k, c in self.columns.items():
            cols[k] = column_take(c, idx)
        return RecordBatch(cols, n, self.type)

    def slice(self, s: int, e: int) -> "RecordBatch":
        cols = {k: column_slice(c, s, e) for k, c in self.columns.items()}
        return RecordBatch(cols, max(0, min(e, self.n) - s), self.type)

    def to(self, device) -> "RecordBatch":
        cols = {k: _col_to(c, device) for k, c in self.columns.items()}
        return RecordBatch(cols, self.n, self.type)

    def nbytes(self) -> int:
        cols = self.columns
        if isinstance(cols, LazyTakeColumns):
            # columns not gathered yet: their source's bytes scaled to the selected rows (no gather to measure)
            total = 0
            for k in cols.keys():
                if dict.__contains__(cols, k):
                    total += _col_nbytes(dict.__getitem__(cols, k))
                else:
                    src = cols._src[k]
                    total += _col_nbytes(src) * self.n // max(1, column_len(src))
            return total
        return sum(_col_nbytes(c) for c in cols.values())

    def materialize(self) -> "RecordBatch":
        """This batch with every lazily gathered column gathered (drops the reference to the source columns)."""
        if isinstance(self.columns, LazyTakeColumns):
            return RecordBatch(dict(self.columns.items()), self.n, self.type)
        return self

    @staticmethod
    def concat(batches: Sequence["RecordBatch"]) -> "RecordBatch":
        batches = [b for b in batches if b is not None]
        if not batches:
            raise ValueError("nothing to concatenate")
        nonempty = [b for b in batches if b.n > 0] or batches[:1]
        first = nonempty[0]
        if len(nonempty) == 1:               # nothing to join: a shallow copy (a lazy selection stays lazy)
            c = first.columns
            if isinstance(c, LazyTakeColumns):
                cp = LazyTakeColumns(c._src, c._idx, c._idxs)
                cp._gone = set(c._gone)
                dict.update(cp, dict.items(c))
            else:
                cp = dict(c)
            return RecordBatch(cp, first.n, first.type)
        cols = {}
        for k in first.columns:
            parts = [b.columns[k] for b in nonempty]
            cols[k] = column_concat(parts)
        return RecordBatch(cols, sum(b.n for b in nonempty), first.type)

    def __repr__(self):
        t = self.type.type_name() if self.type else "tuple"
        return f"RecordBatch<{t}>(n={self.n}, cols={list(self.columns)})"


def _col_nbytes(c) -> int:
    if isinstance(c, torch.Tensor):
        return c.numel() * c.element_size()
    if isinstance(c, RecordBatch):
        return c.nbytes()
    if isinstance(c, StringColumn) or hasattr(c, "offsets"):
        return c.nbytes
    if isinstance(c, tuple):
        return sum(x.numel() * x.element_size() if isinstance(x, torch.Tensor) else 16 * len(x) for x in c)
    return 16 * len(c) + sum(_obj_size(x) for x in c[:64]) * max(1, len(c) // max(1, min(64, len(c))))


def _col_to(c, device):
    if isinstance(c, torch.Tensor):
        return c.to(device, non_blocking=True)
    if isinstance(c, StringColumn):
        return c.to(device)
    if is_string_list(c) and use_device_strings(device):
        return StringColumn.from_list(c, device)
    if isinstance(c, RecordBatch):
        return c.to(device)
    if isinstance(c, tuple):
        return tuple(_col_to(x, device) for x in c)
    if hasattr(c, "offsets") and hasattr(c, "to"):        # NestedColumn / MapColumn
        return c.to(device)
    return c


def _obj_size(x) -> int:
    if isinstance(x, (bytes, str)):
        return len(x)
    if isinstance(x, torch.Tensor):
        return x.numel() * x.element_size()
    if isinstance(x, (list, tuple)):
        return 8 * len(x)
    return 16


def make_column(vals: List[Any], ft, device=None):
    kind = column_kind(ft)
    if kind == "scalar":
        return torch.tensor(vals, dtype=SCALAR_TYPES[ft], device=device) if vals else \
            torch.empty(0, dtype=SCALAR_TYPES[ft], device=device)
    if kind == "tensor":
        if not vals:
            shape = ft.shape if isinstance(ft, Tensor) and ft.shape else (0,)
            dt = ft.dtype if isinstance(ft, Tensor) else torch.float32
            return torch.empty((0,) + tuple(shape), dtype=dt, device=device)
        ts = [v if isinstance(v, torch.Tensor) else torch.as_tensor(v) for v in vals]
        if all(t.shape == ts[0].shape for t in ts):
            out = torch.stack(ts)
            if isinstance(ft, Tensor) and ft.dtype is not None:
                out = out.to(ft.dtype)
            return out.to(device) if device is not None else out
        return [t.to(device) if device is not None else t for t in ts]
    if kind == "nested":
        from .nested import NestedColumn

        return NestedColumn.from_lists([list(v) if v is not None else [] for v in vals], ft.elem, device)
    if kind == "map":
        from .nested import MapColumn

        return MapColumn.from_dicts([dict(v) if v is not None else {} for v in vals], device)
    if kind == "struct":
        objs = [v.materialize() if isinstance(v, RecordView) else v for v in vals]
        return RecordBatch.from_objects(objs, ft, device)
    if ft is str or (vals and all(isinstance(v, str) for v in vals) and ft is not object):
        return list(vals)
    return list(vals)


def _adjacent_tensors(parts, check: bool = True) -> Optional[torch.Tensor]:
    """One view over row-slices that sit back to back in one storage (pages cut from one loaded batch), else None.
    ``check=False``: the caller already verified the layout (a cached scan plan)."""
    p0 = parts[0]
    if p0.dim() == 0:
        return None
    if check:
        ptr, stride, inner = p0.untyped_storage().data_ptr(), p0.stride(), p0.shape[1:]
        off = p0.storage_offset() + p0.shape[0] * stride[0]
        for p in parts[1:]:
            if (p.untyped_storage().data_ptr() != ptr or p.dtype != p0.dtype or p.stride() != stride
                    or p.shape[1:] != inner or p.storage_offset() != off):
                return None
            off += p.shape[0] * stride[0]
    n = sum(p.shape[0] for p in parts)
    return p0.as_strided((n,) + tuple(p0.shape[1:]), p0.stride(), p0.storage_offset())


def merge_adjacent_column(parts, check: bool = True):
    """Zero-copy merge of one column's page slices (None when they are not views of one buffer)."""
    c0 = parts[0]
    if isinstance(c0, torch.Tensor):
        return _adjacent_tensors(parts, check) if all(isinstance(p, torch.Tensor) for p in parts) else None
    if isinstance(c0, StringColumn):
        if not all(isinstance(p, StringColumn) and p.data is c0.data for p in parts):
            return None
        if all(p.is_packed for p in parts):
            offs = [p._off for p in parts]
            o0 = offs[0]
            ok = True
            if check:
                ptr, pos = o0.untyped_storage().data_ptr(), o0.storage_offset() + o0.numel() - 1
                for o in offs[1:]:
                    if o.untyped_storage().data_ptr() != ptr or o.stride() != (1,) or o.storage_offset() != pos:
                        ok = False
                        break
                    pos += o.numel() - 1
            if not ok:
                return None
            n = sum(len(p) for p in parts)
            return StringColumn(c0.data, o0.as_strided((n + 1,), (1,), o0.storage_offset()),
                                max(p.payload for p in parts), c0.buf_rows, StringColumn.max_bound(parts))
        # views: their row-bound arrays must themselves be adjacent slices (no copy is ever made here)
        st = _adjacent_tensors([p.starts for p in parts], check)
        en = _adjacent_tensors([p.ends for p in parts], check) if st is not None else None
        if st is None or en is None:
            return None
        return StringColumn.view(c0.data, st, en, max(p.payload for p in parts), max(p.buf_rows for p in parts),
                                 StringColumn.max_bound(parts))
    if isinstance(c0, tuple):
        subs = [merge_adjacent_column([p[i] for p in parts], check) for i in range(len(c0))]
        return None if any(x is None for x in subs) else tuple(subs)
    if isinstance(c0, RecordBatch):
        return merge_adjacent_batches(parts, check)
    return None


def merge_adjacent_batches(batches: Sequence["RecordBatch"], check: bool = True) -> Optional["RecordBatch"]:
    """The batches as ONE batch without copying row data, when every column of each is a row-slice of the same
    buffer as the previous one's (device pages of one set loaded from one batch); None otherwise."""
    b0 = batches[0]
    cols = {}
    for k in b0.columns:
        parts = [b.columns.get(k) for b in batches]
        if any(x is None for x in parts):
            return None
        m = merge_adjacent_column(parts, check)
        if m is None:
            return None
        cols[k] = m
    return RecordBatch(cols, sum(b.n for b in batches), b0.type)


def column_slice(c, s, e):
    if isinstance(c, RecordBatch):
        return c.slice(s, e)
    if isinstance(c, tuple):
        return tuple(column_slice(x, s, e) for x in c)
    return c[s:e]


def column_len(c) -> int:
    if isinstance(c, tuple):
        return column_len(c[0]) if c else 0
    return len(c)


def column_item(c, i):
    if isinstance(c, RecordBatch):
        return RecordView(c, i)
    if isinstance(c, tuple):
        return tuple(column_item(x, i) for x in c)
    if isinstance(c, torch.Tensor):
        v = c[i]
        return v.item() if v.dim() == 0 else v
    return c[i]


def column_take(c, idx):
    from .nested import NestedColumn

    if isinstance(c, (RecordBatch, StringColumn, NestedColumn)):
        return c.take(idx)
    if isinstance(c, tuple):
        return tuple(column_take(x, idx) for x in c)
    if isinstance(c, torch.Tensor):
        if not isinstance(idx, torch.Tensor):
            idx = torch.as_tensor(idx, dtype=torch.long)
        return c.index_select(0, idx.to(c.device))
    if isinstance(idx, torch.Tensor):
        idx = idx.tolist()
    return [c[i] for i in idx]


def column_concat(parts):
    from .nested import MapColumn, NestedColumn

    if parts and all(isinstance(p, RecordBatch) for p in parts):
        return RecordBatch.concat(parts)
    if parts and all(isinstance(p, MapColumn) for p in parts):
        return MapColumn.concat(parts)
    if parts and all(isinstance(p, NestedColumn) for p in parts):
        return NestedColumn.concat(parts)
    if parts and all(isinstance(p, tuple) for p in parts):
        return tuple(column_concat([p[i] for p in parts]) for i in range(len(parts[0])))
    if parts and any(isinstance(p, StringColumn) for p in parts):
        sc = next(p for p in parts if isinstance(p, StringColumn))
        return StringColumn.concat([p if isinstance(p, StringColumn) else StringColumn.from_list(p, sc.device)
                                    for p in parts])
    if all(isinstance(p, torch.Tensor) for p in parts):
        if len(parts) == 1:
            return parts[0]
        if all(p.shape[1:] == parts[0].shape[1:] for p in parts):
            dev = parts[0].device
            return torch.cat([p.to(dev) for p in parts])
        out = []
        for p in parts:
            out.extend(list(p))
        return out
    out = []
    for p in parts:
        out.extend(list(p) if not isinstance(p, torch.Tensor) else list(p))
    return out


class RecordView:
    """Object-at-a-time view of row ``i`` of a batch (what a ``Handle<T>`` dereference gives)."""

    __slots__ = ("_b", "_i")

    def __init__(self, batch: RecordBatch, i: int):
        object.__setattr__(self, "_b", batch)
        object.__setattr__(self, "_i", i)

    def __getattr__(self, name):
        b = object.__getattribute__(self, "_b")
        i = object.__getattribute__(self, "_i")
        if name in b.columns:
            return column_item(b.columns[name], i)
        t = b.type
        if t is not None and hasattr(t, name):
            attr = getattr(t, name)
            if callable(attr):
                return lambda *a, **k: attr(self, *a, **k)
            return attr
        raise AttributeError(name)

    def materialize(self):
        b = object.__getattribute__(self, "_b")
        i = object.__getattribute__(self, "_i")
        if b.type is None:
            return self.as_tuple()
        o = b.type.__new__(b.type)
        for name in b.type.__fields__:
            setattr(o, name, column_item(b.columns[name], i))
        return o

    def as_tuple(self):
        b = object.__getattribute__(self, "_b")
        i = object.__getattribute__(self, "_i")
        return tuple(column_item(c, i) for c in b.columns.values())

    def __repr__(self):
        return f"RecordView({self.materialize()!r})"


def batch_of(records: Iterable[Any], type_=None, device=None) -> RecordBatch:
    """Build a batch from PDBObjects or RecordViews."""
    objs = [r.materialize() if isinstance(r, RecordView) else r for r in records]
    return RecordBatch.from_objects(objs, type_, device)


__all__ = ["PDBObject", "Tensor", "Vector", "Map", "RecordBatch", "RecordView", "register_type", "lookup_type",
           "registered_types", "batch_of", "make_column", "column_item", "column_take", "column_concat",
           "column_kind", "column_slice", "column_len"]
