"""Device-resident string columns.

The reference stores ``pdb::String`` objects inside pages (src/objectModel/headers/PDBString.h) and
evaluates string predicates, hash-map keys and joins on them one object at a time on the CPU
(tpchBench selections, StringIntPair maps in serviceBenchmarks/StringHashMapTest). Here a ``str`` column
that lives on a GPU is one :class:`StringColumn`: the UTF-8 bytes of every row packed into one uint8
buffer plus int64 row bounds, both in HBM (packed: ``offsets[n+1]``; a row selection is a view of
starts / ends into the source buffer, see :class:`StringColumn`). Predicates (=, IN, LIKE, prefix/suffix/contains),
hashing for group-by/join keys and gathers are single HIP launches over the whole column
(``csrc/kernels/strings.hip``); Python strings appear only when a caller iterates the column.

The same class runs on CPU tensors (numpy paths with identical results) so the CPU test-suite covers the
logic; on a GPU box the HIP path is mandatory (``_ext.hip()`` raises if the kernels are missing).

Policy: :func:`use_device_strings` decides whether ``RecordBatch.to(device)`` packs ``list[str]`` columns
into a StringColumn — by default only for GPU devices; ``NSDB_DEVICE_STRINGS=1`` forces it everywhere
(used to run the CPU suite through this path), ``=0`` disables it.
"""
from __future__ import annotations

import os
import re
from typing import Iterable, List, Optional, Sequence

import numpy as np
import torch

from .. import _ext

_PAD = 16                        # bytes after the payload that the kernels' dword loads may touch
_ANY = 0xFF                      # '_' wildcard byte in a compiled LIKE pattern (never valid UTF-8)
_M1, _M2, _SEED = 0xBF58476D1CE4E5B9, 0x94D049BB133111EB, 0x9E3779B97F4A7C15
_MASK = (1 << 64) - 1


def to_host(*ts: torch.Tensor) -> List[torch.Tensor]:
    """Host copies of several tensors with ONE synchronisation: device tensors are copied asynchronously (into
    pinned buffers) and the stream is synchronised once, instead of one blocking read per tensor."""
    out = [t.to("cpu", non_blocking=True) if t.device.type == "cuda" else t for t in ts]
    devs = {t.device for t in ts if t.device.type == "cuda"}
    # the multi-column gathers' out-of-range words ride along (record.take_many): a bad row id fails loudly at the
    # next batched host read instead of leaving zeros behind, at no extra synchronisation
    from .record import _TAKE_BAD

    flags = [(d, _TAKE_BAD[d], _TAKE_BAD[d].to("cpu", non_blocking=True)) for d in devs if d in _TAKE_BAD]
    for d in devs:                                              # every device the copies were queued on
        torch.cuda.current_stream(d).synchronize()
    for d, dev_word, host_word in flags:
        if int(host_word[0]) != 0:
            dev_word.zero_()
            raise IndexError(f"take_many: a row id was out of range on {d} (a lazily gathered column)")
    return out


def use_device_strings(device) -> bool:
    flag = os.environ.get("NSDB_DEVICE_STRINGS")
    if flag is not None:
        return flag == "1"
    return device is not None and torch.device(device).type == "cuda"


def _mix_py(x: int) -> int:
    x ^= x >> 30
    x = (x * _M1) & _MASK
    x ^= x >> 27
    x = (x * _M2) & _MASK
    x ^= x >> 31
    return x


def hash_str(s) -> int:
    """Host twin of the kernel's string hash (signed int64, as stored in hash columns)."""
    b = s.encode() if isinstance(s, str) else bytes(s)
    h = _mix_py(len(b) ^ _SEED)
    for p in range(0, len(b), 8):
        h = _mix_py(h ^ int.from_bytes(b[p:p + 8], "little"))
    return h - (1 << 64) if h >= (1 << 63) else h


def _mix_np(x: np.ndarray) -> np.ndarray:
    x = x ^ (x >> np.uint64(30))
    x = x * np.uint64(_M1)
    x = x ^ (x >> np.uint64(27))
    x = x * np.uint64(_M2)
    return x ^ (x >> np.uint64(31))


def _hash_np(buf: np.ndarray, starts: np.ndarray, ends: np.ndarray) -> np.ndarray:
    lens = ends - starts
    with np.errstate(over="ignore"):
        h = _mix_np(lens.astype(np.uint64) ^ np.uint64(_SEED))
        nch = int((lens.max() + 7) // 8) if lens.size else 0
        j = np.arange(8)
        for k in range(nch):
            active = lens > 8 * k
            if not active.any():
                break
            rem = lens - 8 * k
            idx = np.minimum(starts[:, None] + 8 * k + j[None, :], buf.size - 1)
            byts = buf[idx].astype(np.uint64)
            byts[j[None, :] >= rem[:, None]] = 0
            c = (byts << (np.uint64(8) * j.astype(np.uint64))[None, :]).sum(1, dtype=np.uint64)
            h = np.where(active, _mix_np(h ^ c), h)
    return h.view(np.int64)


def _compile_like(pattern: str):
    """LIKE pattern -> (pattern bytes, segment starts, segment lengths, anchor_start, anchor_end)."""
    parts = pattern.split("%")
    anchor_start, anchor_end = not pattern.startswith("%"), not pattern.endswith("%")
    if pattern == "":
        return b"", [], [], True, True
    segs = [p for p in parts if p]
    buf, st, ln = bytearray(), [], []
    for p in segs:
        b = bytes(_ANY if ch == ord("_") else ch for ch in p.encode())
        st.append(len(buf))
        ln.append(len(b))
        buf += b
    return bytes(buf), st, ln, anchor_start, anchor_end


def _literal(segs: Sequence[str], anchor_start: bool, anchor_end: bool):
    buf, st, ln = bytearray(), [], []
    for p in segs:
        b = p.encode()
        if _ANY in b:
            raise ValueError("literal contains byte 0xFF")
        st.append(len(buf))
        ln.append(len(b))
        buf += b
    return bytes(buf), st, ln, anchor_start, anchor_end


def _like_regex(pat, st, ln, a0, a1) -> "re.Pattern[bytes]":
    pieces = [re.escape(pat[s:s + n]).replace(re.escape(bytes([_ANY])), b".") for s, n in zip(st, ln)]
    body = b".*".join(pieces)
    if not pieces:
        return re.compile(rb"\A\Z" if (a0 and a1) else rb"", re.S)
    return re.compile((rb"\A" if a0 else b"") + (body if a0 else b".*" + body) + (rb"\Z" if a1 else b""), re.S)


class StringColumn:
    """n strings over one uint8 buffer ``data`` [>= payload + 16] (4-byte multiple): row i is
    ``data[starts[i]:ends[i]]``. A PACKED column (built from a list, gathered, read from a page) also keeps
    ``offsets`` [n+1] with starts = offsets[:-1], ends = offsets[1:]; a VIEW (the result of :meth:`take`, a
    filter, a join probe) keeps only the index_select'ed starts / ends into its source's buffer, so selecting
    rows costs two device gathers and no device->host read. Kernels take (starts, ends) and so run on either
    form; :attr:`offsets` (serialisation, shuffles) packs a view in place on first use."""

    __slots__ = ("data", "starts", "ends", "_off", "payload", "buf_rows", "_maxlen", "_codes")

    def __init__(self, data: torch.Tensor, offsets: torch.Tensor, payload: int, buf_rows: Optional[int] = None,
                 maxlen: Optional[int] = None):
        self.data, self._off, self.payload = data, offsets, int(payload)
        self.starts, self.ends = offsets[:-1], offsets[1:]
        self.buf_rows = max(1, offsets.numel() - 1) if buf_rows is None else buf_rows   # rows sharing data
        if maxlen is None and offsets.device.type == "cpu" and offsets.numel() > 1:
            maxlen = int(np.diff(offsets.numpy()).max())       # host offsets: free to bound here
        self._maxlen = maxlen     # upper bound of the row lengths (None: not known yet, see max_len)
        self._codes = None        # (L, short codes) once computed: the column's fixed-width encoding, kept

    @staticmethod
    def view(data: torch.Tensor, starts: torch.Tensor, ends: torch.Tensor, payload: int,
             buf_rows: int, maxlen: Optional[int] = None) -> "StringColumn":
        c = StringColumn.__new__(StringColumn)
        c.data, c.starts, c.ends, c._off, c.payload, c.buf_rows = data, starts, ends, None, int(payload), buf_rows
        c._maxlen = maxlen
        c._codes = None
        return c

    # ------------------------------------------------------------------ construction
    @staticmethod
    def _alloc_size(payload: int) -> int:
        return ((payload + _PAD + 3) // 4) * 4

    @staticmethod
    def from_list(strs: Iterable, device=None) -> "StringColumn":
        enc = [s.encode() if isinstance(s, str) else bytes(s) for s in strs]
        lens = np.fromiter((len(b) for b in enc), dtype=np.int64, count=len(enc))
        off = np.zeros(len(enc) + 1, dtype=np.int64)
        np.cumsum(lens, out=off[1:])
        payload = int(off[-1])
        buf = np.zeros(StringColumn._alloc_size(payload), dtype=np.uint8)
        if payload:
            buf[:payload] = np.frombuffer(b"".join(enc), dtype=np.uint8)
        data, offs = torch.from_numpy(buf), torch.from_numpy(off)
        if device is not None and torch.device(device).type != "cpu":
            data, offs = data.pin_memory().to(device, non_blocking=True), offs.pin_memory().to(device, non_blocking=True)
        return StringColumn(data, offs, payload, maxlen=int(lens.max()) if len(enc) else 0)

    @staticmethod
    def empty(device=None) -> "StringColumn":
        return StringColumn.from_list([], device)

    # ------------------------------------------------------------------ sequence protocol
    @property
    def device(self) -> torch.device:
        return self.data.device

    def __len__(self) -> int:
        return self.starts.numel()

    @property
    def is_packed(self) -> bool:
        return self._off is not None

    @property
    def offsets(self) -> torch.Tensor:
        """[n+1] row offsets; a view is packed into its own buffer first (one device->host read of the size)."""
        if self._off is None:
            p = self.compact()
            self.data, self.starts, self.ends, self._off, self.payload, self.buf_rows = (
                p.data, p.starts, p.ends, p._off, p.payload, p.buf_rows)
        return self._off

    def lengths(self) -> torch.Tensor:
        return self.ends - self.starts

    def _host(self):
        d, st, en = to_host(self.data[: self.payload], self.starts, self.ends)
        return d.numpy(), st.numpy(), en.numpy()

    def tolist(self) -> List[str]:
        buf, st, en = self._host()
        raw = buf.tobytes()
        return [raw[s:e].decode() for s, e in zip(st.tolist(), en.tolist())]

    def __iter__(self):
        return iter(self.tolist())

    def __array__(self, dtype=None, copy=None):
        return np.array(self.tolist(), dtype=object)

    def __getitem__(self, i):
        if isinstance(i, slice):
            s, e, step = i.indices(len(self))
            if step != 1:
                return self.take(torch.arange(s, e, step, dtype=torch.long))
            e = max(e, s)
            if self._off is not None:
                out = StringColumn(self.data, self._off[s:e + 1], self.payload, self.buf_rows, self._maxlen)
            else:
                out = StringColumn.view(self.data, self.starts[s:e], self.ends[s:e], self.payload, self.buf_rows,
                                        self._maxlen)
            if self._codes is not None:
                out._codes = (self._codes[0], self._codes[1][s:e])
            return out
        if isinstance(i, (torch.Tensor, list, np.ndarray)):
            return self.take(i)
        n = len(self)
        if i < 0:
            i += n
        if not 0 <= i < n:
            raise IndexError(i)
        s, e = int(self.starts[i]), int(self.ends[i])
        return bytes(self.data[s:e].cpu().numpy()).decode()

    def __repr__(self):
        kind = "packed" if self.is_packed else "view"
        return f"StringColumn(n={len(self)}, {kind}, buffer_bytes={self.payload}, device={self.device})"

    @property
    def nbytes(self) -> int:
        """Bytes this column accounts for: a slice / view of a shared buffer is charged its row share,
        estimated without reading the device offsets."""
        return self.data.numel() * len(self) // max(1, self.buf_rows) + 16 * len(self)

    def to(self, device) -> "StringColumn":
        device = torch.device(device)
        if device == self.device:
            return self
        if self._off is None and len(self) < self.buf_rows // 2:
            return self.compact().to(device)          # do not move a large shared buffer for a few rows
        # host sources are staged through pinned memory so the copies stay asynchronous (no stream sync)
        mv = ((lambda t: t.pin_memory().to(device, non_blocking=True)) if self.device.type == "cpu"
              and device.type == "cuda" else (lambda t: t.to(device, non_blocking=True)))
        data = mv(self.data)
        if self._off is not None:
            return StringColumn(data, mv(self._off), self.payload, self.buf_rows, self._maxlen)
        return StringColumn.view(data, mv(self.starts), mv(self.ends), self.payload, self.buf_rows, self._maxlen)

    def compact(self) -> "StringColumn":
        """Own packed buffer holding exactly these rows (one device->host read of the byte total)."""
        dev, n = self.device, len(self)
        lens = self.ends - self.starts
        out_off = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        if n:
            torch.cumsum(lens, 0, out=out_off[1:])
        total = int(out_off[-1]) if n else 0
        if dev.type == "cuda":
            data = _ext.hip().str_gather(self.data, self.starts.contiguous(), self.ends.contiguous(), None,
                                         out_off, total)
        else:
            data_np = np.zeros(self._alloc_size(total), dtype=np.uint8)
            if total:
                st, ln = self.starts.numpy(), lens.numpy()
                pos = np.repeat(st - out_off[:-1].numpy(), ln) + np.arange(total)
                data_np[:total] = self.data.numpy()[pos]
            data = torch.from_numpy(data_np)
        return StringColumn(data, out_off, total, maxlen=self._maxlen)

    # ------------------------------------------------------------------ relational ops
    def take(self, idx) -> "StringColumn":
        """Rows ``idx`` (int positions or a bool mask) as a view over this buffer: two index_selects (bounds are
        checked by index_select itself), no device->host read for int indices."""
        dev = self.device
        if not isinstance(idx, torch.Tensor):
            idx = torch.as_tensor(np.asarray(idx, dtype=np.int64) if len(idx) else np.zeros(0, np.int64))
        idx = idx.to(dev)
        if idx.dtype == torch.bool:
            idx = idx.nonzero().flatten()
        idx = idx.long()
        if dev.type != "cuda" and idx.numel():
            ii = idx.numpy()
            if ii.min() < -len(self) or ii.max() >= len(self):
                raise IndexError("string take index out of range")
        return StringColumn.view(self.data, self.starts.index_select(0, idx), self.ends.index_select(0, idx),
                                 self.payload, self.buf_rows, self._maxlen)

    def substr(self, start: int, length: int) -> "StringColumn":
        """SQL SUBSTRING(s FROM start + 1 FOR length) of every row, on bytes (0-based ``start``): lengths clamped
        and prefix-summed on the device, one copy launch, no device->host read (the output buffer is sized by the
        host-known bound n * length)."""
        if start < 0 or length < 0:
            raise ValueError("substr: start and length must be >= 0")
        dev, n = self.device, len(self)
        new = (self.ends - self.starts - start).clamp(min=0, max=length)
        out_off = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        if n:
            torch.cumsum(new, 0, out=out_off[1:])
        cap = n * length
        if dev.type == "cuda":
            data = _ext.hip().str_slice(self.data, self.starts.contiguous(), self.ends.contiguous(), int(start),
                                        out_off, cap)
        else:
            src, st, oo = self.data.numpy(), self.starts.numpy(), out_off.numpy()
            data_np = np.zeros(self._alloc_size(cap), dtype=np.uint8)
            total = int(oo[-1])
            if total:
                ln = oo[1:] - oo[:-1]
                pos = np.repeat(st + start - oo[:-1], ln) + np.arange(total)
                data_np[:total] = src[pos]
            data = torch.from_numpy(data_np)
        bound = length if self._maxlen is None else max(0, min(length, self._maxlen - start))
        return StringColumn(data, out_off, cap, maxlen=bound)

    @staticmethod
    def concat(parts: Sequence["StringColumn"]) -> "StringColumn":
        parts = [p for p in parts if len(p)] or list(parts[:1])
        if not parts:
            return StringColumn.empty()
        if len(parts) == 1:
            return parts[0]                  # nothing to join (a one-batch group-by used to copy its row bounds here)
        dev = parts[0].device
        parts = [p.to(dev) for p in parts]
        d0 = parts[0].data
        if all(p.data is d0 for p in parts):
            # rows of one buffer (the pages / filtered slices of one set): concatenate the row bounds only
            return StringColumn.view(d0, torch.cat([p.starts for p in parts]), torch.cat([p.ends for p in parts]),
                                     max(p.payload for p in parts), max(p.buf_rows for p in parts),
                                     StringColumn.max_bound(parts))
        parts = [p if p.is_packed else p.compact() for p in parts]
        datas, offs, base = [], [torch.zeros(1, dtype=torch.int64, device=dev)], 0
        for p in parts:
            o0 = p._off[:1]
            o = p._off - o0
            datas.append((p.data, o0, p._off[-1:]))
            offs.append(o[1:] + base)
            base = base + (o[-1])
        # byte ranges: each packed part's rows are contiguous in its buffer from offsets[0] to offsets[-1]
        bounds = torch.stack([torch.cat([s, e]) for _, s, e in datas]).cpu().tolist()
        total = sum(e - s for s, e in bounds)
        data = torch.zeros(StringColumn._alloc_size(total), dtype=torch.uint8, device=dev)
        pos = 0
        for (d, _, _), (s, e) in zip(datas, bounds):
            data[pos:pos + e - s] = d[s:e]
            pos += e - s
        return StringColumn(data, torch.cat(offs), total, maxlen=StringColumn.max_bound(parts))

    @staticmethod
    def max_bound(parts: Sequence["StringColumn"]) -> Optional[int]:
        """Largest row-length bound of several columns (None if any is unknown)."""
        b = [p._maxlen for p in parts]
        return None if any(x is None for x in b) else max(b, default=0)

    def max_len(self) -> int:
        """An upper bound of the row lengths (exact when computed here: one device reduction + host read, cached)."""
        if self._maxlen is None:
            self._maxlen = int((self.ends - self.starts).amax()) if len(self) else 0
        return self._maxlen

    def short_codes(self, L: Optional[int] = None) -> Optional[torch.Tensor]:
        """Exact int64 code per row when every row is <= 7 bytes, else None: bytes big-endian in the low 8L bits
        (L = :meth:`max_len`, or a larger given bound), shifted left 3, OR the length. Equal codes <=> equal
        strings and code order = byte order, so short string keys group, join and sort as integers (no hash, no
        byte re-check).

        The codes are the column's fixed-width encoding (8 bytes a row, like the dictionary / inline encoding a
        column store keeps for short strings): computed once per column and bound L, then kept with the column, so
        a scan that groups or filters on a short string reads one int64 per row instead of two offsets and the
        bytes. Callers must not modify the returned tensor in place."""
        ml = self.max_len()
        L = ml if L is None else L
        if L > 7 or ml > L:
            return None
        if self._codes is not None and self._codes[0] == L and self._codes[1].device == self.device:
            return self._codes[1]
        if self.device.type == "cuda":
            codes = _ext.hip().str_pack(self.data, self.starts.contiguous(), self.ends.contiguous(), L)
            self._codes = (L, codes)
            return codes
        st, en, buf = self.starts.numpy(), self.ends.numpy(), self.data.numpy()
        ln = en - st
        be = np.zeros(len(st), dtype=np.int64)
        for j in range(L):
            b = buf[np.minimum(st + j, buf.size - 1)].astype(np.int64)
            be |= np.where(ln > j, b, 0) << (8 * (L - 1 - j))
        return torch.from_numpy((be << 3) | ln)

    def short_codes32(self, L: Optional[int] = None) -> Optional[torch.Tensor]:
        """:meth:`short_codes` as int32 when every code fits (L <= 3: at most 27 bits), kept with the column like
        the int64 codes: a fused scan reads 4 instead of 8 bytes per row of a flag / mode column. None otherwise."""
        L = self.max_len() if L is None else L
        if L > 3:
            return None
        c = self.short_codes(L)
        if c is None:
            return None
        kept = self._codes is not None and self._codes[0] == L and self._codes[1] is c
        if kept and len(self._codes) > 2 and self._codes[2] is not None:
            return self._codes[2]
        c32 = c.to(torch.int32)
        if kept:
            self._codes = (self._codes[0], self._codes[1], c32)
        return c32

    @staticmethod
    def from_short_codes(codes: torch.Tensor, L: int) -> "StringColumn":
        """Inverse of :meth:`short_codes` (codes made with bound ``L``), on the codes' device."""
        dev, n = codes.device, codes.numel()
        if dev.type == "cpu" and n <= 65536:
            # a fused aggregation's few decoded group keys: numpy (torch's per-op CPU dispatch is ~10x slower here)
            c = codes.numpy().astype(np.int64, copy=False)
            ln = c & 7
            off = np.zeros(n + 1, dtype=np.int64)
            np.cumsum(ln, out=off[1:])
            total = int(off[-1]) if n else 0
            data = np.zeros(StringColumn._alloc_size(total), dtype=np.uint8)
            if total:
                j = np.arange(L, dtype=np.int64)
                byts = (c[:, None] >> (3 + 8 * (L - 1 - j))[None, :]) & 0xFF
                data[:total] = byts[j[None, :] < ln[:, None]].astype(np.uint8)
            return StringColumn(torch.from_numpy(data), torch.from_numpy(off), total, maxlen=L)
        lens = codes & 7
        off = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        if n:
            torch.cumsum(lens, 0, out=off[1:])
        total = int(off[-1]) if n else 0
        data = torch.zeros(StringColumn._alloc_size(total), dtype=torch.uint8, device=dev)
        if total:
            j = torch.arange(L, device=dev, dtype=torch.int64)
            byts = (codes.unsqueeze(1) >> (3 + 8 * (L - 1 - j)).unsqueeze(0)) & 0xFF
            data[:total] = byts[j.unsqueeze(0) < lens.unsqueeze(1)].to(torch.uint8)
        return StringColumn(data, off, total, maxlen=L)

    def hash64(self) -> torch.Tensor:
        """int64 hash per row (== :func:`hash_str` of the row)."""
        if self.device.type == "cuda":
            return _ext.hip().str_hash(self.data, self.starts.contiguous(), self.ends.contiguous(), self.payload)
        return torch.from_numpy(_hash_np(self.data.numpy(), self.starts.numpy(), self.ends.numpy()).copy())

    def eq_rows(self, ia: Optional[torch.Tensor], other: "StringColumn", ib: Optional[torch.Tensor]) -> torch.Tensor:
        """Byte-exact ``self[ia[i]] == other[ib[i]]`` for every i (ia / ib None: the identity), as a bool mask: the
        exact check behind hash-decided group-by / join / IN (reference pdb::String equality, PDBString.h:46-48)."""
        m = len(self) if ia is None else ia.numel()
        dev = self.device
        other = other.to(dev)
        if m == 0:
            return torch.zeros(0, dtype=torch.bool, device=dev)
        # resolve the indices into row bounds with index_select (bounds-checked by torch, no host read)
        sa, ea = (self.starts, self.ends) if ia is None else (self.starts.index_select(0, ia.to(dev).long()),
                                                              self.ends.index_select(0, ia.to(dev).long()))
        sb, eb = (other.starts, other.ends) if ib is None else (other.starts.index_select(0, ib.to(dev).long()),
                                                                other.ends.index_select(0, ib.to(dev).long()))
        if sb.numel() < m:
            raise IndexError("eq_rows: other has fewer rows than compared")
        if dev.type == "cuda":
            return _ext.hip().str_eq_pairs(self.data, sa.contiguous(), ea.contiguous(), None, other.data,
                                           sb.contiguous(), eb.contiguous(), None, m)
        sa, la = sa.numpy()[:m], (ea - sa).numpy()[:m]
        sb, lb = sb.numpy()[:m], (eb - sb).numpy()[:m]
        eq = la == lb
        idx = np.nonzero(eq & (la > 0))[0]
        if idx.size:
            ln = la[idx]
            tot = int(ln.sum())
            rel = np.arange(tot) - np.repeat(np.cumsum(ln) - ln, ln)
            da, db = self.data.numpy(), other.data.numpy()
            same = da[np.repeat(sa[idx], ln) + rel] == db[np.repeat(sb[idx], ln) + rel]
            ok = np.minimum.reduceat(same, np.cumsum(ln) - ln)
            eq[idx] = ok.astype(bool)
        return torch.from_numpy(eq)

    def _match(self, compiled, negate=False) -> torch.Tensor:
        pat, st, ln, a0, a1 = compiled
        if self.device.type == "cuda":
            return _ext.hip().str_like(self.data, self.starts.contiguous(), self.ends.contiguous(), self.payload,
                                       pat, st, ln, a0, a1, negate)
        rx = _like_regex(pat, st, ln, a0, a1)
        buf, ss, ee = self._host()
        raw = buf.tobytes()
        out = np.fromiter((rx.search(raw[s:e]) is not None for s, e in zip(ss.tolist(), ee.tolist())),
                          dtype=bool, count=len(self))
        return torch.from_numpy(out != negate)

    def like(self, pattern: str, negate: bool = False) -> torch.Tensor:
        """SQL ``LIKE`` ('%' any run, '_' any single byte) -> bool mask on the column's device."""
        c = _compile_like(pattern)
        if len(c[0]) > 224 or len(c[1]) > 16:
            raise ValueError("LIKE pattern longer than 224 bytes / 16 segments")
        return self._match(c, negate)

    def eq(self, s: str) -> torch.Tensor:
        return self._match(_literal([s], True, True))

    def startswith(self, s: str) -> torch.Tensor:
        return self._match(_literal([s], True, False))

    def endswith(self, s: str) -> torch.Tensor:
        return self._match(_literal([s], False, True))

    def contains(self, s: str) -> torch.Tensor:
        return self._match(_literal([s], False, False))

    def isin(self, values: Sequence[str]) -> torch.Tensor:
        """Exact membership: a 64-bit hash decides the candidate value (one launch + a sort/search of the
        list's hashes), then every candidate row is byte-compared with that value (str_eq_pairs), so two strings
        with equal hashes are never confused."""
        values = list(dict.fromkeys(values))
        n = len(self)
        if n == 0 or not values:
            return torch.zeros(n, dtype=torch.bool, device=self.device)
        codes = self.short_codes()
        if codes is not None:       # short rows: exact integer membership (values longer than any row never match)
            L = self.max_len()
            fit = [v for v in values if len(v.encode() if isinstance(v, str) else bytes(v)) <= L]
            if not fit:
                return torch.zeros(n, dtype=torch.bool, device=self.device)
            ref = StringColumn.from_list(fit, self.device).short_codes(L)
            return torch.isin(codes, ref)
        h = self.hash64()
        ref = StringColumn.from_list(values, self.device)
        sh, order = torch.sort(ref.hash64())
        pos = torch.searchsorted(sh, h).clamp_(max=len(values) - 1)
        cand = sh.index_select(0, pos) == h
        if bool(torch.unique(sh).numel() != sh.numel()):
            # two listed values share a hash: decide on the host (exact, and never hit in practice)
            allowed = set(values)
            return torch.tensor([s in allowed for s in self.tolist()], dtype=torch.bool, device=self.device)
        return cand & self.eq_rows(None, ref, order.index_select(0, pos))

    def dict_encode(self):
        """(codes int64 [n], dictionary list[str]): device unique over the hashes; only the distinct
        strings cross to the host."""
        from ..execution.kernels import group_ids   # exact (hash + byte re-check) grouping

        inv, reps, _ = group_ids(self)
        return inv, reps.tolist()


def is_string_list(c) -> bool:
    return isinstance(c, list) and len(c) > 0 and all(isinstance(x, str) for x in c)


def as_strings(c, device=None) -> StringColumn:
    return c if isinstance(c, StringColumn) else StringColumn.from_list(c, device)


__all__ = ["StringColumn", "hash_str", "use_device_strings", "is_string_list", "as_strings"]
