"""dbgen ``.tbl`` text ingestion: pipe-delimited TPC-H rows parsed into device columns.

Reference: src/tpch/source/tpchDataLoader.cc — a per-line C++ tokenizer (``:65``, split on '|') that builds one
``Handle<LineItem>`` / ``Handle<Order>`` ... per row and ships them page by page (``:480-653`` load the eight
tables ``customer/lineitem/nation/orders/part/partsupp/region/supplier.tbl``).

MI355X-native design: nothing is parsed per row on the host. The file is streamed in line-aligned chunks
(``chunk_bytes``, default 256 MiB, memory-mapped, pinned, one H2D copy each) and every chunk is parsed by
whole-column tensor operations ON THE DEVICE:

* delimiter and newline positions come from one compare + nonzero over the chunk's bytes; the [rows, fields]
  matrix of field bounds follows from a reshape (every row has exactly one '|' per field, dbgen writes a trailing
  one), validated once per chunk against the newline positions;
* numeric fields are decoded column-wise from a [rows, width] byte window: digits weighted by a power-of-ten table
  indexed by "digits after this one" (a reversed cumulative sum), an optional '-' sign, and decimals divided by
  10^(digits after the '.') — the division of two exact integers, so a value parses to exactly the double Python's
  ``float()`` gives; dates ``YYYY-MM-DD`` become ``int`` yyyymmdd (the digits alone);
* text fields become :class:`StringColumn` views over the chunk buffer (start / end per row), compacted into
  their own packed buffers by the byte-gather kernel so the raw chunk can be freed.

``write_tbl`` writes generated tables in dbgen's format (dates as YYYY-MM-DD, money with two decimals) so the
round trip is testable without dbgen (there is no network to fetch dbgen output).
"""
from __future__ import annotations

import os
import time
from typing import Dict, Iterator, Optional, Sequence

import numpy as np
import torch

from ..objects.record import RecordBatch
from ..objects.strings import StringColumn, use_device_strings
from . import tpch as T

BAR, NL, DOT, MINUS = 124, 10, 46, 45
_POW10 = [10 ** k for k in range(19)]


def _is_date(name: str) -> bool:
    return name.endswith("date")


# ------------------------------------------------------------------------------------------------ writer
def write_tbl(tables: Dict[str, Dict[str, object]], out_dir: str, only: Optional[Sequence[str]] = None) -> Dict[str, str]:
    """Write ``{table: {column: values}}`` (models.tpch.generate / tpch_gen.generate_fast) as dbgen ``<table>.tbl``
    files. Returns {table: path}."""
    import pandas as pd

    os.makedirs(out_dir, exist_ok=True)
    paths = {}
    for name, typ in T.TABLES.items():
        if only is not None and name not in only:
            continue
        cols = {}
        for f, ft in typ.fields().items():
            v = tables[name][f]
            if ft is str:
                cols[f] = v.tolist() if hasattr(v, "tolist") and not isinstance(v, list) else list(v)
            elif ft is float:
                a = np.asarray(v, dtype=np.float64)
                cols[f] = np.char.mod("%.2f", a)
            elif _is_date(f):
                a = np.asarray(v, dtype=np.int64)
                y, m, d = a // 10000, (a // 100) % 100, a % 100
                cols[f] = np.char.add(np.char.add(np.char.add(np.char.zfill(y.astype(str), 4), "-"),
                                                  np.char.add(np.char.zfill(m.astype(str), 2), "-")),
                                      np.char.zfill(d.astype(str), 2))
            else:
                cols[f] = np.asarray(v, dtype=np.int64)
        df = pd.DataFrame(cols)
        df[""] = ""                                  # dbgen's trailing '|'
        path = os.path.join(out_dir, f"{name}.tbl")
        df.to_csv(path, sep="|", header=False, index=False, quoting=3, escapechar=None, lineterminator="\n")
        paths[name] = path
    return paths


# ------------------------------------------------------------------------------------------------ parser
def _field_bounds(buf: torch.Tensor, nc: int):
    """[rows, nc] start / end (exclusive) byte offsets of every field of a chunk of whole lines."""
    bars = (buf == BAR).nonzero().flatten()
    nls = (buf == NL).nonzero().flatten()
    nrows = int(nls.numel())
    if nrows == 0:
        e = torch.empty(0, nc, dtype=torch.int64, device=buf.device)
        return e, e
    if bars.numel() != nrows * nc:
        raise ValueError(f".tbl chunk: {bars.numel()} delimiters for {nrows} rows x {nc} fields")
    ends = bars.view(nrows, nc)
    starts = torch.empty_like(ends)
    starts[:, 1:] = ends[:, :-1] + 1
    starts[0, 0] = 0
    if nrows > 1:
        starts[1:, 0] = nls[:-1] + 1
    # every row's last delimiter lies before its newline and after the previous one
    ok = (ends[:, -1] < nls).all() & (starts[:, 0] <= ends[:, 0]).all()
    if not bool(ok):
        raise ValueError(".tbl chunk: a row does not have exactly one '|' per field")
    return starts, ends


def _parse_numeric(buf: torch.Tensor, s: torch.Tensor, e: torch.Tensor, as_float: bool) -> torch.Tensor:
    """Decode decimal / integer / date fields [s, e) column-wise (no per-row host work)."""
    n = s.numel()
    dev = buf.device
    if n == 0:
        return torch.empty(0, dtype=torch.float64 if as_float else torch.int64, device=dev)
    L = e - s
    W = int(L.max())
    pos = torch.arange(W, device=dev)
    valid = pos.unsqueeze(0) < L.unsqueeze(1)
    idx = (s.unsqueeze(1) + pos.unsqueeze(0)).clamp_(max=buf.numel() - 1)
    b = buf[idx].to(torch.int64)
    isdig = valid & (b >= 48) & (b <= 57)
    d = (b - 48) * isdig
    after = torch.flip(torch.cumsum(torch.flip(isdig.to(torch.int64), [1]), 1), [1]) - isdig.to(torch.int64)
    p10 = torch.tensor(_POW10, dtype=torch.int64, device=dev)
    val = (d * p10[after.clamp_(max=18)]).sum(1)
    neg = b[:, 0] == MINUS
    val = torch.where(neg, -val, val)
    if not as_float:
        return val
    isdot = valid & (b == DOT)
    has_dot = isdot.any(1)
    dot_at = torch.where(has_dot, isdot.to(torch.int64).argmax(1), L)
    frac = (isdig & (pos.unsqueeze(0) > dot_at.unsqueeze(1))).sum(1)
    return val.to(torch.float64) / p10[frac].to(torch.float64)


def parse_tbl(buf: torch.Tensor, table: str, device=None) -> RecordBatch:
    """One chunk of whole ``.tbl`` lines (uint8 tensor) -> a RecordBatch of ``table``'s schema (numbers as int64 /
    float64 tensors, dates as int yyyymmdd, text as StringColumns on the chunk's device, or host lists on a CPU
    device when device strings are off)."""
    typ = T.TABLES[table]
    fields = list(typ.fields().items())
    starts, ends = _field_bounds(buf, len(fields))
    n = starts.shape[0]
    nb = int(buf.numel())
    sbuf = buf                                 # the string kernels read whole words: a padded copy of the chunk
    if StringColumn._alloc_size(nb) != nb:
        sbuf = torch.zeros(StringColumn._alloc_size(nb), dtype=torch.uint8, device=buf.device)
        sbuf[:nb] = buf
    cols = {}
    for j, (f, ft) in enumerate(fields):
        s, e = starts[:, j].contiguous(), ends[:, j].contiguous()
        if ft is str:
            view = StringColumn.view(sbuf, s, e, nb, max(1, n))
            col = view.compact()
            cols[f] = col if use_device_strings(device or buf.device) else col.tolist()
        else:
            cols[f] = _parse_numeric(buf, s, e, ft is float)
            if ft is T.Date32:
                cols[f] = cols[f].to(torch.int32)
    return RecordBatch(cols, n, typ)


def chunk_bounds(path: str, chunk_bytes: int = 256 << 20):
    """[(lo, hi)] byte ranges of line-aligned chunks of a file (each ends after a newline, or at EOF)."""
    size = os.path.getsize(path)
    if size == 0:
        return []
    mm = np.memmap(path, dtype=np.uint8, mode="r")
    out, lo = [], 0
    while lo < size:
        hi = min(size, lo + chunk_bytes)
        while hi < size:
            win = mm[max(lo, hi - (1 << 20)): hi]
            k = np.flatnonzero(win == NL)
            if k.size:
                hi = hi - win.size + int(k[-1]) + 1
                break
            hi = min(size, hi + (1 << 20))            # a line longer than the window: widen
        out.append((lo, hi))
        lo = hi
    return out


def read_chunk(path: str, lo: int, hi: int) -> np.ndarray:
    """Bytes [lo, hi) of a file, newline-terminated."""
    mm = np.memmap(path, dtype=np.uint8, mode="r")
    seg = np.array(mm[lo: hi])
    if seg.size and seg[-1] != NL:                    # last line without a newline
        seg = np.concatenate([seg, np.array([NL], dtype=np.uint8)])
    return seg


def load_tbl(client, db: str, tbl_dir: str, device=None, only: Optional[Sequence[str]] = None,
             chunk_bytes: int = 256 << 20) -> Dict[str, dict]:
    """Create the TPC-H sets of ``db`` and ingest ``<tbl_dir>/<table>.tbl`` (tpchDataLoader.cc). Rank 0 reads and
    parses each chunk on ``device`` (default: the client's) and dispatches it by the set's partition policy
    (send_data: a collective, so every rank takes part chunk by chunk). Returns per-table {rows, bytes, seconds}."""
    dev = torch.device(device) if device is not None else client.device
    client.create_database(db)
    stats = {}
    for name, typ in T.TABLES.items():
        if only is not None and name not in only:
            continue
        path = os.path.join(tbl_dir, f"{name}.tbl")
        client.create_set(db, name, typ)
        t0 = time.perf_counter()
        bounds = chunk_bounds(path, chunk_bytes) if client.ctx.rank == 0 else None
        nchunks = len(bounds) if bounds is not None else 0
        if client.ctx.distributed:
            nchunks = int(client.ctx.all_reduce_scalar(float(nchunks), "max"))
        rows = nbytes = 0
        for i in range(nchunks):
            b = None
            if client.ctx.rank == 0:
                seg = read_chunk(path, *bounds[i])
                host = torch.from_numpy(seg)
                if dev.type == "cuda":
                    host = host.pin_memory()
                buf = host.to(dev, non_blocking=True)
                b = parse_tbl(buf, name, dev)
                del buf
                rows += b.n
                nbytes += seg.size
            client.send_data(db, name, b)
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        stats[name] = {"rows": rows, "bytes": nbytes, "seconds": time.perf_counter() - t0}
    return stats


__all__ = ["write_tbl", "parse_tbl", "chunk_bounds", "read_chunk", "load_tbl"]
