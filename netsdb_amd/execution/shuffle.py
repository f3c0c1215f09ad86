"""Streaming, page-wise distributed hash shuffle (the engine's ShuffleSink).

Reference: src/queryExecution/headers/PipelineStage.h:93-167 (``storeShuffleData``, the combiner circular
buffers and ``runPipelineWithShuffleSink``: shuffle pages leave for their node WHILE the pipeline runs),
ShuffleSink.h, CombinedShuffleSink.h, HashPartitionWork.h and HermesExecutionServer.cc:1270-1274.

MI355X-native form. The pipeline's output batches are hash-partitioned on the device as they are produced
and appended to a local chunk. Once the chunk reaches ``chunk_bytes`` it is sealed: its rows are sorted by
destination rank and every fixed-width column is packed into ONE byte matrix [rows, row_bytes] (all columns
of a row side by side), and the per-destination row counts start an asynchronous device-to-host copy.
A chunk goes on the wire one chunk later (when the next one is sealed, or at the end of the input), so the
host never waits for fresh GPU work: by then its counts have long landed. One round is

  * ONE host all-gather of (send counts, "more rounds follow") over the gloo metadata group (no device
    tensor, no GPU stream sync), then
  * ONE ``all_to_all_single`` of the packed rows, issued asynchronously (RCCL runs it on its own stream
    while the compute stream goes on with the next pipeline batches).

Completed rounds are unpacked into record batches and handed to the consumer (a join build that spills to
a partitioned spool, the final aggregation, the probe side of a partitioned join, a partition sink), so the
per-rank memory of a shuffle is O(chunk) plus what the consumer keeps. Ranks run a different number of
pipeline batches: every rank keeps entering rounds (sending nothing once its input is exhausted) until a
round in which no rank announces more data; the round sequence is the same on every rank, so collectives
stay in lock-step. Columns that are not fixed-width tensors (objects, strings, nested) fall back to the
per-column record-batch exchange of ``ClusterContext.exchange``, still round by round.
"""
from __future__ import annotations

from collections import deque
from typing import Callable, Iterator, List, Optional, Tuple

import torch

from ..objects.record import RecordBatch
from . import kernels as K


class PackedSchema:
    """Fixed-width row image of a flat record batch whose columns are all tensors."""

    def __init__(self, meta: dict):
        self.meta = meta
        self.cols = []          # (name, dtype, shape, byte offset, byte width)
        off = 0
        for cm in meta["columns"]:
            dt = getattr(torch, cm["dtype"])
            shape = tuple(cm["shape"])
            n = 1
            for s in shape:
                n *= s
            w = n * torch.empty((), dtype=dt).element_size()
            self.cols.append((cm["name"], dt, shape, off, w))
            off += w
        self.row_bytes = max(1, off)

    @staticmethod
    def supports(meta: Optional[dict]) -> bool:
        return meta is not None and bool(meta["columns"]) and all(c["kind"] == "tensor" for c in meta["columns"])

    def pack(self, b: RecordBatch) -> torch.Tensor:
        n = b.n
        parts = []
        for name, dt, shape, off, w in self.cols:
            c = b.columns[name]
            if w == 0:
                continue
            cc = c.contiguous().reshape(n, w // c.element_size())
            if cc.stride(-1) != 1:     # one-row views count as contiguous whatever their stride
                cc = cc.clone(memory_format=torch.contiguous_format)
            parts.append(cc.view(torch.uint8).reshape(n, w))
        if not parts:
            return torch.zeros(n, self.row_bytes, dtype=torch.uint8, device=b.device)
        return parts[0] if len(parts) == 1 else torch.cat(parts, dim=1)

    def unpack(self, mat: torch.Tensor, type_=None) -> RecordBatch:
        n = mat.shape[0]
        cols = {}
        for name, dt, shape, off, w in self.cols:
            if w == 0:
                cols[name] = torch.empty((n,) + shape, dtype=dt, device=mat.device)
                continue
            flat = mat[:, off: off + w].reshape(-1)
            if n == 0 or flat.storage_offset() % torch.empty((), dtype=dt).element_size():
                flat = flat.clone()               # a view into the received buffer at an unaligned byte offset
            cols[name] = flat.view(dt).reshape((n,) + shape)
        return RecordBatch(cols, n, type_)


class _Chunk:
    __slots__ = ("packed", "batch", "meta", "counts", "host", "event", "rows")

    def __init__(self):
        self.packed = None      # [rows, row_bytes] uint8 sorted by destination (packed path)
        self.batch = None       # the flat chunk sorted by destination
        self.meta = None        # its schema
        self.counts = None      # device int64 [ws]
        self.host = None        # pinned host int64 [ws] (async copy target)
        self.event = None
        self.rows = 0


class StreamingShuffle:
    """Hash shuffle of a stream of (batch, hash) pairs; yields the batches this rank receives."""

    def __init__(self, ctx, chunk_bytes: int = 64 << 20, combine: Optional[Callable] = None, tag: str = "shuffle"):
        self.ctx = ctx
        self.ws = ctx.world_size
        self.chunk_bytes = max(1, int(chunk_bytes))
        self.combine = combine          # CombinerProcessor: applied to a chunk before it is sealed
        self.tag = tag
        self.pending: List[Tuple[RecordBatch, torch.Tensor]] = []
        self.pending_bytes = 0
        self.sealed: "deque[_Chunk]" = deque()
        self.inflight: deque = deque()
        self.meta = None                # agreed flat batch schema (None: no rank has rows)
        self.schema: Optional[PackedSchema] = None    # agreed (first round)
        self._local: Optional[PackedSchema] = None    # this rank's chunk layout
        self.type_ = None
        self._agreed = False
        self.done = False               # every rank announced its last round
        self.input_done = False
        self.stats = {"rounds": 0, "rounds_while_pipeline": 0, "chunks_sealed": 0, "rows_sent": 0,
                      "bytes_sent": 0, "rows_received": 0, "packed": 0, "fallback_rounds": 0}

    # ------------------------------------------------------------------ producer side
    def _seal(self):
        if not self.pending:
            return
        from ..parallel.comm import _flatten

        bs = [b for b, _ in self.pending]
        hs = [h for _, h in self.pending]
        self.pending, self.pending_bytes = [], 0
        batch = RecordBatch.concat(bs) if len(bs) > 1 else bs[0]
        h = None if self.combine is not None else (torch.cat(hs) if len(hs) > 1 else hs[0])
        if self.combine is not None:
            batch, h = self.combine(batch)
        if batch.n == 0:
            return
        flat = _flatten(batch)
        if self.type_ is None:
            self.type_ = flat.type
        dest = K.partition_of(h.to(flat.device), self.ws)
        ch = _Chunk()
        ch.rows = flat.n
        order, ch.counts = K.partition_perm(dest, self.ws)   # device partition+pack permutation, counts stay on device
        sorted_b = flat.take(order)
        from ..parallel.comm import _batch_meta

        ch.batch = sorted_b
        ch.meta = _batch_meta(sorted_b)
        if PackedSchema.supports(ch.meta):
            if self._local is None or self._local.meta != ch.meta:
                self._local = PackedSchema(ch.meta)
            ch.packed = self._local.pack(sorted_b)          # device work, overlapped with the pipeline
        if self.meta is None:
            self.meta = ch.meta
        if ch.counts.is_cuda:
            ch.host = torch.empty(self.ws, dtype=torch.int64, pin_memory=True)
            ch.host.copy_(ch.counts, non_blocking=True)
            ch.event = torch.cuda.Event()
            ch.event.record()
        else:
            ch.host = ch.counts
        self.sealed.append(ch)
        self.stats["chunks_sealed"] += 1

    # ------------------------------------------------------------------ rounds
    def _agree(self):
        """First round: every rank learns the batch schema (ranks without rows send none)."""
        ref = self.ctx._agree_schema(self.meta)
        self._agreed = True
        if ref is None:
            self.done = True
            return
        self.meta = ref
        self.schema = PackedSchema(ref) if PackedSchema.supports(ref) else None

    def _round(self, ch: Optional[_Chunk], more: bool):
        if not self._agreed:
            self._agree()
            if self.done:
                return
        ws, ctx = self.ws, self.ctx
        if ch is not None and ch.event is not None:
            ch.event.synchronize()             # the chunk sealed one step ago: its counts have landed
        send = [int(x) for x in ch.host.tolist()] if ch is not None else [0] * ws
        # a chunk whose schema differs from the agreed one is flagged in the same all-gather, so every rank
        # learns it together and takes the record-exchange path for this round (never a one-rank raise that
        # leaves the peers blocked in the all-to-all)
        odd = int(self.schema is not None and ch is not None and ch.meta != self.schema.meta)
        rows = ctx.all_gather_ints(send + [1 if more else 0, odd])
        recv = [r[ctx.rank] for r in rows]
        any_more = any(r[ws] for r in rows)
        any_odd = any(r[ws + 1] for r in rows)
        self.stats["rounds"] += 1
        if not self.input_done:
            self.stats["rounds_while_pipeline"] += 1
        self.stats["rows_sent"] += sum(send) - send[ctx.rank]
        self.stats["rows_received"] += sum(recv) - recv[ctx.rank]
        if self.schema is not None and not any_odd:   # every rank: all columns fixed-width tensors, same schema
            rb = self.schema.row_bytes
            if ch is not None and ch.packed is None:
                ch.packed = self.schema.pack(ch.batch)
            src = ch.packed.reshape(-1) if ch is not None else torch.empty(0, dtype=torch.uint8, device=ctx.device)
            out = torch.empty(sum(recv) * rb, dtype=torch.uint8, device=src.device)
            work = ctx.all_to_all_bytes_async(out, src, [c * rb for c in recv], [c * rb for c in send])
            self.stats["bytes_sent"] += (sum(send) - send[ctx.rank]) * rb
            self.stats["packed"] += 1
            self.inflight.append(("packed", work, out, recv))
        else:
            parts: List[Optional[RecordBatch]] = [None] * ws
            if ch is not None:
                s = 0
                for d, c in enumerate(send):
                    parts[d] = ch.batch.slice(s, s + c)
                    s += c
            from ..parallel.comm import _empty_like_meta

            tmpl = _empty_like_meta(self.meta, ctx.device) if self.meta is not None else None
            got = ctx._exchange_flat(parts, tmpl)
            self.stats["fallback_rounds"] += 1
            self.inflight.append(("batches", None, got, recv))
        if not any_more:
            self.done = True

    def _drain(self, block: bool) -> Iterator[RecordBatch]:
        from ..parallel.comm import _unflatten

        while self.inflight:
            kind, work, out, recv = self.inflight[0]
            if kind == "packed" and work is not None and not block and not work.is_completed():
                return
            self.inflight.popleft()
            if kind == "packed":
                self.ctx._wait(work)
                mat = out.reshape(-1, self.schema.row_bytes) if out.numel() else out.reshape(0, self.schema.row_bytes)
                off = 0
                for c in recv:
                    if c:
                        yield _unflatten(self.schema.unpack(mat[off: off + c], self.type_))
                    off += c
            else:
                for g in out:
                    if g is not None and g.n:
                        yield _unflatten(g)

    # ------------------------------------------------------------------ driver
    def run(self, items: Iterator[Tuple[RecordBatch, torch.Tensor]]) -> Iterator[RecordBatch]:
        """Consume (batch, hash) pairs; yield received batches as rounds complete."""
        if not self.ctx.distributed:
            for b, _ in items:
                if b is not None and b.n:
                    yield b
            return
        # Two shuffles on one context must never have rounds in flight at once: their collectives share the
        # metadata group, and rank A could enter this shuffle's round while rank B is still in the other's.
        # A shuffle started while another one runs (an upstream shuffle feeding a shuffling sink: a partitioned
        # probe under a distributed aggregate / partition / partitioned build) therefore seals its chunks
        # locally and starts its rounds only once its input is exhausted, and yields only after its last
        # round; the plan nests shuffles the same way on every rank, so every rank takes the same mode.
        active = getattr(self.ctx, "_active_shuffles", 0)
        deferred = active > 0
        self.stats["deferred"] = int(deferred)
        self.ctx._active_shuffles = active + 1
        try:
            yield from self._run(items, deferred)
        finally:
            self.ctx._active_shuffles = getattr(self.ctx, "_active_shuffles", 1) - 1

    def _run(self, items, deferred: bool) -> Iterator[RecordBatch]:
        for b, h in items:
            if b is None or b.n == 0:
                continue
            self.pending.append((b, h))
            self.pending_bytes += b.nbytes()
            if self.pending_bytes >= self.chunk_bytes:
                self._seal()
            if deferred:
                continue
            # lag one sealed chunk: the host reads counts only of chunks whose copy was issued a step ago
            while len(self.sealed) > 1 and not self.done:
                self._round(self.sealed.popleft(), more=True)
            yield from self._drain(block=False)
        self.input_done = True
        self._seal()
        while self.sealed and not self.done:
            ch = self.sealed.popleft()
            self._round(ch, more=bool(self.sealed))
        while not self.done:
            self._round(None, more=False)
        if deferred:
            # hold every received batch until the rounds are over (the outer shuffle may start rounds as soon
            # as this one yields)
            got = list(self._drain(block=True))
            yield from got
            return
        yield from self._drain(block=True)


def shuffle_stream(ctx, batches: Iterator[RecordBatch], key: Callable[[RecordBatch], torch.Tensor],
                   chunk_bytes: int = 64 << 20, stats: Optional[dict] = None, combine=None) -> Iterator[RecordBatch]:
    """Convenience: stream ``batches`` through a StreamingShuffle keyed by ``key(batch)`` (a hash column)."""
    sh = StreamingShuffle(ctx, chunk_bytes, combine=combine)
    try:
        yield from sh.run((b, key(b)) for b in batches if b is not None and b.n)
    finally:
        if stats is not None:
            for k, v in sh.stats.items():
                stats[k] = stats.get(k, 0) + v


__all__ = ["StreamingShuffle", "PackedSchema", "shuffle_stream"]
