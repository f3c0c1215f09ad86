"""Home-tier page arena: page columns are sub-allocated from large arena chunks by the native slab allocator.

Reference: ``src/memory`` (the slab allocator behind every PDB object page) and ``src/bufferMgr`` (pages
carved out of one shared-memory pool). On an MI355X node the home tier is HBM: the manager reserves arena
chunks (256 MiB by default, more on demand up to the device budget) and every device-resident page's
tensor columns live in slab-allocated, 256-B-aligned regions of them (``SlabAllocator``: best-fit free
list with coalescing, ``csrc/runtime/storage.cpp``). The torch caching allocator never sees page memory,
fragmentation is visible (``largest_free``), and freeing is explicit: when a page is spilled, dropped or
its set removed, its regions go back to the slab allocator.

Frees are stream-ordered: a region is released only after an event recorded on the releasing stream (and,
for a spill, on the copy stream reading the page) has completed, so queued kernels that still read the page
and the D2H copy of an eviction never see the region reused under them. On a CPU pseudo-cluster node the
same arena runs in host memory (frees are immediate), so the CPU test suite exercises the allocator path.
"""
from __future__ import annotations

from collections import deque
from typing import Any, List, Optional, Tuple

import torch

from .. import _ext
from ..objects.record import RecordBatch

Handle = Tuple[int, int]          # (chunk index, byte offset)


class DevicePagePool:
    def __init__(self, device, chunk_bytes: int = 256 << 20, max_bytes: Optional[int] = None, alignment: int = 256):
        self.device = torch.device(device)
        self.chunk_bytes = int(chunk_bytes)
        self.max_bytes = int(max_bytes) if max_bytes else (1 << 62)
        self.alignment = alignment
        self.arenas: List[torch.Tensor] = []
        self.slabs: List[Any] = []
        self._pending: "deque[Tuple[Optional[torch.cuda.Event], List[Handle]]]" = deque()
        self.stats = {"allocs": 0, "frees": 0, "chunks": 0, "fallbacks": 0, "adopted_bytes": 0}

    # ------------------------------------------------------------- chunks / raw regions
    @property
    def is_cuda(self) -> bool:
        return self.device.type == "cuda"

    def capacity(self) -> int:
        return sum(int(s.capacity) for s in self.slabs)

    def used(self) -> int:
        return sum(int(s.used) for s in self.slabs)

    def largest_free(self) -> int:
        return max((int(s.largest_free) for s in self.slabs), default=0)

    def _add_chunk(self, nbytes: int) -> bool:
        # a page larger than a chunk gets a dedicated chunk of its own (2 MiB granules)
        size = self.chunk_bytes if nbytes <= self.chunk_bytes else (nbytes + (2 << 20) - 1) // (2 << 20) * (2 << 20)
        if self.capacity() + size > self.max_bytes:
            return False
        try:
            arena = torch.empty(size, dtype=torch.uint8, device=self.device)
        except RuntimeError:          # the device cannot back another chunk: callers fall back
            return False
        self.arenas.append(arena)
        self.slabs.append(_ext.native().SlabAllocator(size, self.alignment))
        self.stats["chunks"] += 1
        return True

    def _reclaim(self, block: bool = False) -> bool:
        """Return completed stream-ordered frees to the slab allocators; ``block`` waits for the oldest."""
        progressed = False
        while self._pending:
            ev, handles = self._pending[0]
            if ev is not None and not ev.query():
                if not block:
                    break
                ev.synchronize()
                block = False
            self._pending.popleft()
            for c, off in handles:
                self.slabs[c].free(off)
                self.stats["frees"] += 1
            progressed = True
        return progressed

    def alloc(self, nbytes: int) -> Optional[Handle]:
        self._reclaim()
        while True:
            for c, slab in enumerate(self.slabs):
                off = slab.alloc(nbytes)
                if off >= 0:
                    self.stats["allocs"] += 1
                    return c, int(off)
            # grow before blocking: waiting on a pending free would stall the host until the GPU drains
            if self._add_chunk(nbytes):
                continue
            if self._pending and self._reclaim(block=True):
                continue
            return None

    def view(self, h: Handle, dtype: torch.dtype, shape) -> torch.Tensor:
        c, off = h
        n = 1
        for s in shape:
            n *= int(s)
        nbytes = n * torch.empty((), dtype=dtype).element_size()
        return self.arenas[c][off: off + nbytes].view(dtype).view(tuple(shape))

    def release(self, handles: List[Handle], events=()):
        """Free ``handles`` once the current stream has reached this point and every event in ``events`` (e.g.
        the D2H copy of an eviction on the tier's copy stream) has completed."""
        if not handles:
            return
        if not self.is_cuda:
            for c, off in handles:
                self.slabs[c].free(off)
                self.stats["frees"] += 1
            return
        cur = torch.cuda.current_stream(self.device)
        for e in events:
            if e is not None:
                cur.wait_event(e)
        ev = torch.cuda.Event()
        ev.record(cur)
        self._pending.append((ev, list(handles)))

    # ------------------------------------------------------------- pages
    def adopt(self, batch: RecordBatch, move: bool = False) -> Tuple[RecordBatch, List[Handle]]:
        """Copy ``batch``'s home-tier tensor columns (and, with ``move``, its host tensor columns: one H2D copy
        straight into the arena) into slab regions; string / nested column objects stay as they are.
        Returns the pool-backed batch and its regions."""
        handles: List[Handle] = []

        def put(t: torch.Tensor) -> torch.Tensor:
            home = t.device.type == self.device.type and (t.device.index or 0) == (self.device.index or 0)
            if t.numel() == 0 or not (home or (move and t.device.type == "cpu")):
                return t
            h = self.alloc(t.numel() * t.element_size())
            if h is None:
                self.stats["fallbacks"] += 1
                return t
            v = self.view(h, t.dtype, t.shape)
            v.copy_(t, non_blocking=True)
            handles.append(h)
            self.stats["adopted_bytes"] += t.numel() * t.element_size()
            return v

        cols = {k: (put(v) if isinstance(v, torch.Tensor) else v) for k, v in batch.columns.items()}
        return RecordBatch(cols, batch.n, batch.type), handles

    def summary(self) -> dict:
        return {"capacity": self.capacity(), "used": self.used(), "largest_free": self.largest_free(),
                "pending_frees": len(self._pending), **self.stats}


__all__ = ["DevicePagePool"]
