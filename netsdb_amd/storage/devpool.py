"""Home-tier page arena: page columns are sub-allocated from large arena chunks by the native slab allocator.

Reference: ``src/memory`` (the slab allocator behind every PDB object page) and ``src/bufferMgr`` (pages
carved out of one shared-memory pool). On an MI355X node the home tier is HBM: the manager reserves arena
chunks (256 MiB by default, more on demand up to the device budget) and every device-resident page's
tensor columns live in one slab-allocated, 256-B-aligned region of them (``SlabAllocator``: best-fit free
list with coalescing, ``csrc/runtime/storage.cpp``). The torch caching allocator never sees page memory and
fragmentation is visible (``largest_free``).

Region lifetime follows the TENSORS, not page residency. A region is exposed as a tensor with a storage of
its own (``__cuda_array_interface__`` / ``__array_interface__`` over the arena bytes, owned by a
:class:`Region` object), and every column of a page is a view of that one base tensor. The region goes
back to the slab allocator only when the last tensor that views it is gone — so a batch a scan yielded
earlier stays valid after its page was spilled, and a later page load can never be handed bytes that a
held batch still reads (the reference's page pins have the same role: a page is not recycled while an
iterator holds it).

Frees are stream-ordered: when the last view dies the pool records an event on the current stream and keeps
the region, together with every event attached to it (e.g. the D2H copy of an eviction on the pinned tier's
copy stream), until ALL of them have completed. No stream ever waits for another here, so a spill does not
stall compute. Chunks whose slab becomes empty are handed back to the device (the first chunk is kept).
On a CPU pseudo-cluster node the same arena runs in host memory (no events), so the CPU test suite
exercises the allocator and lifetime path.
"""
from __future__ import annotations

import threading
from collections import deque
from typing import Any, Dict, List, Optional, Tuple

import numpy as np
import torch

from .. import _ext
from ..objects.record import RecordBatch

Handle = Tuple[int, int]          # (chunk id, byte offset)


class Region:
    """Owner of one slab region. Tensors made from it keep it alive; when the last one dies the region
    is returned to the pool (after the attached events and the current stream position)."""

    __slots__ = ("pool", "handle", "ptr", "nbytes", "arena", "events", "__weakref__")

    def __init__(self, pool: "DevicePagePool", handle: Handle, nbytes: int):
        self.pool = pool
        self.handle = handle
        self.arena = pool.arenas[handle[0]]             # the chunk stays allocated while a view is alive
        self.ptr = self.arena.data_ptr() + handle[1]
        self.nbytes = nbytes
        self.events: List[Any] = []

    def attach_event(self, ev):
        """The region may be reused only after ``ev`` (e.g. a D2H copy reading it) has completed."""
        if ev is not None:
            self.events.append(ev)

    @property
    def __cuda_array_interface__(self):
        return {"shape": (self.nbytes,), "typestr": "|u1", "data": (self.ptr, False), "version": 2}

    @property
    def __array_interface__(self):
        return {"shape": (self.nbytes,), "typestr": "|u1", "data": (self.ptr, False), "version": 3}

    def tensor(self) -> torch.Tensor:
        """A uint8 tensor over the region whose storage owns this object."""
        if self.pool.is_cuda:
            return torch.as_tensor(self, device=self.pool.device)
        return torch.from_numpy(np.asarray(self))

    def __del__(self):
        pool = self.pool
        if pool is not None and self.handle is not None:
            pool._retire(self.handle, self.events)
            self.handle = None


class DevicePagePool:
    def __init__(self, device, chunk_bytes: int = 256 << 20, max_bytes: Optional[int] = None, alignment: int = 256):
        self.device = torch.device(device)
        self.chunk_bytes = int(chunk_bytes)
        self.max_bytes = int(max_bytes) if max_bytes else (1 << 62)
        self.alignment = alignment
        self.arenas: Dict[int, torch.Tensor] = {}
        self.slabs: Dict[int, Any] = {}
        self._next_chunk = 0
        # retired regions: (events that must complete, handle). Appended from Region finalisers (any thread
        # that drops the last view), consumed by _reclaim.
        self._retired: "deque[Tuple[List[Any], Handle]]" = deque()
        self._pending: "deque[Tuple[List[Any], Handle]]" = deque()
        self._lock = threading.RLock()
        self.stats = {"allocs": 0, "frees": 0, "chunks": 0, "chunks_released": 0, "fallbacks": 0,
                      "adopted_bytes": 0}

    # ------------------------------------------------------------- chunks / raw regions
    @property
    def is_cuda(self) -> bool:
        return self.device.type == "cuda"

    def capacity(self) -> int:
        self._reclaim()
        return sum(int(s.capacity) for s in self.slabs.values())

    def used(self) -> int:
        self._reclaim()
        return sum(int(s.used) for s in self.slabs.values())

    def largest_free(self) -> int:
        self._reclaim()
        return max((int(s.largest_free) for s in self.slabs.values()), default=0)

    def _add_chunk(self, nbytes: int) -> bool:
        # a page larger than a chunk gets a dedicated chunk of its own (2 MiB granules)
        size = self.chunk_bytes if nbytes <= self.chunk_bytes else (nbytes + (2 << 20) - 1) // (2 << 20) * (2 << 20)
        if sum(int(s.capacity) for s in self.slabs.values()) + size > self.max_bytes:
            return False
        try:
            arena = torch.empty(size, dtype=torch.uint8, device=self.device)
        except RuntimeError:          # the device cannot back another chunk: callers fall back
            return False
        cid = self._next_chunk
        self._next_chunk += 1
        self.arenas[cid] = arena
        self.slabs[cid] = _ext.native().SlabAllocator(size, self.alignment)
        self.stats["chunks"] += 1
        return True

    def _retire(self, handle: Handle, events: List[Any]):
        """Called when the last view of a region died: free it once the current stream and ``events`` are done."""
        evs = [e for e in events if e is not None]
        if self.is_cuda:
            try:
                ev = torch.cuda.Event()
                ev.record(torch.cuda.current_stream(self.device))
                evs.append(ev)
            except Exception:        # interpreter shutdown: nothing can reuse the region any more
                return
        self._retired.append((evs, handle))

    def _release_empty_chunks(self):
        """Hand chunks with no live region back to the device (keep the first one as the warm arena)."""
        live = {h[0] for _, h in self._pending} | {h[0] for _, h in self._retired}
        for cid in sorted(self.slabs)[1:]:
            if int(self.slabs[cid].used) == 0 and cid not in live:
                del self.slabs[cid]
                del self.arenas[cid]
                self.stats["chunks_released"] += 1

    def _reclaim(self, block: bool = False) -> bool:
        """Return completed stream-ordered frees to the slab allocators; ``block`` waits for the oldest."""
        with self._lock:
            while self._retired:
                self._pending.append(self._retired.popleft())
            progressed = False
            while self._pending:
                evs, (c, off) = self._pending[0]
                if any(not e.query() for e in evs):
                    if not block:
                        break
                    for e in evs:
                        e.synchronize()
                    block = False
                self._pending.popleft()
                self.slabs[c].free(off)
                self.stats["frees"] += 1
                progressed = True
            if progressed:
                self._release_empty_chunks()
            return progressed

    def alloc(self, nbytes: int) -> Optional[Handle]:
        """Raw region handle (caller frees with :meth:`release`). Pages use :meth:`alloc_region`."""
        self._reclaim()
        with self._lock:
            while True:
                for c, slab in self.slabs.items():
                    off = slab.alloc(nbytes)
                    if off >= 0:
                        self.stats["allocs"] += 1
                        return c, int(off)
                # grow before blocking: waiting on a pending free would stall the host until the GPU drains
                if self._add_chunk(nbytes):
                    continue
                if (self._pending or self._retired) and self._reclaim(block=True):
                    continue
                return None

    def alloc_region(self, nbytes: int) -> Optional[Region]:
        h = self.alloc(nbytes)
        return None if h is None else Region(self, h, nbytes)

    def view(self, h: Handle, dtype: torch.dtype, shape) -> torch.Tensor:
        c, off = h
        n = 1
        for s in shape:
            n *= int(s)
        nbytes = n * torch.empty((), dtype=dtype).element_size()
        return self.arenas[c][off: off + nbytes].view(dtype).view(tuple(shape))

    def release(self, handles: List[Handle], events=()):
        """Free raw ``handles`` once the current stream has reached this point and every event in ``events``
        has completed (no stream waits on another)."""
        for h in handles:
            self._retire(h, list(events))
        if not self.is_cuda:
            self._reclaim()

    # ------------------------------------------------------------- pages
    def adopt(self, batch: RecordBatch, move: bool = False) -> Tuple[RecordBatch, List[Region]]:
        """Copy ``batch``'s home-tier tensor columns (and, with ``move``, its host tensor columns: one H2D copy
        straight into the arena) into ONE region; each column becomes a view of the region's base tensor.
        String / nested column objects stay as they are. Returns the pool-backed batch and its regions."""
        al = self.alignment

        def eligible(t) -> bool:
            if not isinstance(t, torch.Tensor) or t.numel() == 0:
                return False
            home = t.device.type == self.device.type and (t.device.index or 0) == (self.device.index or 0)
            return home or (move and t.device.type == "cpu")

        names = [k for k, v in batch.columns.items() if eligible(v)]
        if not names:
            return batch, []
        offs, total = {}, 0
        for k in names:
            t = batch.columns[k]
            offs[k] = total
            total += (t.numel() * t.element_size() + al - 1) // al * al
        reg = self.alloc_region(total)
        if reg is None:
            self.stats["fallbacks"] += 1
            return batch, []
        base = reg.tensor()
        cols = dict(batch.columns)
        for k in names:
            t = cols[k]
            nb = t.numel() * t.element_size()
            v = base[offs[k]: offs[k] + nb].view(t.dtype).view(tuple(t.shape))
            v.copy_(t, non_blocking=True)
            cols[k] = v
            self.stats["adopted_bytes"] += nb
        return RecordBatch(cols, batch.n, batch.type), [reg]

    def summary(self) -> dict:
        return {"capacity": self.capacity(), "used": self.used(), "largest_free": self.largest_free(),
                "pending_frees": len(self._pending) + len(self._retired), **self.stats}


__all__ = ["DevicePagePool", "Region"]
