"""Pinned host spill tier for device-resident pages.

Reference: the page cache evicts pages to disk through PDBFlushProducerWork / PDBEvictWork
(src/storage); its pages live in shared memory, so eviction is a memcpy.  On MI355X the hot tier is
HBM (288 GB), the warm tier host DRAM.  Moving a page between them should be a DMA, not a CPU
serialisation: a device page evicted under HBM pressure is copied device->host into page-locked
(pinned) buffers with asynchronous copies on a dedicated copy stream (hipMemcpyAsync under
``Tensor.copy_(non_blocking=True)``), the device memory is handed back to the caching allocator once
that stream has consumed it (``record_stream``), and a scan copies the page back host->device the
same way, ordered before the consuming kernels by a stream wait instead of a host sync.  Pages
that do not fit the pinned budget fall through to the serialised BufferManager/page-file path.
"""
from __future__ import annotations

from typing import Any, Optional

import torch

from ..objects.record import RecordBatch


def _map_tensors(c: Any, fn):
    if isinstance(c, torch.Tensor):
        return fn(c)
    if isinstance(c, RecordBatch):
        return RecordBatch({k: _map_tensors(v, fn) for k, v in c.columns.items()}, c.n, c.type)
    if isinstance(c, tuple):
        return tuple(_map_tensors(x, fn) for x in c)
    return c


class PinnedHostTier:
    """Budgeted pinned-memory tier with its own copy stream (one per GPU)."""

    def __init__(self, device, budget_bytes: int):
        self.device = torch.device(device)
        self.budget = int(budget_bytes)
        self.used = 0
        self.stream = torch.cuda.Stream(self.device)
        self.stats = {"offloads": 0, "fetches": 0, "bytes_out": 0, "bytes_in": 0}

    def admit(self, nbytes: int) -> bool:
        return self.used + nbytes <= self.budget

    def offload(self, batch: RecordBatch, nbytes: int):
        """Device batch -> pinned host batch (async D2H). Returns (host batch, completion event)."""
        producer = torch.cuda.current_stream(self.device)
        self.stream.wait_stream(producer)          # the kernels that wrote the page come first

        def d2h(t: torch.Tensor) -> torch.Tensor:
            if t.device.type != "cuda":
                return t
            h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
            h.copy_(t, non_blocking=True)
            t.record_stream(self.stream)            # allocator must not recycle t before the copy ran
            return h

        with torch.cuda.stream(self.stream):
            host = _map_tensors(batch, d2h)
            ev = torch.cuda.Event()
            ev.record(self.stream)
        self.used += nbytes
        self.stats["offloads"] += 1
        self.stats["bytes_out"] += nbytes
        return host, ev

    def fetch(self, host: RecordBatch, ev: Optional[torch.cuda.Event], nbytes: int, pool=None):
        """Pinned host batch -> device batch (async H2D), ordered before the consumer stream's next work.
        With the manager's page arena (``pool``) the copies land in slab-allocated regions. Returns
        (batch, regions); regions is empty without a pool."""
        consumer = torch.cuda.current_stream(self.device)
        regions = []

        def h2d(t: torch.Tensor) -> torch.Tensor:
            if pool is not None and t.device.type == "cpu" and t.numel() > 0:
                r = pool.alloc_region(t.numel() * t.element_size())
                if r is not None:
                    d = r.tensor().view(t.dtype).view(tuple(t.shape))
                    d.copy_(t, non_blocking=True)
                    regions.append(r)
                    return d
            d = t.to(self.device, non_blocking=True)
            # d is allocated on the copy stream's pool; the consumer reads it, so a free must wait for the
            # consumer's queued kernels too (else the next fetch's H2D may overwrite it under them)
            if d.device.type == "cuda":
                d.record_stream(consumer)
            return d

        with torch.cuda.stream(self.stream):
            if ev is not None:
                self.stream.wait_event(ev)
            dev = _map_tensors(host, h2d)
        consumer.wait_stream(self.stream)
        self.used = max(0, self.used - nbytes)
        self.stats["fetches"] += 1
        self.stats["bytes_in"] += nbytes
        return dev, regions

    def release(self, nbytes: int):
        self.used = max(0, self.used - nbytes)

    @staticmethod
    def host_view(host: RecordBatch, ev: Optional[torch.cuda.Event]) -> RecordBatch:
        """Host batch of an offloaded page once its D2H copy landed (for serialising it to the page pool)."""
        if ev is not None:
            ev.synchronize()
        return host


__all__ = ["PinnedHostTier"]
