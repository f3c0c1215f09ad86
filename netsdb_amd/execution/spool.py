"""Spillable intermediate storage for out-of-core execution.

Reference: src/queryExecution/headers/PartitionedHashSet.h (hash sets whose pages are allocated from the
buffer pool and spill), src/storage/source/PageCache.cc (page eviction) and the TupleSetJobStage sinks that
write intermediate tuple sets into temp sets.  A :class:`Spool` is a temp (never flushed) set of the
node's StorageManager: batches appended to it become pages charged to the device budget, and the
manager spills the least-recently-used ones to the pinned host tier / native page pool; iterating the
spool reloads them one page at a time.  :class:`PartitionedSpool` hash-partitions batches into P
spools so that each partition (a join build side, a group-by input) can later be processed alone
within the budget (Grace-style).
"""
from __future__ import annotations

import itertools
from typing import Iterator, List, Optional

import torch

from ..objects.record import RecordBatch
from . import kernels as K

_ids = itertools.count()
SPOOL_DB = "__spool"
# partition hashes are re-mixed with a salt so Grace partitions are independent of the rank shuffle
# (h % world_size) that already happened upstream
_SALT = 0x5851F42D4C957F2D


def grace_partition(h: torch.Tensor, nparts: int) -> torch.Tensor:
    return torch.remainder(K.mix64(h ^ _SALT), nparts)


class Spool:
    def __init__(self, storage, tag: str = "spool", page_size: Optional[int] = None, locality: str = "temp"):
        self.storage = storage
        self.name = f"{tag}_{next(_ids)}"
        # temp / partition locality: MRU replacement and a low reuse prior in the cost-based page cache
        self.set = storage.create_set(SPOOL_DB, self.name, None, page_size=page_size, persistent=False,
                                      locality=locality)
        self.n = 0
        self.bytes = 0

    def add(self, b: RecordBatch):
        if b is None or b.n == 0:
            return
        self.set.add_batch(b)
        self.n += b.n
        self.bytes += b.nbytes()

    def __iter__(self) -> Iterator[RecordBatch]:
        for b in self.set.scan():
            yield b

    def batches(self) -> List[RecordBatch]:
        return list(self)

    def concat(self) -> Optional[RecordBatch]:
        bs = [b for b in self if b.n]
        return RecordBatch.concat(bs) if bs else None

    def drop(self):
        if self.set is not None:
            self.storage.remove_set(SPOOL_DB, self.name)
            self.set = None


class PartitionedSpool:
    """P spools filled by the hash of one key column (PartitionedHashSet's page partitions)."""

    def __init__(self, storage, nparts: int, tag: str = "part", page_size: Optional[int] = None):
        self.nparts = nparts
        self.parts = [Spool(storage, f"{tag}{i}", page_size, locality="partition") for i in range(nparts)]

    def add(self, b: RecordBatch, h: torch.Tensor):
        if b is None or b.n == 0:
            return
        dest = grace_partition(h, self.nparts)
        for i, part in enumerate(K.split_by_dest(b, dest, self.nparts)):
            if part.n:
                self.parts[i].add(part)

    def drop(self):
        for p in self.parts:
            p.drop()

    @property
    def n(self) -> int:
        return sum(p.n for p in self.parts)


__all__ = ["Spool", "PartitionedSpool", "grace_partition", "SPOOL_DB"]
