"""Per-node storage manager (reference: src/serverFunctionalities/source/PangeaStorageServer.cc,
src/storage/source/PageCache.cc, PDBEvictWork.cc, src/bufferMgr/*).

Owns the node's sets, the HBM budget (288 GB per MI355X: the default budget is 85 % of device
memory), the native :class:`BufferManager` page pool (host memory, LRU-spills to disk), and the
device->host eviction of unpinned pages when the HBM budget is exceeded.
"""
from __future__ import annotations

import itertools
import os
import tempfile
import threading
from collections import OrderedDict
from typing import Dict, Optional, Tuple

import torch

from .. import _ext
from .sets import DenseMatrixSet, Page, UserSet

DEFAULT_PAGE_SIZE = 64 << 20


class StorageManager:
    def __init__(self, root: Optional[str] = None, device=None, page_size: int = DEFAULT_PAGE_SIZE,
                 pool_pages: int = 16, device_budget: Optional[int] = None, rank: int = 0, io_workers: int = 2,
                 read_ahead: int = 4, pinned_budget: Optional[int] = None, page_pool_chunk: Optional[int] = None):
        self.root = root or tempfile.mkdtemp(prefix="netsdb_amd_")
        os.makedirs(self.root, exist_ok=True)
        self.device = torch.device(device) if device is not None else None
        # the "device tier" whose bytes the budget governs: the GPU, or the CPU for a CPU pseudo-cluster
        # node (out-of-core tests run the same spill/reload code with a CPU home device)
        self.home = self.device if self.device is not None else torch.device("cpu")
        self.page_size = page_size
        self.rank = rank
        spill = os.path.join(self.root, f"node{rank}")
        os.makedirs(spill, exist_ok=True)
        self.buffer_manager = _ext.native().BufferManager(page_size, pool_pages, spill)
        # native I/O workers (src/work PDBWorkerQueue): page read-ahead for scans, background flushes
        self.workers = _ext.native().WorkerQueue(io_workers)
        self.read_ahead = max(0, min(read_ahead, pool_pages // 2))
        if device_budget is None and self.device is not None and self.device.type == "cuda":
            total = torch.cuda.get_device_properties(self.device).total_memory
            device_budget = int(total * 0.85)
        self.device_budget = device_budget or (1 << 62)
        # warm tier: evicted device pages go to pinned host memory by async DMA (hosttier.py)
        self.host_tier = None
        if self.device is not None and self.device.type == "cuda" and pinned_budget != 0:
            from .hosttier import PinnedHostTier

            if pinned_budget is None:
                try:
                    pinned_budget = min(64 << 30, os.sysconf("SC_PAGE_SIZE") * os.sysconf("SC_PHYS_PAGES") // 8)
                except (ValueError, OSError):
                    pinned_budget = 8 << 30
            self.host_tier = PinnedHostTier(self.device, pinned_budget)
        # home-tier page arena: page columns are carved out of arena chunks by the native slab allocator
        # (src/memory + bufferMgr page pool); page_pool_chunk=0 disables it
        self.page_pool = None
        if page_pool_chunk != 0:
            from .devpool import DevicePagePool

            chunk = page_pool_chunk or ((256 << 20) if self.home.type == "cuda" else (16 << 20))
            self.page_pool = DevicePagePool(self.home, chunk, max_bytes=self.device_budget)
        self.device_bytes = 0
        # LRU of everything resident on the device tier (pages and dense panels), oldest first: eviction
        # pops from the front instead of scanning every page of every set (PageCache's LRU list)
        self._lru: "OrderedDict[int, object]" = OrderedDict()
        self.sets: Dict[Tuple[str, str], UserSet] = {}
        self._ids = itertools.count(1)
        # sets created without a catalog id (temp sets, spools) draw from a disjoint range: their pool pages
        # are keyed by set id and must never alias a catalog set's pages
        self._temp_ids = itertools.count(1 << 32)
        self._clock = itertools.count()
        self.lock = threading.RLock()
        self.stats = {"evicted_pages": 0, "evicted_bytes": 0}

    # ----------------------------------------------------------- sets
    def create_set(self, db: str, name: str, type_=None, page_size: Optional[int] = None, device="default",
                   dense: bool = False, set_id: Optional[int] = None, persistent: bool = True) -> UserSet:
        with self.lock:
            key = (db, name)
            if key in self.sets:
                return self.sets[key]
            dev = self.device if device == "default" else device
            sid = set_id if set_id is not None else (next(self._ids) if persistent else next(self._temp_ids))
            cls = DenseMatrixSet if dense else UserSet
            s = cls(self, db, name, type_, sid, page_size or self.page_size, dev, persistent)
            self.sets[key] = s
            return s

    def get_set(self, db: str, name: str) -> UserSet:
        try:
            return self.sets[(db, name)]
        except KeyError:
            raise KeyError(f"set {db}.{name} does not exist on node {self.rank}") from None

    def has_set(self, db: str, name: str) -> bool:
        return (db, name) in self.sets

    def remove_set(self, db: str, name: str):
        with self.lock:
            s = self.sets.pop((db, name), None)
            if s is not None:
                self._release_pages(s)
                s.clear()

    def remove_database(self, db: str):
        for (d, n) in list(self.sets):
            if d == db:
                self.remove_set(d, n)

    def clear_set(self, db: str, name: str):
        s = self.get_set(db, name)
        self._release_pages(s)
        s.clear()

    def _release_pages(self, s: UserSet):
        if isinstance(s, DenseMatrixSet):
            s.release_storage()
            self.untrack(s)
        for p in s.pages:
            self.untrack(p)
            if p.location == "device" and p.batch is not None:
                self.device_bytes -= p.nbytes
            elif p.location == "pinned" and self.host_tier is not None:
                self.host_tier.release(p.nbytes)
            p.release_regions()
            p.batch = None          # the region returns once no held batch views it any more

    # ----------------------------------------------------------- memory accounting / eviction
    def on_home(self, device) -> bool:
        """True when ``device`` is the budgeted device tier of this node."""
        if device is None:
            return False
        d, h = torch.device(device), self.home
        if d.type != h.type:
            return False
        return d.type != "cuda" or (d.index or 0) == (h.index or 0)

    def track(self, obj):
        """``obj`` (a page or dense set) is resident on the device tier: most recently used."""
        obj.last_use = next(self._clock)
        self._lru[id(obj)] = obj
        self._lru.move_to_end(id(obj))

    def untrack(self, obj):
        self._lru.pop(id(obj), None)

    def account(self, page: Page):
        page.last_use = next(self._clock)
        if page.location == "device":
            self.track(page)
            self.account_bytes(page.nbytes, self.home, keep=page)

    def account_bytes(self, nbytes: int, device=None, keep=None):
        """Charge ``nbytes`` on ``device``; over budget, spill LRU pages / dense panels (never ``keep``)."""
        if not self.on_home(device):
            return
        with self.lock:
            self.device_bytes += nbytes
            if self.device_bytes > self.device_budget:
                self.evict(self.device_bytes - self.device_budget, keep=keep)

    def release_bytes(self, nbytes: int, device=None):
        if self.on_home(device):
            with self.lock:
                self.device_bytes = max(0, self.device_bytes - nbytes)

    def available(self) -> int:
        """Bytes the budget still admits on the device tier."""
        return max(0, self.device_budget - self.device_bytes)

    def touch(self, page):
        page.last_use = next(self._clock)
        if id(page) in self._lru:
            self._lru.move_to_end(id(page))

    def evict(self, need: int, keep=None) -> int:
        """Spill least-recently-used unpinned device pages (to the pinned tier / page pool) and dense
        panels (in block-row slabs, PageCache/PDBEvictWork style) until ``need`` bytes are free."""
        freed = 0
        kept = 0                     # pinned / kept entries stay at the front of the LRU
        while freed < need:
            chunk = list(itertools.islice(self._lru.items(), kept, kept + 32))
            if not chunk:
                break
            for key, p in chunk:
                if freed >= need:
                    break
                if p is keep:
                    kept += 1
                    continue
                if isinstance(p, DenseMatrixSet):
                    if not p.resident_on_home():
                        self.untrack(p)
                        continue
                elif p.location != "device" or p.batch is None:
                    self.untrack(p)
                    continue
                if p.pins:
                    kept += 1
                    continue
                f = p.spill()
                if f or not (p.resident_on_home() if isinstance(p, DenseMatrixSet) else p.location == "device"):
                    self.untrack(p)
                else:
                    kept += 1
                freed += f
                if isinstance(p, DenseMatrixSet):
                    self.stats["evicted_panels"] = self.stats.get("evicted_panels", 0) + 1
                else:
                    self.stats["evicted_pages"] += 1
        self.device_bytes -= freed
        self.stats["evicted_bytes"] += freed
        return freed

    def flush(self):
        """Write every persistent page image to the pool, then let the native workers write the pool's
        dirty frames to the page files (set by set) and wait for them (checkpoint barrier)."""
        buzzers = []
        for s in self.sets.values():
            if s.persistent:
                s.persist_pages()
                buzzers.append(self.workers.submit_flush(self.buffer_manager, s.set_id))
        for b in buzzers:
            b.wait()
            if b.error:
                raise RuntimeError(f"page flush failed: {b.error}")
        self.buffer_manager.flush_all()

    def flush_async(self):
        """Background checkpoint: persist page images now, return the buzzers of the file writes."""
        out = []
        for s in self.sets.values():
            if s.persistent:
                s.persist_pages()
                out.append(self.workers.submit_flush(self.buffer_manager, s.set_id))
        return out

    def prefetch(self, uset, page_nos):
        """Queue native read-ahead of evicted pages (page file -> pool slot) for an upcoming scan."""
        if page_nos:
            return self.workers.submit_prefetch(self.buffer_manager, uset.set_id, list(page_nos))
        return None

    def summary(self) -> dict:
        return {
            "sets": {f"{d}.{n}": {"records": s.num_records(), "bytes": s.nbytes(), "pages": len(s.pages)}
                     for (d, n), s in self.sets.items()},
            "device_bytes": self.device_bytes,
            "device_budget": self.device_budget,
            "pool_resident_pages": self.buffer_manager.resident_pages,
            "pool_evictions": self.buffer_manager.evictions,
            "pool_loads": self.buffer_manager.loads,
            "io_work_completed": self.workers.completed,
            "pinned_tier": dict(self.host_tier.stats, used=self.host_tier.used) if self.host_tier is not None else None,
            "page_pool": self.page_pool.summary() if self.page_pool is not None else None,
            **self.stats,
        }


__all__ = ["StorageManager", "DEFAULT_PAGE_SIZE"]
