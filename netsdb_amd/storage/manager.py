"""Per-node storage manager (reference: src/serverFunctionalities/source/PangeaStorageServer.cc,
src/storage/source/PageCache.cc, PDBEvictWork.cc, src/bufferMgr/*).

Owns the node's sets, the HBM budget (288 GB per MI355X: the default budget is 85 % of device
memory), the native :class:`BufferManager` page pool (host memory, LRU-spills to disk), and the
device->host eviction of unpinned pages when the HBM budget is exceeded.

Eviction is cost-based per locality set (reference: src/storage/headers/PageCache.h:28-38 cost-based
policy and CompareLocalitySets, LocalitySet.h:158-210 locality / replacement / durability types). Every
set has a locality type (``LOCALITY``): model weights reused every step, job inputs/outputs, shuffle
data, hash-partition spools and temp data. Within a set the replacement policy picks the candidate —
LRU for reused sets, MRU for sequential one-pass data (a spool page just written is the one read last).
Across sets the victim is the candidate with the lowest eviction cost per byte freed

    cost = (write_cost + reuse_prob * read_cost) / min(bytes, need),  reuse_prob = prior(locality) / (1 + distance / n)

in microseconds (reference LocalitySet::writeCost / readCost, PageCache.h:345-368):

  * write_cost: moving the object out. 0 for a CLEAN object — a page whose serialised image is already in the
    page pool / page file (loaded from it or persisted since its last change), or a "model" panel unchanged
    since it was persisted: eviction just drops it. A dirty object pays its tier: an async D2H copy into the
    pinned host tier when the tier admits it (~25 GB/s + 10 us), else serialisation into the native page pool
    (~3 GB/s + 50 us, and the pool writes it to the page file).
  * read_cost: bringing it back if it is reused, from the tier it will sit in (pinned: H2D ~25 GB/s; pool or
    page file: ~3 GB/s + deserialisation), so a 64 MiB panel costs ~16000x a 4 KiB spool page to reload.
  * per-set multipliers (``StorageManager.set_costs``, LocalitySet::setWriteCost / setReadCost) scale both;
    distance is the number of accesses since the candidate was last touched (the reference distance),
    normalised by the number n of resident objects.

A spool-heavy job under a tight budget thus spills its own spool pages before it touches an FF weight panel
that every step re-reads (which a single global LRU would evict first because it was touched longest ago),
and among equally old objects a clean one goes before a dirty one.
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

# eviction tiers: bytes per microsecond and fixed microseconds per transfer (module doc)
TIER_BW = {"pinned": 25e3, "pool": 3e3}
TIER_T0 = {"pinned": 10.0, "pool": 50.0}

# locality type -> (reuse prior, replacement policy within the set)
LOCALITY = {
    "model": (8.0, "lru"),        # weights / lookup tables re-read by every job step
    "job": (1.0, "lru"),          # job inputs and outputs
    "shuffle": (0.1, "mru"),      # shuffle data (read once by the receiving stage)
    "partition": (0.1, "mru"),    # hash-partition spools (Grace join / partitioned aggregation)
    "temp": (0.05, "mru"),        # spooled tuple sets and other job-scoped temp data
}


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
        self.world_size = 1            # set by the client from its cluster context
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
        # the device relational kernels charge their scratch to this manager's budget (execution/kernels.py)
        from ..execution.kernels import register_scratch_accounting

        register_scratch_accounting(self)
        # per locality set: everything of it resident on the device tier (pages and dense panels) in recency
        # order, oldest first (LocalitySet::cachedPages: pop_front for LRU, pop_back for MRU)
        self._resident: Dict[int, Tuple[object, "OrderedDict[int, object]"]] = {}
        self.eviction_policy = "cost"     # "cost" (per-locality-set costs) or "lru" (one global LRU, A/B tests)
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
                   dense: bool = False, set_id: Optional[int] = None, persistent: bool = True,
                   locality: Optional[str] = None) -> UserSet:
        with self.lock:
            key = (db, name)
            if key in self.sets:
                return self.sets[key]
            dev = self.device if device == "default" else device
            sid = set_id if set_id is not None else (next(self._ids) if persistent else next(self._temp_ids))
            cls = DenseMatrixSet if dense else UserSet
            s = cls(self, db, name, type_, sid, page_size or self.page_size, dev, persistent)
            s.locality = locality or ("job" if persistent else "temp")
            self.sets[key] = s
            return s

    def set_locality(self, db: str, name: str, locality: str):
        """Declare how a set is used (``LOCALITY`` keys): e.g. ``model`` for weights every step re-reads."""
        if locality not in LOCALITY:
            raise ValueError(f"unknown locality {locality!r}: one of {sorted(LOCALITY)}")
        self.get_set(db, name).locality = locality

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
        if hasattr(s, "drop_scan_views"):
            s.drop_scan_views()
        else:
            s.__dict__.pop("_merged_runs", None)
        for p in s.pages:
            self.untrack(p)
            if p.location == "device" and p.batch is not None:
                self.device_bytes -= p.nbytes
            elif p.location == "pinned" and self.host_tier is not None:
                self.host_tier.release(p.nbytes)
            p.release_regions()
            p.batch = None          # the region returns once no held batch views it any more

    def set_costs(self, db: str, name: str, write_cost: Optional[float] = None, read_cost: Optional[float] = None):
        """Per-set multipliers of the write / read cost (LocalitySet::setWriteCost / setReadCost)."""
        st = self.get_set(db, name)
        if write_cost is not None:
            st.write_cost = float(write_cost)
        if read_cost is not None:
            st.read_cost = float(read_cost)

    # ----------------------------------------------------------- memory accounting / eviction
    def on_home(self, device) -> bool:
        """True when ``device`` is the budgeted device tier of this node."""
        if device is None:
            return False
        d, h = torch.device(device), self.home
        if d.type != h.type:
            return False
        return d.type != "cuda" or (d.index or 0) == (h.index or 0)

    @staticmethod
    def _set_of(obj):
        return obj if isinstance(obj, DenseMatrixSet) else obj.set

    # The resident-set dicts are shared by every job lane (concurrent server requests): track / untrack / touch
    # and the victim scan all hold self.lock (an RLock, re-entered by evict -> untrack).
    def track(self, obj):
        """``obj`` (a page or dense set) is resident on the device tier: most recently used."""
        with self.lock:
            obj.last_use = next(self._clock)
            s = self._set_of(obj)
            ent = self._resident.get(id(s))
            if ent is None:
                ent = self._resident[id(s)] = (s, OrderedDict())
            ent[1][id(obj)] = obj
            ent[1].move_to_end(id(obj))

    def untrack(self, obj):
        with self.lock:
            s = self._set_of(obj)
            ent = self._resident.get(id(s))
            if ent is not None:
                ent[1].pop(id(obj), None)
                if not ent[1]:
                    del self._resident[id(s)]

    def resident_objects(self) -> int:
        with self.lock:
            return sum(len(od) for _, od in self._resident.values())

    def account(self, page: Page):
        with self.lock:
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
        with self.lock:
            page.last_use = next(self._clock)
            ent = self._resident.get(id(self._set_of(page)))
            if ent is not None and id(page) in ent[1]:
                ent[1].move_to_end(id(page))

    def touch_run(self, pages, ids=None):
        """touch() of consecutive pages of ONE set, oldest first, under one lock acquisition (a coalesced scan's run
        of hundreds of pages). ``ids``: the pages' id()s, when the caller keeps them."""
        if not pages:
            return
        with self.lock:
            ent = self._resident.get(id(self._set_of(pages[0])))
            od = ent[1] if ent is not None else None
            t = next(self._clock)                # one stamp for the run: ties inside it fall back to the set's order
            for p in pages:
                p.last_use = t
            if od is None:
                return
            if ids is None:
                ids = [id(p) for p in pages]
            if len(od) >= len(ids) and list(itertools.islice(reversed(od), len(ids))) == ids[::-1]:
                return                           # the run already is the set's most recent tail, in order
            for k in ids:
                if k in od:
                    od.move_to_end(k)

    @staticmethod
    def _resident_on_device(p) -> bool:
        return p.resident_on_home() if isinstance(p, DenseMatrixSet) else (p.location == "device" and p.batch is not None)

    @staticmethod
    def _nbytes(p) -> int:
        return max(1, p._charged if isinstance(p, DenseMatrixSet) else p.nbytes)

    def _candidate(self, s, od: "OrderedDict[int, object]", keep, skip: set):
        """The set's replacement candidate (LRU: oldest; MRU: newest) that may be evicted now."""
        policy = LOCALITY.get(getattr(s, "locality", "job"), LOCALITY["job"])[1]
        seq = reversed(od.values()) if policy == "mru" else od.values()
        for p in seq:
            if p is keep or p.pins or id(p) in skip:
                continue
            return p
        return None

    @staticmethod
    def is_clean(p) -> bool:
        """Evicting ``p`` needs no write: its image is already persisted (module doc)."""
        if isinstance(p, DenseMatrixSet):
            return p.is_clean()
        return not p.dirty

    def _spill_tier(self, p) -> str:
        """Where a dirty ``p`` goes when evicted now: the pinned host tier if it admits the bytes, else the pool."""
        tier = self.host_tier
        if tier is not None and self.home.type == "cuda" and tier.used + self._nbytes(p) <= tier.budget:
            return "pinned"
        return "pool"

    def write_cost(self, s, p) -> float:
        """Microseconds to move ``p`` out of the device tier (0 when clean), times the set's multiplier."""
        if self.is_clean(p):
            return 0.0
        t = self._spill_tier(p)
        return (self._nbytes(p) / TIER_BW[t] + TIER_T0[t]) * getattr(s, "write_cost", 1.0)

    def read_cost(self, s, p) -> float:
        """Microseconds to bring ``p`` back from where eviction puts it, times the set's multiplier."""
        t = "pool" if self.is_clean(p) else self._spill_tier(p)
        return (self._nbytes(p) / TIER_BW[t] + TIER_T0[t]) * getattr(s, "read_cost", 1.0)

    def evict_cost(self, s, p, need: Optional[int] = None) -> float:
        """Eviction cost per byte freed of candidate ``p`` of locality set ``s`` (module doc)."""
        prior = LOCALITY.get(getattr(s, "locality", "job"), LOCALITY["job"])[0]
        n = max(1, self.resident_objects())
        distance = max(0, self._clock_now() - p.last_use)
        reuse_prob = prior / (1.0 + distance / n)
        freed = self._nbytes(p) if need is None else max(1, min(self._nbytes(p), need))
        return (self.write_cost(s, p) + reuse_prob * self.read_cost(s, p)) / freed

    def _clock_now(self) -> int:
        return getattr(self, "_last_clock", 0)

    def _pick_victim(self, keep, skip: set, need: Optional[int] = None):
        if self.eviction_policy == "lru":
            best = None
            for s, od in self._resident.values():
                for p in od.values():
                    if p is keep or p.pins or id(p) in skip:
                        continue
                    if best is None or p.last_use < best.last_use:
                        best = p
                    break                      # the set's oldest unpinned object
            return best
        best, best_cost = None, None
        for s, od in self._resident.values():
            p = self._candidate(s, od, keep, skip)
            if p is None:
                continue
            c = self.evict_cost(s, p, need)
            if best is None or c < best_cost or (c == best_cost and p.last_use < best.last_use):
                best, best_cost = p, c
        return best

    def evict(self, need: int, keep=None) -> int:
        """Spill device pages (to the pinned tier / page pool) and dense panels (in block-row slabs,
        PageCache/PDBEvictWork style) until ``need`` bytes are free: victims by per-locality-set cost."""
        with self.lock:
            return self._evict(need, keep)

    def _evict(self, need: int, keep=None) -> int:
        freed = 0
        skip = set()                 # objects that could not be spilled this round
        self._last_clock = next(self._clock)
        while freed < need:
            p = self._pick_victim(keep, skip, need - freed)
            if p is None:
                break
            if not self._resident_on_device(p):
                self.untrack(p)
                continue
            f = p.spill()
            if f or not self._resident_on_device(p):
                self.untrack(p)
                self.stats.setdefault("evicted_by_locality", {})
                loc = getattr(self._set_of(p), "locality", "job")
                self.stats["evicted_by_locality"][loc] = self.stats["evicted_by_locality"].get(loc, 0) + 1
            else:
                skip.add(id(p))
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
            "sets": {f"{d}.{n}": {"records": s.num_records(), "bytes": s.nbytes(), "pages": len(s.pages),
                                  "locality": getattr(s, "locality", "job")}
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


__all__ = ["StorageManager", "DEFAULT_PAGE_SIZE", "LOCALITY", "TIER_BW", "TIER_T0"]
