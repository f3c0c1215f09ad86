"""Sets and pages (reference: src/storage/headers/UserSet.h, LocalitySet.h, TempSet.h, PDBPage.h,
PageCache.h, PDBFlushProducerWork/ConsumerWork, PDBEvictWork).

A :class:`UserSet` is one node's partition of a stored set: an ordered list of :class:`Page` s,
each holding a RecordBatch of at most ``page_size`` bytes.  Pages are resident in HBM (device
sets), in host memory, or spilled: a spilled page's serialised image lives in the native
:class:`BufferManager` page pool, which itself LRU-evicts to the set's page file on disk.

:class:`DenseMatrixSet` is the MI355X-native physical layout for block-partitioned matrices
(MatrixBlock / FFMatrixBlock sets): the node's row-slab of the matrix is ONE dense, 16-B-aligned
row-major HBM panel that the MFMA kernels read directly with buffer loads; the MatrixBlock
records the UDFs see are slices of it.  This replaces netsDB's per-block heap objects and avoids
assembling blocks before every block GEMM.
"""
from __future__ import annotations

import math
import itertools
import threading
import weakref
from typing import Dict, Iterator, List, Optional, Tuple

import torch

from ..objects.record import RecordBatch, merge_adjacent_batches
from .serde import deserialize_batch, serialize_batch

_BATCH_GEN = itertools.count(1)


class Page:
    __slots__ = ("set", "page_no", "_batch", "gen", "nbytes", "pins", "location", "dirty", "last_use", "n", "event",
                 "regions")

    @property
    def batch(self) -> Optional[RecordBatch]:
        return self._batch

    @batch.setter
    def batch(self, b: Optional[RecordBatch]):
        # every (re)assignment gets a new generation: cached scan plans key on it (object ids can be reused); the
        # set's layout version follows, so a scan can tell in O(1) that none of its pages changed
        self._batch = b
        self.gen = next(_BATCH_GEN)
        st = getattr(self, "set", None)
        if st is not None:
            st._layout_version = self.gen
            # the scan fast path's merged views are stale now, and they would keep this page's old buffers (and the
            # short-code encodings derived from them) alive after a spill credited their bytes back
            st.__dict__.pop("_scan_fast", None)

    def __init__(self, uset: "UserSet", page_no: int, batch: RecordBatch, to_pool: bool = False):
        self.set = uset
        self.page_no = page_no
        self.nbytes = batch.nbytes()
        self.n = batch.n
        self.pins = 0
        mgr = getattr(uset, "manager", None)
        pool = getattr(mgr, "page_pool", None)
        # pages arriving from the host (sendData / add_batch of host records, page reloads) are copied straight
        # into slab-allocated regions of the manager's HBM page arena (storage/devpool.py); a page a device
        # kernel just produced keeps its tensors (no extra device copy); on a CPU node every page is in the
        # host arena
        self.regions = []
        if to_pool and pool is not None:
            batch, self.regions = pool.adopt(batch, move=True)
            batch = batch.to(uset.device)        # string / nested column objects (tensor columns: no-op)
        home = mgr.on_home(batch.device) if mgr is not None and hasattr(mgr, "on_home") else batch.device.type == "cuda"
        if home and pool is not None and not self.regions and not pool.is_cuda:
            batch, self.regions = pool.adopt(batch)
        self.location = "device" if home else "host"
        self.dirty = True
        self.last_use = 0
        self.event = None      # pinned tier: completion event of the page's D2H copy
        self.batch: Optional[RecordBatch] = batch

    def release_regions(self, events=()):
        """Drop the page's hold on its arena regions. A region returns to the slab allocator when the last
        tensor viewing it is gone (batches a scan yielded earlier stay valid) and every event in ``events``
        (e.g. the eviction's D2H copy) has completed (storage/devpool.py)."""
        for r in self.regions:
            for e in events:
                r.attach_event(e)
        self.regions = []

    def is_resident(self) -> bool:
        return self.batch is not None

    def spill(self):
        """Evict from HBM: to the pinned host tier (async DMA) when it has room, else serialise into the
        native page pool (LRU -> disk) and drop the in-memory batch."""
        if self.batch is None or self.pins > 0:
            return 0
        self.set.drop_scan_views()                       # kept scan views would hold this page's buffers alive
        if self.location == "device" and not self.dirty:
            # clean: the page's serialised image is already in the pool / page file (write cost 0) -> just drop it
            self.release_regions()
            self.batch = None
            self.location = "pool"
            return self.nbytes
        tier = getattr(self.set.manager, "host_tier", None)
        if self.location == "device" and tier is not None and tier.admit(self.nbytes):
            self.batch, self.event = tier.offload(self.batch, self.nbytes)
            self.release_regions((self.event,))          # reusable once the D2H copy has read them
            self.location = "pinned"
            return self.nbytes
        if self.location == "pinned":
            self.batch = tier.host_view(self.batch, self.event)
            tier.release(self.nbytes)
            self.event = None
        bm = self.set.manager.buffer_manager
        data = serialize_batch(self.batch)
        if len(data) > bm.page_size:
            raise RuntimeError(f"page image {len(data)} B exceeds pool page size {bm.page_size}")
        slot = bm.pin(self.set.set_id, self.page_no, True)
        view = bm.slot_view(slot)
        view[: len(data)] = data
        bm.unpin(self.set.set_id, self.page_no, True, len(data))
        freed = self.nbytes if self.location == "device" else 0
        self.release_regions()
        self.batch = None
        self.location = "pool"
        self.dirty = False
        return freed

    def load(self, device) -> RecordBatch:
        if self.location == "pinned":
            tier = self.set.manager.host_tier
            if device is not None and torch.device(device).type == "cuda":
                pool = getattr(self.set.manager, "page_pool", None)
                self.batch, self.regions = tier.fetch(self.batch, self.event, self.nbytes, pool=pool)
                self.event = None
                self.location = "device"
                self.set.manager.track(self)
                self.pins += 1
                try:
                    self.set.manager.account_bytes(self.nbytes, device, keep=self)
                finally:
                    self.pins -= 1
            else:
                self.batch = tier.host_view(self.batch, self.event)
            return self.batch
        if self.batch is not None:
            return self.batch
        bm = self.set.manager.buffer_manager
        slot = bm.pin(self.set.set_id, self.page_no, False)
        try:
            n = bm.bytes_used(self.set.set_id, self.page_no)
            data = bytes(bm.slot_view(slot)[:n])
        finally:
            bm.unpin(self.set.set_id, self.page_no, False, 0)
        b = deserialize_batch(data)
        mgr = self.set.manager
        if device is not None and torch.device(device).type == "cuda":
            pool = getattr(mgr, "page_pool", None)
            if pool is not None and mgr.on_home(device):
                b, self.regions = pool.adopt(b, move=True)     # H2D straight into the page arena
            b = b.to(device)
        elif mgr.on_home(b.device) and getattr(mgr, "page_pool", None) is not None:
            b, self.regions = mgr.page_pool.adopt(b)
        self.batch = b
        self.location = "device" if mgr.on_home(b.device) else "host"
        self.dirty = False
        if self.location == "device":
            mgr.track(self)
            self.pins += 1            # the reload is charged to the budget; never evict the page being loaded
            try:
                mgr.account_bytes(self.nbytes, mgr.home, keep=self)
            finally:
                self.pins -= 1
        return b

    def persist(self):
        """Write the page image to the pool (and from there to disk on flush) without dropping it."""
        if self.batch is None or not self.dirty:
            return
        bm = self.set.manager.buffer_manager
        if self.location == "pinned":
            self.set.manager.host_tier.host_view(self.batch, self.event)
        data = serialize_batch(self.batch)
        slot = bm.pin(self.set.set_id, self.page_no, True)
        bm.slot_view(slot)[: len(data)] = data
        bm.unpin(self.set.set_id, self.page_no, True, len(data))
        self.dirty = False


class SharedLink:
    """Pages of a shared set linked into a sharing set (reference: PDBClient::addSharedPage /
    addSharedMapping, src/deduplication SharedFFMatrixBlockSet + PartitionTensorBlockSharedPageIterator).

    The sharing set scans its own pages, then the linked pages of the shared set.  With a block
    mapping (distinct block id -> target (block_row, block_col, total_rows, total_cols)) the shared
    blocks' metadata is rewritten on the fly, exactly as the reference's shared-page iterator does;
    a block without an entry gets block_row = block_col = -1 (the reference's "not found" marker)."""

    def __init__(self, shared: "UserSet"):
        self.shared = shared
        self.pages: List[int] = []
        self.keys: Optional[torch.Tensor] = None      # sorted distinct block ids
        self.targets: Optional[torch.Tensor] = None   # [n, 4] int64 (block_row, block_col, total_rows, total_cols)

    def set_mapping(self, mapping: dict):
        """distinct block id -> target (block_row, block_col, total_rows, total_cols), or a list of targets
        when one stored block appears at several places of the sharing model (exact dedup of repeated
        blocks inside one model); keys are kept sorted with repeats."""
        rows = []
        for k, v in mapping.items():
            for t in (v if v and isinstance(v, list) else [v]):
                rows.append((int(k), *[int(x) for x in t]))
        rows.sort()
        self.keys = torch.tensor([r[0] for r in rows], dtype=torch.int64)
        self.targets = torch.tensor([list(r[1:]) for r in rows], dtype=torch.int64).reshape(-1, 4)

    def batches(self, device=None) -> Iterator[RecordBatch]:
        sh = self.shared
        if isinstance(sh, DenseMatrixSet):
            src = [sh.to_blocks(device)] if sh.has_data() and (not self.pages or 0 in self.pages) else []
        else:
            src = []
            for pno in self.pages:
                if 0 <= pno < len(sh.pages):
                    pg = sh.pages[pno]
                    pg.pins += 1
                    try:
                        src.append(pg.load(device if device is not None else sh.device))
                    finally:
                        pg.pins -= 1
        for b in src:
            yield self._remap(b) if self.keys is not None else b

    def _remap(self, b: RecordBatch) -> RecordBatch:
        if b.n == 0 or "distinct_block_id" not in b.columns:
            return b
        ids = b.columns["distinct_block_id"]
        dev = ids.device
        keys, tg = self.keys.to(dev), self.targets.to(dev)
        if keys.numel() == 0:
            lo = torch.zeros(b.n, dtype=torch.int64, device=dev)
            cnt = torch.zeros(b.n, dtype=torch.int64, device=dev)
        else:
            lo = torch.searchsorted(keys, ids, right=False)
            cnt = torch.searchsorted(keys, ids, right=True) - lo
        # a block with k targets becomes k rows; a block without one keeps a single (-1, -1) row
        rep = cnt.clamp_min(1)
        row = torch.repeat_interleave(torch.arange(b.n, device=dev), rep)
        start = torch.cumsum(rep, 0) - rep
        within = torch.arange(row.numel(), device=dev) - start.index_select(0, row)
        found = cnt.index_select(0, row) > 0
        tpos = (lo.index_select(0, row) + within).clamp(max=max(0, keys.numel() - 1))
        out = b.take(row) if row.numel() != b.n or bool((cnt > 1).any()) else b
        cols = dict(out.columns)
        for j, name in enumerate(("block_row", "block_col", "total_rows", "total_cols")):
            miss = -1 if j < 2 else 0
            val = tg[tpos, j] if keys.numel() else torch.zeros_like(row)
            cols[name] = torch.where(found, val, torch.full_like(row, miss))
        return RecordBatch(cols, int(row.numel()), b.type)

    def num_records(self) -> int:
        sh = self.shared
        if isinstance(sh, DenseMatrixSet):
            return sh.num_blocks() if sh.has_data() else 0
        return sum(sh.pages[p].n for p in self.pages if 0 <= p < len(sh.pages))


def _same_device(a: torch.device, b: torch.device) -> bool:
    return a.type == b.type and (a.index == b.index or a.index is None or b.index is None)


class UserSet:
    """One node's partition of a stored set."""

    def __init__(self, manager, db: str, name: str, type_, set_id: int, page_size: int, device=None,
                 persistent: bool = True):
        self.manager = manager
        self.db, self.name = db, name
        self.type = type_
        self.set_id = set_id
        self.page_size = page_size
        self.device = device
        self.pages: List[Page] = []
        self.persistent = persistent
        self.lock = threading.RLock()
        self.partition_key = None       # (computation, lambda) describing how the set is partitioned
        # hash placement of the rows across ranks: (key kind, key name, world size) when every row came
        # through a dispatch by that key (send_data with a key LambdaPolicy); None once anything else
        # (round-robin dispatch, local adds, engine outputs) put rows here
        self.placement = None
        self.stats = {"records": 0, "bytes": 0}
        self.shared_links: Dict[Tuple[str, str], SharedLink] = {}   # dedup: pages linked from shared sets

    # -------------------------------------------------------------- dedup page sharing
    def link(self, shared: "UserSet") -> SharedLink:
        key = (shared.db, shared.name)
        if key not in self.shared_links:
            self.shared_links[key] = SharedLink(shared)
        return self.shared_links[key]

    def add_shared_page(self, shared: "UserSet", page_no: int):
        ln = self.link(shared)
        if page_no not in ln.pages:
            ln.pages.append(page_no)
        self._shared_dirty = True

    def set_shared_mapping(self, shared: "UserSet", mapping: dict):
        self.link(shared).set_mapping(mapping)
        self._shared_dirty = True

    def shared_batches(self, device=None) -> Iterator[RecordBatch]:
        for ln in list(self.shared_links.values()):
            yield from ln.batches(device)

    # -------------------------------------------------------------- writes
    def note_placement(self, placement):
        """A collective dispatch into this set (called on every rank, rows or not): an empty set takes the
        dispatch's placement; a different placement on a non-empty set makes it unknown."""
        if self.stats["records"] == 0 and not getattr(self, "_placed", False):
            self.placement = placement
        elif placement != self.placement:
            self.placement = None
        self._placed = True

    def add_batch(self, batch: RecordBatch, placement="unknown"):
        if placement == "unknown":
            self.placement = None
            self._placed = True
        if batch.n == 0:
            return
        batch = batch.materialize()          # a stored page never holds a lazy selection's source columns
        pool = getattr(self.manager, "page_pool", None)
        to_pool = (pool is not None and pool.is_cuda and self.device is not None and batch.device.type == "cpu"
                   and self.manager.on_home(self.device))
        if self.device is not None and batch.device != torch.device(self.device) and not to_pool:
            batch = batch.to(self.device)
        with self.lock:
            per_row = max(1, batch.nbytes() // max(1, batch.n))
            # leave room for the serialised page header/column directory when the page spills to the pool
            usable = max(per_row, self.page_size - max(2048, self.page_size // 16))
            rows_per_page = max(1, usable // per_row)
            for s in range(0, batch.n, rows_per_page):
                part = batch.slice(s, min(batch.n, s + rows_per_page)) if batch.n > rows_per_page else batch
                p = Page(self, len(self.pages), part, to_pool=to_pool)
                self.pages.append(p)
                self.stats["records"] += part.n
                self.stats["bytes"] += p.nbytes
                self.manager.account(p)

    def drop_scan_views(self):
        """Forget the merged scan views (and the fast-path list holding them, with the string short-code encodings
        cached on their columns): after a spill, drop or clear their HBM must actually be released."""
        self.__dict__.pop("_merged_runs", None)
        self.__dict__.pop("_scan_fast", None)

    def clear(self):
        with self.lock:
            self.drop_scan_views()
            for p in self.pages:
                self.manager.untrack(p)
            self.pages = []
            self._layout_version = next(_BATCH_GEN)
            self.stats = {"records": 0, "bytes": 0}
            self.placement = None
            self._placed = False
            self.manager.buffer_manager.drop_set(self.set_id)

    # -------------------------------------------------------------- reads
    def scan(self, device=None) -> Iterator[RecordBatch]:
        device = device if device is not None else self.device
        pages = list(self.pages)
        if device is not None and (torch.device(device).type == "cuda" or self.COALESCE_ANY_DEVICE) and len(pages) > 1:
            yield from self._scan_coalesced(pages, torch.device(device))
            yield from self.shared_batches(device)
            return
        ra = getattr(self.manager, "read_ahead", 0)
        queued = 0
        for i, p in enumerate(pages):
            if ra and i >= queued:
                # native read-ahead: evicted pages among the next `ra` are pulled from the page file into
                # pool slots by the I/O workers while this page is deserialised / consumed
                nxt = [q.page_no for q in pages[i: i + ra] if q.batch is None]
                if nxt:
                    self.manager.prefetch(self, nxt)
                queued = i + ra
            p.pins += 1
            try:
                b = p.load(device)
                self.manager.touch(p)
                yield b
            finally:
                p.pins -= 1
        yield from self.shared_batches(device)

    # resident device pages merged per scanned batch (bytes): 64 MiB pages are a storage / spill unit, not a good
    # kernel size on a 288 GB GPU; pages cut from one loaded batch are merged back without a copy. 16 GiB keeps a
    # TPC-H SF 10 lineitem scan one batch (one launch per operator instead of three; its intermediates stay far
    # below the engine's out-of-core limit, a quarter of the device budget)
    SCAN_COALESCE_BYTES = 16 << 30
    COALESCE_ANY_DEVICE = False      # tests: run the merge on CPU pages too

    def coalesce_cap(self) -> int:
        """Merged-batch cap: SCAN_COALESCE_BYTES, but never more than the engine's out-of-core share of the node's
        device budget (``coalesce_fraction`` of it, default 1/8): per-batch intermediates (join expansion, gathers,
        group-by work buffers) scale with the merged batch and must stay inside what the spill logic assumes free."""
        budget = getattr(self.manager, "device_budget", None) or (1 << 62)
        frac = getattr(self.manager, "coalesce_fraction", 0.125)
        return int(max(self.page_size, min(self.SCAN_COALESCE_BYTES, budget * frac)))

    def _coalesce_runs(self, pages, device) -> List[Tuple[int, int]]:
        """[i, j) runs of consecutive resident pages whose columns are adjacent slices of one buffer (checked once;
        the plan is cached while the pages and their resident batches stay the same objects)."""
        key = tuple((id(p), p.gen, p.n) for p in pages) + (str(device),)
        if getattr(self, "_coalesce_key", None) == key:
            return self._coalesce_plan
        runs, i = [], 0
        cap = self.coalesce_cap()
        while i < len(pages):
            j, nbytes = i, 0
            while j < len(pages) and nbytes < cap:
                b = pages[j].batch
                if b is None or not _same_device(b.device, device):
                    break
                if j > i and merge_adjacent_batches([pages[j - 1].batch, b]) is None:
                    break                          # not a continuation of the previous page's buffers
                nbytes += pages[j].nbytes
                j += 1
            if j - i > 1 and merge_adjacent_batches([p.batch for p in pages[i:j]]) is not None:
                runs.append((i, j))
                i = j
            else:
                runs.append((i, i + 1))
                i += 1
        self._coalesce_key, self._coalesce_plan = key, runs
        return runs

    def _scan_coalesced(self, pages, device) -> Iterator[RecordBatch]:
        """Runs of consecutive pages resident on ``device`` whose columns are adjacent slices of one buffer are
        yielded as ONE batch (zero-copy views, up to SCAN_COALESCE_BYTES); any other page is yielded alone."""
        # fast path: no page of the set changed since a scan that merged every page into cached runs
        ver = (getattr(self, "_layout_version", None), len(pages), str(device))
        fast = self.__dict__.get("_scan_fast")
        if fast is not None and fast[0] == ver and ver[0] is not None:
            touch_run = getattr(self.manager, "touch_run", None)
            for run, merged, ids in fast[1]:
                for p in run:
                    p.pins += 1
                try:
                    if touch_run is not None:
                        touch_run(run, ids)
                    yield merged
                finally:
                    for p in run:
                        p.pins -= 1
            return
        all_merged = []
        plan = self._coalesce_runs(pages, device)
        gens = [p.gen for p in pages]          # the layout the plan was checked against
        for i, j in plan:
            run = pages[i:j]
            if j - i > 1:
                # a page spilled / reloaded while earlier runs were consumed no longer matches the plan: page by page
                # (one pass: the run's identity and its validity together)
                ident = tuple((id(p.batch), p.gen) for p in run)
                ok = all(p.batch is not None for p in run) and [g for _, g in ident] == gens[i:j]
            if j - i > 1 and ok:
                for p in run:
                    p.pins += 1
                try:
                    # the merged view of an unchanged run is kept: a re-scan costs no per-page work, and what a
                    # query derives from its columns (a string column's short-code encoding) survives the scan
                    cache = self.__dict__.setdefault("_merged_runs", {})
                    hit = cache.get((i, j))
                    if hit is not None and hit[0] == ident:
                        merged = hit[1]
                    else:
                        merged = merge_adjacent_batches([p.batch for p in run], check=False)
                        cache[(i, j)] = (ident, merged)
                    touch_run = getattr(self.manager, "touch_run", None)
                    if touch_run is not None:
                        touch_run(run)
                    else:
                        for p in run:
                            self.manager.touch(p)
                    if all_merged is not None:
                        all_merged.append((run, merged))
                    yield merged
                finally:
                    for p in run:
                        p.pins -= 1
                continue
            all_merged = None                  # a page-by-page run: no fast path for this layout
            for p in run:
                p.pins += 1
                try:
                    b = p.load(device)
                    self.manager.touch(p)
                    yield b
                finally:
                    p.pins -= 1
        if all_merged is not None and ver[0] is not None and getattr(self, "_layout_version", None) == ver[0]:
            self._scan_fast = (ver, [(run, merged, [id(p) for p in run]) for run, merged in all_merged])

    def all(self, device=None) -> Optional[RecordBatch]:
        bs = list(self.scan(device))
        if not bs:
            return None
        return RecordBatch.concat(bs)

    def num_records(self) -> int:
        return self.stats["records"] + sum(ln.num_records() for ln in self.shared_links.values())

    def nbytes(self) -> int:
        return self.stats["bytes"]

    def persist_pages(self):
        for p in self.pages:
            p.persist()

    def flush(self):
        self.persist_pages()
        self.manager.buffer_manager.flush_set(self.set_id)

    def page_meta(self) -> list:
        return [[p.page_no, p.n, p.nbytes] for p in self.pages]

    def restore(self, pages: list):
        """Re-attach persisted pages lazily (they load from the page file on first scan)."""
        for page_no, n, nbytes in pages:
            p = Page.__new__(Page)
            p.set, p.page_no, p.batch, p.nbytes, p.n = self, page_no, None, nbytes, n
            p.pins, p.location, p.dirty, p.last_use = 0, "pool", False, 0
            p.event, p.regions = None, []
            self.pages.append(p)
            self.stats["records"] += n
            self.stats["bytes"] += nbytes
        return self

    def __repr__(self):
        return f"UserSet({self.db}.{self.name}, pages={len(self.pages)}, records={self.num_records()})"


class DenseMatrixSet(UserSet):
    """A block-partitioned matrix stored as one dense row-slab panel per node.

    The panel is charged to the node's device budget and is evictable like any page
    (PageCache.cc / PDBEvictWork): under HBM pressure the storage manager spills it in block-row
    slabs of about one page — to the pinned host tier by async D2H copies when the panel is on a GPU,
    else serialised into the native page pool — and the next access of :attr:`panel` brings it back
    (H2D copies on the copy stream, ordered before the consumer by a stream wait).  Out-of-core
    consumers read row ranges with :meth:`load_rows` without making the whole panel resident."""

    def __init__(self, manager, db, name, type_, set_id, page_size, device=None, persistent=True):
        super().__init__(manager, db, name, type_, set_id, page_size, device, persistent)
        self._panel: Optional[torch.Tensor] = None    # [local_rows_padded, ld] when resident
        self._spilled: Optional[list] = None          # [(row0, rows, where, handle, event)] when evicted
        self._shape = None                            # (rows, ld, dtype, device) of the spilled panel
        self._charged = 0                             # bytes charged to the device budget
        self.pins = 0
        self.last_use = 0
        self.total_rows = 0
        self.total_cols = 0
        self.block_rows = 0
        self.block_cols = 0
        self.row_offset = 0                           # first global row held by this node
        self.local_rows = 0
        self.transposed = False                       # panel holds the logical matrix transposed
        self.replicated = False                       # every rank holds the full matrix
        self.stats_io = {"spills": 0, "reloads": 0, "slab_loads": 0}
        # spilled slabs go to the page pool under a temp set id of their own with page numbers from 0 (the
        # persisted chunks use this set's id): the page file offset is page_no * page_size, so the slabs must
        # not sit at large page numbers of the set's own file
        self._spill_id: Optional[int] = None
        self._clean_key = None                        # (panel id, version) persisted by persist_pages
        self._clean_geo = None                        # geometry of a clean panel dropped by eviction

    # residency -------------------------------------------------------
    def is_clean(self) -> bool:
        """A "model" panel (read-only weights by contract) unchanged since persist_pages wrote its image: evicting
        it needs no write (storage/manager.py cost model); its version counter catches in-place tensor writes."""
        t = self._panel
        key = self._clean_key
        return (t is not None and getattr(self, "locality", "job") == "model" and key is not None
                and key[0]() is t and key[1] == t._version)

    @property
    def panel(self) -> Optional[torch.Tensor]:
        if self._panel is None and self._clean_geo is not None:
            geo, self._clean_geo = self._clean_geo, None
            self.restore(geo)                          # clean drop: rebuild from the persisted chunks
            self.stats_io["reloads"] += 1
            if self._panel is not None:                # restored from the persisted image: clean again
                self._clean_key = (weakref.ref(self._panel), self._panel._version)
        if self._panel is None and self._spilled is not None:
            self.reload()
        if self._panel is not None:
            self.manager.touch(self)
        return self._panel

    @panel.setter
    def panel(self, t: Optional[torch.Tensor]):
        self._install(t)

    def _install(self, t: Optional[torch.Tensor]):
        # a new panel invalidates any persisted clean image: a dropped clean panel must never come back over it
        self._drop_spilled()
        self._clean_geo = None
        self._clean_key = None
        old = self._charged
        self._panel = t
        self._charged = 0
        if old:
            self.manager.release_bytes(old, self.manager.home)
        if t is None or not self.manager.on_home(t.device):
            self.manager.untrack(self)
        if t is not None and self.manager.on_home(t.device):
            self._charged = t.numel() * t.element_size()
            self.manager.track(self)
            self.pins += 1
            try:
                self.manager.account_bytes(self._charged, self.manager.home, keep=self)
            finally:
                self.pins -= 1

    def is_resident(self) -> bool:
        return self._panel is not None

    def is_spilled(self) -> bool:
        return self._spilled is not None or self._clean_geo is not None

    def resident_on_home(self) -> bool:
        return self._panel is not None and self._charged > 0

    def has_data(self) -> bool:
        return self._panel is not None or self._spilled is not None or self._clean_geo is not None

    def panel_nbytes(self) -> int:
        if self._panel is not None:
            return self._panel.numel() * self._panel.element_size()
        if self._shape is not None:
            r, ld, dt, _ = self._shape
            return r * ld * torch.empty(0, dtype=dt).element_size()
        return 0

    def row_bytes(self) -> int:
        if self._panel is not None:
            return self._panel.shape[1] * self._panel.element_size()
        if self._shape is not None:
            return self._shape[1] * torch.empty(0, dtype=self._shape[2]).element_size()
        return 0

    def _slab_rows(self, ld: int, esize: int) -> int:
        """Rows per spill slab: whole block rows when a block row fits a page, else as many rows as fit (a slab
        must fit one pool page; load_rows assembles any row range from slabs of any height)."""
        per = max(1, self.page_size // max(1, ld * esize))
        if self.block_rows and per >= self.block_rows:
            per = per // self.block_rows * self.block_rows
        return per

    def spill(self) -> int:
        """Evict the panel in block-row slabs; returns the device bytes freed (0 if pinned/absent)."""
        t = self._panel
        if t is None or self.pins > 0:
            return 0
        if self.is_clean():
            # write cost 0: the image persisted by persist_pages is current -> drop, restore on next access
            self._clean_geo = self.geometry()
            freed = self._charged
            self._charged = 0
            self._panel = None
            self._clean_key = None
            self.stats_io["spills"] += 1
            return freed
        tier = getattr(self.manager, "host_tier", None)
        rows, ld = t.shape
        es = t.element_size()
        step = self._slab_rows(ld, es)
        slabs = []
        bm = self.manager.buffer_manager
        for i, r0 in enumerate(range(0, rows, step)):
            part = t[r0: r0 + step]
            nb = part.numel() * es
            if t.is_cuda and tier is not None and tier.admit(nb):
                from ..objects.record import RecordBatch

                host, ev = tier.offload(RecordBatch({"x": part}, part.shape[0]), nb)
                slabs.append((r0, part.shape[0], "pinned", host.columns["x"], ev))
                continue
            data = part.contiguous().cpu().view(torch.uint8).numpy().tobytes()
            if len(data) > bm.page_size:
                raise RuntimeError(f"dense slab {len(data)} B exceeds the pool page size {bm.page_size}")
            pno = i
            if self._spill_id is None:
                self._spill_id = next(self.manager._temp_ids)
            slot = bm.pin(self._spill_id, pno, True)
            bm.slot_view(slot)[: len(data)] = data
            bm.unpin(self._spill_id, pno, True, len(data))
            slabs.append((r0, part.shape[0], "pool", pno, None))
        self._shape = (rows, ld, t.dtype, t.device)
        self._spilled = slabs
        freed = self._charged
        self._charged = 0
        self._panel = None
        self.stats_io["spills"] += 1
        return freed

    def _slab_tensor(self, slab, device) -> torch.Tensor:
        r0, n, where, h, ev = slab
        _, ld, dt, _ = self._shape
        if where == "pinned":
            tier = self.manager.host_tier
            if device is not None and torch.device(device).type == "cuda":
                from ..objects.record import RecordBatch

                return tier.fetch(RecordBatch({"x": h}, n), ev, 0)[0].columns["x"]
            if ev is not None:
                ev.synchronize()
            return h
        bm = self.manager.buffer_manager
        slot = bm.pin(self._spill_id, h, False)
        try:
            nb = bm.bytes_used(self._spill_id, h)
            raw = bytearray(bm.slot_view(slot)[:nb])
        finally:
            bm.unpin(self._spill_id, h, False, 0)
        x = torch.frombuffer(raw, dtype=torch.uint8).view(dt).reshape(n, ld)
        return x.to(device) if device is not None else x

    def reload(self):
        """Bring a spilled panel back to its device (charged to the budget, may evict others)."""
        if self._spilled is None:
            return self._panel
        rows, ld, dt, dev = self._shape
        self.pins += 1
        try:
            if self.manager.on_home(dev):
                self.manager.track(self)
                self.manager.account_bytes(rows * ld * torch.empty(0, dtype=dt).element_size(), self.manager.home,
                                           keep=self)
                self._charged = rows * ld * torch.empty(0, dtype=dt).element_size()
            t = torch.empty(rows, ld, dtype=dt, device=dev)
            for sl in self._spilled:
                t[sl[0]: sl[0] + sl[1]].copy_(self._slab_tensor(sl, dev), non_blocking=True)
        finally:
            self.pins -= 1
        self._drop_spilled(keep_charge=True)
        self._panel = t
        self.stats_io["reloads"] += 1
        return t

    def load_rows(self, r0: int, r1: int, device=None) -> torch.Tensor:
        """Rows [r0, r1) of the panel on ``device`` (a view when resident, else assembled from the spilled
        slabs without reloading the rest): the out-of-core block GEMM's operand slabs."""
        if self._panel is None and self._clean_geo is not None:
            self.panel                                   # noqa: B018  (restore the dropped clean panel)
        if self._panel is not None:
            v = self._panel[r0:r1]
            return v if device is None or v.device == torch.device(device) else v.to(device)
        if self._spilled is None:
            raise RuntimeError(f"set {self.db}.{self.name} holds no panel")
        rows, ld, dt, dev = self._shape
        device = dev if device is None else device
        out = torch.empty(r1 - r0, ld, dtype=dt, device=device)
        for sl in self._spilled:
            a, b = max(r0, sl[0]), min(r1, sl[0] + sl[1])
            if a < b:
                out[a - r0: b - r0].copy_(self._slab_tensor(sl, device)[a - sl[0]: b - sl[0]], non_blocking=True)
        self.stats_io["slab_loads"] += 1
        return out

    def _drop_spilled(self, keep_charge: bool = False):
        if self._spilled is None:
            return
        tier = getattr(self.manager, "host_tier", None)
        for r0, n, where, h, ev in self._spilled:
            if where == "pinned" and tier is not None:
                tier.release(h.numel() * h.element_size())
        if any(sl[2] == "pool" for sl in self._spilled) and self._spill_id is not None:
            self.manager.buffer_manager.drop_set(self._spill_id)
        self._spilled = None
        if not keep_charge:
            self._shape = None

    def release_storage(self):
        """Return the panel's device bytes and spilled slabs (set removed or cleared)."""
        self._drop_spilled()
        self._clean_geo = None
        self._clean_key = None
        if self._charged:
            self.manager.release_bytes(self._charged, self.manager.home)
        self._charged = 0
        self._panel = None

    # geometry -------------------------------------------------------
    def define(self, total_rows: int, total_cols: int, block_rows: int, block_cols: int, row_offset: int = 0,
               local_rows: Optional[int] = None, dtype=torch.bfloat16, device=None, ld_align: int = 64,
               zero: bool = True):
        self.total_rows, self.total_cols = total_rows, total_cols
        self.block_rows, self.block_cols = block_rows, block_cols
        self.row_offset = row_offset
        self.local_rows = total_rows - row_offset if local_rows is None else local_rows
        ld = max(8, math.ceil(total_cols / ld_align) * ld_align)
        dev = device if device is not None else self.device
        alloc = torch.zeros if zero else torch.empty
        self.panel = alloc(self.local_rows, ld, dtype=dtype, device=dev)
        self.stats = {"records": self.num_blocks(), "bytes": self._panel.numel() * self._panel.element_size()}
        return self

    def set_panel(self, panel: torch.Tensor, total_rows: int, total_cols: int, block_rows: int, block_cols: int,
                  row_offset: int = 0, transposed: bool = False, replicated: bool = False):
        """Install a physical panel. ``transposed``: panel is [cols, rows] of the logical matrix."""
        self.panel = panel
        self.total_rows, self.total_cols = total_rows, total_cols
        self.block_rows, self.block_cols = block_rows, block_cols
        self.row_offset = row_offset
        self.transposed = transposed
        self.replicated = replicated
        self.local_rows = panel.shape[1] if transposed else panel.shape[0]
        self.stats = {"records": self.num_blocks(), "bytes": panel.numel() * panel.element_size()}
        return self

    def matrix(self) -> torch.Tensor:
        """Logical [local_rows, total_cols] view (a transposed view when the panel is transposed)."""
        if self.shared_links:
            self.resolve_shared()
        if self.transposed:
            return self.panel[: self.total_cols, : self.local_rows].t()
        return self.panel[:, : self.total_cols]

    def num_blocks(self) -> int:
        if self.block_rows == 0:
            return 0
        return math.ceil(self.local_rows / self.block_rows) * math.ceil(self.total_cols / self.block_cols)

    def block_grid(self) -> Tuple[int, int]:
        return math.ceil(self.total_rows / self.block_rows), math.ceil(self.total_cols / self.block_cols)

    # record view ------------------------------------------------------
    def add_batch(self, batch: RecordBatch):
        """Scatter MatrixBlock records into the panel."""
        if batch.n == 0:
            return
        if not self.has_data():
            b0 = batch.columns
            self.define(int(b0["total_rows"][0]), int(b0["total_cols"][0]), int(b0["row_nums"][0]),
                        int(b0["col_nums"][0]), dtype=batch.columns["data"].dtype if isinstance(
                            batch.columns["data"], torch.Tensor) else torch.float32)
        data = batch.columns["data"]
        todo = self._scatter_full_blocks(batch) if isinstance(data, torch.Tensor) else None
        rows = batch.columns["block_row"].tolist() if todo is None else batch.columns["block_row"][todo].tolist()
        cols = batch.columns["block_col"].tolist() if todo is None else batch.columns["block_col"][todo].tolist()
        if todo is not None:
            data = data[todo]
        for i, (r, c) in enumerate(zip(rows, cols)):
            r0 = r * self.block_rows - self.row_offset
            c0 = c * self.block_cols
            blk = data[i]
            h = min(blk.shape[0], self.local_rows - r0)
            w = min(blk.shape[1], self.total_cols - c0)
            if h > 0 and w > 0:
                self.panel[r0:r0 + h, c0:c0 + w] = blk[:h, :w].to(self.panel.device, self.panel.dtype)

    def _scatter_full_blocks(self, batch: RecordBatch):
        """Vectorised part of add_batch: every block that lies wholly inside the panel and on the block grid is
        written by ONE index_put over a [block-rows, br, block-cols, bc] strided view of the panel (no per-block
        host loop). Returns the indices of the remaining (edge / off-grid) blocks for the element-wise path, or
        None when the batch does not have the uniform [n, br, bc] form (everything goes element-wise)."""
        data = batch.columns["data"]
        br, bc = self.block_rows, self.block_cols
        if data.dim() != 3 or data.shape[1] != br or data.shape[2] != bc or self.row_offset % br != 0 or \
                self.panel.dim() != 2 or self.panel.stride(1) != 1:
            return None
        dev = self.panel.device
        r = batch.columns["block_row"].to(dev, torch.long) - self.row_offset // br
        c = batch.columns["block_col"].to(dev, torch.long)
        nfr, nfc = self.local_rows // br, self.total_cols // bc
        if r.numel() > 1 and torch.unique(r * max(1, nfc + 1) + c).numel() < r.numel():
            return None      # a block written twice: keep the element-wise path's last-writer-wins order
        full = (r >= 0) & (r < nfr) & (c >= 0) & (c < nfc)
        if nfr > 0 and nfc > 0:
            ld = self.panel.stride(0)
            grid = self.panel.as_strided((nfr, br, nfc, bc), (br * ld, ld, bc, 1))
            sel = full.nonzero().flatten()
            if sel.numel():
                grid[r[sel], :, c[sel], :] = data[sel.to(data.device)].to(dev, self.panel.dtype)
        return (~full).nonzero().flatten().to(batch.columns["block_row"].device)

    def resolve_shared(self):
        """Scatter the linked shared blocks (metadata remapped) into this set's dense panel — the
        HBM-resident form the MFMA kernels read.  Done once per change of the links."""
        if not self.shared_links or not getattr(self, "_shared_dirty", False):
            return self
        for b in self.shared_batches():
            if b.n == 0:
                continue
            keep = b.columns["block_row"] >= 0
            if self.has_data() and self.block_rows:
                r0 = b.columns["block_row"] * self.block_rows
                keep &= (r0 >= self.row_offset) & (r0 < self.row_offset + self.local_rows)
            if not bool(keep.all()):
                b = b.take(keep.nonzero().flatten())
            if b.n:
                self.add_batch(b)
        self._shared_dirty = False
        return self

    def scan(self, device=None) -> Iterator[RecordBatch]:
        """The panel as MatrixBlock records. A replicated panel (every rank holds the whole matrix) yields only this
        rank's share of the blocks on a multi-rank node set, so an SPMD pipeline over it processes each block once
        cluster-wide (and a gathered read returns each block once)."""
        self.resolve_shared()
        if not self.has_data():
            return
        b = self.to_blocks(device)
        ws = getattr(self.manager, "world_size", 1)
        if self.replicated and ws > 1:
            rank = getattr(self.manager, "rank", 0)
            b = b.take(torch.arange(rank, b.n, ws, device=b.columns["block_row"].device))
        yield b

    def num_records(self) -> int:
        self.resolve_shared()
        return self.num_blocks()

    def to_blocks(self, device=None) -> RecordBatch:
        from ..objects.builtin import MatrixBlock

        br, bc = self.block_rows, self.block_cols
        nbr = math.ceil(self.local_rows / br)
        nbc = math.ceil(self.total_cols / bc)
        m = self.matrix()
        pr, pc = nbr * br - self.local_rows, nbc * bc - self.total_cols
        if pr or pc:
            m = torch.nn.functional.pad(m, (0, pc, 0, pr))
        blocks = m.reshape(nbr, br, nbc, bc).permute(0, 2, 1, 3).reshape(nbr * nbc, br, bc)
        if device is not None:
            blocks = blocks.to(device)
        dev = blocks.device
        first_br = self.row_offset // br
        r_idx = torch.arange(nbr, device=dev).repeat_interleave(nbc) + first_br
        c_idx = torch.arange(nbc, device=dev).repeat(nbr)
        n = nbr * nbc
        full = lambda v: torch.full((n,), v, dtype=torch.int64, device=dev)  # noqa: E731
        cols = {"block_row": r_idx, "block_col": c_idx, "row_nums": full(br), "col_nums": full(bc),
                "total_rows": full(self.total_rows), "total_cols": full(self.total_cols), "data": blocks}
        t = self.type if self.type is not None else MatrixBlock
        for f in t.__fields__:
            if f not in cols:
                cols[f] = torch.zeros(n, dtype=torch.int64, device=dev)
        return RecordBatch(cols, n, t)

    def clear(self):
        self.release_storage()
        self.stats = {"records": 0, "bytes": 0}

    def flush(self):
        """Persist the panel (as its MatrixBlock records) through the page pool into the set's page file."""
        if not self.has_data():
            return
        self.persist_pages()
        self.manager.buffer_manager.flush_set(self.set_id)

    def persist_pages(self):
        if not self.has_data():
            return
        b = self.to_blocks("cpu")
        bm = self.manager.buffer_manager
        data = serialize_batch(b)
        page = 0
        # dense images may exceed one pool page: store in page-size chunks
        for s in range(0, len(data), bm.page_size):
            chunk = data[s: s + bm.page_size]
            slot = bm.pin(self.set_id, page, True)
            bm.slot_view(slot)[: len(chunk)] = chunk
            bm.unpin(self.set_id, page, True, len(chunk))
            page += 1
        self.flushed_chunks = page
        t = self._panel
        self._clean_key = (weakref.ref(t), t._version) if t is not None else None

    def geometry(self) -> dict:
        return {"total_rows": self.total_rows, "total_cols": self.total_cols, "block_rows": self.block_rows,
                "block_cols": self.block_cols, "row_offset": self.row_offset, "local_rows": self.local_rows,
                "replicated": self.replicated, "dtype": str(self._dtype()).replace("torch.", ""),
                "chunks": getattr(self, "flushed_chunks", 0)}

    def _dtype(self):
        if self._panel is not None:
            return self._panel.dtype
        return self._shape[2] if self._shape is not None else torch.bfloat16

    def restore(self, geo: dict):
        """Rebuild the panel from the chunks written by :meth:`flush` (checkpoint/resume)."""
        bm = self.manager.buffer_manager
        data = bytearray()
        for page in range(int(geo.get("chunks", 0))):
            slot = bm.pin(self.set_id, page, False)
            n = bm.bytes_used(self.set_id, page)
            data += bytes(bm.slot_view(slot)[:n])
            bm.unpin(self.set_id, page, False, 0)
        if not data:
            return self
        b = deserialize_batch(bytes(data))
        self.define(geo["total_rows"], geo["total_cols"], geo["block_rows"], geo["block_cols"],
                    row_offset=geo["row_offset"], local_rows=geo["local_rows"], dtype=getattr(torch, geo["dtype"]))
        self.replicated = geo.get("replicated", True)
        self.transposed = False          # the persisted blocks are logical: the rebuilt panel is row-major
        self.add_batch(b)
        self.flushed_chunks = int(geo.get("chunks", 0))
        return self


__all__ = ["Page", "UserSet", "DenseMatrixSet"]
