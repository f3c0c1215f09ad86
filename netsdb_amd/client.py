"""PDBClient — the user-facing API (reference: src/mainClient/headers/PDBClient.h,
PDBClientTemplate.cc; CatalogClient, DispatcherClient, DistributedStorageManagerClient,
QueryClient).

netsDB runs a master + worker daemons and the client talks to the master over sockets.  The
MI355X-native deployment is SPMD: one process per GPU launched by torchrun; every process
builds a ``PDBClient`` and calls the API collectively (identical calls on every rank).  Metadata
operations are replicated, data operations act on the rank's partition, and queries run as the
stage pipeline on all ranks with RCCL collectives between them.  For a single process it is
simply an embedded database.  (A socket front end for remote clients lives in
:mod:`netsdb_amd.server`.)
"""
from __future__ import annotations

import os
from typing import Iterable, Iterator, List, Optional, Sequence

import torch

from .execution.engine import QueryEngine
from .objects.record import PDBObject, RecordBatch
from .parallel.comm import ClusterContext
from .parallel.dispatcher import PartitionPolicy, make_policy
from .execution import kernels as K
from .storage.catalog import Catalog
from .storage.manager import DEFAULT_PAGE_SIZE, StorageManager
from .utils.trace import Tracer


class PDBClient:
    def __init__(self, ctx: Optional[ClusterContext] = None, root: Optional[str] = None, device=None,
                 page_size: int = DEFAULT_PAGE_SIZE, pool_pages: int = 16, catalog_path: Optional[str] = None,
                 trace: bool = False, broadcast_threshold: int = 2 << 30, fusion: bool = True,
                 device_budget: Optional[int] = None, resume: bool = False):
        self.ctx = ctx or ClusterContext(device=torch.device(device) if device is not None else torch.device("cpu"))
        dev = device if device is not None else self.ctx.device
        self.device = torch.device(dev)
        self.tracer = Tracer(enabled=trace, rank=self.ctx.rank)
        self.storage = StorageManager(root=root, device=self.device, page_size=page_size, pool_pages=pool_pages,
                                      rank=self.ctx.rank, device_budget=device_budget)
        self.catalog = Catalog(catalog_path or os.path.join(self.storage.root, f"catalog_r{self.ctx.rank}.db"))
        self.engine = QueryEngine(self.storage, self.ctx, self.catalog, self.tracer, broadcast_threshold, fusion)
        self.policies = {}
        self.catalog.register_node(self.ctx.rank, os.environ.get("MASTER_ADDR", "127.0.0.1"), str(self.device),
                                   torch.cuda.get_device_properties(self.device).total_memory
                                   if self.device.type == "cuda" else 0)
        self.learning = None
        if resume:
            self._resume()

    # ------------------------------------------------------------------ checkpoint / resume
    def _resume(self):
        """Re-open every set recorded in the catalog from its page files (after flush_data)."""
        import itertools

        max_id = 0
        for meta in self.catalog.sets():
            max_id = max(max_id, meta["set_id"])
            t = self.catalog.resolve_type(meta["type"]) if meta["type"] else None
            dense = meta["layout"] == "dense"
            s = self.storage.create_set(meta["db"], meta["name"], t, meta["page_size"], dense=dense,
                                        set_id=meta["set_id"])
            m = meta.get("meta") or {}
            if dense and m.get("dense"):
                s.restore(m["dense"])
            elif m.get("pages"):
                s.restore(m["pages"])
        self.storage._ids = itertools.count(max_id + 1)

    # ------------------------------------------------------------------ catalog
    def register_type(self, cls: type) -> bool:
        self.catalog.register_type(cls)
        return True

    registerType = register_type

    def create_database(self, name: str) -> bool:
        return self.catalog.create_database(name)

    createDatabase = create_database

    def remove_database(self, name: str) -> bool:
        self.storage.remove_database(name)
        self.catalog.remove_database(name)
        return True

    removeDatabase = remove_database

    def create_set(self, db: str, name: str, type_=None, page_size: Optional[int] = None, dense: bool = False,
                   policy=None, device="default") -> bool:
        if not self.catalog.has_database(db):
            self.catalog.create_database(db)
        if policy == "auto":
            # Lachesis: ask the self-learning advisor for the partition key of this set
            policy = self.learning.advise(db, name) if self.learning is not None else None
        if type_ is not None:
            self.catalog.register_type(type_)
        sid = self.catalog.create_set(db, name, type_.type_name() if type_ else None, page_size or self.storage.page_size,
                                      "dense" if dense else "pages",
                                      {"policy": getattr(policy, "name", policy) if policy is not None else "roundrobin"})
        self.storage.create_set(db, name, type_, page_size, device=device, dense=dense, set_id=sid)
        if policy is not None:
            self.policies[(db, name)] = make_policy(policy)
        return True

    createSet = create_set

    def remove_set(self, db: str, name: str) -> bool:
        self.storage.remove_set(db, name)
        self.catalog.remove_set(db, name)
        self.policies.pop((db, name), None)
        return True

    removeSet = remove_set

    def clear_set(self, db: str, name: str) -> bool:
        self.storage.clear_set(db, name)
        return True

    clearSet = clear_set

    def get_set(self, db: str, name: str):
        return self.storage.get_set(db, name)

    def list_sets(self, db: Optional[str] = None) -> List[dict]:
        return self.catalog.sets(db)

    def list_nodes(self) -> List[dict]:
        return self.catalog.nodes()

    listNodes = list_nodes

    def print_catalog(self) -> str:
        return self.catalog.print_catalog()

    # ------------------------------------------------------------------ data
    def send_data(self, db: str, name: str, data, policy: Optional[PartitionPolicy] = None, src_rank: int = 0) -> int:
        """Dispatch records from ``src_rank`` to all ranks by the set's partition policy (collective).
        ``data``: list of PDBObjects or a RecordBatch (only read on ``src_rank``)."""
        uset = self.storage.get_set(db, name)
        batch = None
        if self.ctx.rank == src_rank and data is not None:
            batch = data if isinstance(data, RecordBatch) else RecordBatch.from_objects(list(data), uset.type)
        if not self.ctx.distributed:
            if batch is not None:
                uset.add_batch(batch)
            return batch.n if batch is not None else 0
        pol = policy or self.policies.get((db, name)) or make_policy(None)
        ws = self.ctx.world_size
        if batch is not None:
            loads = [0] * ws
            dest = pol.assign(batch, ws, loads).to(torch.int64)
            parts = K.split_by_dest(batch, dest.to(batch.device), ws)
            if self.device.type == "cuda":
                parts = [p.to(self.device) for p in parts]
        else:
            parts = [None] * ws
        got = self.ctx.exchange(parts, template=batch)
        n = 0
        for g in got:
            if g is not None and g.n:
                uset.add_batch(g)
                n += g.n
        return n

    sendData = send_data

    def add_local_data(self, db: str, name: str, data) -> int:
        """Append records to THIS rank's partition (no dispatch)."""
        uset = self.storage.get_set(db, name)
        batch = data if isinstance(data, RecordBatch) else RecordBatch.from_objects(list(data), uset.type)
        uset.add_batch(batch)
        return batch.n

    def get_set_batches(self, db: str, name: str, gather: bool = False) -> List[RecordBatch]:
        uset = self.storage.get_set(db, name)
        local = [b for b in uset.scan()]
        if not gather or not self.ctx.distributed:
            return local
        merged = RecordBatch.concat(local) if local else None
        return [g for g in self.ctx.broadcast_batch_all(merged) if g is not None and g.n]

    def get_set_iterator(self, db: str, name: str, gather: bool = False) -> Iterator[PDBObject]:
        for b in self.get_set_batches(db, name, gather):
            for o in b.to_objects():
                yield o

    getSetIterator = get_set_iterator

    def flush_data(self) -> bool:
        """Persist every set (pages -> native page pool -> page files) and record the layout in the
        catalog so a new PDBClient(root=..., resume=True) can reopen them (checkpoint)."""
        from .storage.sets import DenseMatrixSet

        self.storage.flush()
        for (db, name), s in self.storage.sets.items():
            if not s.persistent or self.catalog.get_set(db, name) is None:
                continue
            meta = dict(self.catalog.get_set(db, name)["meta"])
            if isinstance(s, DenseMatrixSet):
                meta["dense"] = s.geometry()
            else:
                meta["pages"] = s.page_meta()
            self.catalog.update_set_meta(db, name, meta)
        return True

    flushData = flush_data

    # ------------------------------------------------------------------ queries
    def execute_computations(self, *sinks, job_name: str = "job"):
        flat: List = []
        for s in sinks:
            if isinstance(s, (list, tuple)):
                flat.extend(s)
            else:
                flat.append(s)
        return self.engine.execute(flat, job_name)

    def executeComputations(self, *sinks, job_name: str = "job"):
        return self.execute_computations(*sinks, job_name=job_name)

    def explain(self, *sinks) -> str:
        from .logical_plan.tcap import compile_tcap
        from .query_planning.planner import Planner
        from . import _ext

        plan = compile_tcap(list(sinks))
        atoms = _ext.native().parse_tcap(plan.tcap)
        pp = Planner(self.engine._scan_size, self.ctx.world_size, self.engine.broadcast_threshold).plan(atoms)
        return plan.tcap + "\n" + pp.explain()

    # ------------------------------------------------------------------ dedup / shared pages
    def add_shared_mapping(self, db, set_name, shared_db, shared_set, meta=None):
        self.catalog.add_shared_mapping(db, set_name, shared_db, shared_set, meta)
        return True

    addSharedMapping = add_shared_mapping

    def enable_self_learning(self, path: str = ":memory:", learned: bool = False):
        """Record job history and let create_set(..., policy='auto') pick partition keys."""
        from .selflearning import SelfLearningHook

        return SelfLearningHook(self, path, learned)

    def barrier(self):
        self.ctx.barrier()


__all__ = ["PDBClient"]

_ = (Iterable, Sequence)
