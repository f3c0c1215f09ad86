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

import contextlib
import threading

import os
from typing import Iterator, List, Optional

import torch

from .execution.engine import QueryEngine
from .objects.record import PDBObject, RecordBatch
from .parallel.comm import ClusterContext
from .parallel.dispatcher import PartitionPolicy, make_policy
from .execution import kernels as K
from .storage.catalog import Catalog
from .storage.manager import DEFAULT_PAGE_SIZE, StorageManager
from .utils.trace import Tracer


def _placement_of(policy, world_size: int):
    """(key kind, key name, world size) of a key-hash dispatch policy (Lachesis LambdaPolicy built by
    selflearning.key_policy, description 'att:<field>' / 'method:<name>'), else None."""
    desc = getattr(policy, "description", "") or ""
    kind, _, name = desc.partition(":")
    if getattr(policy, "name", None) == "lambda" and kind in ("att", "method") and name:
        return (kind, name, int(world_size))
    return None


class PDBClient:
    def __init__(self, ctx: Optional[ClusterContext] = None, root: Optional[str] = None, device=None,
                 page_size: int = DEFAULT_PAGE_SIZE, pool_pages: int = 16, catalog_path: Optional[str] = None,
                 trace: bool = False, broadcast_threshold: int = 2 << 30, fusion: bool = True,
                 device_budget: Optional[int] = None, resume: bool = False, pinned_budget: Optional[int] = None):
        self.ctx = ctx or ClusterContext(device=torch.device(device) if device is not None else torch.device("cpu"))
        dev = device if device is not None else self.ctx.device
        self.device = torch.device(dev)
        self.tracer = Tracer(enabled=trace, rank=self.ctx.rank)
        self.storage = StorageManager(root=root, device=self.device, page_size=page_size, pool_pages=pool_pages,
                                      rank=self.ctx.rank, device_budget=device_budget, pinned_budget=pinned_budget)
        self.storage.world_size = self.ctx.world_size
        self.catalog = Catalog(catalog_path or os.path.join(self.storage.root, f"catalog_r{self.ctx.rank}.db"))
        self._engine = QueryEngine(self.storage, self.ctx, self.catalog, self.tracer, broadcast_threshold, fusion)
        self._lane = threading.local()    # per-thread job lane (server requests running concurrently)
        self.policies = {}
        self.catalog.register_node(self.ctx.rank, os.environ.get("MASTER_ADDR", "127.0.0.1"), str(self.device),
                                   torch.cuda.get_device_properties(self.device).total_memory
                                   if self.device.type == "cuda" else 0)
        self.learning = None
        self.job_streams = None
        self.job_stream_priority = 0
        self.job_lanes = 2               # job streams (in-order job queues) created on first submit_job
        self.job_lane_priority = {}      # lane -> HIP stream priority (default job_stream_priority)
        if resume:
            self._resume()

    @property
    def engine(self):
        """The query engine of the calling thread's job lane (``job_lane``), else the client's engine."""
        e = getattr(self._lane, "engine", None)
        return e if e is not None else self._engine

    @engine.setter
    def engine(self, e):
        self._engine = e

    @contextlib.contextmanager
    def job_lane(self, lane: int):
        """Run this thread's jobs on lane ``lane``: an engine of its own (same storage / catalog / plan cache and
        configuration) and, on a GPU, a HIP stream of its own (JobStreams lane), so requests touching disjoint
        sets execute concurrently (the reference's QuerySchedulerServer running independent jobs)."""
        prev = getattr(self._lane, "engine", None)
        self._lane.engine = self._engine.clone()
        try:
            if self.device is not None and torch.device(self.device).type == "cuda":
                if self.job_streams is None:
                    from .execution.streams import JobStreams

                    self.job_streams = JobStreams(self.device, lanes=max(self.job_lanes, 4),
                                                  priority=self.job_stream_priority,
                                                  lane_priority=self.job_lane_priority)
                s = self.job_streams.stream(lane)
                s.wait_stream(torch.cuda.current_stream(self.device))
                with torch.cuda.stream(s):
                    yield
                    s.synchronize()
            else:
                yield
        finally:
            self._lane.engine = prev

    @classmethod
    def from_config(cls, conf, **kwargs) -> "PDBClient":
        """A client built from a :class:`~netsdb_amd.utils.config.Configuration` (or a settings-file path);
        keyword arguments override the file."""
        from .utils.config import Configuration

        if isinstance(conf, str):
            conf = Configuration.load(conf)
        kw = conf.client_kwargs()
        kw.setdefault("root", conf.root_directory)
        kw.update(kwargs)
        return cls(**kw)

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
                   policy=None, device="default", locality: Optional[str] = None) -> bool:
        """Create a set. ``locality`` tells the page cache how the set is used (storage/manager.py LOCALITY:
        "model" for weights every step re-reads, "job" (default), "shuffle", "partition", "temp")."""
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
        self.storage.create_set(db, name, type_, page_size, device=device, dense=dense, set_id=sid, locality=locality)
        if policy is not None:
            self.policies[(db, name)] = make_policy(policy)
        return True

    createSet = create_set

    def set_locality(self, db: str, name: str, locality: str):
        """Declare how an existing set is used (see create_set): the cost-based page cache keeps "model" sets
        resident under pressure from one-pass job data."""
        self.storage.set_locality(db, name, locality)

    def set_costs(self, db: str, name: str, write_cost: Optional[float] = None, read_cost: Optional[float] = None):
        """Per-set multipliers of the page cache's eviction write / read costs (LocalitySet::setWriteCost /
        setReadCost, src/storage/headers/LocalitySet.h:122-139)."""
        self.storage.set_costs(db, name, write_cost=write_cost, read_cost=read_cost)

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
        placement = _placement_of(pol, ws)
        if hasattr(uset, "note_placement"):
            uset.note_placement(placement)
        n = 0
        for g in got:
            if g is not None and g.n:
                if hasattr(uset, "note_placement"):
                    uset.add_batch(g, placement=placement)
                else:
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
        self.catalog.checkpoint()
        return True

    flushData = flush_data

    # ------------------------------------------------------------------ queries
    def execute_computations(self, *sinks, job_name: str = "job", pre_compile: bool = False):
        """Run the computation graph ending in ``sinks``. ``pre_compile``: only compile + parse it into the
        engine's pre-compiled workload cache (PDBClient::executeComputations(preCompile=true)); later
        executions of a structurally identical graph skip TCAP compilation and parsing."""
        flat: List = []
        for s in sinks:
            if isinstance(s, (list, tuple)):
                flat.extend(s)
            else:
                flat.append(s)
        return self.engine.execute(flat, job_name, pre_compile=pre_compile)

    def executeComputations(self, *sinks, job_name: str = "job", pre_compile: bool = False):
        return self.execute_computations(*sinks, job_name=job_name, pre_compile=pre_compile)

    def explain(self, *sinks) -> str:
        from .logical_plan.tcap import compile_tcap
        from .query_planning.planner import Planner
        from . import _ext

        plan = compile_tcap(list(sinks))
        atoms = _ext.native().parse_tcap(plan.tcap)
        pp = Planner(self.engine._scan_size, self.ctx.world_size, self.engine.broadcast_threshold,
                     distributed=self.ctx.distributed).plan(atoms)
        return plan.tcap + "\n" + pp.explain()

    # ------------------------------------------------------------------ dedup / shared pages
    def add_shared_page(self, sharing_db: str, sharing_set: str, sharing_type, shared_db: str, shared_set: str,
                        shared_type, page_id: int, partition_id: int = 0, page_seq_id: Optional[int] = None,
                        add_shared_set: bool = False, node_id: int = -1) -> bool:
        """Link page ``page_seq_id`` (default ``page_id``) of the shared set into the sharing set on node
        ``node_id`` (-1: every rank).  PDBClient::addSharedPage; ``add_shared_set`` mirrors
        whetherToAddSharedSet (records the shared set in the catalog on first link)."""
        if node_id >= 0 and node_id != self.ctx.rank:
            return True
        sharing = self.storage.get_set(sharing_db, sharing_set)
        shared = self.storage.get_set(shared_db, shared_set)
        sharing.add_shared_page(shared, int(page_seq_id if page_seq_id is not None else page_id))
        if add_shared_set:
            self.catalog.add_shared_mapping(sharing_db, sharing_set, shared_db, shared_set,
                                            {"kind": "pages", "partition": partition_id})
        return True

    addSharedPage = add_shared_page

    def add_shared_mapping(self, sharing_db: str, sharing_set: str, sharing_type, shared_db: str, shared_set: str,
                           shared_type, file_name: Optional[str] = None, total_rows: int = 0, total_cols: int = 0,
                           transpose: bool = False, mapping: Optional[dict] = None) -> bool:
        """Remap the shared set's blocks (by distinct block id) to their place in the sharing set:
        PDBClient::addSharedMapping -> SharedFFMatrixBlockSet::loadIndexFromFile.  ``file_name``
        holds 'blockKey,blockRow,blockCol' lines; ``mapping`` may give {key: (row, col)} directly."""
        from .models.dedup import TensorBlockIndex

        sharing = self.storage.get_set(sharing_db, sharing_set)
        shared = self.storage.get_set(shared_db, shared_set)
        idx = TensorBlockIndex(0, 0)
        key = TensorBlockIndex.set_key(0, 0, sharing.set_id)
        if file_name is not None:
            idx.load_index_file(key, file_name, total_rows, total_cols, transpose)
        multi = {}
        for k, v in (mapping or {}).items():
            if isinstance(v, list):       # one stored block at several places of the sharing model
                multi[int(k)] = [(c, r, total_rows, total_cols) if transpose else (r, c, total_rows, total_cols)
                                 for r, c in v]
                continue
            r, c = v
            idx.insert_index(key, k, (c, r, total_rows, total_cols) if transpose else (r, c, total_rows, total_cols))
        targets = dict(idx.targets.get(key, {}))
        targets.update(multi)
        sharing.set_shared_mapping(shared, targets)
        if not sharing.link(shared).pages:
            # a mapping alone shares every page of the shared set (the reference links pages first)
            for p in range(max(1, len(shared.pages))):
                sharing.add_shared_page(shared, p)
        self.catalog.add_shared_mapping(sharing_db, sharing_set, shared_db, shared_set,
                                        {"kind": "mapping", "file": file_name, "entries": len(targets),
                                         "total_rows": total_rows, "total_cols": total_cols, "transpose": transpose})
        return True

    addSharedMapping = add_shared_mapping

    # ------------------------------------------------------------------ remaining PDBClient surface
    def create_temp_set(self, db: str, name: str, type_=None, page_size: Optional[int] = None) -> bool:
        """createTempSet: a storage-only set (not in the catalog, never flushed)."""
        self.storage.create_set(db, name, type_, page_size, persistent=False)
        return True

    createTempSet = create_temp_set

    def remove_temp_set(self, db: str, name: str, type_=None) -> bool:
        self.storage.remove_set(db, name)
        return True

    removeTempSet = remove_temp_set

    def remove_hash_set(self, name: str) -> bool:
        """removeHashSet: join/aggregation hash tables live only inside one job here (device tensors
        freed with the job), so there is no persistent hash set to drop."""
        return True

    removeHashSet = remove_hash_set

    def delete_set(self, db: str, name: str) -> bool:
        return self.remove_set(db, name)

    deleteSet = delete_set

    def export_set(self, db: str, name: str, path: str, fmt: str = "csv") -> bool:
        """exportSet: schema line + one value line per object (ExportableObject::toSchemaString /
        toValueString; objects may define ``to_schema_string(fmt)`` / ``to_value_string(fmt)``)."""
        import json as _json

        head = False
        with open(path, "w") as f:
            for b in self.get_set_batches(db, name):
                for o in b.to_objects():
                    fields = list(type(o).fields()) if hasattr(type(o), "fields") else []
                    if not head:
                        hs = o.to_schema_string(fmt) if hasattr(o, "to_schema_string") else \
                            (",".join(fields) + "\n" if fmt == "csv" else "")
                        f.write(hs)
                        head = True
                    if hasattr(o, "to_value_string"):
                        f.write(o.to_value_string(fmt))
                        continue
                    vals = {k: getattr(o, k) for k in fields}
                    vals = {k: (v.tolist() if isinstance(v, torch.Tensor) else v) for k, v in vals.items()}
                    if fmt == "json":
                        f.write(_json.dumps(vals, default=str) + "\n")
                    else:
                        f.write(",".join(str(vals[k]) for k in fields) + "\n")
        return True

    exportSet = export_set

    def register_node(self, address: str, port: int = 0, name: str = "", node_type: str = "worker",
                      status: int = 0) -> bool:
        self.catalog.register_node(self.ctx.rank, f"{address}:{port}", name or node_type, 0)
        return True

    registerNode = register_node

    def register_set(self, set_and_db, policy) -> bool:
        """registerSet(pair(set, db), policy): the dispatcher partition policy of a set."""
        name, db = set_and_db
        self.policies[(db, name)] = make_policy(policy)
        return True

    registerSet = register_set

    def send_bytes(self, set_and_db, data: bytes) -> int:
        """sendBytes: a serialised page image (storage.serde) appended to this rank's partition."""
        from .storage.serde import deserialize_batch

        name, db = set_and_db
        b = deserialize_batch(data)
        self.storage.get_set(db, name).add_batch(b)
        return b.n

    sendBytes = send_bytes

    def list_registered_databases(self) -> str:
        return "\n".join(self.catalog.databases())

    listRegisteredDatabases = list_registered_databases

    def list_registered_sets_for_database(self, db: str) -> str:
        return "\n".join(f"{s['db']}.{s['name']} ({s['type']})" for s in self.catalog.sets(db))

    listRegisteredSetsForADatabase = list_registered_sets_for_database

    def list_nodes_in_cluster(self) -> str:
        return "\n".join(str(n) for n in self.catalog.nodes())

    listNodesInCluster = list_nodes_in_cluster

    def list_user_defined_types(self) -> str:
        return "\n".join(sorted(self.catalog.types()))

    listUserDefinedTypes = list_user_defined_types

    def list_all_registered_metadata(self) -> str:
        return self.catalog.print_catalog()

    listAllRegisteredMetadata = list_all_registered_metadata
    printCatalogMetadata = list_all_registered_metadata

    def enable_self_learning(self, path: str = ":memory:", learned=False):
        """Record job history and let create_set(..., policy='auto') pick partition keys.
        ``learned``: False rule-based, True bandit, "drl" the Q-network agent (selflearning.DRLAdvisor)."""
        from .selflearning import SelfLearningHook

        return SelfLearningHook(self, path, learned)

    def barrier(self):
        self.ctx.barrier()

    # ------------------------------------------------------------------ concurrent jobs
    def capture_job(self, fn, *args, warmup: int = 1, inputs=(), **kwargs):
        """Record ``fn(*args, **kwargs)`` (a job-issuing callable) into a HIP graph and return a
        :class:`~netsdb_amd.execution.graphs.CapturedJob` whose ``replay()`` re-runs its kernels with no host
        work (pre-compiled workloads, taken to the kernel-launch level; see that module for the contract)."""
        from .execution.graphs import CapturedJob

        return CapturedJob(self, fn, *args, warmup=warmup, inputs=inputs, **kwargs)

    def submit_job(self, fn, *args, lane: int = 0, independent: bool = False, **kwargs):
        """Run ``fn(*args, **kwargs)`` (any job-issuing callable, e.g. a model's inference entry point)
        with its kernels enqueued on a job stream, concurrently with work on the caller's stream.
        Returns a :class:`~netsdb_amd.execution.streams.JobHandle`; see that module for the ordering
        contract (QuerySchedulerServer's concurrent job scheduling, on HIP queues)."""
        if self.job_streams is None:
            from .execution.streams import JobStreams

            self.job_streams = JobStreams(self.device, lanes=self.job_lanes, priority=self.job_stream_priority,
                                          lane_priority=self.job_lane_priority)
        return self.job_streams.submit(fn, *args, lane=lane, independent=independent, **kwargs)

    def wait_jobs(self):
        """The caller's stream waits (stream-ordered) for every submitted job."""
        if self.job_streams is not None:
            self.job_streams.wait_all()


__all__ = ["PDBClient"]
