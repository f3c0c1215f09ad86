"""Query execution engine (reference: src/serverFunctionalities/source/{QuerySchedulerServer,
HermesExecutionServer,FrontendQueryTestServer}.cc, src/queryExecution/source/PipelineStage.cc,
src/lambdas/headers/{Pipeline,ComputePlan,TupleSetMachine,*Executor,*Sink}.h).

``execute(sinks)``: computation graph -> (tensor-pattern fusion) -> TCAP -> native parser ->
physical stages -> run every stage on every rank (SPMD).  Each stage streams the pages of its
source through its atoms batch-at-a-time (a batch is a whole page, so each atom is one big
vectorised/GPU op) and ends in a sink.  Collectives (shuffle, broadcast, aggregation exchange)
happen exactly once per sink on every rank, so ranks stay in lock-step.
"""
from __future__ import annotations

import os
import time
from typing import Dict, List, Optional

import torch

from .. import _ext
from ..computations import AggregateComp, Computation, TopKComp
from ..lambdas import Literal, SelfRef
from ..logical_plan.tcap import bind_atoms, compile_tcap, graph_signature
from ..objects.nested import NestedColumn
from ..objects.record import PDBObject, RecordBatch, RecordView, batch_of, column_concat, column_take, LazyTakeColumns
from ..objects.strings import StringColumn
from ..parallel.comm import ClusterContext
from ..storage.sets import DenseMatrixSet
from ..query_planning.planner import AdaptivePlanner, PhysicalPlan, Planner
from ..utils.trace import DeviceTimer, Tracer
from . import kernels as K


class _One:
    """inputs[] shim for a leaf lambda that reads one object column."""

    __slots__ = ("b",)

    def __init__(self, b):
        self.b = b

    def __getitem__(self, i):
        return self.b


def _normalize(val, n: int, device):
    if isinstance(val, SelfRef):
        return val.batch
    if isinstance(val, (RecordBatch, torch.Tensor, tuple, StringColumn, NestedColumn)):
        return val
    if isinstance(val, list):
        if val and isinstance(val[0], PDBObject):
            return RecordBatch.from_objects(val, type(val[0]))
        if val and isinstance(val[0], RecordView):
            return batch_of(val)
        if val and isinstance(val[0], bool):
            return torch.tensor(val, dtype=torch.bool)
        if val and isinstance(val[0], int) and not isinstance(val[0], bool):
            return torch.tensor(val, dtype=torch.int64)
        if val and isinstance(val[0], float):
            return torch.tensor(val, dtype=torch.float64)
        return val
    # scalar literal -> broadcast column
    if isinstance(val, bool):
        return torch.full((n,), val, dtype=torch.bool, device=device)
    if isinstance(val, int):
        return torch.full((n,), val, dtype=torch.int64, device=device)
    if isinstance(val, float):
        return torch.full((n,), val, dtype=torch.float64, device=device)
    return [val] * n


class BuildTable:
    """An in-memory join build side: its tuple set plus a hash table over the join-hash column, built on the
    first probe and reused by every later probe batch (device table on the GPU, kernels.JoinTable)."""

    def __init__(self, batch: Optional[RecordBatch], hash_col: str):
        self.batch = batch
        self.hash_col = hash_col
        self.h = batch.columns[hash_col] if batch is not None and batch.n else torch.empty(0, dtype=torch.int64)
        self._table = None

    def table(self, device) -> "K.JoinTable":
        if self._table is None:
            self._table = K.JoinTable(self.h.to(device))
        return self._table


class PartitionedBuild:
    """An out-of-core join build side: hash partitions in spillable spools (PartitionedHashSet)."""

    def __init__(self, parts, hash_col: str):
        self.parts = parts
        self.hash_col = hash_col


# NSDB_STAGE_SYNC=1: every stage is bracketed by device syncs and logged here (scripts/bench_tpch.py --stage-times)
STAGE_SYNC = bool(int(__import__("os").environ.get("NSDB_STAGE_SYNC", "0") or 0))
STAGE_LOG: List[dict] = []


class JobStats(dict):
    """Per-job statistics. On a GPU each stage record carries ``device_seconds``: the stage's time on the device
    stream from a HIP event pair (utils/trace.DeviceTimer), None until resolved — :meth:`device_times` resolves
    them (``block=False``: only pairs that already completed; the engine also resolves completed pairs at the start
    of every later job), with no synchronisation inside the job."""

    def device_times(self, block: bool = True) -> list:
        timer = getattr(self, "_timer", None)
        if timer is not None:
            timer.resolve(block)
        return [st.get("device_seconds") for st in self.get("stages", [])]


class QueryEngine:
    def __init__(self, storage, ctx: Optional[ClusterContext] = None, catalog=None, tracer: Optional[Tracer] = None,
                 broadcast_threshold: int = 2 << 30, fusion: bool = True):
        self.storage = storage
        self.ctx = ctx or ClusterContext()
        self.catalog = catalog
        self.tracer = tracer or Tracer(enabled=False)
        # per-stage device time from HIP event pairs (JobStats.device_times); no synchronisation inside a job
        self.device_timing = True
        self.device_timer = DeviceTimer()
        self.broadcast_threshold = broadcast_threshold
        self.fusion = fusion
        self.last_plan = None
        self.adaptive = True              # statistics-driven stage selection (AdaptivePlanner)
        self.plan_cache_enabled = True
        self._plan_cache = {}
        self.cache_stats = {"tcap_compiles": 0, "tcap_cache_hits": 0}
        self.ooc_stats = {}
        self.shuffle_count = 0            # all-to-all repartitions of join inputs (per job: stats["shuffles"])
        self._copart = set()
        self.ooc_fraction = 0.25          # of the device budget: in-memory build / group-by / tuple-set limit
        self._spools = []
        # streaming shuffle (execution/shuffle.py): chunk size per round and cumulative round statistics
        self.shuffle_chunk_bytes = 64 << 20
        self.shuffle_stats = {}
        # in-kernel operand prefetch: the weight of such a later GEMM is read into the Infinity Cache by the
        # workgroups of the long GEMM before it as they finish (ops.gemm_nt / gemm.hip GemmParams::pf_ptr)
        self.operand_prefetch = True
        self.last_tcap = None
        self._last_comps = None
        # fused filter -> project -> aggregate stages (execution/pipeline.py, csrc/kernels/pipeline.hip)
        self.fused_pipelines = True
        # [filter ->] join probe runs outside aggregation stages as one compiled launch emitting (probe, build) rows
        self.fused_probes = os.environ.get("NSDB_FUSED_PROBES", "1") != "0"
        self.pipeline_stats = {"fused_stages": 0, "fused_batches": 0, "fallback_batches": 0}

    def clone(self) -> "QueryEngine":
        """An engine for another job lane: same storage, context, catalog, tracer, configuration and plan cache
        (dict access under the GIL); its own per-job state (spools, statistics)."""
        e = QueryEngine(self.storage, self.ctx, self.catalog, self.tracer, self.broadcast_threshold, self.fusion)
        for k in ("adaptive", "plan_cache_enabled", "ooc_fraction", "shuffle_chunk_bytes",
                  "operand_prefetch", "fused_pipelines", "fused_probes", "device_timing"):
            setattr(e, k, getattr(self, k))
        e._plan_cache = self._plan_cache
        e.__dict__["meta_cache"] = self.__dict__.setdefault("meta_cache", {})
        return e

    # ------------------------------------------------------------------ entry
    def _compile(self, sinks, job_name, stats):
        """TCAP for the graph: from the pre-compiled workload cache when a structurally identical graph
        ran (or was pre-compiled) before — no TCAP emission, no parse — else compile + native parse.  Also returns
        the graph key (signature + lambda constants) later per-graph caches use, or None."""
        sig, comps, sets = (None, None, None)
        gkey = None
        if self.plan_cache_enabled:
            vals: list = []
            try:
                sig, comps, sets = graph_signature(sinks, vals)
                gkey = (sig, tuple(vals))
                hash(gkey)
            except Exception:          # a graph the signature walk cannot key: always compile
                sig = gkey = None
        hit = self._plan_cache.get(sig) if sig is not None else None
        if hit is not None:
            self.cache_stats["tcap_cache_hits"] += 1
            stats["tcap_cached"] = True
            tcap, atoms = hit
            return bind_atoms(atoms, sets), comps, tcap, gkey
        plan = compile_tcap(sinks)
        with self.tracer.span("parse_tcap", job=job_name):
            atoms = _ext.native().parse_tcap(plan.tcap)
        self.cache_stats["tcap_compiles"] += 1
        stats["tcap_cached"] = False
        if sig is not None:
            self._plan_cache[sig] = (plan.tcap, atoms)
            while len(self._plan_cache) > 256:
                self._plan_cache.pop(next(iter(self._plan_cache)))
        return atoms, plan.computations, plan.tcap, gkey

    def _capturing(self) -> bool:
        """A HIP-graph capture is recording on this thread's stream (event queries / timing records must wait)."""
        return self.ctx.device.type == "cuda" and torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()

    def _device_timed(self) -> bool:
        """Stage device timing on: a GPU engine outside a HIP-graph capture (a captured job replays no host code)."""
        return self.device_timing and self.ctx.device.type == "cuda" and torch.cuda.is_available() and \
            not self._capturing()

    def _timed_stage(self, st, state, stats, job_name):
        sync = STAGE_SYNC and torch.cuda.is_available()
        if sync:   # profiling: device time per stage (serialises the stream at stage boundaries)
            torch.cuda.synchronize()
        dev_t = self._device_timed()
        ev0 = self.device_timer.start() if dev_t else None
        ts = time.perf_counter()
        with self.tracer.span(f"stage{st.id}", job=job_name, sink=st.sink.get("kind")):
            n = self._run_stage(st, state)
        if sync:
            torch.cuda.synchronize()
        rec = {"id": st.id, "desc": st.describe(), "rows_in": n, "seconds": time.perf_counter() - ts}
        if ev0 is not None:
            self.device_timer.stop(ev0, rec, "device_seconds")
        stats["stages"].append(rec)
        if sync:
            STAGE_LOG.append(dict(rec, job=job_name))
        return n

    def _run_adaptive(self, atoms, state, stats, job_name):
        """Stage-at-a-time execution driven by measured statistics (AdaptivePlanner): each finished
        stage's materialised output is measured (bytes, summed over ranks so every rank takes the same
        decisions) and costed for the next source selection."""
        ap = AdaptivePlanner(atoms, self._scan_size, self.ctx.world_size, self.broadcast_threshold, self._copart,
                             distributed=self.ctx.distributed)
        stages = []
        while ap.has_work():
            st = ap.next_stage()
            if st is None:
                break
            self._timed_stage(st, state, stats, job_name)
            stages.append(st)
            measured = None
            sk = st.sink.get("kind")
            if sk in ("materialize", "aggregate", "partition"):
                out = st.sink["ts"] if sk == "materialize" else st.sink["atom"]["output"]["name"]
                m = state.materialized.get(out, [])
                measured = m.bytes if hasattr(m, "bytes") else sum(b.nbytes() for b in m if b is not None)
                if self.ctx.distributed:
                    measured = int(self.ctx.all_reduce_scalar(float(measured), "sum"))
                stats.setdefault("measured_bytes", {})[out] = measured
            ap.complete(st, measured)
        if ap.decisions:
            stats["join_decisions"] = ap.decisions
        return PhysicalPlan(stages, atoms, {d["join"]: d for d in ap.decisions})

    def execute(self, sinks: List[Computation], job_name: str = "job", pre_compile: bool = False) -> JobStats:
        t0 = time.perf_counter()
        stats = JobStats(job=job_name, stages=[])
        stats._timer = self.device_timer
        if self.device_timer.pending and not self._capturing():
            self.device_timer.resolve(block=False)      # earlier jobs' stage times whose events have completed
        sinks = list(sinks)
        if self.fusion and not pre_compile:       # (fusion executes the matched kernels: not on pre-compile)
            from ..query_planning.fusion import fuse_tensor_patterns

            ooc0 = dict(self.ooc_stats)
            sinks, fused = fuse_tensor_patterns(sinks, self)
            stats["fused_ops"] = fused
            ooc = {k: v - ooc0.get(k, 0) for k, v in self.ooc_stats.items() if v - ooc0.get(k, 0)}
            if ooc:
                stats["out_of_core"] = ooc
            if not sinks:
                stats["seconds"] = time.perf_counter() - t0
                self.last_plan = self.last_tcap = self._last_comps = None
                return stats
        atoms, comps, tcap, gkey = self._compile(sinks, job_name, stats)
        self.last_tcap = tcap
        self._last_comps = comps
        if pre_compile:
            stats["pre_compiled"] = True
            stats["seconds"] = time.perf_counter() - t0
            return stats
        state = _JobState(comps)
        state.graph_key = gkey
        ooc0 = dict(self.ooc_stats)
        self._copart = self._copartitioned_joins(atoms, comps) if self.ctx.distributed else set()
        if self._copart:
            stats["copartitioned_joins"] = sorted(self._copart)
        shuffles0 = self.shuffle_count
        try:
            if self.adaptive:
                pplan = self._run_adaptive(atoms, state, stats, job_name)
            else:
                planner = Planner(self._scan_size, self.ctx.world_size, self.broadcast_threshold, self._copart,
                                      distributed=self.ctx.distributed)
                pplan = planner.plan(atoms)
                for st in pplan.stages:
                    self._timed_stage(st, state, stats, job_name)
            self.last_plan = pplan
        finally:
            for sp in self._spools:        # job-scoped spills (builds, spooled tuple sets) end with the job
                sp.drop()
            self._spools = []
        ooc = {k: v - ooc0.get(k, 0) for k, v in self.ooc_stats.items() if v - ooc0.get(k, 0)}
        if ooc:
            stats["out_of_core"] = dict(stats.get("out_of_core", {}), **ooc)
        stats["seconds"] = time.perf_counter() - t0
        stats["tcap_atoms"] = len(atoms)
        stats["shuffles"] = self.shuffle_count - shuffles0
        return stats

    def _copartitioned_joins(self, atoms, comps) -> set:
        """Joins whose two inputs are scans of sets already hash-placed by exactly the join key of their
        side (Lachesis placement, ``UserSet.placement``) with this world size: the hash atom's key lambda
        reads a field / method of the scanned object itself and the dispatcher hashed the same column
        with the same function, so matching rows already share a rank.  The decision is agreed over all
        ranks (min of the local flags) because a set's placement is tracked per rank."""
        from ..selflearning import _key_of, _producer_map, _source_scan

        by_out = _producer_map(atoms)
        cands = []
        for a in atoms:
            if a["type"] != "JOIN":
                continue
            ok = True
            for key in ("input", "input2"):
                h = by_out.get(a[key]["name"])
                if h is None or h["type"] not in ("HASHLEFT", "HASHRIGHT") or len(h["input"]["atts"]) != 1:
                    ok = False
                    break
                scan = _source_scan(by_out, h["input"]["name"])
                comp = comps.get(h["comp"])
                k = _key_of(comp, by_out, h["input"]["name"], h["input"]["atts"][0], scan) if (scan and comp) else None
                try:
                    s = self.storage.get_set(scan["db"], scan["set"]) if scan else None
                except KeyError:
                    s = None
                pl = getattr(s, "placement", None)
                if k is None or k[0] not in ("att", "method") or pl is None or \
                        (pl[0], pl[1], pl[2]) != (k[0], k[1], self.ctx.world_size):
                    ok = False
                    break
            cands.append((a["output"]["name"], ok))
        if not cands:
            return set()
        flags = [self.ctx.all_reduce_scalar(1.0 if ok else 0.0, "min") for _, ok in cands]
        return {name for (name, _), f in zip(cands, flags) if f > 0.5}

    def _scan_size(self, atom) -> int:
        try:
            s = self.storage.get_set(atom["db"], atom["set"])
        except KeyError:
            return 0
        return int(self.ctx.all_reduce_scalar(float(s.nbytes()), "sum")) if self.ctx.distributed else s.nbytes()

    # ------------------------------------------------------------------ stages
    def _source_batches(self, st, state):
        src = st.source
        if src["kind"] == "scan":
            a = src["atom"]
            s = self.storage.get_set(a["db"], a["set"])
            col = a["output"]["atts"][0]
            for b in s.scan():
                yield RecordBatch({col: b}, b.n)
        else:
            for b in state.materialized.get(src["ts"], []):
                yield b

    def _ooc_limit(self) -> int:
        """Bytes an in-memory join build / group-by / materialised tuple set may take before it is
        hash-partitioned into spillable spools (a fraction of the node's device budget)."""
        return max(1 << 14, int(self.storage.device_budget * self.ooc_fraction))

    def _run_stage(self, st, state) -> int:
        # split ops at partitioned-join probes (inputs shuffled collectively first) and at probes of
        # out-of-core (partitioned) builds (probe side hash-partitioned into spools, Grace join)
        segments: List[List[dict]] = [[]]
        for o in st.ops:
            if o["type"] == "JOIN" and (o.get("_strategy") == "partitioned" or
                                        isinstance(state.builds.get(o["output"]["name"]), PartitionedBuild)):
                segments.append([o])
            else:
                segments[-1].append(o)
        rows = [0]
        # a stage ending in an aggregation whose trailing atoms are lambda trees runs them as ONE fused launch per
        # batch (filter -> key / value row -> per-workgroup pre-aggregation); the atoms before them run as usual
        fplan = None
        if self.fused_pipelines and st.sink.get("kind") == "aggregate":
            from . import pipeline as PL

            fplan = PL.plan_stage(segments[-1], state.comps, st.sink["atom"], state.graph_key)
            if fplan is not None:
                fplan.builds = state.builds          # a fused join probe reads its build table from the job state
                if fplan.alt is not None:
                    fplan.alt.builds = state.builds
                segments[-1] = fplan.prefix
                # one rank: the launches' few pre-aggregated rows stay on the host, the sink reduces them there
                # and its result goes back to the device in one asynchronous upload (no device round trips)
                fplan.host_out = not self.ctx.distributed
                if fplan.alt is not None:
                    fplan.alt.host_out = fplan.host_out

        def source():
            for b in self._source_batches(st, state):
                rows[0] += b.n
                yield b

        it = source()
        for si, seg in enumerate(segments):
            ops = seg
            if si > 0:
                probe = seg[0]
                hcol = probe["input"]["atts"][0] if probe["_probe_side"] == "left" else probe["input2"]["atts"][0]
                if probe.get("_strategy") == "partitioned":
                    # streaming repartition of the probe side by its join hash: chunks leave while the
                    # source pipeline still runs, received batches flow into the probe
                    it = self._stream_shuffle(it, hcol, "probe")
                pb = state.builds.get(probe["output"]["name"])
                if isinstance(pb, PartitionedBuild):
                    it = self._grace_probe(probe, it, pb, hcol, state)
                    ops = seg[1:]
            it = self._apply_ops(ops, it, state)
        if fplan is not None:
            it = self._fused_stream(fplan, it, state)
        self._sink(st, it, state)
        return rows[0]

    def _fused_stream(self, fplan, it, state):
        """Batches through a fused stage suffix: one pipeline launch each (pre-aggregated key / value batch out), or
        the suffix's atoms eagerly for a batch the kernel does not take."""
        from . import pipeline as PL

        used = False
        for b in it:
            if b is None or b.n == 0:
                continue
            r = PL.run_batch(fplan, b)
            if r is None and fplan.alt is not None and fplan.disabled:
                # the fused probe could not run (no compiled kernel, an out-of-core build, ...): the atoms up to the
                # alternative plan's suffix eagerly (the probe among them), then that plan's fused launch
                alt = fplan.alt
                head = fplan.suffix[: len(fplan.suffix) - len(alt.suffix)]
                for o in head:
                    if b.n == 0 and o["type"] != "JOIN":
                        break
                    b = self._apply_atom(o, b, state)
                if b.n == 0:
                    continue
                r = PL.run_batch(alt, b)
                if r is None:
                    self.pipeline_stats["fallback_batches"] += 1
                    for o in alt.suffix:
                        if b.n == 0:
                            break
                        b = self._apply_atom(o, b, state)
                    yield b
                    continue
            if r is not None and getattr(r, "emitted", False):
                # the stage's emitted (key parts, values) rows: device columns, reduced by the sink's group-by
                if fplan.join is not None:
                    self.pipeline_stats["fused_join_batches"] = self.pipeline_stats.get("fused_join_batches", 0) + 1
                self.pipeline_stats["emitted_batches"] = self.pipeline_stats.get("emitted_batches", 0) + 1
                used = True
                self.pipeline_stats["fused_batches"] += 1
                yield r
                continue
            if r is not None:
                if fplan.join is not None and not fplan.disabled:
                    self.pipeline_stats["fused_join_batches"] = self.pipeline_stats.get("fused_join_batches", 0) + 1
                if getattr(fplan, "host_out", False) and b.device.type == "cuda":
                    state.fused_out_device = b.device
                state.unique_kv.append(r.columns[fplan.kcol])   # one row per key (the kernel's global table)
                used = True
                self.pipeline_stats["fused_batches"] += 1
                yield r
                continue
            self.pipeline_stats["fallback_batches"] += 1
            for o in fplan.suffix:
                if b.n == 0:
                    break
                b = self._apply_atom(o, b, state)
            yield b
        if used:
            self.pipeline_stats["fused_stages"] += 1

    def _apply_ops(self, ops, it, state):
        """Stream batches through a segment's atoms (generator: one page in flight per stage). Runs of lambda-tree
        APPLYs ending in their FILTER execute as one fused predicate launch (execution/pipeline.py)."""
        if self.fused_pipelines and any(o["type"] in ("FILTER", "JOIN") for o in ops):
            from . import pipeline as PL

            ops = PL.fuse_filters(ops, state.comps)
            if self.fused_probes:
                ops = PL.fuse_probes(ops)
        for b in it:
            for o in ops:
                if b.n == 0 and o["type"] != "JOIN":
                    break
                b = self._apply_atom(o, b, state)
            yield b

    def _grace_probe(self, a, it, pb: "PartitionedBuild", hcol: str, state):
        """Out-of-core hash join (PartitionedHashSet): the probe side is hash-partitioned into spools with
        the build side's partition function, then each partition's build table is built alone and probed."""
        from .spool import PartitionedSpool

        name = a["output"]["name"]
        probe_parts = PartitionedSpool(self.storage, pb.parts.nparts, "probe")
        try:
            for b in it:
                if b.n:
                    probe_parts.add(b, b.columns[hcol])
            self.ooc_stats["grace_joins"] = self.ooc_stats.get("grace_joins", 0) + 1
            for p in range(pb.parts.nparts):
                if probe_parts.parts[p].n == 0 or pb.parts.parts[p].n == 0:
                    continue
                state.builds[name] = BuildTable(pb.parts.parts[p].concat(), pb.hash_col)
                self.ooc_stats["grace_partitions"] = self.ooc_stats.get("grace_partitions", 0) + 1
                for b in probe_parts.parts[p]:
                    yield self._probe(a, b, state)
                state.builds[name] = pb
        finally:
            state.builds[name] = pb
            probe_parts.drop()

    def _stream_shuffle(self, batches, hcol: Optional[str], tag: str, combine=None, key=None):
        """Hash-shuffle a batch stream across ranks in chunk rounds (StreamingShuffle); yields received batches."""
        from .shuffle import shuffle_stream

        if not self.ctx.distributed:
            yield from (b for b in batches if b is not None and b.n)
            return
        if tag in ("probe", "build"):
            self.shuffle_count += 1         # repartitions of join inputs (JobStats["shuffles"])
        keyf = key if key is not None else (lambda b: b.columns[hcol])
        st = {}
        try:
            yield from shuffle_stream(self.ctx, batches, keyf, self.shuffle_chunk_bytes, stats=st, combine=combine)
        finally:
            st["shuffles"] = 1
            for k, v in st.items():
                self.shuffle_stats[k] = self.shuffle_stats.get(k, 0) + v
            self.shuffle_stats.setdefault("by_tag", {})
            self.shuffle_stats["by_tag"][tag] = self.shuffle_stats["by_tag"].get(tag, 0) + 1

    def _shuffle_by(self, batches: List[RecordBatch], hcol: str) -> List[RecordBatch]:
        ws = self.ctx.world_size
        if not self.ctx.distributed:
            return batches
        self.shuffle_count += 1
        merged = RecordBatch.concat(batches) if batches else None
        if merged is None:
            parts = [None] * ws
        else:
            dest = K.partition_of(merged.columns[hcol], ws)
            parts = K.split_by_dest(merged, dest, ws)
        return [b for b in self.ctx.exchange(parts) if b is not None]

    # ------------------------------------------------------------------ atoms
    def _apply_atom(self, a: dict, b: RecordBatch, state) -> RecordBatch:
        t = a["type"]
        comp = state.comps.get(a.get("comp"))
        if t == "APPLY":
            args = a["input"]["atts"]
            carry = a["projection"]["atts"]
            out_col = a["output"]["atts"][-1]
            lname = a["lambda"]
            if lname.startswith("self_in"):
                val = b.columns[args[0]]
            else:
                node = comp.extract_lambdas()[lname]
                if node.children:
                    val = node.eval_node(None, [b.columns[x] for x in args])
                elif isinstance(node, Literal):
                    val = node.value
                else:
                    val = node.eval_node(_One(b.columns[args[0]]), [])
            val = _normalize(val, b.n, b.device)
            cols = {c: b.columns[c] for c in carry}
            cols[out_col] = val
            return RecordBatch(cols, b.n)
        if t == "FILTER":
            mask = b.columns[a["input"]["atts"][0]]
            if not isinstance(mask, torch.Tensor):
                mask = torch.tensor([bool(x) for x in mask], dtype=torch.bool)
            idx = K.selected_rows(mask.bool())
            keep = RecordBatch({c: b.columns[c] for c in a["projection"]["atts"]}, b.n)
            return keep.take(idx)
        if t in ("HASHLEFT", "HASHRIGHT"):
            keys = [b.columns[c] for c in a["input"]["atts"]]
            h = K.hash_keys(keys[0] if len(keys) == 1 else tuple(keys), b.device)
            cols = {c: b.columns[c] for c in a["projection"]["atts"]}
            cols[a["output"]["atts"][-1]] = h
            return RecordBatch(cols, b.n)
        if t == "HASHONE":
            cols = {c: b.columns[c] for c in a["projection"]["atts"]}
            cols[a["output"]["atts"][-1]] = torch.zeros(b.n, dtype=torch.int64, device=b.device)
            return RecordBatch(cols, b.n)
        if t == "FLATTEN":
            vcol = b.columns[a["input"]["atts"][0]]
            carry = a["projection"]["atts"]
            if isinstance(vcol, NestedColumn):
                # device FLATTEN: the element column as rows, carried columns gathered by parent index
                vals, parent = vcol.flatten()
                cols = {c: column_take(b.columns[c], parent) for c in carry}
                cols[a["output"]["atts"][-1]] = vals
                return RecordBatch(cols, int(parent.numel()))
            lens, flat = [], []
            for v in (vcol if not isinstance(vcol, RecordBatch) else [vcol]):
                items = list(v) if not isinstance(v, RecordBatch) else [RecordView(v, i) for i in range(v.n)]
                lens.append(len(items))
                flat.extend(items)
            rep = torch.repeat_interleave(torch.arange(len(lens)), torch.tensor(lens, dtype=torch.int64)) \
                if lens else torch.empty(0, dtype=torch.int64)
            cols = {c: RecordBatch({c: b.columns[c]}, b.n).take(rep).columns[c] for c in carry}
            out_col = a["output"]["atts"][-1]
            cols[out_col] = _normalize(flat, len(flat), b.device) if flat else []
            return RecordBatch(cols, len(flat))
        if t == "JOIN":
            return self._probe(a, b, state)
        if t == "FUSED_PROBE":
            from . import pipeline as PL

            plan = a["plan"]
            plan.builds = state.builds
            r = PL.run_probe(plan, b)
            if r is not None:
                self.pipeline_stats["fused_probes"] = self.pipeline_stats.get("fused_probes", 0) + 1
                return self._join_output(a["join"], b, r[0], r[1], state.builds[a["join"]["output"]["name"]])
            for o in a["atoms"]:
                if b.n == 0 and o["type"] != "JOIN":
                    break
                b = self._apply_atom(o, b, state)
            return b
        if t == "FUSED_FILTER":
            from . import pipeline as PL

            r = PL.run_filter(a["plan"], b)
            if r is not None:
                self.pipeline_stats["fused_filters"] = self.pipeline_stats.get("fused_filters", 0) + 1
                return r
            for o in a["atoms"]:
                if b.n == 0:
                    break
                b = self._apply_atom(o, b, state)
            return b
        raise ValueError(f"atom {t} is not streaming")

    def _probe(self, a, b: RecordBatch, state) -> RecordBatch:
        bt: BuildTable = state.builds[a["output"]["name"]]
        side = a["_probe_side"]
        lh, rh = a["input"]["atts"][0], a["input2"]["atts"][0]
        lcols, rcols = a["projection"]["atts"], a["projection2"]["atts"]
        probe_h = b.columns[lh if side == "left" else rh]
        if bt.batch is None or bt.batch.n == 0 or b.n == 0:
            bi = pi = torch.empty(0, dtype=torch.int64, device=b.device)
        else:
            bi, pi = bt.table(probe_h.device).probe(probe_h)
        return self._join_output(a, b, pi, bi, bt)

    def _join_output(self, a, b: RecordBatch, pi, bi, bt: "BuildTable") -> RecordBatch:
        """The JOIN's output batch: its probe-side projection at probe rows ``pi`` of ``b`` next to its build-side
        projection at build rows ``bi`` (row selections; columns materialise lazily)."""
        side = a["_probe_side"]
        lcols, rcols = a["projection"]["atts"], a["projection2"]["atts"]
        pb = RecordBatch({c: b.columns[c] for c in (lcols if side == "left" else rcols)}, b.n).take(pi)
        if bt.batch is None:
            bb_cols = {c: [] for c in (rcols if side == "left" else lcols)}
            bbat = RecordBatch(bb_cols, 0)
        else:
            bbat = RecordBatch({c: bt.batch.columns[c] for c in (rcols if side == "left" else lcols)}, bt.batch.n).take(bi)
        left, right = (pb, bbat) if side == "left" else (bbat, pb)
        if isinstance(pb.columns, LazyTakeColumns) or isinstance(bbat.columns, LazyTakeColumns):
            # both sides stay row selections: a column is gathered when a later atom or sink reads it (a materialised
            # join output used for one key and two fields gathers those three, not every projected column)
            return RecordBatch(LazyTakeColumns.merged([(left, lcols), (right, rcols)]), int(pi.numel()))
        cols = {}
        for c in lcols:
            cols[c] = left.columns[c]
        for c in rcols:
            cols[c] = right.columns[c]
        return RecordBatch(cols, int(pi.numel()))

    # ------------------------------------------------------------------ sinks
    def _sink(self, st, batches, state):
        sk = st.sink
        kind = sk["kind"]
        if kind == "discard":
            for _ in batches:
                pass
            return
        if kind == "materialize":
            state.materialized[sk["ts"]] = self._collect(batches, "mat")
            return
        if kind == "output":
            a = sk["atom"]
            col = a["input"]["atts"][0]
            uset = self.storage.get_set(a["db"], a["set"])
            dense = isinstance(uset, DenseMatrixSet)
            written = []        # (block_row, block_col) this rank wrote into a dense set
            for x in batches:
                if x is None or x.n == 0:
                    continue
                v = x.columns[col]
                if not isinstance(v, RecordBatch):
                    v = RecordBatch({"value": v}, x.n)
                uset.add_batch(v)
                if dense and "block_row" in v.columns:
                    written.append((v.columns["block_row"], v.columns["block_col"]))
            if self.ctx.distributed and dense:
                self._merge_dense_output(uset, written)
            return
        if kind == "join_build":
            a = sk["atom"]
            side = sk["side"]
            hcol = a["input"]["atts"][0] if side == "left" else a["input2"]["atts"][0]
            cols = (a["projection"]["atts"] if side == "left" else a["projection2"]["atts"]) + [hcol]
            parts = (RecordBatch({c: x.columns[c] for c in cols}, x.n) for x in batches if x is not None and x.n)
            strat = sk["strategy"]
            name = a["output"]["name"]
            if self.ctx.distributed and strat == "broadcast":
                parts = list(parts)
                local = RecordBatch.concat(parts) if parts else None
                got = self.ctx.broadcast_batch_all(local)
                parts = iter([g for g in got if g is not None and g.n])
            elif self.ctx.distributed and strat == "partitioned":
                # streaming shuffle straight into the (spillable) build table
                parts = self._stream_shuffle(parts, hcol, "build")
            state.builds[name] = self._build_table(parts, hcol, st)
            return
        if kind == "aggregate":
            self._aggregate(sk["atom"], batches, state)
            return
        if kind == "partition":
            self._partition(sk["atom"], batches, state)
            return
        raise ValueError(kind)

    _DTYPES = (torch.float32, torch.bfloat16, torch.float16, torch.float64)
    MERGE_BAND_BYTES = 64 << 20        # _merge_dense_output: bytes of one band's contribution buffer

    def _merge_dense_output(self, s, written=()):
        """A dense matrix written block by block by an SPMD pipeline: every rank wrote the blocks it produced. Agree
        on the geometry, then merge by block OWNERSHIP: each block takes the value of the rank(s) that wrote it in
        this job (averaged when several ranks emitted the same block), every other block keeps the panel's previous
        value. A rerun into the same set, or a panel that already held a replicated matrix, is therefore not summed
        across ranks. Afterwards every rank holds the whole matrix (replicated), as a fused GEMM's output would."""
        geo = [0] * 5
        if s.has_data():
            dt = s.panel.dtype
            geo = [s.total_rows, s.total_cols, s.block_rows, s.block_cols,
                   self._DTYPES.index(dt) + 1 if dt in self._DTYPES else 1]
        rows = self.ctx.all_gather_ints(geo)
        ref = next((r for r in rows if r[0] > 0), None)
        if ref is None:
            return
        if not s.has_data():
            s.define(ref[0], ref[1], ref[2], ref[3], dtype=self._DTYPES[ref[4] - 1])
        panel = s.panel
        if s.row_offset != 0 or s.local_rows != ref[0]:
            raise RuntimeError(f"dense output {s.db}.{s.name}: a row-partitioned panel cannot be merged")
        tr, tc, br, bc = ref[0], ref[1], ref[2], ref[3]
        nbr, nbc = -(-tr // br), -(-tc // bc)
        dev = panel.device
        mask = torch.zeros(nbr, nbc, dtype=torch.float32, device=dev)
        for r, c in written:
            r = torch.as_tensor(r, device=dev).long()
            c = torch.as_tensor(c, device=dev).long()
            ok = (r >= 0) & (r < nbr) & (c >= 0) & (c < nbc)
            mask[r[ok], c[ok]] = 1.0
        cnt = mask.clone()
        self.ctx.all_reduce(cnt)
        view = s.matrix()                                 # logical [rows, cols] (a transposed view if need be)
        # the masked all-reduce runs in the panel's own precision (float64 panels stay float64; bf16 / fp16 panels
        # combine in f32 and round once), band by band of whole block rows (<= MERGE_BAND_BYTES per band, the same
        # bands on every rank), so no full-size [rows, cols] mask / contribution / count temporaries are built
        acc_dt = torch.float64 if view.dtype == torch.float64 else torch.float32
        esz = torch.tensor([], dtype=acc_dt).element_size()
        band_blocks = max(1, self.MERGE_BAND_BYTES // max(1, br * tc * esz))
        for b0 in range(0, nbr, band_blocks):
            b1 = min(nbr, b0 + band_blocks)
            r0, r1 = b0 * br, min(tr, b1 * br)
            rows_of = lambda m: m[b0:b1].repeat_interleave(br, 0)[: r1 - r0].repeat_interleave(bc, 1)[:, :tc]  # noqa: E731
            band = view[r0:r1]
            mine = rows_of(mask) > 0
            contrib = torch.where(mine, band.to(acc_dt), torch.zeros((), dtype=acc_dt, device=dev))
            self.ctx.all_reduce(contrib)
            c_el = rows_of(cnt).to(acc_dt)
            band.copy_(torch.where(c_el > 0, contrib / c_el.clamp(min=1.0), band.to(acc_dt)).to(view.dtype))
        s.replicated = True

    def _collect(self, batches, tag: str):
        """Keep a tuple set in memory while it is small; past the out-of-core limit continue it in a
        spillable spool (pages charged to the budget, LRU-spilled, re-read page by page)."""
        from .spool import Spool

        limit = self._ooc_limit()
        held, size, spool = [], 0, None
        for b in batches:
            if b is None:
                continue
            if spool is not None:
                spool.add(b)
                continue
            held.append(b)
            size += b.nbytes()
            if size > limit:
                spool = Spool(self.storage, tag)
                for h in held:
                    spool.add(h)
                held = []
                self.ooc_stats["spooled_sets"] = self.ooc_stats.get("spooled_sets", 0) + 1
        if spool is not None:
            self._spools.append(spool)
            return spool
        return held

    def _build_table(self, parts, hcol: str, st) -> "BuildTable":
        """In-memory build table, or — past the out-of-core limit — a hash-partitioned build whose
        partitions live in spillable spools (probed partition by partition: Grace hash join)."""
        from .spool import PartitionedSpool

        limit = self._ooc_limit()
        held, size, pspool = [], 0, None
        for b in parts:
            if pspool is not None:
                pspool.add(b, b.columns[hcol])
                continue
            held.append(b)
            size += b.nbytes()
            if size > limit:
                est = max(size, self._stage_source_bytes(st))
                nparts = int(min(256, max(2, -(-2 * est // limit))))
                pspool = PartitionedSpool(self.storage, nparts, "build")
                for h in held:
                    pspool.add(h, h.columns[hcol])
                held = []
        if pspool is not None:
            self._spools.append(pspool)
            self.ooc_stats["partitioned_builds"] = self.ooc_stats.get("partitioned_builds", 0) + 1
            return PartitionedBuild(pspool, hcol)
        return BuildTable(RecordBatch.concat(held) if held else None, hcol)

    def _stage_source_bytes(self, st) -> int:
        src = st.source
        if src["kind"] == "scan":
            try:
                return self.storage.get_set(src["atom"]["db"], src["atom"]["set"]).nbytes()
            except KeyError:
                return 0
        return 0

    def _aggregate(self, a, batches, state):
        from .spool import PartitionedSpool

        comp: AggregateComp = state.comps[a["comp"]]
        kcol, vcol = a["input"]["atts"]
        out_ts, out_col = a["output"]["name"], a["output"]["atts"][0]
        if isinstance(comp, TopKComp):
            self._topk(comp, [x for x in batches if x is not None and x.n], kcol, vcol, out_ts, out_col, state)
            return
        op = getattr(comp, "reduce_op", "sum")
        combine = comp.combine
        # a comp may reduce a whole group's values at once (group_values(values, inv, ngroups)), e.g.
        # FFAggMatrixToOneMatrix assembling every block of a matrix into one
        group_fn = getattr(comp, "group_values", None)
        kv = (RecordBatch({"k": x.columns[kcol], "v": x.columns[vcol]}, x.n) for x in batches if x is not None and x.n)
        if group_fn is not None:
            if self.ctx.distributed:   # raw values travel to the key's owner; it reduces them whole
                kv = self._stream_shuffle(kv, None, "aggregate", key=lambda b: K.hash_keys(b.columns["k"], b.device))
            reps, agg = self._reduce_kv(kv, op, combine, group_fn)
        elif not self.ctx.distributed:
            kv = list(kv)
            if len(kv) == 1 and any(kv[0].columns["k"] is u for u in state.unique_kv):
                # the single batch is a fused launch's result: its keys are already unique (one global table per
                # launch), so it IS the aggregate (no group-by pass over a handful of groups)
                reps, agg = kv[0].columns["k"], kv[0].columns["v"]
            else:
                reps, agg = self._reduce_kv(kv, op, combine)
            state.unique_kv.clear()
            dev = state.fused_out_device
            if dev is not None:
                state.fused_out_device = None
                reps, agg = _upload(reps, dev), _upload(agg, dev)
        else:
            # CombinerProcessor -> streaming shuffle by key hash -> AggregationProcessor: every chunk of (key,
            # value) pairs is combined locally before it is sent (CombinedShuffleSink), the shuffle rounds leave
            # while the pipeline runs, and the receiving side merges what arrives with the out-of-core
            # (hash-partitioned) reduction
            # 'mean' travels as (sum, count) columns and is divided after the final merge
            mean = op == "mean"
            local_op = "sum" if mean else op
            merge_op = "sum" if op in ("count", "mean") else op
            vmeta = {}                      # value dtype / trailing shape of a mean (the single-rank result's form)

            def combiner(batch):
                vals = batch.columns["v"]
                if mean:
                    if isinstance(vals, torch.Tensor) and "dt" not in vmeta:
                        vmeta["dt"], vmeta["shape"] = vals.dtype, tuple(vals.shape[1:])
                    vals = _sum_count(vals)
                fused = K.group_reduce(batch.columns["k"], vals, local_op)
                if fused is not None:
                    reps_c, agg_c = fused
                else:
                    inv, reps_c, g = K.group_ids(batch.columns["k"])
                    agg_c = K.segment_reduce(vals, inv, g, local_op if isinstance(vals, torch.Tensor) else None,
                                             combine)
                loc = RecordBatch({"k": reps_c, "v": _normalize(agg_c, len(agg_c), None)}, len(agg_c))
                return loc, K.hash_keys(reps_c, loc.device)

            recv = self._stream_shuffle(kv, None, "aggregate", combine=combiner, key=lambda b: None)
            reps, agg = self._reduce_kv(recv, merge_op, combine)
            if mean:
                # every rank learns the value form (a rank may receive groups without having had rows of its own)
                dts = (torch.float16, torch.bfloat16, torch.float32, torch.float64)
                dt0 = vmeta.get("dt")
                code = dts.index(dt0) if dt0 in dts else (-1 if dt0 is not None else -2)   # -2: no rows seen
                shp = list(vmeta.get("shape", ()))[:4]
                got = self.ctx.all_gather_ints([code, len(shp)] + shp + [0] * (4 - len(shp)))
                ref = next((x for x in got if x[0] != -2), None)
                if agg is not None:
                    dt = dts[ref[0]] if ref is not None and ref[0] >= 0 else torch.float64
                    shape = tuple(ref[2: 2 + ref[1]]) if ref is not None else None
                    agg = _mean_of(agg, dt, shape)
        if reps is None:
            state.materialized[out_ts] = []
            return
        out = comp.make_output(reps, agg)
        state.materialized[out_ts] = [RecordBatch({out_col: out}, out.n)]

    def _reduce_kv(self, kv_batches, op, combine, group_fn=None):
        """(key, value) batches -> (representative keys, aggregates). Streamed; past the out-of-core limit the
        pairs are hash-partitioned by key into spools and each partition is reduced alone (its groups are
        disjoint from every other partition's)."""
        from .spool import PartitionedSpool

        limit = self._ooc_limit()
        held, size, pspool = [], 0, None
        # several chunks (a scan split into coalesced batches): each held chunk is pre-reduced on the device when
        # the next arrives (sum / min / max merge with the same op), so the final reduction concatenates a few
        # partial groups instead of every row; stops as soon as a chunk does not shrink (high-cardinality keys)
        prereduce = group_fn is None and op in ("sum", "min", "max")

        def _pre(b):
            nonlocal prereduce
            v = b.columns["v"]
            if not (prereduce and b.n >= (1 << 16) and isinstance(v, torch.Tensor) and v.is_cuda):
                return b
            fused = K.group_reduce(b.columns["k"], v, op)
            if fused is None or len(fused[1]) * 2 > b.n:
                prereduce = False
                return b
            return RecordBatch({"k": fused[0], "v": fused[1]}, len(fused[1]))

        for kv in kv_batches:
            if kv is None or kv.n == 0:
                continue
            if pspool is None and held and prereduce:
                size -= held[-1].nbytes()
                held[-1] = _pre(held[-1])
                size += held[-1].nbytes()
            if pspool is not None:
                pspool.add(kv, K.hash_keys(kv.columns["k"], kv.device))
                continue
            held.append(kv)
            size += kv.nbytes()
            if size > limit:
                nparts = int(min(256, max(2, -(-2 * size // limit))))
                pspool = PartitionedSpool(self.storage, nparts, "agg")
                for h in held:
                    pspool.add(h, K.hash_keys(h.columns["k"], h.device))
                held = []
        groups = [held] if pspool is None else [p for p in pspool.parts if p.n]
        reps_parts, agg_parts = [], []
        try:
            for grp in groups:
                bs = [b for b in grp if b.n]
                if not bs:
                    continue
                devs = {b.device for b in bs}
                if len(devs) > 1:                 # host-resident fused partials beside eager (device) batches
                    dev = next(d for d in devs if d.type != "cpu")
                    bs = [b.to(dev) if b.device.type == "cpu" else b for b in bs]
                keys = column_concat([b.columns["k"] for b in bs])
                vals = column_concat([b.columns["v"] for b in bs])
                fused = None if group_fn is not None else K.group_reduce(keys, vals, op)   # relops.hip, or None
                if group_fn is not None:
                    inv, reps, g = K.group_ids(keys)
                    agg = group_fn(vals, inv, g)
                elif fused is not None:
                    reps, agg = fused
                else:
                    inv, reps, g = K.group_ids(keys)
                    agg = K.segment_reduce(vals, inv, g, op if isinstance(vals, torch.Tensor) else None, combine)
                reps_parts.append(reps)
                agg_parts.append(agg)
        finally:
            if pspool is not None:
                pspool.drop()
                self.ooc_stats["partitioned_aggregations"] = self.ooc_stats.get("partitioned_aggregations", 0) + 1
        if not reps_parts:
            return None, None
        reps = reps_parts[0] if len(reps_parts) == 1 else column_concat(reps_parts)
        agg = agg_parts[0] if len(agg_parts) == 1 else column_concat(agg_parts)
        return reps, agg

    def _topk(self, comp, batches, kcol, vcol, out_ts, out_col, state):
        """TopKComp: per-rank top k by score on the device (torch.topk over the device score column; objects
        gathered with a device take), then the ranks' candidates meet through one packed all-gather and the
        global top k is selected on the device again. No host copy of the scores."""
        objs, scores = [], []
        for x in batches:
            objs.append(x.columns[kcol])
            s = x.columns[vcol]
            scores.append(s if isinstance(s, torch.Tensor) else torch.tensor(s, dtype=torch.float64))
        local = None
        if objs:
            ob = column_concat(objs)
            dev = scores[0].device
            sc = torch.cat([s.to(dev) for s in scores])
            if not sc.is_floating_point():
                sc = sc.double()
            k = min(comp.k, sc.numel())
            top = torch.topk(sc, k).indices
            local = RecordBatch({"o": column_take(ob, top), "s": sc.index_select(0, top)}, k)
        if self.ctx.distributed:
            got = [g for g in self.ctx.broadcast_batch_all(local) if g is not None and g.n]
            local = RecordBatch.concat(got) if got else None
            if local is not None:
                k = min(comp.k, local.n)
                local = local.take(torch.topk(local.columns["s"], k).indices)
            if self.ctx.rank != 0:
                local = None
        if local is None or local.n == 0:
            state.materialized[out_ts] = []
            return
        state.materialized[out_ts] = [RecordBatch({out_col: local.columns["o"]}, local.n)]

    def _partition(self, a, batches, state):
        """PartitionComp: rows go to the rank owning their key hash in streaming shuffle rounds; what arrives is
        appended to the target set (if any) as it comes, never concatenated whole."""
        comp = state.comps[a["comp"]]
        kcol, ocol = a["input"]["atts"]
        kb = (RecordBatch({"k": x.columns[kcol], "o": x.columns[ocol]}, x.n) for x in batches if x is not None and x.n)
        recv = self._stream_shuffle(kb, None, "partition", key=lambda b: K.hash_keys(b.columns["k"], b.device))
        out_ts, out_col = a["output"]["name"], a["output"]["atts"][0]
        target = None
        if getattr(comp, "set_name", "") and self.storage.has_set(comp.db, comp.set_name):
            target = self.storage.get_set(comp.db, comp.set_name)
        outs = []
        for g in recv:
            objs = g.columns["o"]
            if target is not None:
                target.add_batch(objs)
            outs.append(RecordBatch({out_col: objs}, g.n))
        state.materialized[out_ts] = outs


def _sum_count(vals):
    """[n, ...] numeric values -> [n, F + 1] float64 (the values, then a count column of ones)."""
    if not isinstance(vals, torch.Tensor):
        vals = torch.as_tensor(vals, dtype=torch.float64)
    flat = vals.reshape(vals.shape[0], -1).double()
    return torch.cat([flat, torch.ones(flat.shape[0], 1, dtype=torch.float64, device=flat.device)], 1)


def _mean_of(sc, dtype=torch.float64, shape=None):
    """Merged (sum, count) columns -> the mean per group, in the form the single-rank group-by gives: float values
    keep their dtype (integer values average to float64) and the values' trailing shape."""
    m = (sc[:, :-1] / sc[:, -1:]).to(dtype)
    if shape is not None and len(shape) and int(torch.Size(shape).numel()) == m.shape[1]:
        return m.reshape((m.shape[0],) + tuple(shape))
    return m.squeeze(1) if m.shape[1] == 1 else m


class _JobState:
    def __init__(self, comps):
        self.comps = comps
        self.materialized: Dict[str, List[RecordBatch]] = {}
        self.builds: Dict[str, BuildTable] = {}
        self.fused_out_device = None     # a fused stage's host-resident partials: the device its result returns to
        self.unique_kv: List = []        # key columns of fused launch results (unique keys by construction)
        self.graph_key = None            # (graph signature, lambda constants): keys per-graph plan caches


def _upload(x, dev):
    """A host aggregate result (tensor, StringColumn, tuple / list of them, RecordBatch) -> ``dev`` with pinned,
    asynchronous copies (no stream synchronisation)."""
    if isinstance(x, RecordBatch):
        return RecordBatch({k: _upload(c, dev) for k, c in x.columns.items()}, x.n, x.type)
    if isinstance(x, tuple):
        return tuple(_upload(c, dev) for c in x)
    if isinstance(x, torch.Tensor):
        return x.pin_memory().to(dev, non_blocking=True) if x.device.type == "cpu" else x
    if isinstance(x, StringColumn):
        return x.to(dev)
    return x


__all__ = ["QueryEngine", "JobStats"]
