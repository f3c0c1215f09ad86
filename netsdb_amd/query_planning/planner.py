"""Physical planning: TCAP atoms -> pipeline stages (reference: src/queryPlanning/source/
TCAPAnalyzer.cc, QueryGraphAnalyzer.cc; job stages in src/builtInPDBObjects/headers/
TupleSetJobStage.h, AggregationJobStage.h, BroadcastJoinBuildHTJobStage.h,
HashPartitionedJoinBuildHTJobStage.h).

A *stage* is a pipeline: one source (a SCAN, or a tuple set materialised by an earlier stage),
a chain of streaming atoms (APPLY, FILTER, FLATTEN, HASHLEFT/RIGHT/ONE, JOIN-probe) and one
sink (OUTPUT, AGGREGATE, PARTITION, JOIN-build, or MATERIALIZE when a tuple set feeds several
consumers).  The join build side is chosen from set-size statistics (smaller side builds), and
the distribution strategy — broadcast (all-gather) vs hash-partitioned (all-to-all) — from the
build side's size against ``broadcast_threshold`` (netsDB's cost-based choice between
BroadcastJoinBuildHTJobStage and HashPartitionedJoinBuildHTJobStage).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

STREAMING = {"APPLY", "FILTER", "FLATTEN", "HASHLEFT", "HASHRIGHT", "HASHONE"}


@dataclass
class Stage:
    id: int
    source: dict                      # {"kind": "scan", "atom": a} | {"kind": "materialized", "ts": name}
    ops: List[dict] = field(default_factory=list)
    sink: dict = field(default_factory=dict)   # {"kind": ..., "atom": a, "ts": name}
    deps: List[int] = field(default_factory=list)

    def describe(self) -> str:
        src = self.source["atom"]["comp"] if self.source["kind"] == "scan" else f"mat:{self.source['ts']}"
        ops = " -> ".join(f"{o['type']}" + (f"[{o['lambda']}]" if o.get("lambda") else "") for o in self.ops)
        sk = self.sink.get("kind")
        extra = ""
        if sk == "join_build":
            extra = f" ({self.sink['strategy']})"
        return f"stage {self.id}: {src} -> {ops or '(none)'} => {sk}{extra}"


@dataclass
class PhysicalPlan:
    stages: List[Stage]
    atoms: List[dict]
    join_strategy: Dict[str, dict]

    def explain(self) -> str:
        return "\n".join(s.describe() for s in self.stages)


class Planner:
    def __init__(self, size_of_scan: Callable[[dict], int], world_size: int = 1,
                 broadcast_threshold: int = 2 << 30, copartitioned=(), distributed: Optional[bool] = None):
        self.size_of_scan = size_of_scan
        self.world_size = world_size
        # collectives on (a one-rank group with ClusterContext(force_collectives=True) included)
        self.distributed = world_size > 1 if distributed is None else distributed
        self.broadcast_threshold = broadcast_threshold
        # joins whose two inputs are already hash-placed by their join keys on every rank (Lachesis
        # co-partitioning): built and probed where the rows are, no shuffle of either side
        self.copartitioned = set(copartitioned)

    def plan(self, atoms: List[dict]) -> PhysicalPlan:
        producer: Dict[str, dict] = {}
        consumers: Dict[str, List[dict]] = {}
        for a in atoms:
            producer[a["output"]["name"]] = a
            for key in ("input", "input2"):
                nm = a[key]["name"]
                if nm:
                    lst = consumers.setdefault(nm, [])
                    if not any(x is a for x in lst):
                        lst.append(a)

        # --- size estimates per tuple set (bytes of the scans feeding it), for join side selection
        est: Dict[str, int] = {}
        for a in atoms:
            nm = a["output"]["name"]
            if a["type"] == "SCAN":
                est[nm] = self.size_of_scan(a)
            elif a["type"] == "JOIN":
                est[nm] = est.get(a["input"]["name"], 0) + est.get(a["input2"]["name"], 0)
            elif a["type"] in ("AGGREGATE",):
                est[nm] = max(1, est.get(a["input"]["name"], 0) // 4)
            else:
                est[nm] = est.get(a["input"]["name"], 0)

        join_strategy: Dict[str, dict] = {}
        for a in atoms:
            if a["type"] == "JOIN":
                left_sz, right_sz = est.get(a["input"]["name"], 0), est.get(a["input2"]["name"], 0)
                build = "right" if right_sz <= left_sz else "left"
                bsz = right_sz if build == "right" else left_sz
                if not self.distributed:
                    strat = "local"
                elif a["output"]["name"] in self.copartitioned:
                    strat = "copartitioned"
                elif bsz <= self.broadcast_threshold:
                    strat = "broadcast"
                else:
                    strat = "partitioned"
                join_strategy[a["output"]["name"]] = {"build": build, "strategy": strat, "build_bytes": bsz}

        stages: List[Stage] = []
        work: List[tuple] = []
        for a in atoms:
            if a["type"] == "SCAN":
                work.append(({"kind": "scan", "atom": a, "ts": a["output"]["name"]}, None))
        while work:
            src, first = work.pop(0)
            stages.append(self._walk(src, first, consumers, join_strategy, work))
        for st in stages:
            deps = set()
            if st.source["kind"] == "materialized":
                deps.add(("mat", st.source["ts"]))
            for o in st.ops:
                if o["type"] == "JOIN":
                    deps.add(("build", o["output"]["name"]))
            st.deps = deps  # type: ignore[assignment]
        order = self._toposort(stages)
        return PhysicalPlan(order, atoms, join_strategy)

    def _walk(self, src, first, consumers, join_strategy, work) -> Stage:
        st = Stage(0, src)
        ts, c = src["ts"], first
        while True:
            if c is None:
                cons = consumers.get(ts, [])
                if not cons:
                    st.sink = {"kind": "discard", "ts": ts}
                    return st
                if len(cons) > 1:
                    st.sink = {"kind": "materialize", "ts": ts}
                    for cc in cons:
                        work.append(({"kind": "materialized", "ts": ts}, cc))
                    return st
                c = cons[0]
            t = c["type"]
            if t in STREAMING:
                st.ops.append(c)
                ts, c = c["output"]["name"], None
                continue
            if t == "JOIN":
                js = join_strategy[c["output"]["name"]]
                side = "left" if c["input"]["name"] == ts else "right"
                if side == js["build"]:
                    st.sink = {"kind": "join_build", "atom": c, "side": side, "strategy": js["strategy"], "ts": ts}
                    return st
                st.ops.append(dict(c, _probe_side=side, _strategy=js["strategy"], _build=js["build"]))
                ts, c = c["output"]["name"], None
                continue
            if t in ("AGGREGATE", "PARTITION"):
                st.sink = {"kind": t.lower(), "atom": c, "ts": ts}
                work.append(({"kind": "materialized", "ts": c["output"]["name"]}, None))
                return st
            if t == "OUTPUT":
                st.sink = {"kind": "output", "atom": c, "ts": ts}
                return st
            raise ValueError(f"unexpected atom {t}")

    @staticmethod
    def _toposort(stages: List[Stage]) -> List[Stage]:
        provides = {}
        for st in stages:
            sk = st.sink.get("kind")
            if sk == "join_build":
                provides[("build", st.sink["atom"]["output"]["name"])] = st
            elif sk in ("aggregate", "partition"):
                provides[("mat", st.sink["atom"]["output"]["name"])] = st
            elif sk == "materialize":
                provides[("mat", st.sink["ts"])] = st
        done, order = set(), []
        remaining = list(stages)
        while remaining:
            progressed = False
            for st in list(remaining):
                if all(d in done or d not in provides for d in st.deps):
                    order.append(st)
                    remaining.remove(st)
                    sk = st.sink.get("kind")
                    if sk == "join_build":
                        done.add(("build", st.sink["atom"]["output"]["name"]))
                    elif sk in ("aggregate", "partition"):
                        done.add(("mat", st.sink["atom"]["output"]["name"]))
                    elif sk == "materialize":
                        done.add(("mat", st.sink["ts"]))
                    progressed = True
            if not progressed:
                raise RuntimeError("cyclic stage dependencies: " + "; ".join(s.describe() for s in remaining))
        for i, st in enumerate(order):
            st.id = i
        return order


# ---------------------------------------------------------------------------------------------------
class AdaptivePlanner:
    """Statistics-driven, incremental stage planning (reference: TCAPAnalyzer::getBestSource /
    penalizedSourceSets, TCAPAnalyzer.cc:1233-1300, and QuerySchedulerServer's dynamic planning loop,
    QuerySchedulerServer.cc:1033-1260, which materialises intermediate sets and re-analyses the
    remaining TCAP with their measured statistics).

    Stages are emitted one at a time from the sources available now: scans (catalogued set sizes) and
    tuple sets materialised by finished stages (their MEASURED sizes).  Policy:
      1. a source whose pipeline completes without building a join (it ends in an aggregation,
         partition, materialisation or output, probing only built tables) runs first, cheapest first —
         these stages produce the statistics the join decisions need;
      2. otherwise the cheapest source runs and builds the first unbuilt join it reaches (the smaller
         side builds, judged on measured sizes where known);
      3. a pipeline that has already probed a join and would build another stops there and materialises
         its output (the reference's "met a join sink with probing" rule abandons it instead): the next
         decision sees that set's measured size and builds the join from the smaller side.
    """

    PENALTY = 1000.0

    def __init__(self, atoms: List[dict], size_of_scan: Callable[[dict], int], world_size: int = 1,
                 broadcast_threshold: int = 2 << 30, copartitioned=(), distributed: Optional[bool] = None):
        self.atoms = atoms
        self.copartitioned = set(copartitioned)
        self.world_size = world_size
        self.distributed = world_size > 1 if distributed is None else distributed
        self.broadcast_threshold = broadcast_threshold
        self.producer: Dict[str, dict] = {}
        self.consumers: Dict[str, List[dict]] = {}
        for a in atoms:
            self.producer[a["output"]["name"]] = a
            for key in ("input", "input2"):
                nm = a[key]["name"]
                if nm:
                    lst = self.consumers.setdefault(nm, [])
                    if not any(x is a for x in lst):
                        lst.append(a)
        # pending sources: [ts, first consumer (None = all via consumers map), cost, kind]
        self.pending: List[list] = []
        # source costs only matter when there is a choice to make (several sources, or a join whose side /
        # broadcast decision reads them): a single-source pipeline skips the sizing, which on a cluster is a
        # collective per job (every rank sees the same atoms, so every rank skips it)
        scans = [a for a in atoms if a["type"] == "SCAN"]
        costed = len(scans) > 1 or any(a["type"] in ("JOIN", "HASHLEFT", "HASHRIGHT", "HASHONE") for a in atoms)
        for a in scans:
            self.pending.append([a["output"]["name"], None, float(size_of_scan(a)) if costed else 0.0, "scan", a])
        self.built: Dict[str, dict] = {}
        self.penalized: Dict[str, float] = {}
        self.decisions: List[dict] = []
        self.next_id = 0
        self.measured: Dict[str, int] = {}

    def has_work(self) -> bool:
        return bool(self.pending)

    def _cost(self, entry) -> float:
        key = f"{entry[0]}|{id(entry[1])}"
        c = max(1.0, entry[2])
        return c * self.penalized.get(key, 1.0)

    def next_stage(self) -> Optional[Stage]:
        if not self.pending:
            return None
        order = sorted(self.pending, key=self._cost)
        # 1. statistics-producing / join-free pipelines first
        for e in order:
            st, info = self._walk(e, allow_build=False)
            if st is not None:
                return self._take(e, st, info)
        # 2. cheapest source builds; 3. probe-then-build pipelines are abandoned + penalised
        for e in order:
            st, info = self._walk(e, allow_build=True)
            if st is not None:
                if info.get("build") and not self.distributed:
                    alt = self._measure_filtered_side(e, info["build"][0])
                    if alt is not None:
                        return self._take(*alt)
                return self._take(e, st, info)
            self.penalized[f"{e[0]}|{id(e[1])}"] = self.penalized.get(f"{e[0]}|{id(e[1])}", 1.0) * self.PENALTY
        e = order[0]                      # everything penalised: build anyway (forced)
        st, info = self._walk(e, allow_build=True, force=True)
        return self._take(e, st, info)

    # A build side at least this large is not chosen blind against a FILTERed scan on the other side of its join.
    MEASURE_BUILD_MIN = 64 << 20
    MEASURE_RATIO = 16

    def _measure_filtered_side(self, e, join: str):
        """About to build ``join`` from ``e`` (the cheapest source, costed by its size): if the join's other side is
        a scan that passes a FILTER before reaching it, that side's scan size says nothing about what arrives at the
        join. Run it to the join first and materialise it (its measured size then decides the build side: TPC-H
        Q04's quarter of orders, 0.6 M rows, against 15 M distinct late order keys; Q12's 0.3 M late lineitems
        against 15 M orders). Returns (source, stage, info) of that pipeline, or None."""
        if e[2] < self.MEASURE_BUILD_MIN:
            return None
        for e2 in self.pending:
            if e2 is e or e2[3] != "scan":
                continue
            if e[3] == "materialized" and e[2] * self.MEASURE_RATIO <= e2[2]:
                # the build candidate's size is MEASURED and a small fraction of the scan's: the scan side stays the
                # larger one unless its filter keeps less than 1 / MEASURE_RATIO, so it probes straight from the scan
                # (TPC-H Q03: the 1.4 M orders x customer rows build, 32 M late lineitems probe in the fused scan
                # instead of being materialised first)
                continue
            ts, c, seen_filter = e2[0], e2[1], False
            st = Stage(0, {"kind": "scan", "atom": e2[4], "ts": ts})
            while True:
                if c is None:
                    cons = self.consumers.get(ts, [])
                    if len(cons) != 1:
                        break
                    c = cons[0]
                if c["type"] in STREAMING:
                    seen_filter |= c["type"] == "FILTER"
                    st.ops.append(c)
                    ts, c = c["output"]["name"], None
                    continue
                if c["type"] == "JOIN" and c["output"]["name"] == join and join not in self.built and seen_filter:
                    st.sink = {"kind": "materialize", "ts": ts}
                    return e2, st, {"then": [(ts, c)]}
                break
        return None

    def _take(self, e, st: Stage, info: dict) -> Stage:
        self.pending.remove(e)
        st.id = self.next_id
        self.next_id += 1
        if info.get("build"):
            name, side, strat = info["build"]
            self.built[name] = {"build": side, "strategy": strat}
            self.decisions.append({"join": name, "build_side": side, "strategy": strat, "source": e[0],
                                   "cost": e[2], "measured": e[3] == "materialized"})
        return st

    def _walk(self, e, allow_build: bool, force: bool = False):
        ts0, first, cost, kind = e[0], e[1], e[2], e[3]
        src = {"kind": "scan", "atom": e[4], "ts": ts0} if kind == "scan" else {"kind": "materialized", "ts": ts0}
        st = Stage(0, src)
        ts, c = ts0, first
        probed = False
        info: dict = {}
        while True:
            if c is None:
                cons = self.consumers.get(ts, [])
                if not cons:
                    st.sink = {"kind": "discard", "ts": ts}
                    return st, info
                if len(cons) > 1:
                    st.sink = {"kind": "materialize", "ts": ts}
                    info["then"] = [(ts, cc) for cc in cons]
                    return st, info
                c = cons[0]
            t = c["type"]
            if t in STREAMING:
                st.ops.append(c)
                ts, c = c["output"]["name"], None
                continue
            if t == "JOIN":
                name = c["output"]["name"]
                side = "left" if c["input"]["name"] == ts else "right"
                if name in self.built:
                    js = self.built[name]
                    st.ops.append(dict(c, _probe_side=side, _strategy=js["strategy"], _build=js["build"]))
                    probed = True
                    ts, c = name, None
                    continue
                if allow_build and probed and not force:
                    # a probe-then-build pipeline stops at the join and materialises what it produced: the
                    # post-probe set becomes a source with a MEASURED size, and the next decision builds this
                    # join from whichever side is smaller (TPC-H Q03: 1.4 M orders x customer rows instead of
                    # 32 M lineitem rows). The reference abandons such pipelines; measuring first keeps the
                    # small-side choice without building a post-join table blind.
                    st.sink = {"kind": "materialize", "ts": ts}
                    info["then"] = [(ts, c)]
                    return st, info
                if not allow_build or (probed and not force):
                    return None, info
                if not self.distributed:
                    strat = "local"
                elif name in self.copartitioned:
                    strat = "copartitioned"
                elif cost <= self.broadcast_threshold:
                    strat = "broadcast"
                else:
                    strat = "partitioned"
                st.sink = {"kind": "join_build", "atom": c, "side": side, "strategy": strat, "ts": ts}
                info["build"] = (name, side, strat)
                return st, info
            if t in ("AGGREGATE", "PARTITION"):
                st.sink = {"kind": t.lower(), "atom": c, "ts": ts}
                info["then"] = [(c["output"]["name"], None)]
                return st, info
            if t == "OUTPUT":
                st.sink = {"kind": "output", "atom": c, "ts": ts}
                return st, info
            raise ValueError(f"unexpected atom {t}")

    def complete(self, st: Stage, measured_bytes: Optional[int]):
        """A stage finished: its materialised output becomes a new source, costed by its measured size."""
        sk = st.sink.get("kind")
        if sk in ("materialize", "aggregate", "partition"):
            out = st.sink["ts"] if sk == "materialize" else st.sink["atom"]["output"]["name"]
            size = int(measured_bytes or 0)
            self.measured[out] = size
            if sk == "materialize":
                for cc in self.consumers.get(out, []):
                    self.pending.append([out, cc, float(size), "materialized", None])
            else:
                self.pending.append([out, None, float(size), "materialized", None])


__all__ = ["Planner", "PhysicalPlan", "Stage", "AdaptivePlanner"]
