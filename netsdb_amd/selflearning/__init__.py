"""Self-learning data placement (Lachesis) — reference: src/selfLearning (SelfLearningDB,
SelfLearningServer, RuleBasedDataPlacementOptimizerForLoadJob, DRLBasedDataPlacementOptimizerForLoadJob,
JobStageSelfLearningInfo, LambdaContext; docs/selfLearning-database-schema-full.pdf).

Every executed job is recorded into a sqlite history: for each scanned set, which stages consumed
it, what they ended in (hash-partitioned join build/probe, aggregation shuffle, partition, user set)
and the key lambda they hashed it by (attribute/method name — native lambdas cannot be used to
place data and are skipped, as in the reference).  When a set is (re)loaded, the advisor picks the
partition key:

* :class:`RuleBasedAdvisor` — the reference rule: the key of the most frequent shuffle/repartition
  consumer of that set (following one level of indirection through sets derived from it);
* :class:`LearnedAdvisor`  — epsilon-greedy bandit over the candidate keys, rewarded by the observed
  job time of consumers when the set was placed with that key;
* :class:`DRLAdvisor`      — the reference's deep-RL agent: a Q-network over an RLState-style vector
  (candidate-key features + cluster/environment features), trained online from the same rewards.

The chosen key becomes a dispatcher :class:`LambdaPolicy`, so co-partitioned joins run without a
shuffle (the planner sees both sides partitioned by the join key).
"""
from __future__ import annotations

import json
import math
import os
import random
import sqlite3
import threading
import time
from typing import Dict, List, Optional, Tuple

from ..lambdas import AttAccess, MethodCall
from ..parallel.dispatcher import LambdaPolicy

_SCHEMA = """
CREATE TABLE IF NOT EXISTS jobs (id INTEGER PRIMARY KEY AUTOINCREMENT, name TEXT, started REAL, seconds REAL);
CREATE TABLE IF NOT EXISTS stage_use (job_id INTEGER, db TEXT, set_name TEXT, sink TEXT, comp TEXT,
                                      key_kind TEXT, key_name TEXT, input_index INTEGER, seconds REAL);
CREATE TABLE IF NOT EXISTS lineage (job_id INTEGER, src_db TEXT, src_set TEXT, dst_db TEXT, dst_set TEXT);
CREATE TABLE IF NOT EXISTS placements (db TEXT, set_name TEXT, key_kind TEXT, key_name TEXT, t REAL);
CREATE TABLE IF NOT EXISTS rewards (db TEXT, set_name TEXT, key_name TEXT, seconds REAL);
-- job / stage / lambda / data history (the reference SelfLearningDB.cc schema, docs/selfLearning-database-schema)
CREATE TABLE IF NOT EXISTS data (id INTEGER PRIMARY KEY AUTOINCREMENT, db TEXT, set_name TEXT, created_job_id INTEGER,
                                 is_removed INTEGER DEFAULT 0, set_type TEXT, class_name TEXT, size INTEGER,
                                 page_size INTEGER, placement_kind TEXT, placement_key TEXT, modification_time REAL,
                                 UNIQUE(db, set_name));
CREATE TABLE IF NOT EXISTS job (id INTEGER PRIMARY KEY AUTOINCREMENT, name TEXT UNIQUE, tcap TEXT, signature TEXT,
                                initial_latency REAL, initial_job_instance_id INTEGER);
CREATE TABLE IF NOT EXISTS job_instance (id INTEGER PRIMARY KEY AUTOINCREMENT, job_id INTEGER, status TEXT,
                                         submit_time REAL, finish_time REAL, shuffles INTEGER, seconds REAL);
CREATE TABLE IF NOT EXISTS job_stage (id INTEGER PRIMARY KEY AUTOINCREMENT, job_instance_id INTEGER, stage_id INTEGER,
                                      source_type TEXT, sink_type TEXT, strategy TEXT, num_ops INTEGER,
                                      rows_in INTEGER, seconds REAL, description TEXT, device_seconds REAL);
CREATE TABLE IF NOT EXISTS lambda (id INTEGER PRIMARY KEY AUTOINCREMENT, job_id INTEGER, lambda_type TEXT,
                                   lambda_identifier TEXT, computation_name TEXT, lambda_name TEXT,
                                   input_index INTEGER, UNIQUE(job_id, computation_name, lambda_identifier));
CREATE TABLE IF NOT EXISTS data_job_stage (data_id INTEGER, job_stage_id INTEGER, index_in_inputs INTEGER,
                                           data_type TEXT);
-- trace workloads (tpchGenTrace.cc): partition schemes and the measured runs under each
CREATE TABLE IF NOT EXISTS partition_scheme_stat (id INTEGER PRIMARY KEY, scheme TEXT);
CREATE TABLE IF NOT EXISTS run_stat (id INTEGER PRIMARY KEY AUTOINCREMENT, job_name TEXT, partition_scheme_id INTEGER,
                                     environment_id INTEGER, latency REAL, shuffles INTEGER);
"""


def _producer_map(atoms) -> Dict[str, dict]:
    return {a["output"]["name"]: a for a in atoms}


def _source_scan(atoms_by_out, ts: str) -> Optional[dict]:
    """Follow producers back from tuple set ``ts`` to the SCAN feeding it (single-input chains)."""
    seen = set()
    while ts and ts not in seen:
        seen.add(ts)
        a = atoms_by_out.get(ts)
        if a is None:
            return None
        if a["type"] == "SCAN":
            return a
        if a["type"] == "JOIN":
            return None
        ts = a["input"]["name"]
    return None


def _scan_origin(atoms_by_out, ts: str, col: str) -> Optional[dict]:
    """The SCAN whose object column ``col`` of tuple set ``ts`` IS (carried unchanged, or renamed by
    identity ``self`` lambdas of selections/joins), else None (a derived or joined value)."""
    seen = set()
    while ts and (ts, col) not in seen:
        seen.add((ts, col))
        a = atoms_by_out.get(ts)
        if a is None or a["type"] == "JOIN":
            return None
        if a["type"] == "SCAN":
            return a if a["output"]["atts"] and col == a["output"]["atts"][0] else None
        outs = a["output"]["atts"]
        if col not in outs:
            return None
        if a["type"] == "APPLY" and outs[-1] == col and col not in a["projection"]["atts"]:
            if not str(a.get("lambda", "")).startswith("self") or len(a["input"]["atts"]) != 1:
                return None
            col = a["input"]["atts"][0]
        ts = a["input"]["name"]
    return None


def _key_of(comp, atoms_by_out, key_col_ts: str, key_att: str, scan: Optional[dict] = None):
    """The lambda node that produced column ``key_att`` (APPLY atom) -> (kind, name) or None.  With
    ``scan``, the lambda must read the scanned object column itself (not a derived object)."""
    ts = key_col_ts
    seen = set()
    while ts and ts not in seen:
        seen.add(ts)
        a = atoms_by_out.get(ts)
        if a is None:
            return None
        if a["type"] == "APPLY" and a["output"]["atts"] and a["output"]["atts"][-1] == key_att:
            if scan is not None and (len(a["input"]["atts"]) != 1 or
                                     _scan_origin(atoms_by_out, a["input"]["name"], a["input"]["atts"][0]) is not scan):
                return None
            node = comp.extract_lambdas().get(a["lambda"])
            if isinstance(node, AttAccess):
                return ("att", node.field)
            if isinstance(node, MethodCall):
                return ("method", node.method)
            return ("native", a["lambda"])
        ts = a["input"]["name"]
    return None


def extract_uses(atoms, comps, plan) -> List[dict]:
    """Partition-relevant uses of every scanned set in one job."""
    by_out = _producer_map(atoms)
    uses = []
    strat = plan.join_strategy if plan is not None else {}
    for a in atoms:
        if a["type"] in ("HASHLEFT", "HASHRIGHT"):
            scan = _source_scan(by_out, a["input"]["name"])
            if scan is None:
                continue
            comp = comps.get(a["comp"])
            key = _key_of(comp, by_out, a["input"]["name"], a["input"]["atts"][0]) if comp else None
            join_out = next((j["output"]["name"] for j in atoms if j["type"] == "JOIN" and
                             a["output"]["name"] in (j["input"]["name"], j["input2"]["name"])), None)
            # a broadcast join never moves this set; partitioned (or single-node 'local', which would be
            # partitioned at scale) joins hash it by this key -> a placement candidate
            sink = "Broadcast" if strat.get(join_out, {}).get("strategy") == "broadcast" else "Shuffle"
            uses.append({"db": scan["db"], "set": scan["set"], "sink": sink, "comp": a["comp"],
                         "key": key, "index": 0 if a["type"] == "HASHLEFT" else 1})
        elif a["type"] in ("AGGREGATE", "PARTITION"):
            scan = _source_scan(by_out, a["input"]["name"])
            if scan is None:
                continue
            comp = comps.get(a["comp"])
            key = _key_of(comp, by_out, a["input"]["name"], a["input"]["atts"][0]) if comp else None
            uses.append({"db": scan["db"], "set": scan["set"], "sink": "Repartition" if a["type"] == "PARTITION"
                         else "Shuffle", "comp": a["comp"], "key": key, "index": 0})
        elif a["type"] == "OUTPUT":
            scan = _source_scan(by_out, a["input"]["name"])
            if scan is not None:
                uses.append({"db": scan["db"], "set": scan["set"], "sink": "UserSet", "comp": a["comp"], "key": None,
                             "index": 0, "dst": (a["db"], a["set"])})
    return uses


class SelfLearningDB:
    def __init__(self, path: str = ":memory:"):
        self.conn = sqlite3.connect(path, check_same_thread=False)
        self.conn.executescript(_SCHEMA)
        cols = {r[1] for r in self.conn.execute("PRAGMA table_info(job_stage)")}
        if "device_seconds" not in cols:            # a history file written before stages had device times
            self.conn.execute("ALTER TABLE job_stage ADD COLUMN device_seconds REAL")
        self.lock = threading.Lock()
        # stage rows whose device time (HIP event pair, resolved asynchronously) was not known when recorded
        self._pending_dev: List[tuple] = []

    def flush_device_times(self, block: bool = False) -> int:
        """Write the device times of recorded stages whose event pairs have resolved since (``block``: resolve them
        now); returns how many stay pending."""
        keep = []
        for sid, stats, rec in self._pending_dev:
            if rec.get("device_seconds") is None and hasattr(stats, "device_times"):
                stats.device_times(block)
            if rec.get("device_seconds") is None:
                keep.append((sid, stats, rec))
                continue
            with self.lock, self.conn:
                self.conn.execute("UPDATE job_stage SET device_seconds=? WHERE id=?", (rec["device_seconds"], sid))
        self._pending_dev = keep
        return len(keep)

    def record_job(self, name: str, seconds: float, uses: List[dict]) -> int:
        with self.lock, self.conn:
            cur = self.conn.execute("INSERT INTO jobs(name, started, seconds) VALUES (?,?,?)", (name, time.time(), seconds))
            jid = cur.lastrowid
            for u in uses:
                k = u.get("key") or (None, None)
                self.conn.execute("INSERT INTO stage_use VALUES (?,?,?,?,?,?,?,?,?)",
                                  (jid, u["db"], u["set"], u["sink"], u["comp"], k[0], k[1], u["index"], seconds))
                if u.get("dst"):
                    self.conn.execute("INSERT INTO lineage VALUES (?,?,?,?,?)", (jid, u["db"], u["set"], *u["dst"]))
            # reward the current placement of every set this job read
            for u in uses:
                p = self.current_placement(u["db"], u["set"])
                if p is not None:
                    self.conn.execute("INSERT INTO rewards VALUES (?,?,?,?)", (u["db"], u["set"], p[1], seconds))
            return jid

    # ------------------------------------------------------------------ full job history
    def upsert_data(self, db: str, set_name: str, uset=None, job_id: Optional[int] = None) -> int:
        pl = getattr(uset, "placement", None) if uset is not None else None
        typ = getattr(uset, "type", None)
        with self.lock, self.conn:
            self.conn.execute(
                "INSERT INTO data(db, set_name, created_job_id, set_type, class_name, size, page_size, placement_kind,"
                " placement_key, modification_time) VALUES (?,?,?,?,?,?,?,?,?,?) ON CONFLICT(db, set_name) DO UPDATE SET"
                " size=excluded.size, placement_kind=excluded.placement_kind, placement_key=excluded.placement_key,"
                " modification_time=excluded.modification_time, is_removed=0",
                (db, set_name, job_id, type(uset).__name__ if uset is not None else None,
                 typ.type_name() if typ is not None else None,
                 int(uset.nbytes()) if uset is not None and hasattr(uset, "nbytes") else None,
                 getattr(uset, "page_size", None), pl[0] if pl else None, pl[1] if pl else None, time.time()))
            return self.conn.execute("SELECT id FROM data WHERE db=? AND set_name=?", (db, set_name)).fetchone()[0]

    def record_instance(self, name: str, tcap: Optional[str], stats: dict, plan, comps, storage=None) -> int:
        """One executed job: job (first latency), job_instance, job_stage per physical stage (with the
        measured rows/seconds), lambda per computation lambda, data + data_job_stage for every scanned
        and written set."""
        import hashlib

        secs = float(stats.get("seconds", 0.0))
        if self._pending_dev:
            self.flush_device_times(False)
        if hasattr(stats, "device_times"):
            stats.device_times(False)                 # whatever has completed already (no wait)
        sig = hashlib.sha1((tcap or "").encode()).hexdigest()[:16]
        with self.lock, self.conn:
            self.conn.execute("INSERT OR IGNORE INTO job(name, tcap, signature, initial_latency) VALUES (?,?,?,?)",
                              (name, (tcap or "")[:20000], sig, secs))
            jid = self.conn.execute("SELECT id FROM job WHERE name=?", (name,)).fetchone()[0]
            cur = self.conn.execute("INSERT INTO job_instance(job_id, status, submit_time, finish_time, shuffles, seconds)"
                                    " VALUES (?,?,?,?,?,?)", (jid, "finished", time.time() - secs, time.time(),
                                                              int(stats.get("shuffles", 0)), secs))
            iid = cur.lastrowid
            self.conn.execute("UPDATE job SET initial_job_instance_id=COALESCE(initial_job_instance_id, ?) WHERE id=?",
                              (iid, jid))
            for cname, comp in (comps or {}).items():
                try:
                    lams = comp.extract_lambdas()
                except Exception:
                    continue
                for lname, node in lams.items():
                    field = getattr(node, "field", None) or getattr(node, "method", None)
                    self.conn.execute("INSERT OR IGNORE INTO lambda(job_id, lambda_type, lambda_identifier,"
                                      " computation_name, lambda_name, input_index) VALUES (?,?,?,?,?,?)",
                                      (jid, type(node).__name__, lname, cname, field,
                                       getattr(node, "input_index", None)))
        timing = {st["id"]: st for st in stats.get("stages", [])}
        for st in (plan.stages if plan is not None else []):
            sink = st.sink or {}
            t = timing.get(st.id, {})
            with self.lock, self.conn:
                sid = self.conn.execute(
                    "INSERT INTO job_stage(job_instance_id, stage_id, source_type, sink_type, strategy, num_ops,"
                    " rows_in, seconds, description, device_seconds) VALUES (?,?,?,?,?,?,?,?,?,?)",
                    (iid, st.id, st.source.get("kind"), sink.get("kind"), sink.get("strategy"), len(st.ops),
                     t.get("rows_in"), t.get("seconds"), st.describe(), t.get("device_seconds"))).lastrowid
            if "device_seconds" in t and t["device_seconds"] is None:
                self._pending_dev.append((sid, stats, t))
            ios = []
            if st.source.get("kind") == "scan":
                ios.append((st.source["atom"]["db"], st.source["atom"]["set"], 0, "in"))
            if sink.get("kind") == "output":
                ios.append((sink["atom"]["db"], sink["atom"]["set"], 0, "out"))
            for d, sname, idx, kind in ios:
                uset = None
                if storage is not None:
                    try:
                        uset = storage.get_set(d, sname)
                    except KeyError:
                        uset = None
                did = self.upsert_data(d, sname, uset, jid)
                with self.lock, self.conn:
                    self.conn.execute("INSERT INTO data_job_stage VALUES (?,?,?,?)", (did, sid, idx, kind))
        return iid

    def record_scheme(self, scheme_id: int, scheme: dict):
        with self.lock, self.conn:
            self.conn.execute("INSERT OR REPLACE INTO partition_scheme_stat VALUES (?,?)",
                              (scheme_id, json.dumps(scheme, sort_keys=True)))

    def record_run(self, job_name: str, scheme_id: int, env_id: int, latency: float, shuffles: int):
        with self.lock, self.conn:
            self.conn.execute("INSERT INTO run_stat(job_name, partition_scheme_id, environment_id, latency, shuffles)"
                              " VALUES (?,?,?,?,?)", (job_name, scheme_id, env_id, latency, shuffles))

    def record_placement(self, db: str, set_name: str, key: Tuple[str, str]):
        with self.lock, self.conn:
            self.conn.execute("INSERT INTO placements VALUES (?,?,?,?,?)", (db, set_name, key[0], key[1], time.time()))

    def current_placement(self, db, set_name) -> Optional[Tuple[str, str]]:
        r = self.conn.execute("SELECT key_kind, key_name FROM placements WHERE db=? AND set_name=? ORDER BY t DESC LIMIT 1",
                              (db, set_name)).fetchone()
        return tuple(r) if r else None

    def candidates(self, db: str, set_name: str, sinks=("Shuffle", "Repartition")) -> List[Tuple[str, str, int]]:
        q = ("SELECT key_kind, key_name, COUNT(*) FROM stage_use WHERE db=? AND set_name=? AND key_kind IN ('att','method') "
             f"AND sink IN ({','.join('?' * len(sinks))}) GROUP BY key_kind, key_name ORDER BY COUNT(*) DESC, SUM(seconds) DESC")
        return [tuple(r) for r in self.conn.execute(q, (db, set_name, *sinks))]

    def derived_sets(self, db: str, set_name: str) -> List[Tuple[str, str]]:
        return [tuple(r) for r in self.conn.execute(
            "SELECT DISTINCT dst_db, dst_set FROM lineage WHERE src_db=? AND src_set=?", (db, set_name))]

    def mean_reward(self, db, set_name, key_name) -> Optional[float]:
        r = self.conn.execute("SELECT AVG(seconds), COUNT(*) FROM rewards WHERE db=? AND set_name=? AND key_name=?",
                              (db, set_name, key_name)).fetchone()
        return None if not r or not r[1] else float(r[0])

    def export(self) -> dict:
        return {t: [list(r) for r in self.conn.execute(f"SELECT * FROM {t}")]
                for t in ("jobs", "stage_use", "lineage", "placements", "rewards", "data", "job", "job_instance",
                          "job_stage", "lambda", "data_job_stage", "partition_scheme_stat", "run_stat")}


def key_policy(kind: str, name: str, type_=None) -> LambdaPolicy:
    """Dispatcher policy hashing records by an attribute or (vectorised) method."""
    if kind == "att":
        fn = lambda b: b.columns[name]  # noqa: E731
    else:
        def fn(b):
            m = getattr(b.type, name)
            vec = getattr(m, "__vectorized__", None)
            return vec(b) if vec is not None else [m(v) for v in __import__(
                "netsdb_amd.lambdas", fromlist=["SelfRef"]).SelfRef(b).views()]
    return LambdaPolicy(fn, description=f"{kind}:{name}")


class RuleBasedAdvisor:
    def __init__(self, db: SelfLearningDB):
        self.db = db

    def best_key(self, dbname: str, set_name: str) -> Optional[Tuple[str, str]]:
        c = self.db.candidates(dbname, set_name)
        if c:
            return (c[0][0], c[0][1])
        for d, s in self.db.derived_sets(dbname, set_name):        # one level of indirection
            c = self.db.candidates(d, s)
            if c:
                return (c[0][0], c[0][1])
        return None

    def policy(self, dbname: str, set_name: str) -> Optional[LambdaPolicy]:
        k = self.best_key(dbname, set_name)
        return key_policy(*k) if k else None


class LearnedAdvisor(RuleBasedAdvisor):
    """Epsilon-greedy bandit over the candidate keys (reward = -mean consumer job time)."""

    def __init__(self, db: SelfLearningDB, epsilon: float = 0.1, seed: int = 0):
        super().__init__(db)
        self.epsilon = epsilon
        self.rng = random.Random(seed)

    def best_key(self, dbname, set_name):
        cands = [(k, n) for k, n, _ in self.db.candidates(dbname, set_name)]
        if not cands:
            return super().best_key(dbname, set_name)
        untried = [c for c in cands if self.db.mean_reward(dbname, set_name, c[1]) is None]
        if untried:
            return untried[0]
        if self.rng.random() < self.epsilon:
            return self.rng.choice(cands)
        return min(cands, key=lambda c: self.db.mean_reward(dbname, set_name, c[1]))


class DRLAdvisor(RuleBasedAdvisor):
    """Deep-RL placement agent (reference: DRLBasedDataPlacementOptimizerForLoadJob + RLClient/RLState,
    whose state vector goes to an external RL server that answers with the best lambda index).

    Here the agent is in-process: a Q-network (MLP) maps the RLState-style vector — per candidate key
    slot: use frequency, mean consumer-job time, last observed reward and an untried flag; plus input
    size, number of nodes/GPUs, number of candidates, host cores and device memory — to one value per
    candidate slot.  A placement is a one-step episode (its reward, minus the consumer job time, arrives
    when the jobs reading the set run), so the update is a contextual-bandit Q regression over a replay
    buffer (gamma = 0) with epsilon-greedy exploration over the valid slots."""

    SLOTS = 4

    def __init__(self, db: SelfLearningDB, epsilon: float = 0.2, seed: int = 0, hidden: int = 64, lr: float = 3e-3,
                 env: Optional[dict] = None):
        super().__init__(db)
        import torch

        self.torch = torch
        self.rng = random.Random(seed)
        self.epsilon = epsilon
        self.env = dict(env or {})
        g = torch.Generator().manual_seed(seed)
        dim = self.SLOTS * 4 + 6
        self.q = torch.nn.Sequential(torch.nn.Linear(dim, hidden), torch.nn.ReLU(), torch.nn.Linear(hidden, hidden),
                                     torch.nn.ReLU(), torch.nn.Linear(hidden, self.SLOTS))
        with torch.no_grad():
            for p in self.q.parameters():
                p.copy_(torch.empty_like(p).uniform_(-0.1, 0.1, generator=g))
        self.opt = torch.optim.Adam(self.q.parameters(), lr=lr)
        self.replay: List[Tuple[list, int, float]] = []
        self.pending: Dict[Tuple[str, str], Tuple[list, int, List[Tuple[str, str]]]] = {}
        self.scale: Optional[float] = None      # running reward scale (seconds)

    def state(self, dbname: str, set_name: str, cands: List[Tuple[str, str, int]]) -> list:
        """RLState.toVector analogue."""
        total = max(1, sum(c[2] for c in cands))
        s = self.scale or 1.0
        feats: list = []
        for i in range(self.SLOTS):
            if i < len(cands):
                _, n, cnt = cands[i]
                r = self.db.mean_reward(dbname, set_name, n)
                sec = self.db.conn.execute("SELECT AVG(seconds) FROM stage_use WHERE db=? AND set_name=? AND key_name=?",
                                           (dbname, set_name, n)).fetchone()[0] or 0.0
                feats += [cnt / total, sec / s, (r / s) if r is not None else 0.0, 1.0 if r is None else 0.0]
            else:
                feats += [0.0, 0.0, 0.0, 0.0]
        e = self.env
        feats += [math.log1p(e.get("input_records", 0)) / 20.0, e.get("num_nodes", 1) / 8.0, len(cands) / self.SLOTS,
                  (os.cpu_count() or 1) / 256.0, e.get("mem_gb", 0.0) / 288.0, e.get("num_gpus", 1) / 8.0]
        return feats

    def best_key(self, dbname, set_name):
        cands = self.db.candidates(dbname, set_name)[: self.SLOTS]
        if not cands:
            return super().best_key(dbname, set_name)
        torch = self.torch
        s = self.state(dbname, set_name, cands)
        if self.rng.random() < self.epsilon:
            a = self.rng.randrange(len(cands))
        else:
            with torch.no_grad():
                q = self.q(torch.tensor([s], dtype=torch.float32))[0, : len(cands)]
            a = int(q.argmax())
        self.pending[(dbname, set_name)] = (s, a, [(k, n) for k, n, _ in cands])
        return (cands[a][0], cands[a][1])

    def observe(self, dbname: str, set_name: str, key_name: str, seconds: float, steps: int = 20):
        """Reward of the placement last chosen for (db, set): minus the time of a job that read it."""
        p = self.pending.get((dbname, set_name))
        if p is None:
            return
        s, a, cands = p
        if cands[a][1] != key_name:
            return
        self.scale = seconds if self.scale is None else 0.9 * self.scale + 0.1 * seconds
        self.replay.append((s, a, -seconds / max(self.scale, 1e-9)))
        self.replay = self.replay[-512:]
        torch = self.torch
        for _ in range(steps):
            batch = [self.replay[self.rng.randrange(len(self.replay))] for _ in range(min(32, len(self.replay)))]
            S = torch.tensor([b[0] for b in batch], dtype=torch.float32)
            A = torch.tensor([b[1] for b in batch])
            R = torch.tensor([b[2] for b in batch], dtype=torch.float32)
            loss = torch.nn.functional.mse_loss(self.q(S).gather(1, A[:, None])[:, 0], R)
            self.opt.zero_grad()
            loss.backward()
            self.opt.step()

    def fit_offline(self, samples: List[Tuple[str, str, str, float]], epochs: int = 200, batch: int = 32):
        """Train from a recorded trace (tpchTraining.cc): ``samples`` = (db, set, key_name, cost) runs, cost
        = the consumer jobs' latency (or any measured cost such as shuffles) under that placement.  Each
        sample becomes (state of the set's candidate list, index of the key, -cost/scale)."""
        torch = self.torch
        costs = [c for *_, c in samples]
        if not costs:
            return 0
        self.scale = max(1e-9, sum(costs) / len(costs))
        for dbname, set_name, key_name, cost in samples:
            cands = self.db.candidates(dbname, set_name)[: self.SLOTS]
            names = [n for _, n, _ in cands]
            if key_name not in names:
                continue
            self.replay.append((self.state(dbname, set_name, cands), names.index(key_name), -cost / self.scale))
        self.replay = self.replay[-4096:]
        if not self.replay:
            return 0
        for _ in range(epochs):
            bt = [self.replay[self.rng.randrange(len(self.replay))] for _ in range(min(batch, len(self.replay)))]
            S = torch.tensor([b[0] for b in bt], dtype=torch.float32)
            A = torch.tensor([b[1] for b in bt])
            R = torch.tensor([b[2] for b in bt], dtype=torch.float32)
            loss = torch.nn.functional.mse_loss(self.q(S).gather(1, A[:, None])[:, 0], R)
            self.opt.zero_grad()
            loss.backward()
            self.opt.step()
        return len(self.replay)

    def save(self, path: str):
        self.torch.save({"q": self.q.state_dict(), "scale": self.scale}, path)

    def load(self, path: str):
        st = self.torch.load(path, weights_only=True)
        self.q.load_state_dict(st["q"])
        self.scale = st["scale"]


class SelfLearningHook:
    """Attach to a PDBClient: records every job; ``advise(db, set)`` returns a partition policy.
    ``learned``: False = rule-based, True / "bandit" = epsilon-greedy bandit, "drl" = :class:`DRLAdvisor`."""

    def __init__(self, client, path: str = ":memory:", learned=False):
        self.client = client
        self.db = SelfLearningDB(path)
        if learned == "drl":
            budget = client.storage.device_budget
            env = {"num_nodes": client.ctx.world_size, "num_gpus": client.ctx.world_size,
                   "mem_gb": budget / 2 ** 30 if budget < 1 << 60 else 0.0}
            self.advisor = DRLAdvisor(self.db, env=env)
        else:
            self.advisor = LearnedAdvisor(self.db) if learned else RuleBasedAdvisor(self.db)
        eng = client.engine
        orig = eng.execute

        def execute(sinks, job_name="job", **kw):
            st = orig(sinks, job_name, **kw)
            if st.get("pre_compiled"):
                return st
            if eng.last_tcap is not None and eng.last_plan is not None and eng._last_comps is not None:
                atoms = eng.last_plan.atoms
                uses = extract_uses(atoms, eng._last_comps, eng.last_plan)
                secs = st.get("seconds", 0.0)
                self.db.record_job(job_name, secs, uses)
                self.db.record_instance(job_name, eng.last_tcap, st, eng.last_plan, eng._last_comps, client.storage)
                self.last_stats = st
                if isinstance(self.advisor, DRLAdvisor):
                    for u in uses:
                        p = self.db.current_placement(u["db"], u["set"])
                        if p is not None:
                            self.advisor.observe(u["db"], u["set"], p[1], secs)
            return st

        eng.execute = execute
        client.learning = self

    def advise(self, dbname: str, set_name: str) -> Optional[LambdaPolicy]:
        k = self.advisor.best_key(dbname, set_name)
        if k is None:
            return None
        self.db.record_placement(dbname, set_name, k)
        return key_policy(*k)

    def report(self) -> str:
        return json.dumps(self.db.export(), default=str)[:10000]


__all__ = ["SelfLearningDB", "RuleBasedAdvisor", "LearnedAdvisor", "DRLAdvisor", "SelfLearningHook", "extract_uses",
           "key_policy"]
