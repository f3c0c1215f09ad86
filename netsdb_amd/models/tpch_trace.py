"""Self-learning trace workloads over TPC-H (reference: src/tpch/source/tpchGenTrace.cc,
tpchPrepareTraining.cc, tpchTraining.cc; scripts/pangeaDeepRL).

* :func:`gen_trace` — tpchGenTrace: for every partition scheme (one placement key per table, the
  reference's PARTITION_SCHEME_STAT rows), reload the tables dispatched by those keys, run the query mix and
  record one RUN_STAT row per query (latency and the number of all-to-all shuffles the engine performed),
  while the self-learning hook records the full job / stage / lambda / data history of every run.
* :func:`prepare_training` — tpchPrepareTraining: turn RUN_STAT into per-(table, key) training samples
  (the mean cost of the queries that read the table under schemes placing it by that key).
* :func:`train_advisor` — tpchTraining: fit the :class:`~netsdb_amd.selflearning.DRLAdvisor` Q-network
  offline on those samples; afterwards ``create_set(..., policy="auto")`` places each table by the key the
  agent predicts is cheapest, and joins whose inputs end up placed by their join keys run without a
  shuffle (``stats["copartitioned_joins"]``, ``stats["shuffles"]``).
"""
from __future__ import annotations

import itertools
import time
from typing import Dict, List, Optional, Sequence, Tuple

from . import tpch

# candidate placement keys per table (attributes the TPC-H queries join or group on)
CANDIDATE_KEYS: Dict[str, List[Tuple[str, str]]] = {
    "orders": [("att", "o_orderkey"), ("att", "o_custkey")],
    "lineitem": [("att", "l_orderkey"), ("att", "l_partkey"), ("att", "l_suppkey")],
    "customer": [("att", "c_custkey"), ("att", "c_nationkey")],
    "part": [("att", "p_partkey")],
    "supplier": [("att", "s_suppkey"), ("att", "s_nationkey")],
}


def partition_schemes(tables: Sequence[str], keys: Optional[Dict[str, List[Tuple[str, str]]]] = None,
                      limit: Optional[int] = None) -> List[Dict[str, Tuple[str, str]]]:
    """Every combination of candidate keys over ``tables`` (the PARTITION_SCHEME_STAT enumeration)."""
    keys = keys or CANDIDATE_KEYS
    combos = itertools.product(*[keys[t] for t in tables])
    out = [dict(zip(tables, c)) for c in combos]
    return out[:limit] if limit else out


def load_with_scheme(client, db: str, data: Dict[str, Dict[str, object]], scheme: Dict[str, Tuple[str, str]]):
    """(Re)create the scheme's tables, dispatched by their placement keys (the other tables stay as they are)."""
    from ..selflearning import key_policy

    client.create_database(db)
    for table, (kind, name) in scheme.items():
        if client.storage.has_set(db, table):
            client.remove_set(db, table)
        client.create_set(db, table, tpch.TABLES[table], policy=key_policy(kind, name))
        client.send_data(db, table, tpch.to_batch(table, data[table]))
        if getattr(client, "learning", None) is not None:
            client.learning.db.record_placement(db, table, (kind, name))


def gen_trace(client, db: str, data: Dict[str, Dict[str, object]], schemes: List[Dict[str, Tuple[str, str]]],
              queries: Sequence[str] = ("q12", "q03"), env_id: int = 0, repeats: int = 1) -> List[dict]:
    """Run the query mix under every scheme; returns the RUN_STAT rows (also stored in the hook's DB)."""
    hook = getattr(client, "learning", None)
    if hook is None:
        hook = client.enable_self_learning()
    runs = []
    for sid, scheme in enumerate(schemes):
        hook.db.record_scheme(sid, {t: list(k) for t, k in scheme.items()})
        load_with_scheme(client, db, data, scheme)
        for q in queries:
            for _ in range(repeats):
                client.barrier()
                t0 = time.perf_counter()
                tpch.QUERIES[q](client, db)
                lat = time.perf_counter() - t0
                if client.ctx.distributed:
                    lat = client.ctx.all_reduce_scalar(lat, "max")
                st = getattr(hook, "last_stats", {}) or {}
                row = {"job": q, "scheme": sid, "env": env_id, "latency": lat, "shuffles": int(st.get("shuffles", 0)),
                       "copartitioned": list(st.get("copartitioned_joins", []))}
                hook.db.record_run(q, sid, env_id, lat, row["shuffles"])
                runs.append(row)
    return runs


def prepare_training(hook_db, db: str, cost: str = "latency") -> List[Tuple[str, str, str, float]]:
    """(db, table, key name, mean cost) per (table, key) from RUN_STAT x PARTITION_SCHEME_STAT; ``cost``
    = "latency" (the reference's reward) or "shuffles" (data movement: deterministic at test scale)."""
    import json

    col = "latency" if cost == "latency" else "shuffles"
    schemes = {sid: json.loads(js) for sid, js in hook_db.conn.execute("SELECT id, scheme FROM partition_scheme_stat")}
    per: Dict[Tuple[str, str], List[float]] = {}
    for sid, val in hook_db.conn.execute(f"SELECT partition_scheme_id, {col} FROM run_stat"):
        for table, (_, name) in schemes.get(sid, {}).items():
            per.setdefault((table, name), []).append(float(val))
    return [(db, t, k, sum(v) / len(v)) for (t, k), v in sorted(per.items())]


def train_advisor(client, db: str, cost: str = "latency", epochs: int = 300, seed: int = 0):
    """Fit a DRLAdvisor on the recorded trace and install it as the client's placement advisor."""
    from ..selflearning import DRLAdvisor

    hook = client.learning
    samples = prepare_training(hook.db, db, cost)
    adv = DRLAdvisor(hook.db, epsilon=0.0, seed=seed)
    adv.fit_offline(samples, epochs=epochs)
    hook.advisor = adv
    return adv, samples


__all__ = ["CANDIDATE_KEYS", "partition_schemes", "load_with_scheme", "gen_trace", "prepare_training", "train_advisor"]
