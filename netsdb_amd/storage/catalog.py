"""Distributed catalog (reference: src/catalog/source/PDBCatalog.cc — sqlite-backed metadata of
databases, sets, registered types and nodes; CatalogServer/CatalogClient serve it).

Here the master (rank 0) owns the sqlite file; in SPMD mode every rank holds the same in-memory
view and mutations are applied identically on all ranks (the client API is called collectively).
"""
from __future__ import annotations

import importlib
import json
import os
import sqlite3
import threading
from typing import Dict, List, Optional

from ..objects.record import lookup_type, register_type, registered_types

_SCHEMA = """
CREATE TABLE IF NOT EXISTS databases (name TEXT PRIMARY KEY, created REAL DEFAULT (julianday('now')));
CREATE TABLE IF NOT EXISTS sets (db TEXT, name TEXT, type TEXT, set_id INTEGER, page_size INTEGER,
                                 layout TEXT, partition TEXT, meta TEXT, PRIMARY KEY (db, name));
CREATE TABLE IF NOT EXISTS types (name TEXT PRIMARY KEY, module TEXT, qualname TEXT);
CREATE TABLE IF NOT EXISTS nodes (rank INTEGER PRIMARY KEY, address TEXT, device TEXT, hbm_bytes INTEGER);
CREATE TABLE IF NOT EXISTS shared_mappings (db TEXT, set_name TEXT, shared_db TEXT, shared_set TEXT, meta TEXT);
"""


class Catalog:
    def __init__(self, path: Optional[str] = None):
        self.path = path or ":memory:"
        if self.path != ":memory:":
            os.makedirs(os.path.dirname(os.path.abspath(self.path)), exist_ok=True)
        self.conn = sqlite3.connect(self.path, check_same_thread=False)
        if self.path != ":memory:":
            # write-ahead log with synchronous=NORMAL: no fsync per metadata commit (WAL stays corruption-safe;
            # only the last commits before an OS crash can be lost). Jobs create / drop their output sets every
            # run and a synchronous rollback-journal commit (fsyncs each) put ~0.1-7 ms of host time per set
            # operation in front of the GPU queue; flush_data() makes the catalog durable (checkpoint())
            self.conn.execute("PRAGMA journal_mode=WAL")
            self.conn.execute("PRAGMA synchronous=NORMAL")
        self.conn.executescript(_SCHEMA)
        self.lock = threading.RLock()
        self._types_seen = {}
        self._next_set_id = 1 + (self.conn.execute("SELECT COALESCE(MAX(set_id), 0) FROM sets").fetchone()[0])

    # ------------------------------------------------------------ databases
    def create_database(self, name: str) -> bool:
        with self.lock, self.conn:
            cur = self.conn.execute("INSERT OR IGNORE INTO databases(name) VALUES (?)", (name,))
            return cur.rowcount > 0

    def remove_database(self, name: str):
        with self.lock, self.conn:
            self.conn.execute("DELETE FROM sets WHERE db=?", (name,))
            self.conn.execute("DELETE FROM databases WHERE name=?", (name,))

    def databases(self) -> List[str]:
        return [r[0] for r in self.conn.execute("SELECT name FROM databases ORDER BY name")]

    def has_database(self, name: str) -> bool:
        return self.conn.execute("SELECT 1 FROM databases WHERE name=?", (name,)).fetchone() is not None

    # ------------------------------------------------------------ sets
    def create_set(self, db: str, name: str, type_name: Optional[str], page_size: int, layout: str = "pages",
                   partition: Optional[dict] = None, meta: Optional[dict] = None) -> int:
        with self.lock, self.conn:
            if not self.has_database(db):
                raise KeyError(f"database {db} does not exist")
            row = self.conn.execute("SELECT set_id FROM sets WHERE db=? AND name=?", (db, name)).fetchone()
            if row:
                return row[0]
            sid = self._next_set_id
            self._next_set_id += 1
            self.conn.execute("INSERT INTO sets VALUES (?,?,?,?,?,?,?,?)",
                              (db, name, type_name, sid, page_size, layout, json.dumps(partition or {}),
                               json.dumps(meta or {})))
            return sid

    def remove_set(self, db: str, name: str):
        with self.lock, self.conn:
            self.conn.execute("DELETE FROM sets WHERE db=? AND name=?", (db, name))

    def get_set(self, db: str, name: str) -> Optional[dict]:
        r = self.conn.execute("SELECT db,name,type,set_id,page_size,layout,partition,meta FROM sets WHERE db=? AND name=?",
                              (db, name)).fetchone()
        if not r:
            return None
        return {"db": r[0], "name": r[1], "type": r[2], "set_id": r[3], "page_size": r[4], "layout": r[5],
                "partition": json.loads(r[6]), "meta": json.loads(r[7])}

    def update_set_meta(self, db: str, name: str, meta: dict):
        with self.lock, self.conn:
            self.conn.execute("UPDATE sets SET meta=? WHERE db=? AND name=?", (json.dumps(meta), db, name))

    def sets(self, db: Optional[str] = None) -> List[dict]:
        q = "SELECT db, name FROM sets" + (" WHERE db=?" if db else "") + " ORDER BY db, name"
        rows = self.conn.execute(q, (db,) if db else ()).fetchall()
        return [self.get_set(d, n) for d, n in rows]

    # ------------------------------------------------------------ types
    def register_type(self, cls: type) -> str:
        register_type(cls)
        row = (cls.type_name(), cls.__module__, cls.__qualname__)
        if self._types_seen.get(row[0]) == row:          # already registered as this class: no write
            return row[0]
        with self.lock, self.conn:
            self.conn.execute("INSERT OR REPLACE INTO types VALUES (?,?,?)", row)
        self._types_seen[row[0]] = row
        return cls.type_name()

    def checkpoint(self):
        """Make every metadata commit durable (WAL checkpoint + fsync)."""
        if self.path == ":memory:":
            return
        with self.lock:
            self.conn.execute("PRAGMA wal_checkpoint(FULL)")

    def resolve_type(self, name: Optional[str]):
        if name is None:
            return None
        try:
            return lookup_type(name)
        except KeyError:
            r = self.conn.execute("SELECT module, qualname FROM types WHERE name=?", (name,)).fetchone()
            if not r:
                raise
            mod = importlib.import_module(r[0])
            obj = mod
            for part in r[1].split("."):
                obj = getattr(obj, part)
            register_type(obj)
            return obj

    def types(self) -> Dict[str, str]:
        out = {n: f"{c.__module__}.{c.__qualname__}" for n, c in registered_types().items()}
        for n, m, q in self.conn.execute("SELECT name, module, qualname FROM types"):
            out[n] = f"{m}.{q}"
        return out

    # ------------------------------------------------------------ nodes
    def register_node(self, rank: int, address: str, device: str, hbm_bytes: int):
        with self.lock, self.conn:
            self.conn.execute("INSERT OR REPLACE INTO nodes VALUES (?,?,?,?)", (rank, address, device, hbm_bytes))

    def nodes(self) -> List[dict]:
        return [{"rank": r, "address": a, "device": d, "hbm_bytes": h}
                for r, a, d, h in self.conn.execute("SELECT rank, address, device, hbm_bytes FROM nodes ORDER BY rank")]

    # ------------------------------------------------------------ dedup shared mappings
    def add_shared_mapping(self, db, set_name, shared_db, shared_set, meta=None):
        with self.lock, self.conn:
            self.conn.execute("INSERT INTO shared_mappings VALUES (?,?,?,?,?)",
                              (db, set_name, shared_db, shared_set, json.dumps(meta or {})))

    def shared_mappings(self, db, set_name) -> List[dict]:
        return [{"shared_db": a, "shared_set": b, "meta": json.loads(m)} for a, b, m in self.conn.execute(
            "SELECT shared_db, shared_set, meta FROM shared_mappings WHERE db=? AND set_name=?", (db, set_name))]

    def print_catalog(self) -> str:
        lines = ["databases: " + ", ".join(self.databases())]
        for s in self.sets():
            lines.append(f"  set {s['db']}.{s['name']} type={s['type']} id={s['set_id']} layout={s['layout']}")
        lines.append("types: " + ", ".join(sorted(self.types())))
        for n in self.nodes():
            lines.append(f"  node {n['rank']} {n['address']} {n['device']} hbm={n['hbm_bytes']}")
        return "\n".join(lines)


__all__ = ["Catalog"]
