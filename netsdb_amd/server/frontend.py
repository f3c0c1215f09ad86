"""Master front end (rank 0) + SPMD worker loop + remote client.

Security model: the wire protocol never ships code.  Remote clients can
  * invoke jobs the operator registered up front (``PDBFrontend.register_job`` / ``--jobs module``);
  * ``register_type(module)`` (PDBClient::registerType): the server imports the module ONLY if it lies
    under one of the operator's allow-listed module prefixes (``--udf-modules``) and registers the
    record types and computation (UDF) classes it defines;
  * ``execute_computations(graph)`` (PDBClient::executeComputations): a DECLARATIVE computation graph —
    nodes naming registered computation classes with JSON constructor arguments, scan/write nodes
    naming sets — which the server rebuilds and runs through its engine (``pre_compile`` supported).
The listener binds to 127.0.0.1 unless told otherwise.
"""
from __future__ import annotations

import importlib
import inspect
import socket
import socketserver
import itertools
import threading
import traceback
from typing import Any, Callable, Dict, List, Optional, Sequence

import torch

from ..objects.record import PDBObject, lookup_type
from .protocol import recv_msg, send_msg


class UDFRegistry:
    """Computation classes remote graphs may instantiate, by name (server-side allow-list)."""

    def __init__(self, allowed_modules: Sequence[str] = ()):
        from ..computations import Computation

        self.base = Computation
        self.allowed = tuple(allowed_modules)
        self.classes: Dict[str, type] = {}
        self.modules: List[str] = []

    def allowed_module(self, mod: str) -> bool:
        return any(mod == p or mod.startswith(p.rstrip(".") + ".") for p in self.allowed)

    def register_module(self, mod: str) -> dict:
        """registerType: import an allow-listed module; register its record types and UDF classes."""
        if not isinstance(mod, str) or not mod.replace("_", "").replace(".", "").isalnum():
            raise ValueError("module path must be a dotted identifier")
        if not self.allowed_module(mod):
            raise PermissionError(f"module '{mod}' is not under an allow-listed UDF module prefix")
        m = importlib.import_module(mod)
        types, comps = [], []
        for name, obj in vars(m).items():
            if not inspect.isclass(obj) or obj.__module__ != m.__name__:
                continue
            if issubclass(obj, PDBObject):
                types.append(obj.type_name())
            elif issubclass(obj, self.base):
                self.classes[name] = obj
                comps.append(name)
        if mod not in self.modules:
            self.modules.append(mod)
        return {"module": mod, "types": sorted(types), "computations": sorted(comps)}

    def get(self, name: str) -> type:
        if name not in self.classes:
            raise KeyError(f"computation class '{name}' is not registered on this server")
        return self.classes[name]


def _json_args(v):
    if isinstance(v, (str, int, float, bool)) or v is None:
        return v
    if isinstance(v, list):
        return [_json_args(x) for x in v]
    if isinstance(v, dict) and all(isinstance(k, str) for k in v):
        return {k: _json_args(x) for k, x in v.items()}
    raise ValueError("constructor arguments must be JSON values")


def build_graph(spec: dict, registry: UDFRegistry):
    """Rebuild a declarative graph: {"nodes": [{"id", "kind": "scan"|"write"|"comp", ...}], "sinks": [ids]}."""
    from ..computations import ScanSet, WriteSet

    nodes = spec.get("nodes")
    if not isinstance(nodes, list) or len(nodes) > 10000:
        raise ValueError("graph.nodes must be a list")
    built: Dict[int, Any] = {}
    for n in nodes:
        kind, nid = n.get("kind"), n.get("id")
        if not isinstance(nid, int) or nid in built:
            raise ValueError("every node needs a unique integer id")
        if kind in ("scan", "write"):
            t = lookup_type(n["type"]) if n.get("type") else None
            c = (ScanSet if kind == "scan" else WriteSet)(str(n["db"]), str(n["set"]), t)
        elif kind == "comp":
            cls = registry.get(str(n["class"]))
            c = cls(*_json_args(n.get("args") or []), **_json_args(n.get("kwargs") or {}))
        else:
            raise ValueError(f"unknown node kind {kind!r}")
        built[nid] = c
    for n in nodes:
        for i, src in enumerate(n.get("inputs") or []):
            if src not in built:
                raise ValueError(f"node {n['id']}: unknown input {src}")
            built[n["id"]].set_input(i, built[src])
    return [built[s] for s in spec.get("sinks", [])]


class Dispatcher:
    """Executes one request against a PDBClient (runs on every rank)."""

    def __init__(self, client, jobs: Dict[str, Callable], health=None, registry: Optional[UDFRegistry] = None):
        self.client = client
        self.jobs = jobs
        self.health = health
        self.registry = registry or UDFRegistry()
        self.prepared: Dict[int, Any] = {}      # handle -> (CapturedJob | eager closure, input sets)

    def _prepare(self, req: dict):
        """Prepared (captured) job: the registered job's kernels recorded into a HIP graph on a GPU server
        (execution/graphs.py), a plain closure on a CPU server; run_prepared then only feeds inputs + replays."""
        c = self.client
        fn = self._job(req["job"])
        kw = _kwargs(req)
        inputs = [tuple(x) for x in (req.get("inputs") or [])]
        if not all(len(x) == 2 and all(isinstance(v, str) for v in x) for x in inputs):
            raise ValueError("inputs must be [db, set] pairs")
        if torch.device(c.device).type == "cuda":
            runner = c.capture_job(fn, c, inputs=inputs, **kw)
        else:
            fn(c, **kw)
            runner = (lambda: fn(c, **kw))
        h = len(self.prepared) + 1
        self.prepared[h] = (runner, inputs)
        return {"handle": h, "graph": not callable(runner)}

    def _run_prepared(self, req: dict):
        c = self.client
        h = int(req["handle"])
        if h not in self.prepared:
            raise KeyError(f"no prepared job {h}")
        runner, inputs = self.prepared[h]
        for f in req.get("feeds") or []:
            key = (f["db"], f["set"])
            if key not in inputs:
                raise ValueError(f"{key} is not an input of prepared job {h}")
            t = _dec_tensor(f)
            s = c.storage.get_set(*key)
            dst = s.panel
            if t.dim() != 2 or t.shape[0] > dst.shape[0] or t.shape[1] > dst.shape[1]:
                raise ValueError(f"feed {tuple(t.shape)} does not fit the input panel {tuple(dst.shape)}")
            dst[: t.shape[0], : t.shape[1]].copy_(t.to(dst.device, dst.dtype))
        if callable(runner):
            runner()
        else:
            runner.replay()
            torch.cuda.synchronize(runner.device)
        return {"ok": True}

    def handle(self, req: dict):
        op = req["op"]
        c = self.client
        if op == "ping":
            return {"rank": c.ctx.rank, "world_size": c.ctx.world_size, "jobs": sorted(self.jobs)}
        if op == "create_database":
            return c.create_database(req["name"])
        if op == "remove_database":
            return c.remove_database(req["name"])
        if op == "create_set":
            t = lookup_type(req["type"]) if req.get("type") else None   # only server-registered types
            return c.create_set(req["db"], req["set"], t, req.get("page_size"), dense=bool(req.get("dense", False)))
        if op == "remove_set":
            return c.remove_set(req["db"], req["set"])
        if op == "clear_set":
            return c.clear_set(req["db"], req["set"])
        if op == "send_data":
            recs = req.get("records")
            if recs and isinstance(recs[0], dict):
                t = c.get_set(req["db"], req["set"]).type
                recs = [t(**r) for r in recs]
            return c.send_data(req["db"], req["set"], recs if c.ctx.rank == 0 else None)
        if op == "get_set":
            objs: List[Any] = []
            for b in c.get_set_batches(req["db"], req["set"], gather=True):
                if b.type is not None:
                    objs.extend(b.to_objects())
                else:
                    cols = {k: _col_list(v) for k, v in b.columns.items()}
                    objs.extend(dict(zip(cols, row)) for row in zip(*cols.values()))
            lim = req.get("limit")
            return objs[:lim] if lim else objs
        if op == "list_sets":
            return c.list_sets(req.get("db"))
        if op == "list_nodes":
            nodes = c.list_nodes()
            if self.health is not None:
                st = self.health.status()
                for n in nodes:
                    n["health"] = st.get(n["rank"], {}).get("state")
            return nodes
        if op == "print_catalog":
            return c.print_catalog()
        if op == "flush":
            return c.flush_data()
        if op == "run":
            fn = self._job(req["job"])
            return _jsonable(fn(c, **_kwargs(req)))
        if op == "explain":
            sinks = self._job(req["job"])(c, **_kwargs(req))
            return c.explain(*(sinks if isinstance(sinks, (list, tuple)) else [sinks]))
        if op == "register_type":
            info = self.registry.register_module(req["module"])
            for tn in info["types"]:
                t = lookup_type(tn)
                if t is not None:
                    c.register_type(t)
            return info
        if op == "execute":
            sinks = build_graph(req["graph"], self.registry)
            st = c.execute_computations(*sinks, job_name=str(req.get("job_name", "remote-job")),
                                        pre_compile=bool(req.get("pre_compile", False)))
            return _jsonable({k: v for k, v in st.items() if k != "stages"} | {"stages": len(st.get("stages", []))})
        if op == "explain_graph":
            return c.explain(*build_graph(req["graph"], self.registry))
        if op == "prepare":
            return self._prepare(req)
        if op == "run_prepared":
            return self._run_prepared(req)
        raise ValueError(f"unknown request {op}")

    def _job(self, name: str) -> Callable:
        if name not in self.jobs:
            raise KeyError(f"job '{name}' is not registered on this server")
        return self.jobs[name]


def _enc_tensor(t) -> dict:
    """Exact-bytes tensor encoding for prepared-job feeds (raw bytes base64 + dtype + shape; no pickle)."""
    import base64

    t = t.detach().cpu().contiguous()
    return {"data": base64.b64encode(t.view(torch.uint8).numpy().tobytes()).decode("ascii"),
            "dtype": str(t.dtype).replace("torch.", ""), "shape": list(t.shape)}


def _dec_tensor(f: dict):
    import base64

    dt = getattr(torch, str(f["dtype"]), None)
    if not isinstance(dt, torch.dtype):
        raise ValueError(f"bad dtype {f.get('dtype')!r}")
    raw = bytearray(base64.b64decode(f["data"]))
    shape = [int(x) for x in f["shape"]]
    t = torch.frombuffer(raw, dtype=torch.uint8) if raw else torch.empty(0, dtype=torch.uint8)
    return t.view(dt).reshape(shape)


def _kwargs(req) -> dict:
    kw = req.get("kwargs") or {}
    if not isinstance(kw, dict) or not all(isinstance(k, str) for k in kw):
        raise ValueError("kwargs must be a JSON object")
    return kw


def _col_list(v):
    import torch

    if isinstance(v, torch.Tensor):
        return list(v.cpu())
    return list(v)


def _jsonable(v):
    import torch

    if isinstance(v, (str, int, float, bool)) or v is None or isinstance(v, (torch.Tensor, PDBObject)):
        return v
    if isinstance(v, dict):
        return {str(k): _jsonable(x) for k, x in v.items()}
    if isinstance(v, (list, tuple)):
        return [_jsonable(x) for x in v]
    return repr(v)


class _RWLock:
    """Readers-writer lock (writers preferred)."""

    def __init__(self):
        self._c = threading.Condition()
        self._readers = 0
        self._writer = False
        self._waiting_writers = 0

    def acquire(self, write: bool):
        with self._c:
            if write:
                self._waiting_writers += 1
                while self._writer or self._readers:
                    self._c.wait()
                self._waiting_writers -= 1
                self._writer = True
            else:
                while self._writer or self._waiting_writers:
                    self._c.wait()
                self._readers += 1

    def release(self, write: bool):
        with self._c:
            if write:
                self._writer = False
            else:
                self._readers -= 1
            self._c.notify_all()


# Requests answered by rank 0 alone from its catalog / plan state: no data, no collectives, never broadcast, so
# they run at any time, concurrently with jobs.
LOCAL_OPS = frozenset({"ping", "list_sets", "list_nodes", "print_catalog", "explain", "explain_graph"})


def _graph_sets(sinks):
    """(read sets, written sets) of a computation graph: its ScanSets and WriteSets."""
    from ..computations import ScanSet, WriteSet

    reads, writes, seen, todo = set(), set(), set(), list(sinks)
    while todo:
        c = todo.pop()
        if c is None or id(c) in seen:
            continue
        seen.add(id(c))
        if isinstance(c, WriteSet):
            writes.add((c.db, c.set_name))
        elif isinstance(c, ScanSet):
            reads.add((c.db, c.set_name))
        todo.extend(getattr(c, "inputs", []) or [])
    return reads, writes


class PDBFrontend:
    """Rank-0 socket server. ``serve_forever()`` blocks; ``start()`` runs it in a thread.

    Concurrency (reference: QuerySchedulerServer running independent jobs at once). Every connection has a
    handler thread; a request runs under locks of exactly what it touches instead of one global lock:
      * catalog / planning requests (``LOCAL_OPS``) take no lock and are never broadcast;
      * set-scoped requests take a readers-writer lock per (db, set) (ScanSets read, WriteSets write for
        declarative graphs; jobs registered with ``sets=(reads, writes)``), plus the database lock shared;
        requests of unknown footprint (registered jobs without declared sets, flush, prepared jobs) take the
        global lock exclusively. Locks are acquired in one sorted order (no lock-order deadlock);
      * a job runs on a job lane of its own (``PDBClient.job_lane``: its own engine and, on a GPU, its own HIP
        stream), so jobs on disjoint sets overlap;
      * with several ranks, every request that runs on all ranks is broadcast and executed in ONE global
        order (a ticket taken when it is broadcast; such requests run one at a time on every rank), so the
        collectives of different requests never interleave.
    """

    def __init__(self, client, host: str = "127.0.0.1", port: int = 8108, health=None,
                 jobs: Optional[Dict[str, Callable]] = None, udf_modules: Sequence[str] = ()):
        self.client = client
        self.jobs: Dict[str, Callable] = dict(jobs or {})
        self.registry = UDFRegistry(udf_modules)
        self.dispatcher = Dispatcher(client, self.jobs, health, self.registry)
        self.host, self.port = host, port
        self.set_locks: Dict[tuple, _RWLock] = {}
        self._locks_guard = threading.Lock()
        self.coll_lock = threading.Lock()     # multi-rank: broadcast requests execute one at a time, in order
        self.set_footprints: Dict[str, tuple] = {}     # registered job -> (reads, writes)
        self._lanes = itertools.count()
        self.active = 0
        self.max_active = 0                   # most requests executing at once (stats / tests)
        self._active_guard = threading.Lock()
        self._server: Optional[socketserver.ThreadingTCPServer] = None
        self.stopped = threading.Event()
        fe = self

        class Handler(socketserver.BaseRequestHandler):
            def handle(self):
                while True:
                    try:
                        req = recv_msg(self.request)
                    except (ConnectionError, OSError, ValueError):
                        return
                    resp = fe.execute(req)
                    send_msg(self.request, resp)
                    if isinstance(req, dict) and req.get("op") == "shutdown":
                        threading.Thread(target=fe.stop, daemon=True).start()
                        return

        self._handler = Handler

    def register_job(self, name: str, fn: Callable, sets: Optional[tuple] = None):
        """Expose ``fn(client, **kwargs)`` to remote clients under ``name`` (server-side only). ``sets`` =
        (reads, writes), each an iterable of (db, set): the job then runs concurrently with requests on other
        sets; without it the job takes the global lock."""
        self.jobs[name] = fn
        if sets is not None:
            r, w = sets
            self.set_footprints[name] = (frozenset(map(tuple, r)), frozenset(map(tuple, w)))
        return self

    # ------------------------------------------------------------------ locking
    def _lock_of(self, key) -> _RWLock:
        with self._locks_guard:
            lk = self.set_locks.get(key)
            if lk is None:
                lk = self.set_locks[key] = _RWLock()
            return lk

    def _footprint(self, req) -> List[tuple]:
        """[(lock key, write)] of a request, sorted: ("*",) global, ("db", name) database, ("set", db, set)."""
        op = req["op"]
        if op in LOCAL_OPS or op == "shutdown":
            return []
        reads, writes, glob = set(), set(), False
        if op in ("create_set", "remove_set", "clear_set", "send_data"):
            writes.add((req.get("db"), req.get("set")))
        elif op == "get_set":
            reads.add((req.get("db"), req.get("set")))
        elif op in ("create_database", "remove_database"):
            return [(("*",), False), (("db", str(req.get("name"))), True)]
        elif op == "execute":
            try:
                reads, writes = _graph_sets(build_graph(req["graph"], self.registry))
            except Exception:
                glob = True
        elif op == "run" and req.get("job") in self.set_footprints:
            reads, writes = (set(x) for x in self.set_footprints[req["job"]])
        else:
            glob = True
        if glob:
            return [(("*",), True)]
        keys = {("*",): False}
        for db, st in reads | writes:
            keys[("db", str(db))] = False
        for db, st in reads:
            keys[("set", str(db), str(st))] = keys.get(("set", str(db), str(st)), False)
        for db, st in writes:
            keys[("set", str(db), str(st))] = True
        return sorted(keys.items())

    def execute(self, req) -> dict:
        if not isinstance(req, dict) or not isinstance(req.get("op"), str):
            return {"ok": False, "error": "malformed request"}
        ctx = self.client.ctx
        op = req["op"]
        if op == "shutdown":
            with self.coll_lock:
                if ctx.distributed:
                    ctx.broadcast_object(req, src=0)
            return {"ok": True, "result": True}
        fp = self._footprint(req)
        held = []
        try:
            for key, write in fp:
                lk = self._lock_of(key)
                lk.acquire(write)
                held.append((lk, write))
            broadcast = ctx.distributed and op not in LOCAL_OPS
            with self._active_guard:
                self.active += 1
                self.max_active = max(self.max_active, self.active)
            try:
                if broadcast:
                    # one global order for everything every rank executes: broadcast and run under the same lock
                    with self.coll_lock:
                        ctx.broadcast_object(req, src=0)
                        return {"ok": True, "result": self._run(req)}
                return {"ok": True, "result": self._run(req)}
            finally:
                with self._active_guard:
                    self.active -= 1
        except Exception as e:
            return {"ok": False, "error": f"{type(e).__name__}: {e}", "trace": traceback.format_exc()}
        finally:
            for lk, write in reversed(held):
                lk.release(write)

    def _run(self, req):
        if req["op"] in LOCAL_OPS:
            return self.dispatcher.handle(req)
        with self.client.job_lane(next(self._lanes) % 4):
            return self.dispatcher.handle(req)

    def start(self):
        socketserver.ThreadingTCPServer.allow_reuse_address = True
        self._server = socketserver.ThreadingTCPServer((self.host, self.port), self._handler)
        self.port = self._server.server_address[1]
        threading.Thread(target=self._server.serve_forever, name="nsdb-frontend", daemon=True).start()
        return self

    def serve_forever(self):
        self.start()
        self.stopped.wait()

    def stop(self):
        if self._server is not None:
            self._server.shutdown()
            self._server.server_close()
        self.stopped.set()


def serve_worker(client, jobs: Optional[Dict[str, Callable]] = None, health=None, udf_modules: Sequence[str] = ()):
    """Non-zero ranks: execute every broadcast request until shutdown (WorkerMain)."""
    d = Dispatcher(client, dict(jobs or {}), health, UDFRegistry(udf_modules))
    while True:
        req = client.ctx.broadcast_object(None, src=0)
        if req.get("op") == "shutdown":
            return
        try:
            d.handle(req)
        except Exception:
            traceback.print_exc()


class RemotePDBClient:
    """Client side of the socket protocol (mirrors PDBClient's API)."""

    def __init__(self, host: str = "127.0.0.1", port: int = 8108, timeout: float = 600.0):
        self.sock = socket.create_connection((host, port), timeout=timeout)

    def _call(self, **req):
        send_msg(self.sock, req)
        resp = recv_msg(self.sock)
        if not resp.get("ok"):
            raise RuntimeError(resp.get("error"))
        return resp.get("result")

    def ping(self):
        return self._call(op="ping")

    def create_database(self, name):
        return self._call(op="create_database", name=name)

    def remove_database(self, name):
        return self._call(op="remove_database", name=name)

    def create_set(self, db, set_name, type_name=None, page_size=None, dense=False):
        return self._call(op="create_set", db=db, set=set_name, type=type_name, page_size=page_size, dense=dense)

    def remove_set(self, db, set_name):
        return self._call(op="remove_set", db=db, set=set_name)

    def clear_set(self, db, set_name):
        return self._call(op="clear_set", db=db, set=set_name)

    def send_data(self, db, set_name, records: List[Any]):
        return self._call(op="send_data", db=db, set=set_name, records=records)

    def get_set(self, db, set_name, limit: Optional[int] = None):
        return self._call(op="get_set", db=db, set=set_name, limit=limit)

    def list_sets(self, db=None):
        return self._call(op="list_sets", db=db)

    def list_nodes(self):
        return self._call(op="list_nodes")

    def print_catalog(self):
        return self._call(op="print_catalog")

    def flush_data(self):
        return self._call(op="flush")

    def run(self, job: str, **kwargs):
        """executeComputations of a server-registered job ``job(client, **kwargs)``."""
        return self._call(op="run", job=job, kwargs=kwargs)

    def explain(self, job: str, **kwargs):
        return self._call(op="explain", job=job, kwargs=kwargs)

    def register_type(self, module: str) -> dict:
        """PDBClient::registerType: the server imports an allow-listed UDF module (no code is sent)."""
        return self._call(op="register_type", module=module)

    registerType = register_type

    def execute_computations(self, *sinks, job_name: str = "remote-job", pre_compile: bool = False) -> dict:
        """PDBClient::executeComputations on a graph of :class:`RemoteComp` nodes, shipped declaratively."""
        return self._call(op="execute", graph=RemoteComp.graph(sinks), job_name=job_name, pre_compile=pre_compile)

    executeComputations = execute_computations

    def prepare_job(self, job: str, inputs=(), **kwargs) -> dict:
        """Prepare a registered job for repeated runs: on a GPU server its kernels are captured into a HIP
        graph once; returns {"handle", "graph"}."""
        return self._call(op="prepare", job=job, kwargs=kwargs, inputs=[list(x) for x in inputs])

    def run_prepared(self, handle: int, feeds: Optional[dict] = None) -> dict:
        """Write ``feeds`` ({(db, set): 2-D tensor}) into the prepared job's input sets and run it (a graph
        replay on a GPU server)."""
        fs = [dict(db=k[0], set=k[1], **_enc_tensor(v)) for k, v in (feeds or {}).items()]
        return self._call(op="run_prepared", handle=handle, feeds=fs)

    def explain_graph(self, *sinks) -> str:
        return self._call(op="explain_graph", graph=RemoteComp.graph(sinks))

    def shutdown(self):
        try:
            return self._call(op="shutdown")
        finally:
            self.sock.close()

    def close(self):
        self.sock.close()


class RemoteComp:
    """Client-side node of a declarative computation graph: a server-registered computation class name
    + JSON constructor arguments, or a scan / write of a named set.

        scan = RemoteComp.scan("db", "emps", "Employee")
        agg = RemoteComp("SalaryByDept").set_input(RemoteComp("OlderThan", 40).set_input(scan))
        rc.execute_computations(RemoteComp.write("db", "out", "DepartmentTotal").set_input(agg))
    """

    def __init__(self, cls_name: str, *args, **kwargs):
        self.kind = "comp"
        self.cls_name = cls_name
        self.args, self.kwargs = list(args), dict(kwargs)
        self.inputs: Dict[int, "RemoteComp"] = {}
        self.db = self.set_name = self.type_name = None

    @staticmethod
    def scan(db: str, set_name: str, type_name: Optional[str] = None) -> "RemoteComp":
        n = RemoteComp("ScanSet")
        n.kind, n.db, n.set_name, n.type_name = "scan", db, set_name, type_name
        return n

    @staticmethod
    def write(db: str, set_name: str, type_name: Optional[str] = None) -> "RemoteComp":
        n = RemoteComp("WriteSet")
        n.kind, n.db, n.set_name, n.type_name = "write", db, set_name, type_name
        return n

    def set_input(self, *a) -> "RemoteComp":
        i, comp = (0, a[0]) if len(a) == 1 else a
        self.inputs[int(i)] = comp
        return self

    setInput = set_input

    @staticmethod
    def graph(sinks) -> dict:
        ids: Dict[int, int] = {}
        nodes: List[dict] = []

        def visit(n: "RemoteComp") -> int:
            if id(n) in ids:
                return ids[id(n)]
            ins = [visit(n.inputs[i]) for i in sorted(n.inputs)]
            nid = len(nodes)
            ids[id(n)] = nid
            d = {"id": nid, "kind": n.kind, "inputs": ins}
            if n.kind == "comp":
                d.update({"class": n.cls_name, "args": n.args, "kwargs": n.kwargs})
            else:
                d.update({"db": n.db, "set": n.set_name, "type": n.type_name})
            nodes.append(d)
            return nid

        flat = []
        for s in sinks:
            flat.extend(s if isinstance(s, (list, tuple)) else [s])
        return {"nodes": nodes, "sinks": [visit(s) for s in flat]}


__all__ = ["PDBFrontend", "RemotePDBClient", "RemoteComp", "UDFRegistry", "build_graph", "serve_worker",
           "Dispatcher"]
