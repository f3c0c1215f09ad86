"""Master front end (rank 0) + SPMD worker loop + remote client.

Security model: the wire protocol never imports code or names arbitrary functions.  The server
operator registers UDF jobs up front (``PDBFrontend.register_job(name, fn)`` or the
``--jobs module`` flag of server/main.py, resolved on the server at start-up); remote clients can
only invoke those jobs by name with JSON arguments, and can only refer to record types that are
already registered server-side.  The listener binds to 127.0.0.1 unless told otherwise.
"""
from __future__ import annotations

import socket
import socketserver
import threading
import traceback
from typing import Any, Callable, Dict, List, Optional

from ..objects.record import PDBObject, lookup_type
from .protocol import recv_msg, send_msg


class Dispatcher:
    """Executes one request against a PDBClient (runs on every rank)."""

    def __init__(self, client, jobs: Dict[str, Callable], health=None):
        self.client = client
        self.jobs = jobs
        self.health = health

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
        raise ValueError(f"unknown request {op}")

    def _job(self, name: str) -> Callable:
        if name not in self.jobs:
            raise KeyError(f"job '{name}' is not registered on this server")
        return self.jobs[name]


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


class PDBFrontend:
    """Rank-0 socket server. ``serve_forever()`` blocks; ``start()`` runs it in a thread."""

    def __init__(self, client, host: str = "127.0.0.1", port: int = 8108, health=None,
                 jobs: Optional[Dict[str, Callable]] = None):
        self.client = client
        self.jobs: Dict[str, Callable] = dict(jobs or {})
        self.dispatcher = Dispatcher(client, self.jobs, health)
        self.host, self.port = host, port
        self.lock = threading.Lock()
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

    def register_job(self, name: str, fn: Callable):
        """Expose ``fn(client, **kwargs)`` to remote clients under ``name`` (server-side only)."""
        self.jobs[name] = fn
        return self

    def execute(self, req) -> dict:
        if not isinstance(req, dict) or not isinstance(req.get("op"), str):
            return {"ok": False, "error": "malformed request"}
        with self.lock:  # requests are serialised: every rank executes them in the same order
            ctx = self.client.ctx
            if ctx.distributed:
                ctx.broadcast_object(req, src=0)
            if req["op"] == "shutdown":
                return {"ok": True, "result": True}
            try:
                return {"ok": True, "result": self.dispatcher.handle(req)}
            except Exception as e:
                return {"ok": False, "error": f"{type(e).__name__}: {e}", "trace": traceback.format_exc()}

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


def serve_worker(client, jobs: Optional[Dict[str, Callable]] = None, health=None):
    """Non-zero ranks: execute every broadcast request until shutdown (WorkerMain)."""
    d = Dispatcher(client, dict(jobs or {}), health)
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

    def shutdown(self):
        try:
            return self._call(op="shutdown")
        finally:
            self.sock.close()

    def close(self):
        self.sock.close()


__all__ = ["PDBFrontend", "RemotePDBClient", "serve_worker", "Dispatcher"]
