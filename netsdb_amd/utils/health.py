"""Failure detection (reference: the master's worker liveness tracking in
src/serverFunctionalities (ResourceManagerServer / DistributedStorageManagerServer node lists,
scripts/checkProcess.sh) and PDBAlarm/PDBBuzzer work signalling in src/work).

Every rank runs a daemon thread that publishes a heartbeat (monotonic timestamp + progress
counter) into a key-value store (the torch.distributed TCPStore the process group rendezvous
already uses, or a standalone one).  :meth:`HeartbeatMonitor.status` reports each rank alive /
suspect / dead; :meth:`check` raises :class:`NodeFailure` so a driver can abort before entering a
collective that would hang on a dead peer.
"""
from __future__ import annotations

import threading
import time
from typing import Dict, List, Optional


class NodeFailure(RuntimeError):
    pass


class HeartbeatMonitor:
    def __init__(self, store, rank: int, world_size: int, interval: float = 0.5, timeout: float = 5.0,
                 prefix: str = "nsdb_hb"):
        self.store, self.rank, self.world_size = store, rank, world_size
        self.interval, self.timeout, self.prefix = interval, timeout, prefix
        self.progress = 0
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self._t0 = time.time()

    @staticmethod
    def standalone(host: str, port: int, rank: int, world_size: int, **kw) -> "HeartbeatMonitor":
        import torch.distributed as dist

        import datetime

        store = dist.TCPStore(host, port, None, rank == 0, timeout=datetime.timedelta(seconds=30),
                              wait_for_workers=False)
        return HeartbeatMonitor(store, rank, world_size, **kw)

    def beat(self):
        self.store.set(f"{self.prefix}/{self.rank}", f"{time.time():.6f}:{self.progress}")

    def start(self):
        self.beat()

        def loop():
            while not self._stop.wait(self.interval):
                try:
                    self.beat()
                except Exception:
                    return

        self._thread = threading.Thread(target=loop, name="nsdb-heartbeat", daemon=True)
        self._thread.start()
        return self

    def stop(self):
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=2 * self.interval)

    def mark_progress(self):
        self.progress += 1

    def status(self) -> Dict[int, dict]:
        now = time.time()
        out = {}
        for r in range(self.world_size):
            key = f"{self.prefix}/{r}"
            try:
                if not self.store.check([key]):
                    out[r] = {"state": "unknown", "age": None, "progress": None}
                    continue
                ts, prog = self.store.get(key).decode().split(":")
                age = now - float(ts)
                state = "alive" if age < self.timeout else ("suspect" if age < 2 * self.timeout else "dead")
                out[r] = {"state": state, "age": age, "progress": int(prog)}
            except Exception as e:  # store unreachable
                out[r] = {"state": "unreachable", "age": None, "progress": None, "error": str(e)}
        return out

    def dead_ranks(self) -> List[int]:
        return [r for r, s in self.status().items() if s["state"] in ("dead", "unreachable")]

    def check(self):
        dead = self.dead_ranks()
        if dead:
            raise NodeFailure(f"ranks {dead} stopped heartbeating (timeout {self.timeout}s)")


__all__ = ["HeartbeatMonitor", "NodeFailure"]
