"""Tracing (reference: src/pdbServer/headers/PDBLogger.h, PDBDebug.h, gen_trace.sql / tpchGenTrace
job traces used by the self-learning optimizer).

:class:`Tracer` records nested spans (job, stage, op) with host wall time and, with ``device_time=True``, the
device time of each span from a HIP event pair on the current stream (:class:`DeviceTimer`: recorded without a
synchronisation, resolved when the events have completed), exports Chrome-trace JSON (viewable in Perfetto) and
feeds the self-learning history (:mod:`netsdb_amd.selflearning`). The engine times every stage the same way
(``JobStats["stages"][i]["device_seconds"]``).  When ``roctx=True`` spans are also emitted as ROCTx ranges
(``torch.cuda.nvtx`` maps to roctx on ROCm) so they show up in ``rocprofv3 --marker-trace``.
"""
from __future__ import annotations

import contextlib
import json
import logging
import os
import threading
import time
from typing import Any, Dict, List, Optional

_log = logging.getLogger("netsdb_amd")


def get_logger(name: str = "netsdb_amd", level: Optional[str] = None) -> logging.Logger:
    lg = logging.getLogger(name)
    if not lg.handlers:
        h = logging.StreamHandler()
        h.setFormatter(logging.Formatter("[%(asctime)s %(name)s %(levelname)s] %(message)s"))
        lg.addHandler(h)
    lg.setLevel(level or os.environ.get("NSDB_LOG_LEVEL", "WARNING"))
    return lg


class DeviceTimer:
    """Device time of host-side regions from HIP event pairs recorded on the current stream, resolved later without a
    synchronisation per region: :meth:`start` / :meth:`stop` enqueue the two events, :meth:`resolve` turns every pair
    whose end event has completed (``block=True``: waits for the last one) into seconds written to ``rec[key]``.
    The measured span is the stream's time from the first event to the second: the kernels of the region plus any
    time the stream sat idle in between (host work of the region that did not overlap earlier kernels)."""

    def __init__(self):
        self.pending: List[tuple] = []
        self._lock = threading.Lock()

    @staticmethod
    def available(device=None) -> bool:
        try:
            import torch

            if device is not None and torch.device(device).type != "cuda":
                return False
            return torch.cuda.is_available()
        except Exception:
            return False

    def start(self):
        import torch

        e = torch.cuda.Event(enable_timing=True)
        e.record()
        return e

    def stop(self, e0, rec: dict, key: str = "device_seconds"):
        import torch

        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        rec[key] = None
        with self._lock:
            self.pending.append((e0, e1, rec, key))

    def resolve(self, block: bool = False) -> int:
        """Fill in the pairs that have completed (all of them when ``block``); returns how many are still pending.
        A no-op while a HIP-graph capture records on this thread's stream (an event query would invalidate it)."""
        if self.pending:
            import torch

            if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
                return len(self.pending)
        with self._lock:
            todo, self.pending = self.pending, []
        keep = []
        for e0, e1, rec, key in todo:
            if block:
                e1.synchronize()
            elif not e1.query():
                keep.append((e0, e1, rec, key))
                continue
            rec[key] = e0.elapsed_time(e1) / 1e3
        with self._lock:
            self.pending = keep + self.pending
            return len(self.pending)


class Tracer:
    def __init__(self, enabled: bool = True, roctx: bool = False, rank: int = 0, device_time: bool = False):
        self.enabled = enabled
        self.roctx = roctx
        self.rank = rank
        # device_time: every span also carries a HIP event pair; its "device_us" arg is filled in by resolve()
        self.device_time = device_time
        self.device = DeviceTimer()
        self.events: List[Dict[str, Any]] = []
        self._lock = threading.Lock()
        self._t0 = time.perf_counter()

    def resolve(self, block: bool = True) -> int:
        """Resolve the spans' device times (see DeviceTimer.resolve)."""
        n = self.device.resolve(block)
        for e in self.events:
            d = e["args"].pop("_dev", None) if "_dev" in e["args"] else None
            if d is not None:
                if d.get("s") is None:
                    e["args"]["_dev"] = d
                else:
                    e["args"]["device_us"] = d["s"] * 1e6
        return n

    @contextlib.contextmanager
    def span(self, name: str, **args):
        if not self.enabled:
            yield
            return
        dev0 = self.device.start() if self.device_time and DeviceTimer.available() else None
        pushed = False
        if self.roctx:
            try:
                import torch

                torch.cuda.nvtx.range_push(name)
                pushed = True
            except Exception:
                pass
        t = time.perf_counter()
        try:
            yield
        finally:
            dt = time.perf_counter() - t
            if pushed:
                import torch

                torch.cuda.nvtx.range_pop()
            if dev0 is not None:
                box: Dict[str, Any] = {}
                self.device.stop(dev0, box, "s")
                args = dict(args, _dev=box)
            with self._lock:
                self.events.append({"name": name, "ph": "X", "ts": (t - self._t0) * 1e6, "dur": dt * 1e6,
                                    "pid": self.rank, "tid": threading.get_ident() % 100000, "args": args})

    def summary(self) -> Dict[str, Dict[str, float]]:
        agg: Dict[str, Dict[str, float]] = {}
        for e in self.events:
            a = agg.setdefault(e["name"], {"count": 0, "total_us": 0.0})
            a["count"] += 1
            a["total_us"] += e["dur"]
            if "device_us" in e["args"]:
                a["device_us"] = a.get("device_us", 0.0) + e["args"]["device_us"]
        return agg

    def export_chrome(self, path: str):
        if self.device_time:
            self.resolve(block=True)
        evs = [dict(e, args={k: v for k, v in e["args"].items() if k != "_dev"}) for e in self.events]
        with open(path, "w") as f:
            json.dump({"traceEvents": evs}, f, default=str)

    def clear(self):
        self.events.clear()


__all__ = ["Tracer", "DeviceTimer", "get_logger"]
