"""Tracing (reference: src/pdbServer/headers/PDBLogger.h, PDBDebug.h, gen_trace.sql / tpchGenTrace
job traces used by the self-learning optimizer).

:class:`Tracer` records nested spans (job, stage, op) with wall time and optional GPU-event
time, exports Chrome-trace JSON (viewable in Perfetto) and feeds the self-learning history
(:mod:`netsdb_amd.selflearning`).  When ``roctx=True`` spans are also emitted as ROCTx ranges
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


class Tracer:
    def __init__(self, enabled: bool = True, roctx: bool = False, rank: int = 0):
        self.enabled = enabled
        self.roctx = roctx
        self.rank = rank
        self.events: List[Dict[str, Any]] = []
        self._lock = threading.Lock()
        self._t0 = time.perf_counter()

    @contextlib.contextmanager
    def span(self, name: str, **args):
        if not self.enabled:
            yield
            return
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
            with self._lock:
                self.events.append({"name": name, "ph": "X", "ts": (t - self._t0) * 1e6, "dur": dt * 1e6,
                                    "pid": self.rank, "tid": threading.get_ident() % 100000, "args": args})

    def summary(self) -> Dict[str, Dict[str, float]]:
        agg: Dict[str, Dict[str, float]] = {}
        for e in self.events:
            a = agg.setdefault(e["name"], {"count": 0, "total_us": 0.0})
            a["count"] += 1
            a["total_us"] += e["dur"]
        return agg

    def export_chrome(self, path: str):
        with open(path, "w") as f:
            json.dump({"traceEvents": self.events}, f)

    def clear(self):
        self.events.clear()


__all__ = ["Tracer", "get_logger"]
