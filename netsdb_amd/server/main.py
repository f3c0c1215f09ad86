"""Start a netsdb_amd cluster: ``python -m netsdb_amd.server.main --port 8108`` (one process) or
``torchrun --nproc-per-node N --master-addr 127.0.0.1 -m netsdb_amd.server.main --port 8108``
(one process per GPU; rank 0 serves clients, all ranks execute).  Mirrors the reference's
startPseudoCluster.py / startMaster.sh + startWorkers.sh."""
from __future__ import annotations

import argparse
import os


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default=None,
                    help="pdbSettings-style settings file (default: $NSDB_CONF or ./conf/pdbSettings.conf if present); "
                         "command-line flags override it")
    ap.add_argument("--host", default=None)
    ap.add_argument("--port", type=int, default=None)
    ap.add_argument("--root", default=None, help="data directory (catalog + page files)")
    ap.add_argument("--page-size-mb", type=int, default=None)
    ap.add_argument("--resume", action="store_true", help="reopen the sets persisted in --root")
    ap.add_argument("--heartbeat-port", type=int, default=0)
    ap.add_argument("--jobs", action="append", default=[],
                    help="operator-chosen module exposing a JOBS dict {name: fn(client, **kw)} to clients")
    ap.add_argument("--udf-modules", action="append", default=[],
                    help="module prefix remote clients may register_type() (UDF classes + record types)")
    a = ap.parse_args(argv)

    from ..utils.config import Configuration, find_config

    path = find_config(a.config)
    conf = Configuration.load(path) if path else Configuration()
    if a.config and not path:
        ap.error(f"settings file {a.config} not found")
    host = a.host or conf.my_ip
    port = a.port if a.port is not None else conf.port
    page_size = (a.page_size_mb << 20) if a.page_size_mb is not None else conf.page_size

    from ..client import PDBClient
    from ..parallel.comm import ClusterContext
    from ..utils.health import HeartbeatMonitor
    from .frontend import PDBFrontend, serve_worker

    import importlib

    jobs = {}
    for mod in a.jobs:
        jobs.update(getattr(importlib.import_module(mod), "JOBS"))
    ctx = ClusterContext.from_env()
    root = a.root or os.path.join(os.getcwd(), conf.root_directory)
    kw = conf.client_kwargs()
    kw["page_size"] = page_size
    client = PDBClient(ctx=ctx, root=os.path.join(root, f"rank{ctx.rank}"), resume=a.resume, **kw)
    health = None
    if a.heartbeat_port:
        health = HeartbeatMonitor.standalone(host, a.heartbeat_port, ctx.rank, ctx.world_size).start()
        ctx.attach_health(health)      # every engine collective waits under the heartbeat watchdog
    if ctx.rank == 0:
        fe = PDBFrontend(client, host, port, health, jobs=jobs, udf_modules=a.udf_modules)
        print(f"[netsdb_amd] master listening on {host}:{fe.start().port} (world {ctx.world_size})", flush=True)
        fe.stopped.wait()
    else:
        serve_worker(client, jobs, health, a.udf_modules)
    if health:
        health.stop()


if __name__ == "__main__":
    main()
