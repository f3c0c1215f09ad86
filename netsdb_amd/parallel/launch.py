"""Single-node rank launcher for the benchmark entry points (bench.py, scripts/bench_la_matmul.py,
scripts/bench_dedup.py): ``--gpus N`` without torchrun starts N rank processes of the same script, one per GPU.

The launching parent never touches the GPU: it counts devices from the environment / the KFD topology (no HIP
call, no torch.cuda call), starts the ranks as ordinary child processes (no exec of a GPU-initialised process)
with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT set, and returns the first non-zero exit
code. Rank r binds cuda:r (ClusterContext.from_env); on a host without GPUs the ranks run gloo on the CPU, which is
how the CPU contract tests rehearse the 2- and 8-rank launches.

Reference: the netsDB pseudo-cluster start-up scripts (scripts/startPseudoCluster.py, startWorkers.sh) that bring
up one worker process per node.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys
from typing import Optional, Sequence


def visible_gpus() -> int:
    """GPUs a child process would see, WITHOUT any HIP / torch.cuda call: HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES /
    CUDA_VISIBLE_DEVICES when set, else the KFD topology nodes with a non-zero gpu_id. -1 when it cannot be told
    (rank 0's own device check then decides)."""
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            return len([x for x in v.split(",") if x.strip() not in ("", "-1")])
    topo = "/sys/class/kfd/kfd/topology/nodes"
    try:
        n = 0
        for node in os.listdir(topo):
            try:
                with open(os.path.join(topo, node, "gpu_id")) as f:
                    n += int(f.read().strip() or 0) != 0
            except (OSError, ValueError):
                continue
        return n
    except OSError:
        return -1


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def should_launch(n: int) -> bool:
    """True in the parent of a ``--gpus N`` (N > 1) run that was not started by torchrun."""
    return n > 1 and "WORLD_SIZE" not in os.environ


def launch_ranks(script: str, n: int, argv: Sequence[str], quiet_ranks: bool = True,
                 env_extra: Optional[dict] = None) -> int:
    """Start ``n`` ranks of ``script`` with ``argv`` and wait for all of them. Rank 0 keeps this process's stdout
    (its JSON line is the result); the other ranks' stdout is discarded when ``quiet_ranks``. A failing rank kills
    the others (no rank is left waiting in a collective)."""
    ndev = visible_gpus()
    if 0 < ndev < n:
        print(f"[launch] --gpus {n} but only {ndev} GPUs visible", file=sys.stderr)
        return 2
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if env_extra:
            env.update(env_extra)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(script)] + list(argv), env=env,
                                      stdout=None if (r == 0 or not quiet_ranks) else subprocess.DEVNULL))
    import time

    rc = 0
    try:
        while True:                      # poll every rank: whichever fails first ends the run
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = bad[0]
                break
            if all(c == 0 for c in codes):
                break
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return rc


__all__ = ["visible_gpus", "free_port", "should_launch", "launch_ranks"]
