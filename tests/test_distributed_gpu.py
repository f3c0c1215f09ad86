"""Two ranks on the one GPU of a test box (gloo process group: RCCL refuses two ranks on one device; the data
collectives stage through the host): the distributed engine on device-resident sets — hash-partitioned joins and
shuffled aggregations over the device relational kernels, string columns (views) on the wire — checked against
the pandas oracle. The same code runs one rank per GPU over RCCL on an 8-GPU node."""
import math
import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

QUERIES = ("q01", "q03", "q04", "q06", "q12", "q13")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, ws, port, out_dir, device="cuda:0"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(ws),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        from netsdb_amd import _ext
        from netsdb_amd.client import PDBClient
        from netsdb_amd.models import tpch, tpch_gen
        from netsdb_amd.parallel.comm import ClusterContext

        dev = torch.device(device)
        if dev.type == "cuda":
            torch.cuda.set_device(dev)
        ctx = ClusterContext(rank, ws, dev, "gloo")
        t = tpch_gen.generate_fast(0.01, seed=5)
        c = PDBClient(ctx=ctx, root=tempfile.mkdtemp(), device=dev, broadcast_threshold=0)   # partitioned joins
        # rank 0's rows are dispatched over the ranks (send_data, round-robin), each rank's share on the device
        tpch.load(c, "tpch", t, device=dev)
        res = {q: tpch.QUERIES[q](c, "tpch") for q in QUERIES}
        res["_hip"] = _ext.hip() is not None
        torch.save(res, os.path.join(out_dir, f"r{rank}.pt"))
    except BaseException:
        import traceback
        with open(os.path.join(out_dir, f"err{rank}.txt"), "w") as fh:   # every rank's own traceback
            fh.write(traceback.format_exc())
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_tpch_two_ranks_on_one_gpu_vs_pandas():
    from netsdb_amd.models import tpch, tpch_gen

    out = tempfile.mkdtemp()
    try:
        mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    except Exception:
        errs = [open(os.path.join(out, f)).read() for f in sorted(os.listdir(out)) if f.startswith("err")]
        raise AssertionError("rank failures:\n" + "\n".join(errs))
    res = [torch.load(os.path.join(out, f"r{r}.pt"), weights_only=False) for r in range(2)]
    t = tpch_gen.generate_fast(0.01, seed=5)
    f = tpch.frames(t)
    for r in res:
        assert r["_hip"]
    for q in QUERIES:
        ref = tpch.reference(q, t, f=f)
        for r in res:
            got = r[q]
            if isinstance(ref, float):
                assert math.isclose(got, ref, rel_tol=1e-9, abs_tol=1e-6), q
                continue
            if q == "q01":
                ref = sorted(ref, key=lambda x: (x["l_returnflag"], x["l_linestatus"]))
            elif q in ("q04", "q12"):
                ref = sorted(ref, key=lambda x: x[list(x)[0]])
            assert len(got) == len(ref), q
            for g, e in zip(got, ref):
                for k, v in e.items():
                    ok = math.isclose(g[k], v, rel_tol=1e-9, abs_tol=1e-6) if isinstance(v, float) else g[k] == v
                    assert ok, (q, g, e)
