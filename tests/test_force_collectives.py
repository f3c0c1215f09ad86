"""One-rank process groups that run the MULTI-rank code paths (``ClusterContext(force_collectives=True)``).

A one-GPU box cannot host two RCCL ranks (RCCL refuses two ranks on one device), so without this mode the RCCL
branches of the engine — the streaming shuffle's device-buffer all-to-alls, partitioned join builds / probes and
shuffled aggregations, the all-gathered N-chunk matmul pipeline (``_allgather_n``) and the overlapped K-split
reduce-scatter (``_kpartial_overlapped``), the gloo metadata group next to RCCL — would never execute on hardware.
Here a world_size-1 group runs every one of those branches (collectives on, nothing short-circuited) and the
results must equal the single-process run:

* CPU: gloo, world_size 1 (runs in the CPU suite);
* GPU: RCCL (``nccl``) world_size 1 on cuda:0 with the gloo metadata group — device buffers on the wire.

Reference: the worker pipeline's shuffle / broadcast / hash-partition sinks
(src/queryExecution/headers/PipelineStage.h:167-173, ShuffleSink.h:17)."""
import math
import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


TPCH_Q = ("q01", "q03", "q04", "q06", "q12", "q13", "q22")


def _scenarios(ctx, dev):
    """Everything a multi-rank job does, on this context. Returns host-side results."""
    from netsdb_amd.client import PDBClient
    from netsdb_amd.computations import ScanSet, WriteSet
    from netsdb_amd.la import computations as L
    from netsdb_amd.models import blocks as B
    from netsdb_amd.models import ff, tpch, tpch_gen

    res = {"distributed": ctx.distributed}
    # LA: A %*% B over row-partitioned operands (all-gather N-chunk pipeline), A '* B (K-split reduce-scatter)
    c = PDBClient(ctx=ctx, root=tempfile.mkdtemp(), device=dev)
    c.create_database("LA_db")
    g = torch.Generator().manual_seed(7)
    A = torch.rand(80, 80, generator=g) - 0.5
    Bm = torch.rand(80, 48, generator=g) - 0.5
    B.load_tensor(c, "LA_db", "A", A, 16, 16, dtype=torch.float32, partition_rows=True)
    B.load_tensor(c, "LA_db", "B", Bm, 16, 16, dtype=torch.float32, partition_rows=True)
    n0 = ctx.stats["collectives"]
    for tag, jcls, ref in (("mul", L.LAMultiply1Join, A @ Bm), ("tmul", L.LATransposeMultiply1Join, A.t() @ Bm)):
        c.create_set("LA_db", f"C_{tag}", None, dense=True)
        j = jcls()
        j.set_input(0, ScanSet("LA_db", "A"))
        j.set_input(1, ScanSet("LA_db", "B"))
        st = c.execute_computations(WriteSet("LA_db", f"C_{tag}").set_input(L.LAMultiply2Aggregate().set_input(j)))
        C = B.to_tensor(c, "LA_db", f"C_{tag}").float().cpu()
        res[tag] = (C - ref).abs().max().item()
        res[f"{tag}_fused"] = st.get("fused_ops")
    res["la_collectives"] = ctx.stats["collectives"] - n0
    res["C_mul"] = B.to_tensor(c, "LA_db", "C_mul").float().cpu()
    res["dist_stats"] = dict(getattr(c.engine, "dist_stats", {}))
    # a second write into the same dense set: merged by block ownership, not summed
    c.create_set("LA_db", "C_twice", None, dense=True)
    for _ in range(2):
        j = L.LAMultiply1Join()
        j.set_input(0, ScanSet("LA_db", "A"))
        j.set_input(1, ScanSet("LA_db", "B"))
        c.execute_computations(WriteSet("LA_db", "C_twice").set_input(L.LAMultiply2Aggregate().set_input(j)))
    res["twice"] = (B.to_tensor(c, "LA_db", "C_twice").float().cpu() - A @ Bm).abs().max().item()
    # the ownership merge keeps a float64 panel in float64 and works band by band (several bands here)
    c.create_set("LA_db", "C_f64", None, dense=True)
    s64 = c.storage.get_set("LA_db", "C_f64")
    s64.define(70, 50, 16, 16, dtype=torch.float64, device=dev)
    vals = (1.0 + torch.arange(70 * 50, dtype=torch.float64) * 1e-13).reshape(70, 50).to(dev)
    s64.matrix().copy_(vals)
    old_band = c.engine.MERGE_BAND_BYTES
    c.engine.MERGE_BAND_BYTES = 16 * 50 * 8 * 2        # two block rows per band: 3 bands for 5 block rows
    try:
        c.engine._merge_dense_output(s64, written=[(torch.tensor([0, 2, 4]), torch.tensor([1, 3, 0]))])
    finally:
        c.engine.MERGE_BAND_BYTES = old_band
    res["merge_f64"] = (s64.matrix().cpu() - vals.cpu()).abs().max().item()
    res["merge_f64_dtype"] = str(s64.matrix().dtype)
    # FF inference with row-partitioned inputs
    c2 = PDBClient(ctx=ctx, root=tempfile.mkdtemp(), device=dev)
    ff.load_model(c2, "ff", 64, 96, 32, 24, 16, 32, dtype=torch.float32, partition_inputs=True)
    ff.inference_unit(c2, "ff", "w1", "wo", "inputs", "b1", "bo", "output")
    gt = lambda n: B.to_tensor(c2, "ff", n).float().cpu()  # noqa: E731
    out = gt("output")
    ref = ff.reference_inference(gt("inputs"), gt("w1"), gt("b1"), gt("wo"), gt("bo"))
    res["ff"] = (out - ref).abs().max().item()
    res["ff_out"] = out
    # TPC-H through hash-partitioned joins and shuffled aggregations (streaming shuffle)
    t = tpch_gen.generate_fast(0.005, seed=5)
    c3 = PDBClient(ctx=ctx, root=tempfile.mkdtemp(), device=dev, broadcast_threshold=0)
    tpch.load(c3, "tpch", t, device=dev)
    n0 = ctx.stats["collectives"]
    for q in TPCH_Q:
        res[q] = tpch.QUERIES[q](c3, "tpch")
    res["tpch_collectives"] = ctx.stats["collectives"] - n0
    res["shuffles"] = dict(c3.engine.shuffle_stats)
    return res


def _worker(rank, port, out_dir, backend, device):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    try:
        dev = torch.device(device)
        kw = {}
        if dev.type == "cuda":
            torch.cuda.set_device(dev)
            kw["device_id"] = dev
        dist.init_process_group(backend, rank=0, world_size=1, **kw)
        from netsdb_amd.parallel.comm import ClusterContext

        # the single-process run of the same scenarios first (the reference), then the forced-collective run
        single = _scenarios(ClusterContext(device=dev), dev)
        ctx = ClusterContext(0, 1, dev, backend, force_collectives=True).attach_meta_group()
        res = _scenarios(ctx, dev)
        res["single"] = single
        res["meta_group"] = ctx.meta_group is not None
        if dev.type == "cuda":
            torch.cuda.synchronize()
            from netsdb_amd import _ext

            res["_hip"] = _ext.hip() is not None
        torch.save(res, os.path.join(out_dir, "r0.pt"))
    except BaseException:
        import traceback

        with open(os.path.join(out_dir, "err0.txt"), "w") as fh:
            fh.write(traceback.format_exc())
        raise
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def _run(backend, device):
    out = tempfile.mkdtemp()
    try:
        mp.spawn(_worker, args=(_free_port(), out, backend, device), nprocs=1, join=True)
    except Exception:
        errs = [open(os.path.join(out, f)).read() for f in sorted(os.listdir(out)) if f.startswith("err")]
        raise AssertionError("rank failure:\n" + "\n".join(errs))
    return torch.load(os.path.join(out, "r0.pt"), weights_only=False)


def _check(r, tol=1e-4):
    from netsdb_amd.models import tpch, tpch_gen

    assert r["distributed"] is True and r["single"]["distributed"] is False
    # vs fp64 (tol: bf16 MFMA on the GPU), and vs the single-process run of the same scenario
    assert r["mul"] < tol and r["tmul"] < tol and r["twice"] < tol and r["ff"] < tol, r
    assert r["merge_f64"] == 0.0 and r["merge_f64_dtype"] == "torch.float64", r["merge_f64"]
    same = 1e-5 if tol <= 1e-4 else 1e-2     # the GPU's split / chunk order may round differently in bf16
    assert torch.allclose(r["C_mul"], r["single"]["C_mul"], rtol=same, atol=same)
    assert torch.allclose(r["ff_out"], r["single"]["ff_out"], rtol=same, atol=same * 0.1)
    assert any("matmul" in f for f in r["mul_fused"]) and any("matmul" in f for f in r["tmul_fused"])
    assert r["la_collectives"] >= 2, r["la_collectives"]
    # the all-gathered N-chunk pipeline (_allgather_n) and the K-split reduce-scatter (_kpartial_overlapped)
    assert r["dist_stats"].get("allgather_n", 0) >= 1 and r["dist_stats"].get("kpartial", 0) >= 1, r["dist_stats"]
    assert r["tpch_collectives"] > 0
    assert r["shuffles"].get("shuffles", 0) > 0, r["shuffles"]
    t = tpch_gen.generate_fast(0.005, seed=5)
    f = tpch.frames(t)
    for q in TPCH_Q:
        ref = tpch.reference(q, t, f=f)
        got = r[q]
        if isinstance(ref, float):
            assert math.isclose(got, ref, rel_tol=1e-9, abs_tol=1e-6), q
            continue
        if q == "q01":
            ref = sorted(ref, key=lambda x: (x["l_returnflag"], x["l_linestatus"]))
        elif q in ("q04", "q12", "q22"):
            ref = sorted(ref, key=lambda x: x[list(x)[0]])
        assert len(got) == len(ref), q
        for g, e in zip(got, ref):
            for k, v in e.items():
                ok = math.isclose(g[k], v, rel_tol=1e-9, abs_tol=1e-6) if isinstance(v, float) else g[k] == v
                assert ok, (q, g, e)


@pytest.mark.timeout(600)
def test_force_collectives_gloo_one_rank():
    _check(_run("gloo", "cpu"))


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_force_collectives_rccl_one_rank_on_device():
    """RCCL world_size 1 on cuda:0: the streaming shuffle, partitioned joins / aggregations, the all-gather N-chunk
    matmul and the K-split reduce-scatter run their collectives on device buffers."""
    r = _run("nccl", "cuda:0")
    assert r["_hip"] and r["meta_group"]
    _check(r, tol=3e-2)
