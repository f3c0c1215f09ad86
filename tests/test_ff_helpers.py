"""FF helper UDFs and the drivers that use them (reference src/FF/headers: FFMatrixPartitioner, FFMatrixMultiSel,
InferenceResult(Partition), FFAggMatrixToOneMatrix, FFSingleMatrix; src/FF/source/SimpleFF.cc enablePartition;
src/tests/source/RedditFeatureExtractor.cc; heterogeneousModelDeduplication/*.cc), each against an fp32 reference."""
import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from netsdb_amd.client import PDBClient
from netsdb_amd.models import blocks as B
from netsdb_amd.models import ff
from netsdb_amd.models import text_classifier as TC
from netsdb_amd.objects.builtin import FFMatrixBlock


def _ff_partitioned(dev):
    c = PDBClient(root=tempfile.mkdtemp(), device=dev)
    ff.load_model(c, "ff", 40, 200, 48, 20, 8, 32, seed=3, hidden2=24, dtype=torch.float32)
    g = lambda n: B.to_tensor(c, "ff", n)  # noqa: E731
    ref = ff.reference_inference(g("inputs"), g("w1"), g("b1"), g("wo"), g("bo"), g("w2"), g("b2"))
    out = {}
    for ep in (False, True):
        ff.inference(c, "ff", "w1", "w2", "wo", "inputs", "b1", "b2", "bo", "out", enable_partition=ep)
        out[ep] = B.to_tensor(c, "ff", "out").float()
    y1 = c.storage.get_set("ff", "y1")
    return out, ref, y1


def test_inference_enable_partition_cpu():
    out, ref, y1 = _ff_partitioned(None)
    torch.testing.assert_close(out[True].cpu(), ref.cpu(), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(out[True], out[False], rtol=1e-5, atol=1e-6)
    assert y1.num_records() > 0 and not hasattr(y1, "panel")       # block records, not a dense panel


def test_multisel_and_partition_writer_cpu():
    c = PDBClient(root=tempfile.mkdtemp())
    c.create_database("db")
    data = torch.arange(3 * 4 * 5, dtype=torch.float32).reshape(3, 4, 5)
    blk = ff.mk_blocks(torch.tensor([0, 1, 2]), 0, data, 12, 5)
    c.create_set("db", "m", FFMatrixBlock)
    c.send_data("db", "m", blk)
    for writer in (ff.InferenceResultPartition("db", "r"), None):
        if c.storage.has_set("db", "r"):
            c.remove_set("db", "r")
        c.create_set("db", "r", ff.InferenceResult)
        from netsdb_amd.computations import WriteSet

        w = writer if writer is not None else WriteSet("db", "r", ff.InferenceResult)
        c.execute_computations(w.set_input(ff.FFMatrixMultiSel().set_input(ff.FFMatrixBlockScanner("db", "m"))))
        from netsdb_amd.objects.record import RecordBatch

        r = RecordBatch.concat([b for b in c.get_set_batches("db", "r") if b.n])
        order = torch.argsort(r.columns["index"])
        assert r.columns["index"][order].tolist() == list(range(12))
        assert r.columns["block_row_id"][order].tolist() == [i // 4 for i in range(12)]
        torch.testing.assert_close(r.columns["inference"][order].float(), data.reshape(12, 5)[:, :2])
        lab = ff.InferenceResult.getLabel.__vectorized__(r)
        assert lab.tolist() == [-1] * 12                            # score0 < score1 on every row


def test_agg_to_one_matrix_and_single_block_classifier_cpu():
    c = PDBClient(root=tempfile.mkdtemp())
    TC.load_workload(c, "tc", 3000, 30, batch=16, block_x=10, block_y=400, seed=2)
    r = TC.run_workload(c, "tc", 30)
    ref = TC.reference_labels(B.to_tensor(c, "tc", "weights"), B.to_tensor(c, "tc", "inputs"), 30)
    assert r["labels"].shape[-1] == 16
    assert torch.equal(r["labels"].float().reshape(ref.shape).cpu(), ref)
    assert "matmul[FFTransposeMult+FFAggMatrix]" in r["jobs"][0]["fused_ops"]
    # the assembled single matrix equals the intermediate panel
    one = ff.FFAggMatrixToOneMatrix()
    inter = c.storage.get_set("tc", "intermediate")
    blocks = inter.to_blocks()
    mats = one.group_values(blocks, torch.zeros(blocks.n, dtype=torch.int64), 1)
    torch.testing.assert_close(mats[0].float(), B.to_tensor(c, "tc", "intermediate").float())


def test_heterogeneous_dedup_cpu():
    c = PDBClient(root=tempfile.mkdtemp())
    models = {"nnlm-a": (2400, 20), "nnlm-b": (2400, 40), "wiki-c": (2000, 30)}
    res = TC.heterogeneous_dedup(c, models, batch=8, block_x=10, block_y=400, run=list(models))
    assert all(r["match"] for r in res["runs"].values())
    assert res["bytes_pooled"] < res["bytes_private"] and res["dedup_ratio"] < 1.0


def test_reddit_inference_results_cpu():
    from netsdb_amd.models import reddit

    c = PDBClient(root=tempfile.mkdtemp())
    reddit.load(c, "rd", reddit.generate(300, seed=4)) if hasattr(reddit, "generate") else pytest.skip("no generator")
    for ep in (False, True):
        res, ref = reddit.infer_results(c, "rd", 300, enable_partition=ep)
        assert res.columns["index"].tolist() == list(range(res.n))
        torch.testing.assert_close(res.columns["inference"][:300].float(), ref.float(), rtol=1e-4, atol=1e-6)


# ------------------------------------------------------------------------------------------- 2 ranks
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, ws, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(ws),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        from netsdb_amd.parallel.comm import ClusterContext

        ctx = ClusterContext(rank, ws, torch.device("cpu"), "gloo")
        c = PDBClient(ctx=ctx, root=tempfile.mkdtemp(), device="cpu")
        ff.load_model(c, "ff", 32, 160, 40, 16, 8, 32, seed=5, hidden2=24, dtype=torch.float32)
        ff.inference(c, "ff", "w1", "w2", "wo", "inputs", "b1", "b2", "bo", "out", enable_partition=True)
        y1 = c.storage.get_set("ff", "y1")
        rows = sorted({int(x) for b in y1.scan() for x in b.columns["block_row"].tolist()})
        out = B.to_tensor(c, "ff", "out").float()
        g = lambda n: B.to_tensor(c, "ff", n)  # noqa: E731
        ref = ff.reference_inference(g("inputs"), g("w1"), g("b1"), g("wo"), g("bo"), g("w2"), g("b2"))
        torch.save({"err": float((out - ref).abs().max()), "y1_block_rows": rows},
                   os.path.join(out_dir, f"r{rank}.pt"))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_partitioned_ff_2_ranks():
    out = tempfile.mkdtemp()
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    res = [torch.load(os.path.join(out, f"r{r}.pt"), weights_only=True) for r in range(2)]
    assert all(r["err"] < 1e-4 for r in res), res
    rows = [set(r["y1_block_rows"]) for r in res]
    assert rows[0] and rows[1] and not (rows[0] & rows[1])          # y1 block rows split across the ranks
    assert sorted(rows[0] | rows[1]) == list(range(5))                # 40 hidden rows / 8 = 5 block rows


# ------------------------------------------------------------------------------------------- GPU
@pytest.mark.gpu
def test_inference_enable_partition_gpu():
    out, ref, _ = _ff_partitioned("cuda:0")
    torch.testing.assert_close(out[True].cpu(), ref.cpu(), rtol=2e-2, atol=2e-3)


@pytest.mark.gpu
def test_text_classifier_and_dedup_gpu():
    c = PDBClient(root=tempfile.mkdtemp(), device="cuda:0")
    TC.load_workload(c, "tc", 30000, 50, batch=100, block_x=50, block_y=10000, seed=2)
    r = TC.run_workload(c, "tc", 50)
    ref = TC.reference_labels(B.to_tensor(c, "tc", "weights").cpu(), B.to_tensor(c, "tc", "inputs").cpu(), 50)
    agree = (r["labels"].float().reshape(ref.shape).cpu() == ref).float().mean().item()
    assert agree >= 0.98, agree                                        # bf16 GEMM vs fp32 at the 0.5 threshold
    res = TC.heterogeneous_dedup(c, {"a": (30000, 50), "b": (30000, 100)}, batch=100, run=["a"])
    assert res["bytes_pooled"] < res["bytes_private"]
