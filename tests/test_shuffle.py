"""Streaming distributed shuffle (execution/shuffle.py; reference PipelineStage.h:93-167 runPipelineWithShuffleSink,
ShuffleSink.h, CombinedShuffleSink.h): unit checks of the packed row image, and world_size 8 gloo runs in which a
hash-partitioned join build and a group-by each exceed every rank's device budget 4x and still match pandas,
with shuffle rounds sent while the pipelines were still producing (out-of-core execution at N > 1)."""
import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from netsdb_amd.execution.shuffle import PackedSchema
from netsdb_amd.objects.record import RecordBatch
from netsdb_amd.parallel.comm import _batch_meta


def test_packed_row_image_roundtrip():
    n = 37
    b = RecordBatch({"a": torch.arange(n), "b": torch.randn(n, 3), "c": torch.rand(n) > 0.5,
                     "d": torch.randn(n, 2, 2).to(torch.bfloat16), "e": torch.randint(0, 9, (n,), dtype=torch.int8)}, n)
    ps = PackedSchema(_batch_meta(b))
    assert ps.row_bytes == 8 + 12 + 1 + 8 + 1
    rows = ps.pack(b)
    assert rows.shape == (n, ps.row_bytes) and rows.dtype == torch.uint8
    back = ps.unpack(rows[5:20])
    for k in b.columns:
        assert torch.equal(back.columns[k], b.columns[k][5:20]), k
    empty = ps.pack(b.slice(0, 0))
    assert empty.shape == (0, ps.row_bytes) and ps.unpack(empty).n == 0


def test_packed_row_image_of_one_row_strided_columns():
    """A one-row batch of column views (stride 6, e.g. an aggregate's value row split into columns) packs too:
    torch calls a one-element view contiguous whatever its stride."""
    v = torch.rand(1, 6, dtype=torch.float64)
    b = RecordBatch({f"c{j}": v[:, j] for j in range(6)}, 1)
    ps = PackedSchema(_batch_meta(b))
    back = ps.unpack(ps.pack(b))
    assert torch.equal(torch.stack([back.columns[f"c{j}"] for j in range(6)], 1), v)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, ws, port, fn_name, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(ws),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        from netsdb_amd.parallel.comm import ClusterContext

        ctx = ClusterContext(rank, ws, torch.device("cpu"), "gloo")
        res = globals()[fn_name](ctx, out_dir)
        torch.save(res, os.path.join(out_dir, f"r{rank}.pt"))
    finally:
        dist.destroy_process_group()


def _run(fn_name, ws):
    out = tempfile.mkdtemp()
    mp.spawn(_worker, args=(ws, _free_port(), fn_name, out), nprocs=ws, join=True)
    return [torch.load(os.path.join(out, f"r{r}.pt"), weights_only=False) for r in range(ws)]


def _stream_scenario(ctx, out_dir):
    """Each rank shuffles its own (uneven, one empty) stream; every row must arrive at its hash owner."""
    from netsdb_amd.execution.shuffle import StreamingShuffle

    g = torch.Generator().manual_seed(ctx.rank)
    nb = [3, 0, 7, 1, 5, 2, 9, 4][ctx.rank % 8]
    batches = []
    for i in range(nb):
        n = 800 + 53 * i
        k = torch.randint(0, 10 ** 7, (n,), generator=g)
        batches.append(RecordBatch({"k": k, "v": k.double() * 0.25, "w": torch.randn(n, 3, generator=g)}, n))
    sh = StreamingShuffle(ctx, chunk_bytes=24 << 10)
    got = list(sh.run((b, b.columns["k"]) for b in batches))
    keys = torch.cat([b.columns["k"] for b in got]) if got else torch.empty(0, dtype=torch.int64)
    ok = bool((keys % ctx.world_size == ctx.rank).all()) and all(
        torch.equal(b.columns["v"], b.columns["k"].double() * 0.25) for b in got)
    return {"sent": sorted(torch.cat([b.columns["k"] for b in batches]).tolist()) if batches else [],
            "recv": sorted(keys.tolist()), "ok": ok, "stats": sh.stats}


def test_streaming_shuffle_8_ranks_uneven():
    res = _run("_stream_scenario", 8)
    assert all(r["ok"] for r in res)
    sent = sorted(x for r in res for x in r["sent"])
    recv = sorted(x for r in res for x in r["recv"])
    assert sent == recv and len(sent) > 0
    rounds = {r["stats"]["rounds"] for r in res}
    assert len(rounds) == 1                                   # lock-step: every rank ran the same rounds
    assert max(r["stats"]["rounds_while_pipeline"] for r in res) > 0
    assert all(r["stats"]["fallback_rounds"] == 0 for r in res)   # packed path: one all-to-all per round


def _ooc_scenario(ctx, out_dir):
    from netsdb_amd.client import PDBClient
    from netsdb_amd.computations import ScanSet, WriteSet
    from netsdb_amd.models.tpch import _EqJoin, _GroupBy
    from tests.test_out_of_core import OocCust, OocOrder, _join_proj

    budget = 80 << 10
    c = PDBClient(ctx=ctx, root=tempfile.mkdtemp(), device="cpu", device_budget=budget, page_size=16 << 10,
                  broadcast_threshold=0)
    c.engine.shuffle_chunk_bytes = 48 << 10
    c.create_database("db")
    n_orders, n_cust = 160000, 120000
    g = torch.Generator().manual_seed(11)
    if ctx.rank == 0:
        orders = RecordBatch({"okey": torch.arange(n_orders),
                              "cust": torch.randint(0, n_cust + 10000, (n_orders,), generator=g),
                              "amount": torch.rand(n_orders, generator=g, dtype=torch.float64)}, n_orders, OocOrder)
        cust = RecordBatch({"ckey": torch.randperm(n_cust, generator=g),
                            "region": torch.randint(0, 37, (n_cust,), generator=g),
                            "weight": torch.rand(n_cust, generator=g, dtype=torch.float64)}, n_cust, OocCust)
    else:
        orders = cust = None
    for name, t, b in (("orders", OocOrder, orders), ("cust", OocCust, cust)):
        c.create_set("db", name, t)
        c.send_data("db", name, b)
    res = {"local_cust_bytes": c.storage.get_set("db", "cust").nbytes(), "budget": budget}

    c.create_set("db", "joined", None)
    j = _EqJoin(2, [(0, "cust", 1, "ckey")], _join_proj)
    j.set_input(0, ScanSet("db", "orders", OocOrder))
    j.set_input(1, ScanSet("db", "cust", OocCust))
    st = c.execute_computations(WriteSet("db", "joined").set_input(j), job_name="ooc-join-8")
    res["join_stats"] = {k: st.get(k) for k in ("out_of_core", "shuffles", "join_decisions")}
    got = c.get_set_batches("db", "joined")
    res["joined"] = RecordBatch.concat(got) if got else None

    # group-by with many groups (every order key) over the joined rows: the combiner output and the received
    # partial aggregates exceed the budget; hash-partitioned final reduction on every rank
    c.engine.ooc_fraction = 0.1
    c.create_set("db", "by_okey", None)
    gb = _GroupBy(lambda b: b.columns["okey"] % 90001, lambda b: b.columns["value"],
                  lambda k, v: RecordBatch({"k": k, "total": v}, k.numel()))
    j2 = _EqJoin(2, [(0, "cust", 1, "ckey")], _join_proj)
    j2.set_input(0, ScanSet("db", "orders", OocOrder))
    j2.set_input(1, ScanSet("db", "cust", OocCust))
    st2 = c.execute_computations(WriteSet("db", "by_okey").set_input(gb.set_input(j2)), job_name="ooc-agg-8")
    res["agg_stats"] = {k: st2.get(k) for k in ("out_of_core",)}
    tot = c.get_set_batches("db", "by_okey")
    res["agg"] = RecordBatch.concat(tot) if tot else None
    res["shuffle_stats"] = {k: v for k, v in c.engine.shuffle_stats.items() if k != "by_tag"}
    res["device_bytes_after"] = c.storage.device_bytes
    if ctx.rank == 0:
        res["orders"], res["cust"] = orders, cust
    return res


@pytest.mark.timeout(600)
def test_ooc_join_and_groupby_8_ranks_match_pandas():
    pd = pytest.importorskip("pandas")
    res = _run("_ooc_scenario", 8)
    budget = res[0]["budget"]
    # the partitioned build side each rank receives is >= 4x its device budget
    assert min(r["local_cust_bytes"] for r in res) >= 4 * budget, [r["local_cust_bytes"] for r in res]
    for r in res:
        ooc = r["join_stats"]["out_of_core"] or {}
        assert ooc.get("partitioned_builds", 0) >= 1 and ooc.get("grace_joins", 0) >= 1, r["join_stats"]
        assert (r["agg_stats"]["out_of_core"] or {}).get("partitioned_aggregations", 0) >= 1, r["agg_stats"]
        assert r["join_stats"]["shuffles"] >= 1
        assert r["device_bytes_after"] <= budget + (64 << 10)
    # shuffle chunks left while the pipelines were still running
    assert sum(r["shuffle_stats"].get("rounds_while_pipeline", 0) for r in res) > 0
    assert all(r["shuffle_stats"].get("fallback_rounds", 0) == 0 for r in res)

    o, cu = res[0]["orders"], res[0]["cust"]
    od = pd.DataFrame({k: o.columns[k].numpy() for k in ("okey", "cust", "amount")})
    cd = pd.DataFrame({k: cu.columns[k].numpy() for k in ("ckey", "region", "weight")})
    ref = od.merge(cd, left_on="cust", right_on="ckey")
    ref = ref.assign(value=ref.amount * ref.weight)
    joined = RecordBatch.concat([r["joined"] for r in res if r["joined"] is not None])
    gdf = pd.DataFrame({k: joined.columns[k].numpy() for k in ("okey", "region", "value")}).sort_values("okey")
    rj = ref[["okey", "region", "value"]].sort_values("okey")
    assert len(gdf) == len(rj) > 0
    assert (gdf.okey.values == rj.okey.values).all() and (gdf.region.values == rj.region.values).all()
    assert abs(gdf.value.values - rj.value.values).max() < 1e-12

    agg = RecordBatch.concat([r["agg"] for r in res if r["agg"] is not None])
    got = dict(zip(agg.columns["k"].tolist(), agg.columns["total"].tolist()))
    want = ref.assign(k=ref.okey % 90001).groupby("k").value.sum().to_dict()
    assert len(got) == agg.n == len(want)                     # every group on exactly one rank
    assert max(abs(got[k] - want[k]) for k in want) < 1e-9


def _nested_scenario(ctx, out_dir):
    """A partitioned in-memory join (its probe side streamed through one shuffle) feeding a distributed group-by
    (a second shuffle), tiny chunks, skewed per-rank data: the downstream shuffle must not start rounds while
    the upstream one still has rounds in flight (execution/shuffle.py deferred mode)."""
    from netsdb_amd.client import PDBClient
    from netsdb_amd.computations import ScanSet, WriteSet
    from netsdb_amd.models.tpch import _EqJoin, _GroupBy
    from tests.test_out_of_core import OocCust, OocOrder, _join_proj

    c = PDBClient(ctx=ctx, root=tempfile.mkdtemp(), device="cpu", page_size=8 << 10, broadcast_threshold=0)
    c.engine.shuffle_chunk_bytes = 4 << 10
    c.create_database("db")
    g = torch.Generator().manual_seed(100 + ctx.rank)
    n_o = [0, 9000, 1500, 20000][ctx.rank % 4]                # skewed: one rank has no orders at all
    n_c = [3000, 200, 0, 5000][ctx.rank % 4]
    orders = RecordBatch({"okey": torch.arange(n_o) + 100000 * ctx.rank,
                          "cust": torch.randint(0, 9000, (n_o,), generator=g),
                          "amount": torch.rand(n_o, generator=g, dtype=torch.float64)}, n_o, OocOrder)
    ck = torch.arange(ctx.rank, 9000, ctx.world_size)[: n_c]   # each customer key on exactly one rank
    cust = RecordBatch({"ckey": ck, "region": ck % 13, "weight": torch.rand(ck.numel(), generator=g,
                                                                              dtype=torch.float64)}, ck.numel(), OocCust)
    for name, t, b in (("orders", OocOrder, orders), ("cust", OocCust, cust)):
        c.create_set("db", name, t)
        if b.n:
            c.storage.get_set("db", name).add_batch(b)        # rank-local data (no dispatch): skewed sizes
    c.create_set("db", "agg", None)
    j = _EqJoin(2, [(0, "cust", 1, "ckey")], _join_proj)
    j.set_input(0, ScanSet("db", "orders", OocOrder))
    j.set_input(1, ScanSet("db", "cust", OocCust))
    gb = _GroupBy(lambda b: b.columns["region"], lambda b: b.columns["value"],
                  lambda k, v: RecordBatch({"k": k, "total": v}, k.numel()))
    st = c.execute_computations(WriteSet("db", "agg").set_input(gb.set_input(j)), job_name="nested-shuffles")
    tot = c.get_set_batches("db", "agg")
    agg = RecordBatch.concat(tot) if tot else None
    agg = None if agg is None else {"k": agg.columns["k"].tolist(), "total": agg.columns["total"].tolist()}
    return {"agg": agg, "orders": orders, "cust": cust,
            "shuffles": st.get("shuffles"), "deferred": c.engine.shuffle_stats.get("deferred", 0),
            "rounds": c.engine.shuffle_stats.get("rounds", 0)}


@pytest.mark.timeout(300)
def test_nested_shuffles_join_then_groupby_4_ranks():
    pd = pytest.importorskip("pandas")
    res = _run("_nested_scenario", 4)
    assert all(r["shuffles"] >= 1 for r in res)
    assert all(r["deferred"] >= 1 for r in res)               # the upstream probe shuffle ran deferred
    od = pd.concat([pd.DataFrame({k: r["orders"].columns[k].numpy() for k in ("okey", "cust", "amount")})
                    for r in res])
    cd = pd.concat([pd.DataFrame({k: r["cust"].columns[k].numpy() for k in ("ckey", "region", "weight")})
                    for r in res])
    ref = od.merge(cd, left_on="cust", right_on="ckey")
    want = ref.assign(v=ref.amount * ref.weight).groupby("region").v.sum().to_dict()
    ks = [k for r in res if r["agg"] is not None for k in r["agg"]["k"]]
    got = dict(zip(ks, [t for r in res if r["agg"] is not None for t in r["agg"]["total"]]))
    assert len(got) == len(ks) == len(want) > 0
    assert max(abs(got[k] - want[k]) for k in want) < 1e-9
