"""Out-of-core execution: dense panels larger than the device budget spill in block-row slabs (page pool on
a CPU node, pinned host tier on a GPU) and the fused block GEMM streams slab pairs back
(reference: src/storage PageCache eviction + PDBEvictWork; PipelineStage over spilled pages)."""
import tempfile

import pytest
import torch

from netsdb_amd.client import PDBClient
from netsdb_amd.models import ff
from netsdb_amd.models.blocks import load_tensor, to_tensor


def _ff_over_budget(device, budget, page_size):
    c = PDBClient(root=tempfile.mkdtemp(), device=device, device_budget=budget, page_size=page_size)
    g = torch.Generator().manual_seed(0)
    batch, feats, hid, labels = 64, 4096, 256, 96
    X = torch.rand(batch, feats, generator=g) - 0.5
    W1 = (torch.rand(hid, feats, generator=g) - 0.5) * 0.05
    b1 = torch.rand(hid, 1, generator=g) * 0.1
    Wo = (torch.rand(labels, hid, generator=g) - 0.5) * 0.2
    bo = torch.rand(labels, 1, generator=g) * 0.1
    ff.setup(c, "ff")
    dt = torch.float32 if device == "cpu" else torch.bfloat16
    for name, t, bx, by in (("inputs", X, 16, 512), ("w1", W1, 16, 512), ("b1", b1, 16, 1), ("wo", Wo, 16, 16),
                            ("bo", bo, 16, 1)):
        load_tensor(c, "ff", name, t.to(device), bx, by, dtype=dt)
    res = ff.inference_unit(c, "ff", "w1", "wo", "inputs", "b1", "bo", "output")
    out = to_tensor(c, "ff", "output").float().cpu()
    r = lambda t: t.to(dt).float()  # noqa: E731
    ref = ff.reference_inference(r(X), r(W1), r(b1), r(Wo), r(bo))
    return c, res, out, ref


def test_ff_weights_exceed_budget_cpu():
    budget = 3 << 20                       # W1 alone is 4 MB (f32), inputs 1 MB
    c, res, out, ref = _ff_over_budget("cpu", budget, 256 << 10)
    torch.testing.assert_close(out, ref, atol=2e-5, rtol=2e-4)
    ooc = res["jobs"][0].get("out_of_core", {})
    assert ooc.get("ooc_matmuls", 0) >= 1 and ooc.get("ooc_slab_pairs", 0) > 1, res["jobs"][0]
    w1 = c.storage.get_set("ff", "w1")
    assert w1.stats_io["spills"] >= 1 and w1.stats_io["slab_loads"] >= 1
    assert c.storage.stats.get("evicted_panels", 0) >= 1


def test_dense_panel_spill_reload_roundtrip_cpu():
    c = PDBClient(root=tempfile.mkdtemp(), device="cpu", device_budget=900 << 10, page_size=64 << 10)
    c.create_database("db")
    a = torch.randn(300, 500)
    b = torch.randn(200, 500)
    load_tensor(c, "db", "a", a, 10, 100, dtype=torch.float32)
    sa = c.storage.get_set("db", "a")
    assert sa.is_resident()
    load_tensor(c, "db", "b", b, 10, 100, dtype=torch.float32)    # a (614 KB) + b (410 KB) > 900 KB budget
    assert sa.is_spilled() and not sa.is_resident()
    assert c.storage.device_bytes <= c.storage.device_budget
    torch.testing.assert_close(sa.load_rows(37, 211)[:, :500], a[37:211])   # slabs without a reload
    assert sa.is_spilled()
    torch.testing.assert_close(to_tensor(c, "db", "a"), a)                   # full reload on access
    assert sa.is_resident() and c.storage.get_set("db", "b").is_spilled()   # LRU: b made room for a
    torch.testing.assert_close(to_tensor(c, "db", "b"), b)
    c.remove_set("db", "a")
    c.remove_set("db", "b")
    assert c.storage.device_bytes == 0


@pytest.mark.gpu
def test_ff_weights_exceed_budget_gpu_pinned_tier():
    budget = 2 << 20                       # bf16 W1 = 2 MB, inputs 0.5 MB
    c, res, out, ref = _ff_over_budget("cuda:0", budget, 256 << 10)
    err = (out - ref).abs().max().item() / ref.abs().max().item()
    assert err < 2e-2, err
    assert res["jobs"][0].get("out_of_core", {}).get("ooc_matmuls", 0) >= 1
    w1 = c.storage.get_set("ff", "w1")
    assert w1.stats_io["spills"] >= 1
    assert c.storage.host_tier.stats["offloads"] >= 1      # evicted to pinned host memory by async D2H


# ------------------------------------------------------------------ out-of-core join + aggregation
from netsdb_amd.computations import ScanSet, WriteSet  # noqa: E402
from netsdb_amd.models.tpch import _EqJoin, _GroupBy  # noqa: E402
from netsdb_amd.objects import PDBObject, RecordBatch  # noqa: E402


class OocOrder(PDBObject):
    okey: int
    cust: int
    amount: float


class OocCust(PDBObject):
    ckey: int
    region: int
    weight: float


def _ooc_tables(n_orders=60000, n_cust=45000, seed=3):
    g = torch.Generator().manual_seed(seed)
    orders = RecordBatch({"okey": torch.arange(n_orders), "cust": torch.randint(0, n_cust + 5000, (n_orders,), generator=g),
                          "amount": torch.rand(n_orders, generator=g, dtype=torch.float64)}, n_orders, OocOrder)
    cust = RecordBatch({"ckey": torch.randperm(n_cust, generator=g), "region": torch.randint(0, 37, (n_cust,), generator=g),
                        "weight": torch.rand(n_cust, generator=g, dtype=torch.float64)}, n_cust, OocCust)
    return orders, cust


def _join_proj(o, c):
    return RecordBatch({"okey": o.columns["okey"], "region": c.columns["region"],
                        "value": o.columns["amount"] * c.columns["weight"]}, o.n)


def _region_sum():
    return _GroupBy(lambda b: b.columns["region"], lambda b: b.columns["value"],
                    lambda k, v: RecordBatch({"region": k, "total": v}, k.numel()))


def test_hash_join_build_4x_budget_matches_pandas():
    pd = pytest.importorskip("pandas")
    budget = 256 << 10
    c = PDBClient(root=tempfile.mkdtemp(), device="cpu", device_budget=budget, page_size=32 << 10)
    c.create_database("db")
    orders, cust = _ooc_tables()
    assert cust.nbytes() >= 4 * budget                      # the build side (smaller input) is 4x the budget
    for name, t, b in (("orders", OocOrder, orders), ("cust", OocCust, cust)):
        c.create_set("db", name, t)
        c.send_data("db", name, b)
    c.create_set("db", "joined", None)
    j = _EqJoin(2, [(0, "cust", 1, "ckey")], _join_proj)
    j.set_input(0, ScanSet("db", "orders", OocOrder))
    j.set_input(1, ScanSet("db", "cust", OocCust))
    st = c.execute_computations(WriteSet("db", "joined").set_input(j), job_name="ooc-join")
    ooc = st.get("out_of_core", {})
    assert ooc.get("partitioned_builds", 0) == 1 and ooc.get("grace_joins", 0) == 1, st
    assert c.storage.stats["evicted_pages"] > 0            # input / spool pages spilled to the page pool
    got = RecordBatch.concat(c.get_set_batches("db", "joined"))
    gdf = pd.DataFrame({k: got.columns[k].numpy() for k in ("okey", "region", "value")}).sort_values("okey")
    od = pd.DataFrame({k: orders.columns[k].numpy() for k in ("okey", "cust", "amount")})
    cd = pd.DataFrame({k: cust.columns[k].numpy() for k in ("ckey", "region", "weight")})
    ref = od.merge(cd, left_on="cust", right_on="ckey")
    ref = ref.assign(value=ref.amount * ref.weight)[["okey", "region", "value"]].sort_values("okey")
    assert len(gdf) == len(ref) > 0
    assert (gdf.okey.values == ref.okey.values).all() and (gdf.region.values == ref.region.values).all()
    assert abs(gdf.value.values - ref.value.values).max() < 1e-12

    # join -> group-by with the group-by input over the limit: hash-partitioned aggregation
    c.engine.ooc_fraction = 0.1
    j2 = _EqJoin(2, [(0, "cust", 1, "ckey")], _join_proj)
    j2.set_input(0, ScanSet("db", "orders", OocOrder))
    j2.set_input(1, ScanSet("db", "cust", OocCust))
    c.create_set("db", "totals", None)
    st2 = c.execute_computations(WriteSet("db", "totals").set_input(_region_sum().set_input(j2)), job_name="ooc-agg")
    assert st2.get("out_of_core", {}).get("partitioned_aggregations", 0) == 1, st2
    tot = RecordBatch.concat(c.get_set_batches("db", "totals"))
    got_t = dict(zip(tot.columns["region"].tolist(), tot.columns["total"].tolist()))
    ref_t = ref.groupby("region").value.sum().to_dict()
    assert set(got_t) == set(ref_t)
    assert max(abs(got_t[k] - ref_t[k]) for k in ref_t) < 1e-9
    assert c.storage.device_bytes <= budget + (64 << 10)    # spools dropped at job end, within budget
