"""Device nested columns (objects/nested.py): Vector / Map fields as offsets + element columns, their
structural ops against plain-Python answers, serde round trips, the engine's device FLATTEN and map-merge
aggregation (tpchBench's CustomerMultiSelection / CustomerSupplierPartGroupBy, reference src/tpchBench),
and the same on cuda:0 (gpu marker)."""
import random
import tempfile

import pytest
import torch

from netsdb_amd.objects.nested import MapColumn, NestedColumn
from netsdb_amd.objects.record import Map, PDBObject, RecordBatch, Vector
from netsdb_amd.storage.serde import deserialize_batch, serialize_batch


class NPoint(PDBObject):
    x: int
    tag: str


class NBag(PDBObject):
    bid: int
    pts: Vector(NPoint)
    ws: Vector(float)
    m: Map(str, Vector(int))


def _bags(n=20, seed=0):
    r = random.Random(seed)
    out = []
    for i in range(n):
        pts = [NPoint(r.randint(0, 99), f"t{r.randint(0, 4)}") for _ in range(r.randint(0, 4))]
        ws = [r.random() for _ in range(r.randint(0, 3))]
        m = {f"k{r.randint(0, 3)}": [r.randint(0, 9) for _ in range(r.randint(0, 3))] for _ in range(r.randint(0, 3))}
        out.append(NBag(i, pts, ws, m))
    return out


def _plain(b: NBag):
    return (b.bid, [(p.x, p.tag) for p in b.pts], list(b.ws), {k: list(v) for k, v in b.m.items()})


def _rows(batch):
    return [_plain(o) for o in batch.to_objects()]


def test_typed_nested_columns_roundtrip():
    bags = _bags()
    b = RecordBatch.from_objects(bags)
    assert isinstance(b.columns["pts"], NestedColumn) and isinstance(b.columns["pts"].values, RecordBatch)
    assert isinstance(b.columns["ws"].values, torch.Tensor)
    assert isinstance(b.columns["m"], MapColumn)
    assert _rows(b) == [_plain(x) for x in bags]


def test_take_slice_concat():
    bags = _bags(30, seed=1)
    b = RecordBatch.from_objects(bags)
    idx = torch.tensor([5, 0, 29, 5, 17])
    assert _rows(b.take(idx)) == [_plain(bags[i]) for i in idx.tolist()]
    assert _rows(b.slice(7, 19)) == [_plain(x) for x in bags[7:19]]
    cat = RecordBatch.concat([b.slice(0, 10), b.slice(10, 30)])
    assert _rows(cat) == [_plain(x) for x in bags]


def test_flatten_and_segment_sum():
    bags = _bags(25, seed=2)
    b = RecordBatch.from_objects(bags)
    vals, parent = b.columns["pts"].flatten()
    exp = [(i, p.x) for i, bg in enumerate(bags) for p in bg.pts]
    assert list(zip(parent.tolist(), vals.columns["x"].tolist())) == exp
    s = b.columns["ws"].segment_sum(b.columns["ws"].values)
    assert torch.allclose(s, torch.tensor([sum(x.ws) for x in bags], dtype=torch.float64))


def test_map_merge_matches_python():
    bags = _bags(40, seed=3)
    b = RecordBatch.from_objects(bags)
    group = torch.tensor([x.bid % 3 for x in bags])
    merged = MapColumn.merge(b.columns["m"], group, 3)
    ref = [{} for _ in range(3)]
    for x in bags:
        for k, v in x.m.items():
            ref[x.bid % 3].setdefault(k, []).extend(v)
    assert [{k: sorted(v) for k, v in merged.item(g).items()} for g in range(3)] == \
        [{k: sorted(v) for k, v in r.items()} for r in ref]


def test_serde_roundtrip_nested():
    bags = _bags(15, seed=4)
    b = RecordBatch.from_objects(bags)
    for part in (b, b.slice(3, 11), b.take(torch.tensor([9, 2, 2]))):
        back = deserialize_batch(serialize_batch(part))
        assert _rows(RecordBatch(back.columns, back.n, NBag)) == _rows(part)


def _tpch(device=None, vectorized=True):
    from netsdb_amd.client import PDBClient
    from netsdb_amd.models import tpch_nested as T

    cs = T.generate(120, seed=5)
    c = PDBClient(root=tempfile.mkdtemp(), page_size=1 << 14, device=device)
    T.load(c, "bench", cs)
    return c, cs, T


def test_tpch_nested_vectorized_matches_object_path():
    c, cs, T = _tpch()
    ref = T.reference_groupby(cs)
    assert T.supplier_groupby(c, "bench", vectorized=True) == ref
    assert T.supplier_groupby(c, "bench", vectorized=False) == ref


@pytest.mark.gpu
def test_nested_ops_on_gpu():
    bags = _bags(64, seed=6)
    b = RecordBatch.from_objects(bags, device="cuda:0")
    col = b.columns["pts"]
    assert col.offsets.is_cuda and col.values.columns["x"].is_cuda
    vals, parent = col.flatten()
    assert parent.is_cuda
    idx = torch.tensor([3, 63, 0, 3], device="cuda:0")
    assert _rows(b.take(idx).to("cpu")) == [_plain(bags[i]) for i in idx.tolist()]
    group = torch.tensor([x.bid % 4 for x in bags], device="cuda:0")
    merged = MapColumn.merge(b.columns["m"], group, 4)
    assert merged.offsets.is_cuda
    ref = [{} for _ in range(4)]
    for x in bags:
        for k, v in x.m.items():
            ref[x.bid % 4].setdefault(k, []).extend(v)
    assert [{k: sorted(v) for k, v in merged.item(g).items()} for g in range(4)] == \
        [{k: sorted(v) for k, v in r.items()} for r in ref]


@pytest.mark.gpu
def test_tpch_nested_on_gpu():
    c, cs, T = _tpch("cuda:0")
    orders = c.storage.get_set("bench", "customers").all().columns["orders"]
    assert orders.offsets.is_cuda
    assert T.supplier_groupby(c, "bench") == T.reference_groupby(cs)
    q = [1, 3, 5, 7, 9, 11]
    assert T.top_jaccard(c, "bench", 6, q) == T.reference_jaccard(cs, q, 6)
