"""dbgen .tbl ingestion (models/tpch_tbl.py; reference src/tpch/source/tpchDataLoader.cc:65,480-653): generated
tables written in dbgen's pipe-delimited format, loaded back through the vectorised chunked parser, must give the
same columns and the same results for all ten TPC-H queries as the in-memory load."""
import math
import tempfile

import numpy as np
import pytest
import torch

from netsdb_amd.client import PDBClient
from netsdb_amd.models import tpch, tpch_gen, tpch_tbl

QUERIES = ("q01", "q02", "q03", "q04", "q06", "q12", "q13", "q14", "q17", "q22")


def _same(a, b):
    if isinstance(a, float):
        return math.isclose(a, b, rel_tol=1e-12, abs_tol=1e-9)
    if isinstance(a, list):
        return len(a) == len(b) and all(_same(x, y) for x, y in zip(a, b))
    if isinstance(a, dict):
        return a.keys() == b.keys() and all(_same(a[k], b[k]) for k in a)
    return a == b


def _roundtrip(dev, sf, chunk):
    t = tpch_gen.generate_fast(sf, seed=11)
    d = tempfile.mkdtemp()
    tpch_tbl.write_tbl(t, d)
    c_mem = PDBClient(root=tempfile.mkdtemp(), device=dev)
    tpch.load(c_mem, "tpch", t, device=dev)
    c_tbl = PDBClient(root=tempfile.mkdtemp(), device=dev)
    st = tpch_tbl.load_tbl(c_tbl, "tpch", d, device=dev, chunk_bytes=chunk)
    assert st["lineitem"]["rows"] == len(t["lineitem"]["l_orderkey"])
    # columns equal, numbers bit for bit
    li = c_tbl.get_set("tpch", "lineitem").all()
    for col in ("l_orderkey", "l_extendedprice", "l_discount", "l_tax", "l_quantity", "l_shipdate", "l_receiptdate"):
        got = li.columns[col].cpu().numpy()
        assert np.array_equal(got, np.asarray(t["lineitem"][col])), col
    for col in ("l_returnflag", "l_shipmode", "l_comment"):
        got = li.columns[col]
        got = got if isinstance(got, list) else got.tolist()
        assert got == t["lineitem"][col].tolist(), col
    for q in QUERIES:
        a, b = tpch.QUERIES[q](c_mem, "tpch"), tpch.QUERIES[q](c_tbl, "tpch")
        assert _same(a, b), (q, a, b)
    return st


def test_tbl_roundtrip_cpu_all_queries():
    st = _roundtrip("cpu", 0.004, 1 << 20)      # several chunks per large table
    assert st["orders"]["rows"] > 0


def test_tbl_parser_edge_cases():
    txt = b"1|-12.50|1996-03-13|a b|\n22|0.00|2001-12-31||\n-7|1234567.89|1970-01-01|x|y z|"
    # 3rd row has 5 fields: malformed
    with pytest.raises(ValueError):
        tpch_tbl._field_bounds(torch.frombuffer(bytearray(txt + b"\n"), dtype=torch.uint8), 4)
    buf = torch.frombuffer(bytearray(b"1|-12.50|1996-03-13|a b|\n22|0.00|2001-12-31||\n"), dtype=torch.uint8)
    s, e = tpch_tbl._field_bounds(buf, 4)
    assert tpch_tbl._parse_numeric(buf, s[:, 0], e[:, 0], False).tolist() == [1, 22]
    assert tpch_tbl._parse_numeric(buf, s[:, 1], e[:, 1], True).tolist() == [-12.5, 0.0]
    assert tpch_tbl._parse_numeric(buf, s[:, 2], e[:, 2], False).tolist() == [19960313, 20011231]
    assert (e[:, 3] - s[:, 3]).tolist() == [3, 0]


@pytest.mark.gpu
def test_tbl_roundtrip_gpu_all_queries():
    _roundtrip("cuda:0", 0.01, 1 << 20)
