"""Nested-object TPC-H micro-benchmarks (reference src/tpchBench) vs plain-Python answers."""
from netsdb_amd.client import PDBClient
from netsdb_amd.models import tpch_nested as T


def test_tpch_bench_queries(tmp_path):
    cs = T.generate(100, seed=2)
    c = PDBClient(root=str(tmp_path), page_size=1 << 14)
    T.load(c, "bench", cs)
    assert T.count_customers(c, "bench") == 100
    keys = [x.custKey for x in cs]
    for virtual in (False, True):
        assert T.select_customers(c, "bench", T.CustomerIntegerSelection(30, virtual=virtual)) == [k for k in keys if k < 30]
        assert T.select_customers(c, "bench", T.CustomerIntegerSelection(30, True, virtual)) == [k for k in keys if k >= 30]
        assert T.select_customers(c, "bench", T.CustomerStringSelection("Customer#7", virtual=virtual)) == [7]
        assert T.select_customers(c, "bench", T.CustomerStringSelection("Customer#7", True, virtual)) == \
            [k for k in keys if k != 7]
    assert T.supplier_groupby(c, "bench") == T.reference_groupby(cs)
    q = [1, 3, 5, 7, 9, 11]
    assert T.top_jaccard(c, "bench", 6, q) == T.reference_jaccard(cs, q, 6)
