"""The nested-object TPC-H micro-benchmarks (reference: src/tpchBench — Customer{Vector<Order{Vector<LineItem
{Handle<Supplier>, Handle<Part>}>}>}, CustomerIntegerSelection(+Not, +Virtual), CustomerStringSelection(+Not,
+Virtual), CountCustomer / CountAggregation, CustomerMultiSelection -> SupplierInfo,
CustomerSupplierPartGroupBy, TopJaccard/AllParts, tpchDataGenerator).

Customers are stored as nested objects (list columns of nested PDBObjects — the object model's
Vector/Handle support). The heavy queries flatten once and then run columnar:

* ``CustomerMultiSelection`` flattens each customer's orders/lineitems into SupplierInfo records
  (FLATTEN atom);
* ``CustomerSupplierPartGroupBy`` groups them by supplier name, value = {customer: [parts]}
  (the reference's Map<String, Vector<int>> merge in SupplierInfo::operator+);
* ``TopJaccard`` scores every customer's distinct purchased-part set against the query list with a
  vectorised CSR intersection (``torch.isin`` + segment sums) and keeps the top k (TopKComp).
"""
from __future__ import annotations

from typing import Dict, List

import torch

from ..computations import AggregateComp, MultiSelectionComp, ScanSet, SelectionComp, TopKComp, WriteSet
from ..lambdas import make_batch_lambda, make_lambda, make_lambda_from_member, make_lambda_from_method, \
    make_lambda_from_self
from ..objects.record import PDBObject, RecordBatch, Vector


class BPart(PDBObject):
    partKey: int
    name: str


class BSupplier(PDBObject):
    supplierKey: int
    name: str


class BLineItem(PDBObject):
    lineNumber: int
    quantity: float
    supplier: object
    part: object


class BOrder(PDBObject):
    orderKey: int
    lineItems: Vector(object)


class BCustomer(PDBObject):
    orders: Vector(object)
    custKey: int
    name: str
    address: str
    nationKey: int
    phone: str
    accbal: float
    mktsegment: str
    comment: str

    def getName(self):
        return self.name

    def getKey(self):
        return self.custKey

    def getOrders(self):
        return self.orders


class SupplierInfo(PDBObject):
    supplierName: str
    customer: str
    part: int


class SupplierParts(PDBObject):
    supplierName: str
    soldPartIDs: object        # {customer name: [part keys]}


def generate(n_customers: int = 200, n_parts: int = 50, n_suppliers: int = 10, max_orders: int = 4,
             max_lines: int = 4, seed: int = 0) -> List[BCustomer]:
    """tpchDataGenerator: random nested customers."""
    g = torch.Generator().manual_seed(seed)
    parts = [BPart(i, f"part{i}") for i in range(n_parts)]
    sups = [BSupplier(i, f"Supplier#{i}") for i in range(n_suppliers)]
    out = []
    for c in range(n_customers):
        orders = []
        for o in range(int(torch.randint(1, max_orders + 1, (1,), generator=g))):
            lines = [BLineItem(ln, float(torch.randint(1, 50, (1,), generator=g)),
                               sups[int(torch.randint(0, n_suppliers, (1,), generator=g))],
                               parts[int(torch.randint(0, n_parts, (1,), generator=g))])
                     for ln in range(int(torch.randint(1, max_lines + 1, (1,), generator=g)))]
            orders.append(BOrder(c * 100 + o, lines))
        out.append(BCustomer(orders, c, f"Customer#{c}", f"addr{c}", c % 25, f"{10 + c % 25}-555", float(c % 97) * 10.0,
                             ["BUILDING", "MACHINERY", "AUTOMOBILE"][c % 3], "comment"))
    return out


def load(client, db: str, customers: List[BCustomer]):
    client.create_database(db)
    client.create_set(db, "customers", BCustomer)
    client.send_data(db, "customers", customers)


class CustomerIntegerSelection(SelectionComp):
    """custKey < bound (``negate``: the *Not variants; ``virtual``: through a method call)."""

    def __init__(self, bound: int, negate: bool = False, virtual: bool = False):
        super().__init__()
        self.bound, self.negate, self.virtual = bound, negate, virtual

    def get_selection(self, c):
        key = make_lambda_from_method(c, "getKey") if self.virtual else make_lambda_from_member(c, "custKey")
        return (key >= self.bound) if self.negate else (key < self.bound)

    def get_projection(self, c):
        return make_lambda_from_self(c)


class CustomerStringSelection(SelectionComp):
    """name == value (``negate`` / ``virtual`` as above)."""

    def __init__(self, value: str, negate: bool = False, virtual: bool = False):
        super().__init__()
        self.value, self.negate, self.virtual = value, negate, virtual

    def get_selection(self, c):
        name = make_lambda_from_method(c, "getName") if self.virtual else make_lambda_from_member(c, "name")
        return (name != self.value) if self.negate else (name == self.value)

    def get_projection(self, c):
        return make_lambda_from_self(c)


class CountCustomer(AggregateComp):
    def get_key_projection(self, c):
        return make_batch_lambda(c, lambda b: torch.zeros(b.n, dtype=torch.int64))

    def get_value_projection(self, c):
        return make_batch_lambda(c, lambda b: torch.ones(b.n, dtype=torch.int64))


class CustomerMultiSelection(MultiSelectionComp):
    def get_selection(self, c):
        return make_lambda(c, lambda r: True)

    def get_projection(self, c):
        def flat(r):
            return [SupplierInfo(li.supplier.name, r.name, li.part.partKey) for o in r.orders for li in o.lineItems]

        return make_lambda(c, flat)


class CustomerSupplierPartGroupBy(AggregateComp):
    reduce_op = None

    def get_key_projection(self, s):
        return make_lambda_from_member(s, "supplierName")

    def get_value_projection(self, s):
        return make_lambda(s, lambda r: {r.customer: [r.part]})

    def combine(self, a, b):
        out = {k: list(v) for k, v in a.items()}
        for k, v in b.items():
            out.setdefault(k, []).extend(v)
        return out

    def make_output(self, keys, values):
        return RecordBatch.from_objects([SupplierParts(k, v) for k, v in zip(keys, values)], SupplierParts)


class TopJaccard(TopKComp):
    """Top-k customers by Jaccard similarity of their distinct purchased parts to ``parts``."""

    def __init__(self, k: int, parts: List[int]):
        super().__init__(k)
        self.parts = torch.tensor(sorted(set(parts)), dtype=torch.int64)

    def get_value_projection(self, c):
        def score(b):
            keys, lens = [], []
            for orders in b.columns["orders"]:
                s = sorted({li.part.partKey for o in orders for li in o.lineItems})
                keys.extend(s)
                lens.append(len(s))
            flat = torch.tensor(keys, dtype=torch.int64)
            seg = torch.repeat_interleave(torch.arange(b.n), torch.tensor(lens, dtype=torch.int64))
            inter = torch.zeros(b.n, dtype=torch.float64).index_add_(0, seg, torch.isin(flat, self.parts).double())
            union = torch.tensor(lens, dtype=torch.float64) + self.parts.numel() - inter
            return inter / union.clamp_min(1)

        return make_batch_lambda(c, score)


def _run(client, db, out, comp, job):
    if client.storage.has_set(db, out):
        client.remove_set(db, out)
    client.create_set(db, out, None)
    client.execute_computations(WriteSet(db, out).set_input(comp), job_name=job)
    return [b for b in client.get_set_batches(db, out, gather=True) if b.n]


def _objs(batches) -> list:
    out = []
    for b in batches:
        if len(b.columns) == 1 and isinstance(next(iter(b.columns.values())), RecordBatch):
            b = next(iter(b.columns.values()))
        out.extend(b.to_objects() if hasattr(b, "to_objects") else [])
    return out


def select_customers(client, db: str, comp) -> List[int]:
    got = _run(client, db, "bench_sel", comp.set_input(ScanSet(db, "customers", BCustomer)), "tpchbench_select")
    keys = []
    for b in got:
        col = b.columns.get("custKey")
        if col is None:
            inner = next(iter(b.columns.values()))
            col = inner.columns["custKey"]
        keys.extend(col.tolist() if isinstance(col, torch.Tensor) else list(col))
    return sorted(int(k) for k in keys)


def count_customers(client, db: str) -> int:
    got = _run(client, db, "bench_cnt", CountCustomer().set_input(ScanSet(db, "customers", BCustomer)),
               "tpchbench_count")
    return int(sum(int(b.columns["value"].sum()) for b in got))


def supplier_groupby(client, db: str) -> Dict[str, Dict[str, List[int]]]:
    flat = CustomerMultiSelection().set_input(ScanSet(db, "customers", BCustomer))
    got = _run(client, db, "bench_gb", CustomerSupplierPartGroupBy().set_input(flat), "tpchbench_groupby")
    out = {}
    for b in got:
        inner = next(iter(b.columns.values())) if len(b.columns) == 1 else b
        for s, m in zip(inner.columns["supplierName"], inner.columns["soldPartIDs"]):
            out[s] = {k: sorted(v) for k, v in m.items()}
    return out


def top_jaccard(client, db: str, k: int, parts: List[int]):
    """[(custKey, score)] of the k most similar customers (TopKComp output = the customers)."""
    comp = TopJaccard(k, parts)
    got = _run(client, db, "bench_topk", comp.set_input(ScanSet(db, "customers", BCustomer)), "tpchbench_topjaccard")
    score = comp.get_value_projection(None).fn
    res = []
    for b in got:
        inner = next(iter(b.columns.values())) if len(b.columns) == 1 else b
        res.extend(zip(inner.columns["custKey"].tolist(), score(inner).tolist()))
    return sorted(res, key=lambda x: (-x[1], x[0]))[:k]


def reference_groupby(customers: List[BCustomer]):
    out: Dict[str, Dict[str, List[int]]] = {}
    for c in customers:
        for o in c.orders:
            for li in o.lineItems:
                out.setdefault(li.supplier.name, {}).setdefault(c.name, []).append(li.part.partKey)
    return {s: {k: sorted(v) for k, v in m.items()} for s, m in out.items()}


def reference_jaccard(customers: List[BCustomer], parts: List[int], k: int):
    q = set(parts)
    sc = []
    for c in customers:
        s = {li.part.partKey for o in c.orders for li in o.lineItems}
        sc.append((c.custKey, len(s & q) / max(1, len(s | q))))
    return sorted(sc, key=lambda x: (-x[1], x[0]))[:k]
