"""The nested-object TPC-H micro-benchmarks (reference: src/tpchBench — Customer{Vector<Order{Vector<LineItem
{Handle<Supplier>, Handle<Part>}>}>}, CustomerIntegerSelection(+Not, +Virtual), CustomerStringSelection(+Not,
+Virtual), CountCustomer / CountAggregation, CustomerMultiSelection -> SupplierInfo,
CustomerSupplierPartGroupBy, TopJaccard/AllParts, tpchDataGenerator).

Customers are stored with TYPED nested fields: ``orders: Vector(BOrder)`` and ``lineItems: Vector(BLineItem)``
are offsets + element columns (:class:`~netsdb_amd.objects.nested.NestedColumn`) and the supplier / part
``Handle`` fields are struct columns, so a customer set on a GPU is a handful of device tensors.  The heavy
queries never walk records:

* ``CustomerMultiSelection`` projects each customer to a ragged column of SupplierInfo rows built with two
  device FLATTENs (customers -> orders -> line items, parent indices composed) and the engine's FLATTEN atom
  turns it into rows without leaving the device;
* ``CustomerSupplierPartGroupBy`` groups them by supplier name with value ``Map(customer -> Vector(part))``
  (the reference's ``Map<String, Vector<int>>`` merge in SupplierInfo::operator+) — a MapColumn whose
  per-group merge (:meth:`MapColumn.merge`) is a sort + segmented concatenation;
* ``TopJaccard`` scores every customer's distinct purchased-part set against the query list with a
  flattened (customer, part) unique + ``torch.isin`` + segment sums, then keeps the top k (TopKComp).

``vectorized=False`` on the projections selects the object-at-a-time lambdas (RecordView walks), kept for
parity tests.
"""
from __future__ import annotations

from typing import Dict, List

import torch

from ..computations import AggregateComp, MultiSelectionComp, ScanSet, SelectionComp, TopKComp, WriteSet
from ..lambdas import make_batch_lambda, make_lambda, make_lambda_from_member, make_lambda_from_method, \
    make_lambda_from_self
from ..objects.nested import MapColumn, NestedColumn
from ..objects.record import Map, PDBObject, RecordBatch, Vector, column_take


class BPart(PDBObject):
    partKey: int
    name: str


class BSupplier(PDBObject):
    supplierKey: int
    name: str


class BLineItem(PDBObject):
    lineNumber: int
    quantity: float
    supplier: BSupplier          # Handle<Supplier>
    part: BPart                  # Handle<Part>


class BOrder(PDBObject):
    orderKey: int
    lineItems: Vector(BLineItem)


class BCustomer(PDBObject):
    orders: Vector(BOrder)
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
    soldPartIDs: Map(str, Vector(int))        # {customer name: [part keys]}


def _offsets(counts: torch.Tensor) -> torch.Tensor:
    off = torch.zeros(counts.numel() + 1, dtype=torch.int64, device=counts.device)
    torch.cumsum(counts, 0, out=off[1:])
    return off


def line_items(b: RecordBatch):
    """(line-item batch, owning customer row of every line item) by two device FLATTENs."""
    ob, o_par = b.columns["orders"].flatten()
    lb, l_par = ob.columns["lineItems"].flatten()
    return lb, o_par.index_select(0, l_par)


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
    def __init__(self, vectorized: bool = True):
        super().__init__()
        self.vectorized = vectorized

    def get_selection(self, c):
        if self.vectorized:
            return make_batch_lambda(c, lambda b: torch.ones(b.n, dtype=torch.bool, device=b.device))
        return make_lambda(c, lambda r: True)

    def get_projection(self, c):
        if not self.vectorized:
            def flat(r):
                return [SupplierInfo(li.supplier.name, r.name, li.part.partKey) for o in r.orders
                        for li in o.lineItems]

            return make_lambda(c, flat)

        def flat_batch(b):
            lb, cust = line_items(b)
            info = RecordBatch({"supplierName": lb.columns["supplier"].columns["name"],
                                "customer": column_take(b.columns["name"], cust),
                                "part": lb.columns["part"].columns["partKey"]}, int(cust.numel()), SupplierInfo)
            # line items arrive grouped by customer (orders keep customer order), so one count per customer
            counts = torch.bincount(cust, minlength=b.n)
            return NestedColumn(_offsets(counts), info)

        return make_batch_lambda(c, flat_batch)


class CustomerSupplierPartGroupBy(AggregateComp):
    reduce_op = None

    def __init__(self, vectorized: bool = True):
        super().__init__()
        self.vectorized = vectorized

    def get_key_projection(self, s):
        return make_lambda_from_member(s, "supplierName")

    def get_value_projection(self, s):
        if not self.vectorized:
            return make_lambda(s, lambda r: {r.customer: [r.part]})

        def one_entry_maps(b):
            part = b.columns["part"]
            ar = torch.arange(b.n + 1, dtype=torch.int64, device=part.device)
            return MapColumn(ar, b.columns["customer"], NestedColumn(ar.clone(), part))

        return make_batch_lambda(s, one_entry_maps)

    def combine(self, a, b):
        out = {k: list(v) for k, v in a.items()}
        for k, v in b.items():
            out.setdefault(k, []).extend(v)
        return out

    def make_output(self, keys, values):
        if isinstance(values, MapColumn):
            return RecordBatch({"supplierName": keys, "soldPartIDs": values}, len(values), SupplierParts)
        return RecordBatch.from_objects([SupplierParts(k, v) for k, v in zip(keys, values)], SupplierParts)


class TopJaccard(TopKComp):
    """Top-k customers by Jaccard similarity of their distinct purchased parts to ``parts``."""

    def __init__(self, k: int, parts: List[int]):
        super().__init__(k)
        self.parts = torch.tensor(sorted(set(parts)), dtype=torch.int64)

    def get_value_projection(self, c):
        def score(b):
            lb, cust = line_items(b)
            pk = lb.columns["part"].columns["partKey"]
            dev = pk.device
            # distinct (customer, part) pairs
            span = int(pk.max()) + 1 if pk.numel() else 1
            pairs = torch.unique(cust * span + pk)
            pc, pp = pairs // span, pairs % span
            q = self.parts.to(dev)
            inter = torch.zeros(b.n, dtype=torch.float64, device=dev).index_add_(0, pc, torch.isin(pp, q).double())
            size = torch.bincount(pc, minlength=b.n).double()
            return inter / (size + q.numel() - inter).clamp_min(1)

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


def supplier_groupby(client, db: str, vectorized: bool = True) -> Dict[str, Dict[str, List[int]]]:
    flat = CustomerMultiSelection(vectorized).set_input(ScanSet(db, "customers", BCustomer))
    got = _run(client, db, "bench_gb", CustomerSupplierPartGroupBy(vectorized).set_input(flat), "tpchbench_groupby")
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
