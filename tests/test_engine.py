"""End-to-end query tests on the CPU pseudo-cluster path (reference test strategy: src/tests/source
Test*.cc selection/join/aggregation programs checked against expected outputs)."""
import pytest
import torch

from netsdb_amd.client import PDBClient
from netsdb_amd.computations import AggregateComp, JoinComp, MultiSelectionComp, ScanSet, SelectionComp, TopKComp, WriteSet
from netsdb_amd.lambdas import make_lambda, make_lambda_from_member, make_lambda_from_method, make_lambda_from_self
from netsdb_amd.objects import PDBObject, RecordBatch
from netsdb_amd.objects.builtin import DepartmentTotal, Employee, StringIntPair


class Dept(PDBObject):
    name: str
    floor: int


class EmpDept(PDBObject):
    emp: str
    dept: str
    floor: int


class OlderThan(SelectionComp):
    def __init__(self, age):
        super().__init__()
        self.age = age

    def get_selection(self, e):
        return make_lambda_from_member(e, "age") > self.age

    def get_projection(self, e):
        return make_lambda_from_self(e)


class NameOnly(SelectionComp):
    def get_selection(self, e):
        return make_lambda(e, lambda r: r.department == "eng")

    def get_projection(self, e):
        return make_lambda(e, lambda r: StringIntPair(r.name, r.age))


class EmpJoinDept(JoinComp):
    def get_selection(self, e, d):
        return make_lambda_from_member(e, "department") == make_lambda_from_member(d, "name")

    def get_projection(self, e, d):
        return make_lambda(e, d, lambda a, b: EmpDept(a.name, b.name, b.floor))


class SalaryByDept(AggregateComp):
    def get_key_projection(self, e):
        return make_lambda_from_method(e, "getDepartment")

    def get_value_projection(self, e):
        return make_lambda_from_method(e, "getSalary")

    def make_output(self, keys, values):
        return RecordBatch.from_objects([DepartmentTotal(k, float(v)) for k, v in zip(keys, values.tolist())],
                                        DepartmentTotal)


class Explode(MultiSelectionComp):
    def get_projection(self, e):
        return make_lambda(e, lambda r: [StringIntPair(r.name, i) for i in range(r.age % 3)])


class TopSalary(TopKComp):
    def get_value_projection(self, e):
        return make_lambda_from_member(e, "salary")


def _emps(n=50):
    depts = ["eng", "ops", "sales", "hr"]
    return [Employee(f"e{i}", 20 + (i * 7) % 40, depts[i % 4], 1000.0 + i) for i in range(n)]


def _client(tmp_path):
    c = PDBClient(root=str(tmp_path), page_size=1 << 12)
    c.create_database("db")
    c.create_set("db", "emps", Employee)
    c.send_data("db", "emps", _emps())
    return c


def test_selection(tmp_path):
    c = _client(tmp_path)
    c.create_set("db", "old", Employee)
    s = OlderThan(40)
    s.set_input(ScanSet("db", "emps", Employee))
    w = WriteSet("db", "old")
    w.set_input(s)
    c.execute_computations(w)
    got = sorted(o.name for o in c.get_set_iterator("db", "old"))
    exp = sorted(e.name for e in _emps() if e.age > 40)
    assert got == exp and got


def test_native_lambda_selection(tmp_path):
    c = _client(tmp_path)
    c.create_set("db", "names", StringIntPair)
    s = NameOnly()
    s.set_input(ScanSet("db", "emps", Employee))
    w = WriteSet("db", "names").set_input(s)
    c.execute_computations(w)
    got = sorted((o.myString, o.myInt) for o in c.get_set_iterator("db", "names"))
    assert got == sorted((e.name, e.age) for e in _emps() if e.department == "eng")


def test_join(tmp_path):
    c = _client(tmp_path)
    c.create_set("db", "depts", Dept)
    c.send_data("db", "depts", [Dept("eng", 3), Dept("ops", 1), Dept("hr", 2)])
    c.create_set("db", "out", EmpDept)
    j = EmpJoinDept()
    j.set_input(0, ScanSet("db", "emps", Employee))
    j.set_input(1, ScanSet("db", "depts", Dept))
    c.execute_computations(WriteSet("db", "out").set_input(j))
    got = sorted((o.emp, o.dept, o.floor) for o in c.get_set_iterator("db", "out"))
    floors = {"eng": 3, "ops": 1, "hr": 2}
    exp = sorted((e.name, e.department, floors[e.department]) for e in _emps() if e.department in floors)
    assert got == exp


def test_aggregate(tmp_path):
    c = _client(tmp_path)
    c.create_set("db", "totals", DepartmentTotal)
    a = SalaryByDept()
    a.set_input(ScanSet("db", "emps", Employee))
    c.execute_computations(WriteSet("db", "totals").set_input(a))
    got = {o.department: o.total for o in c.get_set_iterator("db", "totals")}
    exp = {}
    for e in _emps():
        exp[e.department] = exp.get(e.department, 0.0) + e.salary
    assert got.keys() == exp.keys()
    for k in exp:
        assert abs(got[k] - exp[k]) < 1e-6


def test_multiselection_and_topk(tmp_path):
    c = _client(tmp_path)
    c.create_set("db", "flat", StringIntPair)
    m = Explode()
    m.set_input(ScanSet("db", "emps", Employee))
    c.execute_computations(WriteSet("db", "flat").set_input(m))
    assert sum(1 for _ in c.get_set_iterator("db", "flat")) == sum(e.age % 3 for e in _emps())
    c.create_set("db", "top", Employee)
    t = TopSalary(5)
    t.set_input(ScanSet("db", "emps", Employee))
    c.execute_computations(WriteSet("db", "top").set_input(t))
    got = sorted(o.salary for o in c.get_set_iterator("db", "top"))
    assert got == sorted(e.salary for e in _emps())[-5:]


def test_tcap_roundtrip(tmp_path):
    c = _client(tmp_path)
    j = EmpJoinDept()
    j.set_input(0, ScanSet("db", "emps", Employee))
    j.set_input(1, ScanSet("db", "emps", Employee))
    text = c.explain(WriteSet("db", "x").set_input(j))
    assert "HASHLEFT" in text and "JOIN" in text and "OUTPUT" in text and "stage" in text


def test_chained_selection_join_aggregate(tmp_path):
    """selection -> join -> aggregate -> write in ONE job (multi-stage pipeline with breakers)."""
    c = _client(tmp_path)
    c.create_set("db", "depts", Dept)
    c.send_data("db", "depts", [Dept("eng", 3), Dept("ops", 1), Dept("sales", 2), Dept("hr", 9)])

    class FloorSum(AggregateComp):
        def get_key_projection(self, r):
            return make_lambda_from_member(r, "dept")

        def get_value_projection(self, r):
            return make_lambda_from_member(r, "floor")

    s = OlderThan(30).set_input(ScanSet("db", "emps", Employee))
    j = EmpJoinDept()
    j.set_input(0, s)
    j.set_input(1, ScanSet("db", "depts", Dept))
    a = FloorSum().set_input(j)
    c.create_set("db", "res", None)
    c.execute_computations(WriteSet("db", "res").set_input(a))
    got = {}
    for b in c.get_set_batches("db", "res"):
        for k, v in zip(b.columns["key"], b.columns["value"].tolist()):
            got[k] = v
    floors = {"eng": 3, "ops": 1, "sales": 2, "hr": 9}
    exp = {}
    for e in _emps():
        if e.age > 30:
            exp[e.department] = exp.get(e.department, 0) + floors[e.department]
    assert got == exp
    _ = torch


@pytest.mark.gpu
def test_topk_on_device_gpu(tmp_path):
    """TopKComp on a device set: scores never leave the GPU (no .cpu()/.tolist()/.item() of them inside the TopK
    sink; string object columns read only their byte bounds), result matches the host top 5."""
    from netsdb_amd.execution.engine import QueryEngine

    c = PDBClient(root=str(tmp_path), page_size=1 << 12, device="cuda:0")
    c.create_database("db")
    c.create_set("db", "emps", Employee)
    c.send_data("db", "emps", _emps(300))
    c.create_set("db", "top", Employee)
    calls = []
    orig_topk = QueryEngine._topk
    orig = {k: getattr(torch.Tensor, k) for k in ("cpu", "tolist", "item")}

    def guard(name):
        def w(self, *a, **kw):
            import traceback

            fr = traceback.extract_stack(limit=3)[0]
            calls.append((name, self.numel(), f"{fr.filename.rsplit('/', 2)[-1]}:{fr.lineno}"))
            return orig[name](self, *a, **kw)
        return w

    def guarded_topk(self, *a, **kw):
        for k in orig:
            setattr(torch.Tensor, k, guard(k))
        try:
            return orig_topk(self, *a, **kw)
        finally:
            for k, f in orig.items():
                setattr(torch.Tensor, k, f)

    QueryEngine._topk = guarded_topk
    try:
        t = TopSalary(5)
        t.set_input(ScanSet("db", "emps", Employee))
        c.execute_computations(WriteSet("db", "top").set_input(t))
    finally:
        QueryEngine._topk = orig_topk
    # the 300 scores never leave the device: the only host reads allowed are the string columns' byte bounds
    # (two int64 per concatenated part) when the winners' object rows are assembled
    assert all(n <= 64 and "engine.py" not in site for _, n, site in calls), calls
    got = sorted(o.salary for o in c.get_set_iterator("db", "top"))
    assert got == sorted(e.salary for e in _emps(300))[-5:]


def test_lazy_take_columns_behave_as_dict(monkeypatch):
    """Row selections of wide batches gather each column on first access (objects/record.py LazyTakeColumns);
    every dict operation the engine and UDFs use sees all columns, with the gathered values."""
    from netsdb_amd.objects import record as R

    monkeypatch.setattr(R, "LAZY_TAKE_ANY_DEVICE", True)
    cols = {f"c{i}": torch.arange(10) * (i + 1) for i in range(6)}
    b = R.RecordBatch(dict(cols), 10)
    idx = torch.tensor([1, 4, 7])
    t = b.take(idx)
    assert isinstance(t.columns, R.LazyTakeColumns) and t.n == 3
    assert dict.__len__(t.columns) == 0                       # nothing gathered yet
    assert t.columns["c2"].tolist() == [3, 12, 21]
    assert dict.__len__(t.columns) == 1
    assert list(t.columns) == list(cols) and len(t.columns) == 6 and "c5" in t.columns
    t.columns["new"] = torch.zeros(3)
    del t.columns["c0"]
    assert "c0" not in t.columns and list(t.columns)[-1] == "new"
    d = dict(t.columns)
    assert set(d) == {"c1", "c2", "c3", "c4", "c5", "new"} and d["c4"].tolist() == [5, 20, 35]
    assert {**t.columns}.keys() == d.keys()
    assert [k for k, _ in t.columns.items()] == list(d)
    assert R.RecordBatch.concat([t, t]).columns["c1"].tolist() == [2, 8, 14] * 2


def test_lazy_take_nbytes_and_storage_do_not_gather(monkeypatch, tmp_path):
    from netsdb_amd.client import PDBClient
    from netsdb_amd.objects import record as R

    monkeypatch.setattr(R, "LAZY_TAKE_ANY_DEVICE", True)
    b = R.RecordBatch({f"c{i}": torch.arange(100, dtype=torch.float64) for i in range(6)}, 100)
    t = b.take(torch.arange(0, 100, 4))
    assert t.nbytes() == 6 * 25 * 8 and dict.__len__(t.columns) == 0     # estimated, nothing gathered
    m = t.materialize()
    assert type(m.columns) is dict and m.columns["c3"].tolist() == list(range(0, 100, 4))
    c = PDBClient(root=str(tmp_path))
    c.create_database("d")
    c.create_set("d", "s", None)
    s = c.storage.get_set("d", "s")
    s.add_batch(t)
    assert all(type(p.batch.columns) is dict for p in s.pages)


def test_lazy_take_device_and_values_gather_only_what_they_touch():
    """RecordBatch.device of a lazy row selection reads its source (no gather); values() / items() gather as they
    iterate, so a loop that stops at the first column gathers one."""
    from netsdb_amd.objects import record as R

    src = {f"c{i}": torch.arange(10) * i for i in range(8)}
    lt = R.LazyTakeColumns(src, torch.tensor([1, 3, 5]))
    b = RecordBatch(lt, 3)
    assert b.device == torch.device("cpu") and not any(dict.__contains__(lt, k) for k in src)
    first = next(iter(lt.values()))
    assert first.tolist() == [0, 0, 0] and sum(dict.__contains__(lt, k) for k in src) == 1
    assert len(lt.values()) == 8 and [k for k, _ in lt.items()] == [f"c{i}" for i in range(8)]
    assert [v.tolist() for v in lt.values()][2] == [2, 6, 10]


def test_stage_records_and_history_device_time_cpu(tmp_path):
    """On the CPU a stage record carries no device time (no event pair), the tracer's device mode is inert, and the
    history's job_stage table has the device_seconds column (NULL here)."""
    from netsdb_amd.client import PDBClient
    from netsdb_amd.models import tpch, tpch_gen
    from netsdb_amd.utils.trace import Tracer

    c = PDBClient(root=str(tmp_path))
    tpch.load(c, "tpch", tpch_gen.generate_fast(0.001, seed=3))
    sl = c.enable_self_learning()
    tpch.QUERIES["q06"](c, "tpch")
    st = sl.last_stats
    assert st["stages"] and all("device_seconds" not in s for s in st["stages"])
    assert st.device_times() == [None] * len(st["stages"])
    cols = {r[1] for r in sl.db.conn.execute("PRAGMA table_info(job_stage)")}
    assert "device_seconds" in cols and sl.db.flush_device_times() == 0
    tr = Tracer(device_time=True)
    with tr.span("x"):
        pass
    assert tr.resolve() == 0 and "device_us" not in tr.events[0]["args"]
    tr.export_chrome(str(tmp_path / "t.json"))
