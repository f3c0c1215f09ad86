"""Fused filter -> project -> aggregate stages (execution/pipeline.py + csrc/kernels/pipeline.hip): the TPC-H Q01 /
Q06 / Q12 / Q14 lambda trees compiled into the device interpreter's register program. On CPU the compiled program
runs on the torch interpreter of the same instruction set (the compiler's check); on the GPU the kernel runs and
must match the eager per-atom path and the pandas oracle. Reference: src/lambdas/headers/Pipeline.h:57,194."""
import math
import tempfile

import pytest
import torch

from netsdb_amd.client import PDBClient
from netsdb_amd.computations import AggregateComp, ScanSet, SelectionComp, WriteSet
from netsdb_amd.execution import pipeline as PL
from netsdb_amd.lambdas import IsIn, KeyTuple, Like, Literal, Select, Values, make_lambda_from_self
from netsdb_amd.models import tpch, tpch_gen

QUERIES = ("q01", "q06", "q12", "q14")
FILTER_QUERIES = ("q03", "q04", "q17", "q13", "q22", "q02")   # tree-lambda FILTERs, joins, emitted aggregations


def _close(a, b):
    if isinstance(a, float):
        return math.isclose(a, b, rel_tol=1e-9, abs_tol=1e-6)
    if isinstance(a, list):
        return len(a) == len(b) and all(_close(x, y) for x, y in zip(a, b))
    if isinstance(a, dict):
        return all(_close(a[k], b[k]) for k in b)
    return a == b


def _ref(q, t, f):
    ref = tpch.reference(q, t, f=f)
    if q == "q01":
        ref = sorted(ref, key=lambda x: (x["l_returnflag"], x["l_linestatus"]))
    elif q in ("q04", "q12", "q22"):
        ref = sorted(ref, key=lambda x: x[list(x)[0]])
    return ref


def _client(dev, t):
    c = PDBClient(root=tempfile.mkdtemp(), device=dev)
    tpch.load(c, "tpch", t, device=dev)
    return c


def test_fused_tpch_cpu_interpreter(monkeypatch):
    monkeypatch.setenv("NSDB_DEVICE_STRINGS", "1")
    monkeypatch.setattr(PL, "CPU_INTERPRETER", True)
    t = tpch_gen.generate_fast(0.003, seed=4)
    f = tpch.frames(t)
    c = _client("cpu", t)
    for q in QUERIES + FILTER_QUERIES:
        got = tpch.QUERIES[q](c, "tpch")
        assert _close(got, _ref(q, t, f)), (q, got)
    st = c.engine.pipeline_stats
    assert st["fused_stages"] >= len(QUERIES) and st["fallback_batches"] == 0, st
    assert st.get("fused_filters", 0) >= 5, st


def test_jit_sources_compile_cpu(monkeypatch):
    """Every TPC-H stage program's run-time kernel source (aggregate and mask forms, early and late columns, both
    string kinds) compiles with hiprtc for gfx950 — no GPU needed to compile; the GPU tests run the kernels."""
    from netsdb_amd import _ext
    if not _ext.hip_available() or not hasattr(_ext.hip(), "jit_compile"):
        pytest.skip("kernel extension not built")
    monkeypatch.setenv("NSDB_DEVICE_STRINGS", "1")
    monkeypatch.setattr(PL, "CPU_INTERPRETER", True)
    PL._PROG_CACHE.clear()
    t = tpch_gen.generate_fast(0.002, seed=4)
    c = _client("cpu", t)
    for q in QUERIES + FILTER_QUERIES:
        tpch.QUERIES[q](c, "tpch")
    progs = list(PL._PROG_CACHE.values())
    assert len(progs) >= len(QUERIES) + len(FILTER_QUERIES), len(progs)
    h, hdr, seen = _ext.hip(), PL._jit_header(), set()
    joins = pairs = 0
    for p in progs:
        kinds = [cc["kind"] for cc in p.cols]
        lates = [cc["late"] for cc in p.cols]
        if p.mode == "pairs":                  # a fused filter + probe outside an aggregation: (probe, build) rows
            pairs += 1
            src = PL.jit_source(p, kinds, lates, "pairs")
            assert "jit_emit_body" in src and "w[1] = (u64)brow" in src
            if src not in seen:
                seen.add(src)
                assert len(h.jit_compile(src, hdr)) > 1000
            continue
        if p.jk_reg >= 0:                      # a fused join probe: the aggregate kernel only (jit_join_agg_body)
            joins += 1
            src = PL.jit_source(p, kinds, lates, "agg", p.key_reg, p.val_regs)
            assert "jit_join_agg_body" in src and "brow[j]" in src
            if src not in seen:
                seen.add(src)
                assert len(h.jit_compile(src, hdr)) > 1000
            continue
        srcs = [PL.jit_source(p, kinds, lates, "mask")]
        if p.val_regs or p.key_reg >= 0:
            srcs.append(PL.jit_source(p, kinds, lates, "agg", p.key_reg, p.val_regs))
            srcs.append(PL.jit_source(p, [PL.C_I64 if k == PL.C_SCODE else k for k in kinds], [1] * len(kinds), "agg",
                                      p.key_reg, p.val_regs))
        for src in srcs:
            if src not in seen:
                seen.add(src)
                assert len(h.jit_compile(src, hdr)) > 1000
    assert len(seen) >= len(progs) - pairs     # pairs programs of one shape share a source
    assert joins >= 2, joins                   # q12 and q14 probe their build tables inside the fused kernel
    assert pairs >= 3, pairs                   # q02 / q03 / q04 filter + probe stages
    # the emitted (high-cardinality) form of every stage: tables capped so each stage overflows once
    PL._PROG_CACHE.clear()
    PL._EMIT_SIGS.clear()
    monkeypatch.setattr(PL, "INTERP_CAP", 0)
    for q in QUERIES:
        tpch.QUERIES[q](c, "tpch")
    emits = [p for p in PL._PROG_CACHE.values() if p.mode == "emit"]
    assert len(emits) >= len(QUERIES), len(emits)
    for p in emits:
        kinds = [cc["kind"] for cc in p.cols]
        src = PL.jit_source(p, kinds, [cc["late"] for cc in p.cols], "emit", -1, p.val_regs)
        assert "jit_emit_body" in src
        assert len(h.jit_compile(src, hdr)) > 1000


class _Sel(SelectionComp):
    def __init__(self, pred):
        super().__init__()
        self.pred = pred

    def get_selection(self, x):
        return self.pred(x)

    def get_projection(self, x):
        return make_lambda_from_self(x)


class _Agg(AggregateComp):
    def __init__(self, key, val, op="sum"):
        super().__init__()
        self.key, self.val, self.reduce_op = key, val, op

    def get_key_projection(self, x):
        return self.key(x)

    def get_value_projection(self, x):
        return self.val(x)


_JOBS = [0]


def _agg_job(c, pred, key, val, op="sum"):
    _JOBS[0] += 1
    out = f"o{_JOBS[0]}"
    c.create_set("tpch", out, None)
    comp = _Agg(key, val, op).set_input(_Sel(pred).set_input(ScanSet("tpch", "lineitem", tpch.LineItem)))
    c.execute_computations(WriteSet("tpch", out).set_input(comp))
    b = [x for x in c.get_set_batches("tpch", out) if x.n]
    assert len(b) == 1
    b = b[0]
    keys = [b.columns[k] for k in sorted(k for k in b.columns if k.startswith("key"))]
    keys = [k.tolist() if hasattr(k, "tolist") else list(k) for k in keys]
    vals = b.columns["value"]
    order = sorted(range(b.n), key=lambda i: tuple(k[i] for k in keys))
    return [tuple(k[i] for k in keys) for i in order], vals[torch.tensor(order)].double().cpu()


CASES = {
    "min_max_int_key": (lambda x: (x.l_quantity > 10) | (x.l_tax == 0.0), lambda x: x.l_linenumber,
                        lambda x: Values(x.l_extendedprice, x.l_discount * 2.0 - x.l_tax), "max"),
    "min": (lambda x: ~(x.l_shipmode == "AIR"), lambda x: KeyTuple(x.l_linestatus, x.l_returnflag),
            lambda x: Values(x.l_quantity / 3, -x.l_tax), "min"),
    "isin_like_select": (lambda x: IsIn(x.l_shipmode, ["MAIL", "TRUCK", "REG AIR"]) & Like(x.l_shipinstruct, "%PERSON"),
                         lambda x: x.l_linestatus,
                         lambda x: Values(Select(x.l_discount < 0.05, x.l_quantity, 0), 1.0),
                         "sum"),
    # general LIKE (contains, several segments, '_', anchored both ends) through the compiled matcher
    "like_general": (lambda x: (Like(x.l_comment, "%ar%ly%") | Like(x.l_shipinstruct, "D_L%SON")) &
                     ~Like(x.l_shipmode, "%AI%"),
                     lambda x: x.l_returnflag, lambda x: Values(x.l_quantity, 1.0), "sum"),
}


@pytest.mark.parametrize("case", sorted(CASES))
def test_fused_operators_cpu_interpreter(case, monkeypatch):
    """Each operator class (or, not, string ==, IN, LIKE suffix, CASE, min / max, int keys, composite string keys)
    through the compiler: fused (torch interpreter) == eager."""
    monkeypatch.setenv("NSDB_DEVICE_STRINGS", "1")
    pred, key, val, op = CASES[case]
    t = tpch_gen.generate_fast(0.002, seed=9)
    c = _client("cpu", t)
    eager = _agg_job(c, pred, key, val, op)
    monkeypatch.setattr(PL, "CPU_INTERPRETER", True)
    n0 = c.engine.pipeline_stats["fused_batches"]
    fused = _agg_job(c, pred, key, val, op)
    assert c.engine.pipeline_stats["fused_batches"] > n0
    assert eager[0] == fused[0]
    assert torch.allclose(eager[1], fused[1], rtol=1e-12, atol=1e-9)


def test_fused_stage_cache_keys_constants(monkeypatch):
    """Repeated graphs re-use their fused stage expressions (plan_stage's cache), but a literal, IN list or LIKE
    pattern that changes between runs of the same graph shape must change the plan: fused == eager for each."""
    monkeypatch.setenv("NSDB_DEVICE_STRINGS", "1")
    t = tpch_gen.generate_fast(0.002, seed=9)
    c = _client("cpu", t)
    variants = [(q, modes, pat) for q in (10, 30) for modes in (["MAIL"], ["TRUCK", "AIR"]) for pat in ("%PERSON", "%RN")]

    def job(q, modes, pat):
        return _agg_job(c, lambda x: (x.l_quantity > q) & IsIn(x.l_shipmode, modes) & Like(x.l_shipinstruct, pat),
                        lambda x: x.l_linestatus, lambda x: Values(x.l_extendedprice), "sum")

    eager = [job(*v) for v in variants]
    monkeypatch.setattr(PL, "CPU_INTERPRETER", True)
    PL._STAGE_CACHE.clear()
    for _ in range(2):                               # the second pass hits the cache for every variant
        for v, e in zip(variants, eager):
            f = job(*v)
            assert e[0] == f[0] and torch.allclose(e[1], f[1], rtol=1e-12, atol=1e-9), v
    assert len(PL._STAGE_CACHE) == len(variants)


def test_fused_program_cache_rechecks_string_key_bound(monkeypatch):
    """A compiled program fixes a string key's short-code bound L. A later batch of the same stage whose string
    lengths are not known yet (same program-cache key) but exceed L must not reuse that program: it recompiles
    (or runs eagerly), and the groups stay distinct — fused == eager after the set's strings got longer."""
    from netsdb_amd.objects.strings import StringColumn

    monkeypatch.setenv("NSDB_DEVICE_STRINGS", "1")
    t = tpch_gen.generate_fast(0.002, seed=9)
    c = _client("cpu", t)
    args = (lambda x: x.l_quantity > 1, lambda x: x.l_returnflag, lambda x: Values(x.l_extendedprice), "sum")
    monkeypatch.setattr(PL, "CPU_INTERPRETER", True)
    PL._PROG_CACHE.clear()
    first = _agg_job(c, *args)
    assert {k[0] for k in first[0]} <= {"A", "N", "R"}
    # the same set, rewritten with longer flags ("A" -> "AX1", "N" -> "N", "R" -> "RYY2"): distinct 1-byte prefixes
    # would merge if the 1-byte program were reused
    b = [x for x in c.get_set_batches("tpch", "lineitem") if x.n]
    rows = {k: v for k, v in b[0].columns.items()}
    flags = rows["l_returnflag"].tolist() if isinstance(rows["l_returnflag"], StringColumn) else list(rows["l_returnflag"])
    longer = {"A": "AX1", "N": "N", "R": "RYY2"}
    new_flags = [longer[f] for f in flags]
    newcol = StringColumn.from_list(new_flags)
    newcol._maxlen = None                              # bound unknown: the cache key cannot tell it apart
    rows["l_returnflag"] = newcol
    c.clear_set("tpch", "lineitem")
    c.send_data("tpch", "lineitem", type(b[0])(rows, b[0].n))
    fused = _agg_job(c, *args)
    monkeypatch.setattr(PL, "CPU_INTERPRETER", False)
    eager = _agg_job(c, *args)
    assert {k[0] for k in fused[0]} == {"AX1", "N", "RYY2"}
    assert eager[0] == fused[0] and torch.allclose(eager[1], fused[1], rtol=1e-12, atol=1e-9)


def test_fused_overflow_falls_back(monkeypatch):
    """More groups than the kernel's per-workgroup tables: the batch takes the eager atoms, same result."""
    monkeypatch.setenv("NSDB_DEVICE_STRINGS", "1")
    t = tpch_gen.generate_fast(0.002, seed=9)
    c = _client("cpu", t)
    args = (lambda x: x.l_quantity > 1, lambda x: x.l_orderkey, lambda x: Values(x.l_extendedprice), "sum")
    eager = _agg_job(c, *args)
    monkeypatch.setattr(PL, "CPU_INTERPRETER", True)
    monkeypatch.setattr(PL, "INTERP_CAP", 64)      # the interpreter models the kernel's table capacity
    monkeypatch.setattr(PL, "EMIT", False)         # without the emitted form: the eager atoms
    fused = _agg_job(c, *args)
    assert c.engine.pipeline_stats["fallback_batches"] >= 1
    assert eager[0] == fused[0] and torch.allclose(eager[1], fused[1])


EMIT_CASES = {
    # one integer key with more groups than the kernel's table: every kept row emitted, reduced by the group-by
    "int_key": (lambda x: x.l_quantity > 1, lambda x: x.l_orderkey, lambda x: Values(x.l_extendedprice, 1.0), "sum"),
    # a composite key of an integer, a float and a short string (not packable into one word), min
    "composite_key": (lambda x: x.l_shipmode == "AIR", lambda x: KeyTuple(x.l_partkey, x.l_discount, x.l_returnflag),
                      lambda x: Values(x.l_quantity * x.l_tax), "min"),
    # a string key part longer than a short code (17-byte ship instructions): emitted as its row, taken afterwards
    "long_string_key": (lambda x: x.l_quantity > 30, lambda x: KeyTuple(x.l_partkey, x.l_shipinstruct),
                        lambda x: Values(x.l_quantity), "sum"),
}


@pytest.mark.parametrize("case", sorted(EMIT_CASES))
def test_fused_emit_cpu_interpreter(case, monkeypatch):
    """High-cardinality stages: the emitted form (torch model of jit_emit_body) == the eager atoms."""
    monkeypatch.setenv("NSDB_DEVICE_STRINGS", "1")
    t = tpch_gen.generate_fast(0.002, seed=9)
    c = _client("cpu", t)
    eager = _agg_job(c, *EMIT_CASES[case])
    monkeypatch.setattr(PL, "CPU_INTERPRETER", True)
    monkeypatch.setattr(PL, "INTERP_CAP", 64)
    PL._EMIT_SIGS.clear()
    e0 = c.engine.pipeline_stats.get("emitted_batches", 0)
    fused = _agg_job(c, *EMIT_CASES[case])
    fused2 = _agg_job(c, *EMIT_CASES[case])        # the stage now starts in the emitted form
    assert c.engine.pipeline_stats.get("emitted_batches", 0) >= e0 + 2, c.engine.pipeline_stats
    for f in (fused, fused2):
        assert eager[0] == f[0]
        assert torch.allclose(eager[1], f[1], rtol=1e-12, atol=1e-9)


@pytest.mark.gpu
@pytest.mark.parametrize("case", sorted(EMIT_CASES))
def test_fused_emit_gpu(case):
    """The compiled emit kernel (per-tile regions, workgroup scan, compaction) == the eager atoms, 10 k+ groups."""
    t = tpch_gen.generate_fast(0.05, seed=9)
    c = _client("cuda:0", t)
    c.engine.fused_pipelines = False
    eager = _agg_job(c, *EMIT_CASES[case])
    c.engine.fused_pipelines = True
    e0 = c.engine.pipeline_stats.get("emitted_batches", 0)
    fused = _agg_job(c, *EMIT_CASES[case])
    fused2 = _agg_job(c, *EMIT_CASES[case])
    assert c.engine.pipeline_stats.get("emitted_batches", 0) >= e0 + 2, c.engine.pipeline_stats
    assert len(eager[0]) > 2048
    for f in (fused, fused2):
        assert eager[0] == f[0]
        assert torch.allclose(eager[1], f[1], rtol=1e-9, atol=1e-9)


@pytest.mark.gpu
def test_fused_emit_gpu_million_groups():
    """1 M+ groups (every order key of SF 0.7) through the emitted form: exact against the eager atoms."""
    t = tpch_gen.generate_fast(0.7, seed=5)
    c = _client("cuda:0", t)
    args = (lambda x: x.l_quantity > 0, lambda x: x.l_orderkey, lambda x: Values(x.l_quantity, 1.0), "sum")
    c.engine.fused_pipelines = False
    eager = _agg_job(c, *args)
    c.engine.fused_pipelines = True
    e0 = c.engine.pipeline_stats.get("emitted_batches", 0)
    fused = _agg_job(c, *args)
    assert c.engine.pipeline_stats.get("emitted_batches", 0) > e0, c.engine.pipeline_stats
    assert len(eager[0]) >= 1_000_000
    assert eager[0] == fused[0]
    assert torch.equal(eager[1], fused[1])         # integer-valued sums: exact whatever the order


@pytest.mark.gpu
@pytest.mark.parametrize("tile,jit", [(-2, True), (-2, False), (-1, False), (0, False)],
                         ids=["compiled", "lds_tile", "hybrid", "register"])
def test_fused_tpch_gpu_vs_eager_and_pandas(tile, jit, monkeypatch):
    """Every kernel shape (run-time compiled; LDS-tile, hybrid and register interpreters) against the eager path and
    pandas."""
    monkeypatch.setattr(PL, "TILE", tile)
    monkeypatch.setattr(PL, "JIT", jit)
    j0 = dict(PL.JIT_STATS)
    t = tpch_gen.generate_fast(0.05, seed=4)
    f = tpch.frames(t)
    c = _client("cuda:0", t)
    for q in QUERIES + FILTER_QUERIES:
        c.engine.fused_pipelines = True
        got = tpch.QUERIES[q](c, "tpch")
        c.engine.fused_pipelines = False
        eager = tpch.QUERIES[q](c, "tpch")
        ref = _ref(q, t, f)
        assert _close(got, ref), (q, got, ref)
        assert _close(eager, ref), q
    st = c.engine.pipeline_stats
    assert st["fused_stages"] >= len(QUERIES), st
    if jit:     # every fused launch took a compiled kernel; the emitted form and join probes exist there only
        assert st["fallback_batches"] == 0, st
        assert st.get("fused_join_batches", 0) >= 3 and st.get("emitted_batches", 0) >= 1, st
        assert st.get("fused_probes", 0) >= 3, st     # q02 / q03 / q04: filter + probe stages as "pairs" launches
        assert PL.JIT_STATS["failed"] == j0["failed"], PL.JIT_STATS
        assert PL.JIT_STATS["launches"] - j0["launches"] >= len(QUERIES) + len(FILTER_QUERIES), PL.JIT_STATS
    else:
        assert PL.JIT_STATS["launches"] == j0["launches"]


@pytest.mark.gpu
@pytest.mark.parametrize("case", sorted(CASES))
def test_fused_operators_gpu(case):
    pred, key, val, op = CASES[case]
    t = tpch_gen.generate_fast(0.01, seed=9)
    c = _client("cuda:0", t)
    c.engine.fused_pipelines = False
    eager = _agg_job(c, pred, key, val, op)
    c.engine.fused_pipelines = True
    n0 = c.engine.pipeline_stats["fused_batches"]
    fused = _agg_job(c, pred, key, val, op)
    assert c.engine.pipeline_stats["fused_batches"] > n0
    assert eager[0] == fused[0]
    assert torch.allclose(eager[1], fused[1], rtol=1e-9, atol=1e-9)


@pytest.mark.gpu
@pytest.mark.parametrize("emit", [True, False], ids=["emitted", "eager"])
def test_fused_overflow_gpu(emit, monkeypatch):
    """A table overflow re-runs the batch in the emitted form, or (emitted form off) through the eager atoms."""
    monkeypatch.setattr(PL, "EMIT", emit)
    PL._EMIT_SIGS.clear()
    t = tpch_gen.generate_fast(0.01, seed=9)
    c = _client("cuda:0", t)
    args = (lambda x: x.l_quantity > 1, lambda x: x.l_orderkey, lambda x: Values(x.l_extendedprice), "sum")
    c.engine.fused_pipelines = False
    eager = _agg_job(c, *args)
    c.engine.fused_pipelines = True
    fused = _agg_job(c, *args)
    st = c.engine.pipeline_stats
    if emit:
        assert st.get("emitted_batches", 0) >= 1 and st["fallback_batches"] == 0, st
    else:
        assert st["fallback_batches"] >= 1, st
    assert eager[0] == fused[0] and torch.allclose(eager[1], fused[1])


def _table_result(table: torch.Tensor, nval: int):
    host = table.cpu()
    gcap = (host.numel() - 2) // 9
    keys = host[2:2 + gcap]
    occ = (keys != -(1 << 63)).nonzero().flatten()
    order = torch.argsort(keys[occ])
    vals = host[2 + gcap:].view(torch.float64).reshape(gcap, 8)
    return int(host[0]), int(host[1]), keys[occ][order], vals[occ[order], :nval]


@pytest.mark.gpu
def test_pipe_kernel_shapes_gpu():
    """pipe_agg / pipe_mask directly: every tile size and the register kernels on the same program (all column kinds,
    a partial last tile, string keys, compare-AND folding) give the torch interpreter's groups and sums."""
    import struct

    from netsdb_amd import _ext
    from netsdb_amd.objects.strings import StringColumn

    h = _ext.hip()
    dev = torch.device("cuda:0")
    n = 100_003
    g = torch.Generator().manual_seed(3)
    a = torch.randint(0, 100, (n,), generator=g, dtype=torch.int32)
    b = torch.rand(n, generator=g, dtype=torch.float32)
    u = torch.randint(0, 4, (n,), generator=g, dtype=torch.uint8)
    d = torch.rand(n, generator=g, dtype=torch.float64) * 100
    words = ["A", "BB", "CCC"]
    s = StringColumn.from_list([words[i % 3] for i in torch.randint(0, 3, (n,), generator=g).tolist()])
    fb = lambda v: struct.unpack("<q", struct.pack("<d", v))[0]  # noqa: E731
    I = PL.IMM
    # regs: 0 s (scode, L=3), 1 a, 2 b, 3 u, 4 d; keep 5 = a < 50 && b >= 0.25; key 6 = pack(s, u); values d, b*2
    ins = [(PL.OP_LTI, 5, 1, I, -1, 50), (PL.OP_GEF, 5, 2, I, 5, fb(0.25)),
           (PL.OP_PACK, 6, 0, 3, -1, 8), (PL.OP_MULF, 7, 2, I, -1, fb(2.0))]
    prog = PL.Program()
    prog.cols = [{"kind": PL.C_SCODE, "late": 0, "L": 3, "obj": s}, {"kind": PL.C_I32, "late": 0, "L": 0, "obj": a},
                 {"kind": PL.C_F32, "late": 0, "L": 0, "obj": b}, {"kind": PL.C_U8, "late": 0, "L": 0, "obj": u},
                 {"kind": PL.C_F64, "late": 0, "L": 0, "obj": d}]
    prog.ins, prog.nins_a, prog.keep_reg, prog.key_reg, prog.val_regs = [t + (0,) for t in ins], 2, 5, 6, [4, 7]
    ref_k, ref_v = PL.interpret(prog, n, "sum")
    ref_mask = PL.interpret_mask(prog, n)
    gprog = PL.Program()
    gprog.cols = [dict(c, obj=c["obj"].to(dev)) for c in prog.cols]
    cols = PL._col_args(gprog, dev)
    lit = torch.zeros(1, dtype=torch.uint8, device=dev)
    pt = torch.tensor(ins, dtype=torch.int64)
    for tile in (0, -1, -2, 512, 768, 1024, 2048):
        st, kept, k, v = _table_result(h.pipe_agg(pt, 2, cols, lit, n, 5, 6, [4, 7], 0, 0, tile), 2)
        assert st == 0 and kept == int(ref_mask.sum()), tile
        assert torch.equal(k, ref_k), tile
        assert torch.allclose(v, ref_v, rtol=1e-12, atol=1e-9), tile
        m = h.pipe_mask(pt[:2], cols, lit, n, 5, tile).bool().cpu()
        assert torch.equal(m, ref_mask), tile
    # the run-time compiled kernels of the same program: all columns early, then d / b late (kept rows only)
    kinds = [cc[0] for cc in cols]
    for lates in ([0, 0, 0, 0, 0], [0, 0, 0, 1, 1]):
        lcols = [(cc[0], lt) + tuple(cc[2:]) for cc, lt in zip(cols, lates)]
        src = PL.jit_source(prog, kinds, lates, "agg", 6, [4, 7])
        fn = PL.jit_kernel(src, "nsdb_jit_agg")
        assert fn, "compiled aggregate kernel"
        nreg = PL.program_nreg(prog, len(kinds), 6, [4, 7])
        st, kept, k, v = _table_result(h.pipe_agg(pt, 2, lcols, lit, n, 5, 6, [4, 7], 0, 0, -2, [], fn, nreg,
                                                  PL.JIT_ROWS), 2)
        assert st == 0 and kept == int(ref_mask.sum()), lates
        assert torch.equal(k, ref_k), lates
        assert torch.allclose(v, ref_v, rtol=1e-12, atol=1e-9), lates
    mprog = PL.Program()
    mprog.cols, mprog.ins, mprog.nins_a, mprog.keep_reg = prog.cols, prog.ins[:2], 2, 5
    fn = PL.jit_kernel(PL.jit_source(mprog, kinds, [0] * 5, "mask"), "nsdb_jit_mask")
    assert fn, "compiled mask kernel"
    m = h.pipe_mask(pt[:2], cols, lit, n, 5, -2, [], fn, PL.program_nreg(mprog, 5, -1, []), PL.JIT_ROWS).bool().cpu()
    assert torch.equal(m, ref_mask)


def test_jit_every_opcode_and_column_kind_compiles_cpu():
    """One program touching every opcode and every column kind (early and late) through jit_source + hiprtc: the
    generated C++ of each instruction form compiles for gfx950 (the GPU tests check the values)."""
    from netsdb_amd import _ext
    if not _ext.hip_available() or not hasattr(_ext.hip(), "jit_compile"):
        pytest.skip("kernel extension not built")
    I = PL.IMM
    kinds = [PL.C_SCODE, PL.C_SREF, PL.C_F64, PL.C_I64, PL.C_I32, PL.C_F32, PL.C_U8]
    p = PL.Program()
    p.cols = [{"kind": k, "late": 0, "L": 3} for k in kinds]
    p.kpool = [100, 7]
    r = 7
    ins = []
    for op in range(PL.OP_RNGI + 1):
        if op in (PL.OP_SEQ, PL.OP_SPRE, PL.OP_SSUF):
            ins.append((op, r, 1, 1, -1, 3, 0))              # bytes of column 1 (SREF) against literal 0..3
        elif op == PL.OP_SEL:
            ins.append((op, r, 8, 2, -1, 9, 0))
        elif op in (PL.OP_RNGF, PL.OP_RNGI):
            ins.append((op, r, 2 if op == PL.OP_RNGF else 3, -1, 8, 5, (op - PL.OP_RNGF) | (3 << 8)))
        elif PL.OP_LTF <= op <= PL.OP_NEI:
            ins.append((op, r, 2, I, 8, 1, 0))               # compare folded with register 8
        else:
            ins.append((op, r, 3, 4 if op != PL.OP_NOT else -1, -1, 2, 0))
        r = 8 + (len(ins) % 7)
    p.ins, p.nins_a, p.keep_reg, p.key_reg, p.val_regs = ins, 20, 9, 10, [11, 12, 13]
    h, hdr = _ext.hip(), PL._jit_header()
    for lates in ([0] * 7, [0, 0, 1, 1, 1, 1, 1]):
        for kind in ("agg", "mask"):
            src = PL.jit_source(p, kinds, lates, kind, p.key_reg if kind == "agg" else -1,
                                p.val_regs if kind == "agg" else ())
            assert len(h.jit_compile(src, hdr)) > 1000, (kind, lates)


# ---------------------------------------------------------------------------------------------- fused join probes
def _join_agg(c, probe, build, keys, pick, key_fn, val_fn, out, op="sum"):
    """probe ⋈ build (tpch _EqJoin + _pick) -> _TreeGroupBy(key, Values): rows sorted by key."""
    j = tpch._EqJoin(2, keys, tpch._pick(pick))
    j.set_input(0, probe)
    j.set_input(1, build)
    agg = tpch._TreeGroupBy(key_fn, val_fn, tpch._rows_out(["a", "b"]), reduce_op=op)
    if c.storage.has_set("tpch", out):
        c.remove_set("tpch", out)
    c.create_set("tpch", out, None)
    c.execute_computations(WriteSet("tpch", out).set_input(agg.set_input(j)))
    b = [x for x in c.get_set_batches("tpch", out) if x.n][0]
    ks = b.columns["k0"]
    ks = ks.tolist() if hasattr(ks, "tolist") else list(ks)
    order = sorted(range(b.n), key=lambda i: ks[i])
    vals = torch.stack([b.columns["a"].double().cpu(), b.columns["b"].double().cpu()], 1)
    return [ks[i] for i in order], vals[torch.tensor(order)]


JOIN_CASES = {
    # build = supplier (the smaller side) on its REPEATED s_nationkey (CSR runs: several suppliers per nation), probe
    # = customer; a build-side integer key, values from both sides
    "repeated_build_keys": (
        lambda db: ScanSet(db, "customer", tpch.Customer),
        lambda db: ScanSet(db, "supplier", tpch.Supplier),
        [(0, "c_nationkey", 1, "s_nationkey")], [["c_custkey", "c_acctbal"], ["s_acctbal", "s_nationkey"]],
        lambda x: x.s_nationkey,
        lambda x: Values(Select(x.s_acctbal > 0.0, x.s_acctbal, 0.0) + x.c_acctbal * 0.5, 1.0), "sum"),
    # build = orders, probe = one week of lineitems (fused predicate before the probe); a key and a value from the
    # build side (string key at the matched build rows)
    "build_side_string_key": (
        lambda db: tpch._TreeFilter(lambda x: (x.l_shipdate >= 19960101) & (x.l_shipdate < 19960301)).set_input(
            ScanSet(db, "lineitem", tpch.LineItem)),
        lambda db: ScanSet(db, "orders", tpch.Order),
        [(0, "l_orderkey", 1, "o_orderkey")], [["l_quantity"], ["o_orderstatus", "o_totalprice"]],
        lambda x: x.o_orderstatus, lambda x: Values(x.l_quantity * 2.0, Select(x.o_totalprice > 100000.0, 1.0, 0.0)),
        "sum"),
    # build = part (unique p_partkey), probe = a quarter of lineitems; a probe-side key, min of a mixed expression
    "unique_build_keys_min": (
        lambda db: tpch._TreeFilter(lambda x: (x.l_shipdate >= 19950101) & (x.l_shipdate < 19950401)).set_input(
            ScanSet(db, "lineitem", tpch.LineItem)),
        lambda db: ScanSet(db, "part", tpch.Part),
        [(0, "l_partkey", 1, "p_partkey")], [["l_linenumber", "l_extendedprice"], ["p_size", "p_retailprice"]],
        lambda x: x.l_linenumber, lambda x: Values(x.l_extendedprice - x.p_retailprice, x.p_size * 1.0), "min"),
}


def _join_case(c, case):
    probe, build, keys, pick, key_fn, val_fn, op = JOIN_CASES[case]
    return _join_agg(c, probe("tpch"), build("tpch"), keys, pick, key_fn, val_fn, f"j_{case}", op)


@pytest.mark.parametrize("late", [True, False], ids=["late_cols", "early_cols"])
@pytest.mark.parametrize("case", sorted(JOIN_CASES))
def test_fused_join_probe_cpu_interpreter(case, late, monkeypatch):
    """A stage probing a build table inside the fused program (torch model of jit_join_agg_body): == the eager atoms.
    ``early_cols``: the selectivity estimate says "load every probe column in the first pass" (what a GPU run's
    measured estimate does on repeats) — build-side columns must still be read at the matched build rows."""
    monkeypatch.setenv("NSDB_DEVICE_STRINGS", "1")
    if not late:
        monkeypatch.setattr(PL, "LATE_MAX_SEL", -1.0)
    t = tpch_gen.generate_fast(0.003, seed=6)
    c = _client("cpu", t)
    eager = _join_case(c, case)
    assert eager[0], "the case must produce groups"
    monkeypatch.setattr(PL, "CPU_INTERPRETER", True)
    j0 = c.engine.pipeline_stats.get("fused_join_batches", 0)
    fused = _join_case(c, case)
    assert c.engine.pipeline_stats.get("fused_join_batches", 0) > j0, c.engine.pipeline_stats
    assert eager[0] == fused[0]
    assert torch.allclose(eager[1], fused[1], rtol=1e-12, atol=1e-9)


@pytest.mark.gpu
@pytest.mark.parametrize("case", sorted(JOIN_CASES))
def test_fused_join_probe_gpu(case):
    """The compiled join kernel (probe, CSR runs of repeated build keys, build-side gathers, post-join predicate)
    against the eager probe / gather / group-by atoms on the same data."""
    t = tpch_gen.generate_fast(0.05, seed=6)
    c = _client("cuda:0", t)
    c.engine.fused_pipelines = False
    eager = _join_case(c, case)
    c.engine.fused_pipelines = True
    j0 = c.engine.pipeline_stats.get("fused_join_batches", 0)
    f0 = PL.JIT_STATS["launches"]
    fused = _join_case(c, case)
    assert c.engine.pipeline_stats.get("fused_join_batches", 0) > j0, c.engine.pipeline_stats
    assert PL.JIT_STATS["launches"] > f0
    assert eager[0] == fused[0]
    assert torch.allclose(eager[1], fused[1], rtol=1e-9, atol=1e-6)


def _join_rows(c, case, name):
    """The JOIN_CASES join written to a set (no aggregation after it: the fused "pairs" probe or the eager atoms),
    as sorted row tuples of the picked columns."""
    probe, build, keys, pick, _k, _v, _op = JOIN_CASES[case]
    j = tpch._EqJoin(2, keys, tpch._pick(pick))
    j.set_input(0, probe("tpch"))
    j.set_input(1, build("tpch"))
    if c.storage.has_set("tpch", name):
        c.remove_set("tpch", name)
    c.create_set("tpch", name, None)
    c.execute_computations(WriteSet("tpch", name).set_input(j))
    cols = [x for side in pick for x in side]
    rows = []
    for b in c.get_set_batches("tpch", name):
        b = tpch._flat(b)
        if b is None or not b.n:
            continue
        vals = [b.columns[x] for x in cols]
        vals = [v.tolist() if hasattr(v, "tolist") else list(v) for v in vals]
        rows.extend(zip(*vals))
    return sorted(rows)


@pytest.mark.parametrize("case", sorted(JOIN_CASES))
def test_fused_probe_pairs_cpu_interpreter(case, monkeypatch):
    """[filter ->] probe with no aggregation after it (torch model of the "pairs" emit form) == the eager atoms,
    repeated build keys included."""
    monkeypatch.setenv("NSDB_DEVICE_STRINGS", "1")
    t = tpch_gen.generate_fast(0.003, seed=6)
    c = _client("cpu", t)
    eager = _join_rows(c, case, "pe")
    assert eager
    monkeypatch.setattr(PL, "CPU_INTERPRETER", True)
    p0 = c.engine.pipeline_stats.get("fused_probes", 0)
    fused = _join_rows(c, case, "pf")
    assert c.engine.pipeline_stats.get("fused_probes", 0) > p0, c.engine.pipeline_stats
    assert eager == fused


@pytest.mark.gpu
@pytest.mark.parametrize("case", sorted(JOIN_CASES))
def test_fused_probe_pairs_gpu(case):
    """The compiled "pairs" kernel (predicate, probe, CSR walk of repeated build keys, per-tile regions + compaction)
    against the eager filter / hash / probe / expand atoms."""
    t = tpch_gen.generate_fast(0.05, seed=6)
    c = _client("cuda:0", t)
    c.engine.fused_pipelines = False
    eager = _join_rows(c, case, "pe")
    c.engine.fused_pipelines = True
    p0 = c.engine.pipeline_stats.get("fused_probes", 0)
    fused = _join_rows(c, case, "pf")
    assert c.engine.pipeline_stats.get("fused_probes", 0) > p0, c.engine.pipeline_stats
    assert eager and eager == fused


LIKE_PATTERNS = ["%ly%re%", "%e_s%", "care%", "%ts", "%furiously%", "%quickly%ideas%", "%c_refully%r%",
                 "%blithely regular pack%", "%", "furiously%deposits", "%a%e%i%o%"]


@pytest.mark.gpu
@pytest.mark.parametrize("pat", LIKE_PATTERNS)
def test_fused_like_patterns_gpu(pat):
    """The compiled general LIKE (register-window search for strings and segments that fit, the memory scan for the
    rest: the 22-byte segment) against the eager column LIKE, as the count of matching rows per return flag."""
    t = tpch_gen.generate_fast(0.02, seed=12)
    c = _client("cuda:0", t)
    args = (lambda x: Like(x.l_comment, pat), lambda x: x.l_returnflag, lambda x: Values(1.0), "sum")
    c.engine.fused_pipelines = False
    eager = _agg_job(c, *args)
    c.engine.fused_pipelines = True
    f0 = c.engine.pipeline_stats["fused_batches"]
    fused = _agg_job(c, *args)
    assert c.engine.pipeline_stats["fused_batches"] > f0
    assert eager[0] == fused[0] and torch.equal(eager[1], fused[1]), (pat, eager, fused)
