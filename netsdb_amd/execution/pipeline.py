"""Fused relational pipelines: a stage's filter -> project -> low-cardinality aggregate compiled into ONE device pass.

Reference: src/lambdas/headers/Pipeline.h:57,194 (a page goes through the whole chain of executors while it is
cache-resident) with the FilterExecutor / ApplyExecutor / aggregation HashSink of the chain
(src/queryExecution/headers/AggregationProcessor.h:16); the TPC-H selections are lambda trees
(src/tpch/headers/Query01.h, Query06.h: makeLambdaFromMember, ==, &&, arithmetic).

The eager engine evaluates every APPLY atom of a stage as its own whole-column operation, so a scan-heavy stage
materialises each intermediate (the filter mask, every comparison, every product of the value row) as a full-length
column in HBM. When a stage ends in an aggregation and every atom after its last join is a lambda-tree node this
module understands (member access, literals, + - * /, comparisons, && || !, string ==, IN, LIKE prefix / suffix,
CASE, and the ``Values`` / ``KeyTuple`` rows of the aggregate), the atoms are compiled into a short register
program for the device interpreter kernel ``pipe_agg`` (csrc/kernels/pipeline.hip): one launch reads each input
column once, evaluates the predicate, key and value row per row in registers, pre-aggregates in registers / LDS and
merges every workgroup into one small global table with device atomics; the host reads that table back in ONE copy
(the launch's only synchronisation). A batch whose groups overflow the kernel's tables, or whose columns are of a
kind the kernel does not read, runs the eager atoms instead.

Program (mirrors pipeline.hip): registers [0, ncol) hold the loaded columns (numeric: f64 / i64 / i32 / f32 / u8;
strings: an exact short code for keys, or a (start, length) reference for byte comparisons), the temporaries follow.
Segment A computes the keep mask from the predicate's ("early") columns; the key / value columns that only segment B
reads are loaded for the kept rows only — when the stage's measured selectivity (the kernel counts the kept rows)
is low enough for that to save bandwidth; a non-selective predicate loads every column in one pass instead (one
memory round trip per row block instead of two).
"""
from __future__ import annotations

import hashlib
import os
import re
import struct
import threading
import warnings

import numpy as np
from typing import Dict, List, Optional, Tuple

import torch

from .. import _ext
from . import kernels as K
from ..lambdas import AttAccess, Binary, IsIn, KeyTuple, Like, Literal, Select, Unary, Values
from ..objects.record import RecordBatch
from ..objects.strings import StringColumn

# ---- must match pipeline.hip ----------------------------------------------------------------------------------
NREG, MAXINS, MAXCOL, FMAX, MAXSTR = 16, 48, 10, 8, 4
IMM = -2                       # operand register number meaning "the instruction's immediate"
(OP_NOP, OP_CONST, OP_ADDF, OP_SUBF, OP_MULF, OP_DIVF, OP_ADDI, OP_SUBI, OP_MULI, OP_I2F,
 OP_LTF, OP_LEF, OP_GTF, OP_GEF, OP_EQF, OP_NEF, OP_LTI, OP_LEI, OP_GTI, OP_GEI, OP_EQI, OP_NEI,
 OP_AND, OP_OR, OP_NOT, OP_PACK, OP_SEQ, OP_SPRE, OP_SSUF, OP_SEL, OP_NEGF, OP_RNGF, OP_RNGI, OP_SLIKE) = range(34)
KPOOL = 16                     # second immediates (range upper bounds), pipeline.hip PipeArgs.kpool
C_F64, C_I64, C_I32, C_F32, C_U8, C_SCODE, C_SREF = range(7)
AGG_OPS = {"sum": 0, "min": 1, "max": 2}

_ARITH = {"+": (OP_ADDF, OP_ADDI), "-": (OP_SUBF, OP_SUBI), "*": (OP_MULF, OP_MULI), "/": (OP_DIVF, None)}
_CMP = {"<": (OP_LTF, OP_LTI), "<=": (OP_LEF, OP_LEI), ">": (OP_GTF, OP_GTI), ">=": (OP_GEF, OP_GEI),
        "==": (OP_EQF, OP_EQI), "!=": (OP_NEF, OP_NEI)}

# test hook: run the compiled program with the torch interpreter on CPU batches too (validates the compiler where
# there is no GPU); the engine never takes the fused path on CPU otherwise
CPU_INTERPRETER = False
# the torch interpreter's model of the kernel's per-workgroup table: more distinct kept keys than this -> overflow
INTERP_CAP = 1 << 30
# late (post-predicate) loads of the key / value columns only when the stage keeps fewer rows than this fraction
LATE_MAX_SEL = 0.25
# kernel shape: -2 (default) the LDS-tile kernels (registers as LDS vectors) when their tile fits, -1 the hybrid kernels
# (LDS-DMA column tiles, registers in VGPRs), 0 the register kernels (plain loads), 512 / 768 / 1024 / 2048 the
# LDS-tile kernels of that tile; every mode falls back to the register kernels. Measured on 60 M rows
# (profiles/r5_tpch/pipe_micro_modes.log): LDS-tile Q06 0.88 ms / Q14 mask 0.18 ms, hybrid 0.92 / 0.29, register
# 1.22 / 0.34; an interpreted instruction costs 32-45 us of dispatch per 60 M rows in every mode.
TILE = -2
_SEL_EST: Dict[tuple, float] = {}          # stage signature -> kept fraction measured by its last launch
_EMPTY = -(1 << 63)                        # free slot of the kernel's global table


class Unfusable(Exception):
    pass


# ---------------------------------------------------------------------------------------------- expression IR
class E:
    """Symbolic column expression of a stage (built from the TCAP atoms' lambda nodes)."""

    __slots__ = ("kind", "args", "val", "_p")

    def __init__(self, kind: str, args=(), val=None):
        self.kind, self.args, self.val = kind, tuple(args), val
        self._p = None

    def __repr__(self):
        return f"{self.kind}{self.args if self.args else ''}{'' if self.val is None else '=' + repr(self.val)}"


def _node_expr(node, argx: List[E]) -> E:
    if isinstance(node, Literal):
        v = node.value
        if not isinstance(v, (bool, int, float, str)):
            raise Unfusable(f"literal {type(v).__name__}")
        return E("const", (), v)
    if isinstance(node, AttAccess):
        return E("field", argx, node.field)
    if isinstance(node, Values):
        return E("vals", argx)
    if isinstance(node, KeyTuple):
        return E("keys", argx)
    if isinstance(node, Like):
        return E("like", argx, (node.pattern, node.negate))
    if isinstance(node, IsIn):
        return E("isin", argx, tuple(node.values))
    if isinstance(node, Select):
        return E("sel", argx)
    if isinstance(node, Unary):
        return E("not", argx)
    if isinstance(node, Binary):
        return E("bin", argx, node.op)
    raise Unfusable(type(node).__name__)


_FUSABLE_NODES = (AttAccess, Values, KeyTuple, Like, IsIn, Select, Unary, Binary)


def _node_ok(node) -> bool:
    """Whether _node_expr takes this lambda node (the same test, without building the expression)."""
    if isinstance(node, Literal):
        return isinstance(node.value, (bool, int, float, str))
    return isinstance(node, _FUSABLE_NODES)


class StagePlan:
    """The fusable suffix of a stage: ``prefix`` atoms run eagerly, the rest is one fused launch per batch.

    ``join`` (a stage probing a build table inside the suffix): {"name": the JOIN's output tuple set (its BuildTable in
    the job state), "key": the probe side's key expression}; ``post`` the predicate conjuncts after the join (the key
    re-check and any condition on build-side columns); expressions rooted at an ``E("bsrc", name)`` read the build
    side's columns at the matched build rows."""

    def __init__(self, prefix, suffix, conj: List[E], key: Optional[E], val: E, op: str, kcol: str, vcol: str,
                 join: Optional[dict] = None, post: Optional[List[E]] = None):
        self.prefix, self.suffix = prefix, suffix
        self.conj, self.key, self.val, self.op = conj, key, val, op
        self.kcol, self.vcol = kcol, vcol
        self.join = join
        self.post = list(post or [])
        self.builds = None              # the job's build tables (engine state.builds), bound before the first batch
        self.alt: Optional["StagePlan"] = None   # join plans: the same stage with the probe left to the eager atoms
        self.disabled = False
        self.reason = None
        self.stats = {"fused_batches": 0, "fallback_batches": 0}
        self._sig = None

    @property
    def sig(self) -> tuple:
        """The stage's expressions (stable across executions of the same query): keys the selectivity estimate."""
        if self._sig is None:
            self._sig = (tuple(_path(c) for c in self.conj), _path(self.key), _path(self.val), self.op,
                         _path(self.join["key"]) if self.join else None, tuple(_path(c) for c in self.post))
        return self._sig

    def build_batch(self) -> Optional[RecordBatch]:
        """The build side's tuple set of a fused join (None: no join, or its build is not an in-memory table)."""
        if not self.join:
            return None
        bt = (self.builds or {}).get(self.join["name"])
        return getattr(bt, "batch", None) if hasattr(bt, "table") else None


_STAGE_CACHE: Dict[tuple, Optional[tuple]] = {}    # (graph key, stage atoms, sink) -> plan_stage's expressions
_STAGE_CACHE_MAX = 512
_MISS = object()


def plan_stage(ops: List[dict], comps: dict, sink_atom: dict, graph_key=None) -> Optional[StagePlan]:
    """The fusable suffix of ``ops`` feeding the aggregation ``sink_atom``, or None.  With ``graph_key`` (the graph's
    structural signature + every lambda constant, engine._compile) a repeated query re-uses the expressions built the
    first time; the returned plan is always new and bound to this execution's atoms."""
    ck = None
    if graph_key is not None:
        ck = (graph_key, tuple(o["output"]["name"] for o in ops), sink_atom["output"]["name"])
        hit = _STAGE_CACHE.get(ck, _MISS)
        if hit is not _MISS:
            return _unfreeze(hit, ops)
    plan = _plan_stage(ops, comps, sink_atom)
    if plan is not None and plan.join is not None:
        # the same stage without the fused probe: what runs when the join cannot be fused at run time (no compiled
        # kernels, an out-of-core or oversized build), its suffix starting after the join
        plan.alt = _plan_stage(ops, comps, sink_atom, allow_join=False)
    if ck is not None:
        if len(_STAGE_CACHE) >= _STAGE_CACHE_MAX:
            _STAGE_CACHE.pop(next(iter(_STAGE_CACHE)))
        _STAGE_CACHE[ck] = _freeze(plan)
    return plan


def _freeze(plan: Optional[StagePlan]):
    if plan is None:
        return None
    return (len(plan.prefix), plan.conj, plan.key, plan.val, plan.op, plan.kcol, plan.vcol, plan.join, plan.post,
            _freeze(getattr(plan, "alt", None)))


def _unfreeze(hit, ops) -> Optional[StagePlan]:
    if hit is None:
        return None
    start, conj, key, val, op, kcol, vcol, join, post, alt = hit
    p = StagePlan(ops[:start], ops[start:], conj, key, val, op, kcol, vcol, join, post)
    p.alt = _unfreeze(alt, ops)
    return p


def _plan_stage(ops: List[dict], comps: dict, sink_atom: dict, allow_join: bool = True) -> Optional[StagePlan]:
    from ..computations import AggregateComp, TopKComp

    comp = comps.get(sink_atom["comp"])
    if not isinstance(comp, AggregateComp) or isinstance(comp, TopKComp) or getattr(comp, "group_values", None):
        return None
    op = getattr(comp, "reduce_op", "sum")
    if op not in AGG_OPS:
        return None
    # the suffix: the longest run of trailing atoms that are lambda-tree APPLYs / FILTERs, plus at most ONE join probe
    # (its probe-side hash, the JOIN against an in-memory build table, the key re-check and a field-picking projection:
    # reference JoinProbe in the pipeline chain, JoinTuple.h:434 / Pipeline.h:194). Other native lambdas (opaque UDFs)
    # end the suffix: it starts after them and reads their output columns.
    def fusable(o) -> bool:
        if o["type"] == "FILTER":
            return True
        if o["type"] in ("HASHLEFT", "HASHRIGHT"):
            return len(o["input"]["atts"]) == 1
        if o["type"] == "JOIN":
            return allow_join and o.get("_probe_side") in ("left", "right") and o.get("_strategy") != "partitioned"
        if o["type"] != "APPLY":
            return False
        if o["lambda"].startswith("self_"):
            return True
        node = comps[o["comp"]].extract_lambdas().get(o["lambda"])
        return node is not None and (_node_ok(node) or _pick_spec(node) is not None)

    start = len(ops)
    joins = 0
    while start > 0 and fusable(ops[start - 1]):
        if ops[start - 1]["type"] == "JOIN":
            if joins:
                break                                 # one fused probe per stage: an earlier join stays eager
            joins += 1
        start -= 1
    suffix = ops[start:]
    env: Dict[str, E] = {}

    def col(name: str) -> E:
        return env[name] if name in env else E("src", (), name)

    conj: List[E] = []
    post: List[E] = []
    join = None
    hashes: Dict[str, E] = {}
    try:
        for o in suffix:
            t = o["type"]
            if t == "FILTER":
                (post if join else conj).append(col(o["input"]["atts"][0]))
                continue
            if t in ("HASHLEFT", "HASHRIGHT"):
                hashes[o["output"]["atts"][-1]] = col(o["input"]["atts"][0])
                continue
            if t == "JOIN":
                side = o["_probe_side"]
                hatt = o["input"]["atts"][0] if side == "left" else o["input2"]["atts"][0]
                if hatt not in hashes:
                    raise Unfusable("join hash computed before the suffix")
                bcols = o["projection2"]["atts"] if side == "left" else o["projection"]["atts"]
                for c in bcols:
                    env[c] = E("bsrc", (), c)
                join = {"name": o["output"]["name"], "key": hashes[hatt]}
                continue
            args = o["input"]["atts"]
            out = o["output"]["atts"][-1]
            lname = o["lambda"]
            if lname.startswith("self_"):
                env[out] = col(args[0])
                continue
            node = comps[o["comp"]].extract_lambdas().get(lname)
            if node is None:
                raise Unfusable(lname)
            spec = _pick_spec(node)
            if spec is not None:
                env[out] = E("pick", [col(a) for a in args], spec)
                continue
            env[out] = _simplify(_node_expr(node, [col(a) for a in args]))
        kcol, vcol = sink_atom["input"]["atts"]
        key, val = col(kcol), col(vcol)
    except Unfusable:
        return None
    if key.kind in ("src", "bsrc") or val.kind in ("src", "bsrc"):
        return None                                  # computed before the suffix: nothing to fuse
    if not suffix:
        return None
    return StagePlan(ops[:start], suffix, conj, key, val, op, kcol, vcol, join, post)


def _pick_spec(node) -> Optional[tuple]:
    """A join projection that only picks named fields of its inputs (models/tpch.py ``_pick``: the function carries
    ``.pick`` = the field names taken from each input): ((names of input 0), (names of input 1), ...), else None."""
    fn = getattr(node, "fn", None)
    spec = getattr(fn, "pick", None)
    if spec is None or not getattr(node, "vectorized", False):
        return None
    return tuple(tuple(x) for x in spec)


def _simplify(e: E) -> E:
    """field(pick(in_0, .., in_k), f) -> field(in_i, f) for the input i the projection took f from; recursively."""
    if e.kind == "field" and e.args and e.args[0].kind == "pick":
        pk = e.args[0]
        for i, names in enumerate(pk.val):
            if e.val in names:
                return E("field", [pk.args[i]], e.val)
        raise Unfusable(f"field {e.val} not in the join projection")
    if any(a.kind == "pick" or a.args for a in e.args):
        return E(e.kind, [_simplify(a) for a in e.args], e.val)
    return e


# ---------------------------------------------------------------------------------------------- binding + codegen
def _resolve(e: E, batch: RecordBatch, build: Optional[RecordBatch] = None):
    """The runtime column of a 'field' / 'src' / 'bsrc' (build side of a fused join) expression."""
    if e.kind in ("src", "bsrc"):
        src = batch if e.kind == "src" else build
        c = src.columns.get(e.val) if src is not None else None
        if c is None:
            raise Unfusable(f"column {e.val}")
        return c
    if e.kind == "field":
        base = _resolve(e.args[0], batch, build)
        if isinstance(base, RecordBatch) and e.val in base.columns:
            return base.columns[e.val]
        raise Unfusable(f"field {e.val}")
    raise Unfusable(e.kind)


def _side(e: E) -> int:
    """0: a probe-side (the stage's own) column; 1: a build-side column of the fused join."""
    while e.kind == "field":
        e = e.args[0]
    return 1 if e.kind == "bsrc" else 0


def _num_kind(t: torch.Tensor) -> Tuple[int, str]:
    if t.dim() != 1:
        raise Unfusable("non-scalar column")
    return {torch.float64: (C_F64, "f"), torch.int64: (C_I64, "i"), torch.int32: (C_I32, "i"),
            torch.float32: (C_F32, "f"), torch.uint8: (C_U8, "i"), torch.bool: (C_U8, "i")}.get(t.dtype) or \
        (_ for _ in ()).throw(Unfusable(str(t.dtype)))


class Program:
    """A compiled program + the column table it reads."""

    def __init__(self):
        self.ins: List[Tuple[int, int, int, int, int, int, int]] = []   # (op, dst, a, b, c, imm, aux)
        self.kpool: List[int] = []            # range ops' upper bounds (aux = pool index | mode << 8)
        self.cols: List[dict] = []            # {"key": (path, usage), "kind", "late", "L", "obj": column}
        self.col_index: Dict[tuple, int] = {}
        self.lit = bytearray()
        self.lit_index: Dict[bytes, int] = {}
        self.free: List[int] = []
        self.pinned = set()                   # common subexpressions kept for their later uses
        self.nins_a = 0
        self.keep_reg = -1
        self.key_reg = -1
        self.val_regs: List[int] = []
        self.key_layout = None                # how to turn the packed key back into columns
        self.nval = 0
        self.val_shape = None
        self.jk_reg = -1                      # fused join: the probe key's column register
        self.mode = "agg"                     # "emit": high-cardinality form (every row's key parts and values out)
        self.emit_keys: List[tuple] = []      # emit: (register, "int" | "float" | "str", dtype | L) per key part
        self.emit_keys_const = None           # emit: a literal key (no key registers)
        self.key_tuple = False
        self.keep2_reg = -1                   # fused join: the post-join predicate (per matched build row)

    # registers
    def temp(self) -> int:
        if not self.free:
            raise Unfusable("registers")
        return self.free.pop()

    def release(self, r: int):
        if r >= len(self.cols) and r not in self.free and r not in self.pinned:
            self.free.append(r)

    def emit(self, op, dst, a=-1, b=-1, imm=0):
        """a / b == IMM: that operand is the 64-bit immediate. ``AND d, r, t`` right after the compare that wrote the
        temporary t folds into that compare (its AND-with field c = r): one instruction per conjunct; and a lower and
        an upper bound of the same register against immediates (``lo <= x`` folded with ``x < hi``) become ONE range
        instruction (RNGF / RNGI)."""
        if op == OP_AND and self.ins:
            po, pd, pa, pb, pc, pimm, _ = self.ins[-1]
            if OP_LTF <= po <= OP_NEI and pc < 0:
                other = a if pd == b else (b if pd == a else None)
                if other is not None and other != pd and pd >= len(self.cols) and pd not in self.pinned:
                    self.ins[-1] = (po, dst, pa, pb, other, pimm, 0)
                    self._range_fold()
                    return
        if len(self.ins) >= MAXINS:
            raise Unfusable("program too long")
        self.ins.append((op, dst, a, b, -1, int(imm), 0))

    _LOWER = {OP_GEF: 1, OP_GTF: 0, OP_GEI: 1, OP_GTI: 0}      # op -> lower bound inclusive?
    _UPPER = {OP_LEF: 2, OP_LTF: 0, OP_LEI: 2, OP_LTI: 0}      # op -> upper bound inclusive (mode bit 1)?

    def _range_fold(self):
        """ins[-2] = (cmp1 r = x ? imm1), ins[-1] = (cmp2 d = (x ? imm2) & r): a lower + upper bound pair on one
        register -> RNG d = lo <(=) x <(=) hi, AND-ed with ins[-2]'s own chain."""
        if len(self.ins) < 2 or len(self.kpool) >= KPOOL:
            return
        o2, d, a2, b2, c2, imm2, _ = self.ins[-1]
        o1, r, a1, b1, c1, imm1, _ = self.ins[-2]
        if c2 != r or a1 != a2 or b1 != IMM or b2 != IMM or r < len(self.cols) or r in self.pinned or a1 < 0:
            return
        fam = lambda o: "f" if OP_LTF <= o <= OP_NEF else ("i" if OP_LTI <= o <= OP_NEI else None)  # noqa: E731
        if fam(o1) is None or fam(o1) != fam(o2):
            return
        if o1 in self._LOWER and o2 in self._UPPER:
            lo_op, lo, hi_op, hi = o1, imm1, o2, imm2
        elif o2 in self._LOWER and o1 in self._UPPER:
            lo_op, lo, hi_op, hi = o2, imm2, o1, imm1
        else:
            return
        mode = self._LOWER[lo_op] | self._UPPER[hi_op]
        self.kpool.append(int(hi))
        aux = (len(self.kpool) - 1) | (mode << 8)
        self.ins[-2:] = [(OP_RNGF if fam(o1) == "f" else OP_RNGI, d, a1, -1, c1, int(lo), aux)]

    def like_literal(self, pattern: str) -> int:
        """A general LIKE pattern in the literal pool as pipeline_core.h str_like reads it: [flags: 1 anchored start,
        2 anchored end][nseg][segment lengths][segment bytes, '_' = 0xFF]."""
        from ..objects.strings import _compile_like

        buf, _st, ln, a0, a1 = _compile_like(pattern)
        if len(ln) > 32 or any(n > 255 for n in ln):
            raise Unfusable("LIKE pattern size")
        blob = bytes([int(a0) | (int(a1) << 1), len(ln)] + list(ln)) + bytes(buf)
        assert len(blob) == 2 + len(ln) + sum(ln)
        return self._pool(blob)

    def literal(self, s: str) -> int:
        return self._pool(s.encode())

    def _pool(self, b: bytes) -> int:
        if len(b) > 0xFFFF:
            raise Unfusable("literal")
        if b not in self.lit_index:
            self.lit_index[b] = len(self.lit)
            self.lit += b
        return (self.lit_index[b] << 16) | len(b)


def _fbits(v: float) -> int:
    return struct.unpack("<q", struct.pack("<d", v))[0]


def _path(e: E) -> tuple:
    """Structural key of an expression (memoised on the node: the compiler asks for it many times)."""
    if e._p is None:
        e._p = (e.kind, e.val) + tuple(_path(a) for a in e.args)
    return e._p


class _Compiler:
    def __init__(self, plan: StagePlan, batch: RecordBatch, build: Optional[RecordBatch] = None, mode: str = "agg"):
        self.plan, self.batch, self.build = plan, batch, build
        self.mode = mode                  # "agg": pre-aggregate in the kernel's tables; "emit": every row out
        if plan.join is not None and build is None:
            raise Unfusable("join without a build table")
        self.p = Program()
        self.cse: Dict[tuple, tuple] = {}
        self.counts: Dict[tuple, int] = {}
        self.late_ok = _SEL_EST.get(plan.sig, 0.0) < LATE_MAX_SEL

    def _count(self, e: E):
        if e.kind in ("bin", "sel", "not", "like", "isin"):
            k = _path(e)
            self.counts[k] = self.counts.get(k, 0) + 1
            if self.counts[k] > 1:
                return
        for a in e.args:
            self._count(a)

    # -- column slots (registers [0, ncol)) are assigned before any temporary
    def _collect(self, e: E, usage: str, seg: str, out: list):
        if e.kind in ("src", "field"):
            out.append((e, usage, seg))
            return
        if e.kind == "bin" and e.val in ("==", "!=") and any(a.kind == "const" and isinstance(a.val, str) for a in e.args):
            for a in e.args:
                if a.kind != "const":
                    self._collect(a, "scmp", seg, out)
            return
        if e.kind == "like" and _floating_like(e.val[0]):
            out.append((e, "likemask", seg))           # precomputed per launch (occurrence bitmaps), read as a column
            return
        if e.kind in ("like", "isin"):
            self._collect(e.args[0], "sref" if e.kind == "like" else "scmp", seg, out)
            return
        for a in e.args:
            self._collect(a, usage, seg, out)

    def _res(self, e: E):
        return _resolve(e, self.batch, self.build)

    def _slot(self, e: E, usage: str, late: bool) -> int:
        if usage == "likemask":
            pat = e.val[0]
            e = e.args[0]
            obj = self._res(e)
            if not isinstance(obj, StringColumn):
                raise Unfusable("LIKE on a non-string")
            key = (_path(e), ("likemask", pat))
            if key in self.p.col_index:
                i = self.p.col_index[key]
                if not late and self.p.cols[i]["late"] != 2:
                    self.p.cols[i]["late"] = 0
                return i
            if len(self.p.cols) >= MAXCOL:
                raise Unfusable("columns")
            self.p.col_index[key] = len(self.p.cols)
            self.p.cols.append({"kind": C_U8, "late": 2 if _side(e) else int(late), "L": 0, "obj": obj, "expr": e,
                                "like": pat})
            return len(self.p.cols) - 1
        obj = self._res(e)
        side = _side(e)
        if usage == "jkey":
            if side or not isinstance(obj, torch.Tensor) or _num_kind(obj)[0] not in (C_I64, C_I32):
                raise Unfusable("join key: a probe-side integer column")
            usage = "num"
        if isinstance(obj, StringColumn):
            if usage == "scmp":
                # == / IN against literals: a column of short strings is compared on its fixed-width code (one integer
                # compare per literal, no offsets or bytes read); longer strings byte by byte
                usage = "key" if obj.max_len() <= 7 else "sref"
            if usage == "isin":
                usage = "sref"
            if usage == "key":
                L = obj.max_len()
                if L > 7:
                    raise Unfusable("long string key")
                kind, u = C_SCODE, ("scode", L)
            elif usage == "sref":
                kind, u, L = C_SREF, ("sref",), 0
            else:
                raise Unfusable("string in arithmetic")
        elif isinstance(obj, torch.Tensor):
            kind, _ = _num_kind(obj)
            u, L = ("num",), 0
        else:
            raise Unfusable(type(obj).__name__)
        key = (_path(e), u)
        if key in self.p.col_index:
            i = self.p.col_index[key]
            if not late and self.p.cols[i]["late"] != 2:   # an early use of a probe column; build columns stay 2
                self.p.cols[i]["late"] = 0
            return i
        if len(self.p.cols) >= MAXCOL:
            raise Unfusable("columns")
        self.p.col_index[key] = len(self.p.cols)
        # late: 0 first pass, 1 probe-side columns loaded for the kept rows, 2 build-side columns (matched build rows)
        self.p.cols.append({"kind": kind, "late": 2 if side else int(late), "L": L, "obj": obj, "expr": e})
        return len(self.p.cols) - 1

    def compile(self) -> Program:
        plan, p = self.plan, self.p
        uses = []
        for c in plan.conj:
            self._collect(c, "num", "A", uses)
            if any(_side(u[0]) for u in uses):
                raise Unfusable("build-side column before the join")
        if plan.join is not None:
            uses.append((plan.join["key"], "jkey", "A"))
        for c in plan.post:
            self._collect(c, "num", "B", uses)
        keys = self._key_fields()
        for k in keys:
            if not self._row_key(k):
                uses.append((k, "key", "B"))
        vals = plan.val.args if plan.val.kind == "vals" else (plan.val,)
        for v in vals:
            self._collect(v, "num", "B", uses)
        for e, usage, seg in [u for u in uses if u[2] == "A"] + [u for u in uses if u[2] == "B"]:
            self._slot(e, usage, late=seg == "B" and self.late_ok)
        self._strings_first()
        ncol = len(p.cols)
        if ncol > NREG:
            raise Unfusable("registers")
        p.free = list(range(NREG - 1, ncol - 1, -1))
        # segment A: the predicate
        if plan.conj:
            r = None
            for c in plan.conj:
                rc, t = self.gen(c)
                if t not in ("i", "b"):
                    rc = self._truthy(rc, t)
                if r is None:
                    r = rc
                else:
                    d = p.temp()
                    p.emit(OP_AND, d, r, rc)
                    p.release(r)
                    p.release(rc)
                    r = d
            p.keep_reg = r
        p.nins_a = len(p.ins)
        if plan.join is not None:
            p.jk_reg = p.col_index[(_path(plan.join["key"]), ("num",))]
        self.cse, self.counts = {}, {}
        for v in vals:
            self._count(v)
        # segment B: the predicate after the join (per matched build row), the key, then the value row
        if plan.post:
            r = None
            for c in plan.post:
                rc, t = self.gen(c)
                if t not in ("i", "b"):
                    rc = self._truthy(rc, t)
                if r is None:
                    r = rc
                else:
                    d = p.temp()
                    p.emit(OP_AND, d, r, rc)
                    p.release(r)
                    p.release(rc)
                    r = d
            if r < len(p.cols):                        # a bare column as the condition: keep it in a temporary
                d = p.temp()
                p.emit(OP_CONST, d, imm=0)
                p.emit(OP_NEI, d, r, d)
                r = d
            p.keep2_reg = r
            p.pinned.add(r)                            # read after the key and values are computed
        p.mode = self.mode
        if self.mode == "emit":
            # key parts leave as they are in their column registers (any mix of integer, float and short-string
            # columns: no packing into one 63-bit word), decoded on the host side of the launch
            p.key_reg = -1
            p.emit_keys = []
            k = plan.key
            if not keys:
                p.emit_keys_const = k.val
            for e in keys:
                obj = self._res(e)
                if self._row_key(e):
                    # a string longer than a short code: the row it comes from (probe row, or the matched build row);
                    # the host takes the key strings by row afterwards (a view: two index gathers, no bytes copied)
                    p.emit_keys.append((-2 if _side(e) else -1, "strrow", e))
                    continue
                slot = p.col_index[(_path(e), self._key_usage(e))]
                if isinstance(obj, StringColumn):
                    p.emit_keys.append((slot, "str", p.cols[slot]["L"]))
                else:
                    p.emit_keys.append((slot, "float" if obj.is_floating_point() else "int", obj.dtype))
            p.key_tuple = k.kind == "keys"
        else:
            p.key_reg = self._gen_key(keys)
        if len(vals) > FMAX:
            raise Unfusable("values")
        for v in vals:
            r, t = self.gen(v)
            if t == "s":
                raise Unfusable("string value")
            if t != "f":
                d = p.temp()
                p.emit(OP_I2F, d, r)
                p.release(r)
                r = d
            p.val_regs.append(r)
        p.nval = len(vals)
        p.val_shape = "row" if plan.val.kind == "vals" else "scalar"
        if p.val_shape == "scalar" and self._static_type(plan.val) != "f":
            raise Unfusable("integer value (the eager path sums it exactly as int64)")
        return p

    def _strings_first(self):
        """String columns take the first column slots (the kernel's 2nd load round only covers MAXSTR slots)."""
        p = self.p
        order = sorted(range(len(p.cols)), key=lambda i: (p.cols[i]["kind"] not in (C_SCODE, C_SREF), i))
        if sum(c["kind"] in (C_SCODE, C_SREF) for c in p.cols) > MAXSTR:
            raise Unfusable("string columns")
        if order != list(range(len(order))):
            where = {old: new for new, old in enumerate(order)}
            p.cols = [p.cols[i] for i in order]
            p.col_index = {k: where[i] for k, i in p.col_index.items()}

    def _truthy(self, r, t):
        p = self.p
        z = p.temp()
        p.emit(OP_CONST, z, imm=0)
        d = p.temp()
        p.emit(OP_NEF if t == "f" else OP_NEI, d, r, z)
        p.release(z)
        p.release(r)
        return d

    # -- keys
    def _key_fields(self) -> List[E]:
        k = self.plan.key
        if k.kind == "const":
            return []
        items = list(k.args) if k.kind == "keys" else [k]
        for it in items:
            if it.kind not in ("src", "field"):
                raise Unfusable("computed key")
        return items

    def _gen_key(self, items: List[E]) -> int:
        p = self.p
        k = self.plan.key
        if not items:
            p.key_layout = ("const", k.val)
            return -1
        slots = [p.col_index[(_path(e), self._key_usage(e))] for e in items]
        objs = [p.cols[s]["obj"] for s in slots]
        if len(items) == 1 and isinstance(objs[0], torch.Tensor):
            if objs[0].is_floating_point():
                raise Unfusable("float key")
            p.key_layout = ("int", objs[0].dtype, k.kind == "keys")
            return slots[0]
        if not all(isinstance(o, StringColumn) for o in objs):
            raise Unfusable("mixed key")
        bits = [8 * p.cols[s]["L"] + 3 for s in slots]
        if sum(bits) > 63:
            raise Unfusable("key too wide")
        p.key_layout = ("strings", [p.cols[s]["L"] for s in slots], k.kind == "keys")
        r = slots[0]
        for s, b in zip(slots[1:], bits[1:]):
            d = p.temp()
            p.emit(OP_PACK, d, r, s, b)
            p.release(r)
            r = d
        return r

    def _row_key(self, e: E) -> bool:
        """Emit mode: a string key part too long for a short code is emitted as its row index instead."""
        if self.mode != "emit":
            return False
        obj = self._res(e)
        return isinstance(obj, StringColumn) and obj.max_len() > 7

    def _key_usage(self, e: E):
        obj = self._res(e)
        return ("scode", obj.max_len()) if isinstance(obj, StringColumn) else ("num",)

    # -- expressions: (register, type) with type f / i / b / s
    def gen(self, e: E):
        key = _path(e) if e.kind in ("bin", "sel", "not", "like", "isin") else None
        if key is not None and key in self.cse:
            return self.cse[key]
        r = self._gen(e)
        if key is not None and self.counts.get(key, 0) > 1:
            self.cse[key] = r
            self.p.pinned.add(r[0])
        return r

    def _gen(self, e: E):
        p = self.p
        if e.kind in ("src", "field"):
            obj = self._res(e)
            if isinstance(obj, StringColumn):
                return p.col_index[(_path(e), ("sref",))], "s"
            i = p.col_index[(_path(e), ("num",))]
            return i, _num_kind(obj)[1]
        if e.kind == "const":
            v = e.val
            if isinstance(v, str):
                raise Unfusable("bare string literal")
            d = p.temp()
            if isinstance(v, float):
                p.emit(OP_CONST, d, imm=_fbits(v))
                return d, "f"
            p.emit(OP_CONST, d, imm=int(v))
            return d, "i"
        if e.kind == "not":
            r, t = self.gen(e.args[0])
            d = p.temp()
            p.emit(OP_NOT, d, r)
            p.release(r)
            return d, "b"
        if e.kind == "bin":
            return self._bin(e)
        if e.kind == "like":
            pat, neg = e.val
            m = p.col_index.get((_path(e.args[0]), ("likemask", pat)))
            if m is not None:                          # the launch's precomputed match column
                if not neg:
                    return m, "b"
                d = p.temp()
                p.emit(OP_NOT, d, m)
                return d, "b"
            r, t = self.gen(e.args[0])
            if t != "s":
                raise Unfusable("LIKE on a non-string")
            body = pat.strip("%")
            d = p.temp()
            if "%" in body or "_" in pat or (pat.startswith("%") and pat.endswith("%")):
                # contains / several segments / '_': the general matcher (pipeline_core.h str_like)
                p.emit(OP_SLIKE, d, r, r, p.like_literal(pat))
            else:
                if pat.endswith("%"):
                    opc = OP_SPRE
                elif pat.startswith("%"):
                    opc = OP_SSUF
                else:
                    opc = OP_SEQ
                p.emit(opc, d, r, r, p.literal(body))
            if neg:
                p.emit(OP_NOT, d, d)
            return d, "b"
        if e.kind == "isin" and self._scode(e.args[0]) is not None:
            r, L = self._scode(e.args[0])
            acc = None
            for v in e.val:
                if not isinstance(v, str):
                    raise Unfusable("IN types")
                d = self._code_eq(r, L, v)
                if acc is None:
                    acc = d
                else:
                    p.emit(OP_OR, acc, acc, d)
                    p.release(d)
            if acc is None:
                acc = p.temp()
                p.emit(OP_CONST, acc, imm=0)
            return acc, "b"
        if e.kind == "isin":
            r, t = self.gen(e.args[0])
            acc = None
            for v in e.val:
                d = p.temp()
                if t == "s":
                    if not isinstance(v, str):
                        raise Unfusable("IN types")
                    p.emit(OP_SEQ, d, r, r, p.literal(v))
                else:
                    z = p.temp()
                    if t == "f":
                        p.emit(OP_CONST, z, imm=_fbits(float(v)))
                        p.emit(OP_EQF, d, r, z)
                    else:
                        if isinstance(v, float):
                            raise Unfusable("IN types")
                        p.emit(OP_CONST, z, imm=int(v))
                        p.emit(OP_EQI, d, r, z)
                    p.release(z)
                if acc is None:
                    acc = d
                else:
                    p.emit(OP_OR, acc, acc, d)
                    p.release(d)
            p.release(r)
            if acc is None:
                acc = p.temp()
                p.emit(OP_CONST, acc, imm=0)
            return acc, "b"
        if e.kind == "sel":
            rc, tc = self.gen(e.args[0])
            ra, ta = self.gen(e.args[1])
            rb, tb = self.gen(e.args[2])
            if "s" in (ta, tb):
                raise Unfusable("string CASE")
            if ta != tb:
                ra, rb = self._promote(ra, ta), self._promote(rb, tb)
                ta = "f"
            d = p.temp()
            p.emit(OP_SEL, d, rc, ra, rb)
            for r in (rc, ra, rb):
                p.release(r)
            return d, ta
        raise Unfusable(e.kind)

    def _scode(self, e: E):
        """(slot, L) when string column ``e`` was registered by its short code (== / IN compares), else None."""
        if e.kind not in ("src", "field"):
            return None
        obj = self._res(e)
        if not isinstance(obj, StringColumn):
            return None
        L = obj.max_len()
        i = self.p.col_index.get((_path(e), ("scode", L)))
        return None if i is None else (i, L)

    def _code_eq(self, r: int, L: int, lit: str) -> int:
        """A temporary holding (code register r == the literal's short code); a literal longer than L never matches."""
        p = self.p
        b = lit.encode()
        d = p.temp()
        if len(b) > L:
            p.emit(OP_CONST, d, imm=0)
            return d
        c = 0
        for i in range(L):
            c |= (b[i] if i < len(b) else 0) << (8 * (L - 1 - i))
        z = p.temp()
        p.emit(OP_CONST, z, imm=(c << 3) | len(b))
        p.emit(OP_EQI, d, r, z)
        p.release(z)
        return d

    def _promote(self, r, t):
        if t == "f":
            return r
        p = self.p
        d = p.temp()
        p.emit(OP_I2F, d, r)
        p.release(r)
        return d

    def _bin(self, e: E):
        p = self.p
        op = e.val
        a, b = e.args
        if op in ("==", "!=") and (a.kind == "const" and isinstance(a.val, str) or b.kind == "const" and isinstance(b.val, str)):
            s, lit = (b, a.val) if a.kind == "const" else (a, b.val)
            sc = self._scode(s)
            if sc is not None:                            # fixed-width code compare
                d = self._code_eq(sc[0], sc[1], lit)
                if op == "!=":
                    p.emit(OP_NOT, d, d)
                return d, "b"
            r, t = self.gen(s)
            if t != "s":
                raise Unfusable("string compare")
            d = p.temp()
            p.emit(OP_SEQ, d, r, r, p.literal(lit))
            if op == "!=":
                p.emit(OP_NOT, d, d)
            p.release(r)
            return d, "b"
        if op in ("&&", "||"):
            ra, _ = self.gen(a)
            rb, _ = self.gen(b)
            d = p.temp()
            p.emit(OP_AND if op == "&&" else OP_OR, d, ra, rb)
            p.release(ra)
            p.release(rb)
            return d, "b"
        # numeric: a literal operand rides in the instruction's immediate and takes the other side's type (an int
        # literal against a float column compares as a float)
        ra, ta, ia = self._operand(a, b, allow_imm=True)
        rb, tb, ib = self._operand(b, a, allow_imm=ra != IMM)
        imm = ia if ra == IMM else ib
        if "s" in (ta, tb):
            raise Unfusable("string arithmetic")
        fl = "f" in (ta, tb) or op == "/"
        if fl:
            if ra == IMM and ta == "i":
                imm = _fbits(float(imm))
            if rb == IMM and tb == "i":
                imm = _fbits(float(imm))
            ra = ra if ra == IMM else self._promote(ra, ta)
            rb = rb if rb == IMM else self._promote(rb, tb)
        d = p.temp()
        if op in _ARITH:
            opc = _ARITH[op][0 if fl else 1]
            if opc is None:
                raise Unfusable(op)
            p.emit(opc, d, ra, rb, imm)
            res = "f" if fl else "i"
        elif op in _CMP:
            p.emit(_CMP[op][0 if fl else 1], d, ra, rb, imm)
            res = "b"
        else:
            raise Unfusable(op)
        p.release(ra)
        p.release(rb)
        return d, res

    def _operand(self, e: E, other: E, allow_imm: bool):
        """(register, type, immediate): a numeric literal becomes the immediate (register IMM) when allowed."""
        if allow_imm and e.kind == "const" and isinstance(e.val, (int, float)) and not isinstance(e.val, bool):
            ot = self._static_type(other)
            if ot == "f" or isinstance(e.val, float):
                return IMM, "f", _fbits(float(e.val))
            return IMM, "i", int(e.val)
        r, t = self._gen_as(e, other)
        return r, t, 0

    def _gen_as(self, e: E, other: E):
        if e.kind == "const" and isinstance(e.val, (int, float)) and not isinstance(e.val, bool):
            ot = self._static_type(other)
            if ot == "f" or isinstance(e.val, float):
                d = self.p.temp()
                self.p.emit(OP_CONST, d, imm=_fbits(float(e.val)))
                return d, "f"
        return self.gen(e)

    def _static_type(self, e: E) -> str:
        if e.kind in ("src", "field"):
            obj = self._res(e)
            return "s" if isinstance(obj, StringColumn) else _num_kind(obj)[1]
        if e.kind == "const":
            return "f" if isinstance(e.val, float) else "i"
        if e.kind == "bin" and e.val in _ARITH:
            ts = [self._static_type(a) for a in e.args]
            return "f" if "f" in ts or e.val == "/" else "i"
        if e.kind == "sel":
            ts = [self._static_type(a) for a in e.args[1:]]
            return "f" if "f" in ts else "i"
        return "b"


# ---------------------------------------------------------------------------------------------- execution
_PROG_CACHE: Dict[tuple, Program] = {}
_PROG_CACHE_MAX = 256


def _schema_key(batch: RecordBatch) -> tuple:
    """What a compiled program depends on besides the stage's expressions: each column's kind (dtype, or string with
    its length bound), never its values."""
    out = []
    for k, c in batch.columns.items():
        if isinstance(c, torch.Tensor):
            out.append((k, str(c.dtype), c.dim()))
        elif isinstance(c, StringColumn):
            out.append((k, "s", c._maxlen))
        else:
            out.append((k, type(c).__name__))
    return tuple(out)


def _compile_cached(plan: StagePlan, batch: RecordBatch, mode: str = "agg") -> Program:
    """The stage's program for this batch: compiled once per (stage expressions, selectivity mode, column kinds, agg /
    emit form) and re-bound to the batch's columns afterwards (repeated queries skip the compiler)."""
    build = plan.build_batch()
    if plan.join is not None and build is None:
        raise Unfusable("the join's build side is not an in-memory table")
    key = (plan.sig, _SEL_EST.get(plan.sig, 0.0) < LATE_MAX_SEL, _schema_key(batch),
           _schema_key(build) if build is not None else None, mode)
    hit = _PROG_CACHE.get(key)
    if hit is not None:
        p = Program.__new__(Program)
        p.__dict__.update(hit.__dict__)
        p.cols = [dict(c, obj=_resolve(c["expr"], batch, build)) for c in hit.cols]
        # A string key column's short-code bound L is fixed at compile time. The key above holds the column's
        # length bound only when it was already known (no device read per batch), so a batch with an unknown bound
        # can meet a program compiled for shorter strings: re-check the bound of every such column (one cached
        # reduction per column) and compile afresh when a row is longer than L.
        if all(c["kind"] != C_SCODE or c["obj"].max_len() <= c["L"] for c in p.cols):
            return p
        return _Compiler(plan, batch, build, mode).compile()
    p = _Compiler(plan, batch, build, mode).compile()
    _prog_tensors(p, batch.device)              # built once here: every cached copy shares them
    if len(_PROG_CACHE) >= _PROG_CACHE_MAX:
        _PROG_CACHE.pop(next(iter(_PROG_CACHE)))
    _PROG_CACHE[key] = p
    return p


_EMIT_SIGS: Dict[tuple, bool] = {}           # stage signatures whose groups overflowed the kernel's tables
_KEY_SHAPE = __import__("re").compile(r"float key|mixed key|key too wide|long string key")
EMIT = os.environ.get("NSDB_PIPE_EMIT", "1") != "0"


def run_batch(plan: StagePlan, batch: RecordBatch) -> Optional[RecordBatch]:
    """One fused launch over ``batch``: the pre-aggregated {kcol: keys, vcol: values} batch; for a stage with more
    groups than the kernel's tables (seen once, remembered per stage signature) the emitted, not yet aggregated
    {kcol, vcol} rows of every kept row (``batch.emitted``, device columns for the sink's group-by); or None when this
    batch must take the eager atoms (columns the kernel cannot read, no compiled kernels for the emitted form)."""
    if plan.disabled or batch.n == 0:
        return None
    dev = batch.device
    on_gpu = dev.type == "cuda" and _ext.hip() is not None and hasattr(_ext.hip(), "pipe_agg")
    if not on_gpu and not (CPU_INTERPRETER and dev.type == "cpu"):
        return None
    if EMIT and _EMIT_SIGS.get(plan.sig):
        return _run_emit(plan, batch, on_gpu)
    try:
        prog = _compile_cached(plan, batch)
    except Unfusable as e:
        if EMIT and _KEY_SHAPE.search(str(e)):
            # a key the kernel's one-word table cannot hold (float, mixed or too wide for one word): emitted form
            _EMIT_SIGS[plan.sig] = True
            return _run_emit(plan, batch, on_gpu)
        plan.disabled = True
        plan.reason = str(e)
        return None
    if on_gpu:
        try:
            parts = _launch(prog, batch.n, dev, plan)
        except Unfusable as e:
            plan.disabled = True
            plan.reason = str(e)
            return None
    elif plan.join is not None:
        parts = interpret_join(prog, batch.n, plan)
    else:
        parts = interpret(prog, batch.n, plan.op)
    if parts is None:
        # more groups than the kernel's tables hold: the emitted form (every row's key parts and values straight from
        # registers into the sink's group-by) for this and every later run of the stage, else the eager atoms
        if EMIT:
            _EMIT_SIGS[plan.sig] = True
            return _run_emit(plan, batch, on_gpu)
        plan.disabled = True
        return None
    keys, vals = parts                  # host tensors (a few rows): decoded on the host
    plan.stats["fused_batches"] += 1
    kc, vc = _key_columns(prog, keys), _value_column(prog, vals)
    if getattr(plan, "host_out", False):
        return RecordBatch({plan.kcol: kc, plan.vcol: vc}, int(keys.numel()))     # the sink reduces on the host
    return RecordBatch({plan.kcol: _to_dev(kc, dev), plan.vcol: _to_dev(vc, dev)}, int(keys.numel()))


EMIT_TILE_BLOCKS = 16                         # row blocks (NTHR x ROWS rows) per emit tile


class EmittedBatch(RecordBatch):
    """A fused launch's emitted rows (key parts, values) — not pre-aggregated: the sink's group-by reduces them."""

    __slots__ = ()
    emitted = True


def _run_emit(plan: StagePlan, batch: RecordBatch, on_gpu: bool) -> Optional[RecordBatch]:
    try:
        prog = _compile_cached(plan, batch, "emit")
        if on_gpu:
            got = _launch_emit(prog, batch.n, batch.device, plan)
        else:
            got = interpret_emit(prog, batch.n, plan)
    except Unfusable as e:
        plan.disabled = True
        plan.reason = str(e)
        return None
    if got is None:
        return None                     # an emit region overflowed (many matches per probe row): eager atoms
    words, m = got
    plan.stats["fused_batches"] += 1
    plan.stats["emitted_rows"] = plan.stats.get("emitted_rows", 0) + m
    nk = len(prog.emit_keys)
    parts = []
    for i, (_reg, kind, info) in enumerate(prog.emit_keys):
        w = words[i]
        if kind == "strrow":                          # the key strings at the emitted rows (probe or build side)
            parts.append(_resolve(info, batch, plan.build_batch()).take(w))
            continue
        if kind == "int":
            parts.append(w.to(info) if info != torch.int64 else w)
        elif kind == "float":
            parts.append(w.view(torch.float64).to(info))
        else:
            parts.append(StringColumn.from_short_codes(w, info))
    if nk == 0:
        v = prog.emit_keys_const
        key = torch.full((m,), v, dtype=torch.float64 if isinstance(v, float) else torch.int64, device=words.device)
    else:
        key = tuple(parts) if prog.key_tuple or nk > 1 else parts[0]
    vals = words[nk:].view(torch.float64).t()        # [rows, F] column-major: the group-by reads it in place
    if prog.val_shape != "row":
        vals = vals[:, 0].contiguous()
    return EmittedBatch({plan.kcol: key, plan.vcol: vals}, m)


def _launch_emit(prog: Program, n: int, dev, plan: StagePlan, kind: str = "emit"):
    """The emitted form's launch: (int64 words [ne, rows] on the device, rows), or None on a region overflow. ``kind``
    "pairs": the (probe row, build row) of every kept, matched row (a fused filter + join probe)."""
    h = _ext.hip()
    if not hasattr(h, "pipe_emit"):
        raise Unfusable("no emit kernels in this build")
    ins, lit = _prog_tensors(prog, dev)
    cargs = _col_args(prog, dev)
    jtab = jperm = jbloom = None
    bn = -1
    mult = 1
    if plan.join is not None:
        jtab, jperm, bn, jbloom = _join_table(plan, dev)
        # every probe row emits at most the build side's largest key multiplicity: regions sized by it never overflow
        mult = plan.builds[plan.join["name"]].table(dev).max_multiplicity()
        if mult > 64:
            raise Unfusable(f"a build key with {mult} rows (emit regions hold at most 64 per probe row)")
    jit = _jit_for(prog, cargs, kind, -1, prog.val_regs if kind == "emit" else (), dev)
    if jit is None:
        raise Unfusable("the emitted form needs the compiled kernels")
    fn, jnreg, jrows = jit
    ne = 2 if kind == "pairs" else len(prog.emit_keys) + len(prog.val_regs)
    tile = 256 * jrows * EMIT_TILE_BLOCKS
    # a tile's region: its rows times the most matches one probe row can have
    cap = tile * max(1, mult)
    words, status = h.pipe_emit(ins, prog.nins_a, cargs, lit, n, prog.keep_reg, -1, prog.val_regs, prog.kpool, fn,
                                jnreg, jrows, max(1, ne), tile, cap, jtab, jperm, bn, jbloom)
    if int(status[0]) != 0:
        return None
    if n:
        _SEL_EST[plan.sig] = int(status[1]) / n
    return words, int(words.shape[1])


def _to_dev(x, dev):
    """Host result -> device without a synchronisation (pinned staging, asynchronous copy)."""
    if isinstance(x, tuple):
        return tuple(_to_dev(c, dev) for c in x)
    if x.device == dev:
        return x
    if isinstance(x, StringColumn):
        return x.to(dev)
    return x.pin_memory().to(dev, non_blocking=True) if dev.type == "cuda" else x.to(dev)


def _col_args(prog: Program, dev):
    out = []
    for c in prog.cols:
        o = c["obj"]
        if getattr(o, "device", dev) != dev:
            raise Unfusable("a column on another device")
        if c.get("like") is not None:
            out.append((C_U8, c["late"], 0, _like_mask(c), None, None, None))
            continue
        if c["kind"] == C_SCODE:
            # the column's kept fixed-width encoding: a plain int32 (codes of <= 3 bytes) or int64 load
            codes = o.short_codes32(c["L"]) if o.device.type == "cuda" else None
            if codes is not None:
                out.append((C_I32, c["late"], 0, codes.contiguous(), None, None, None))
                continue
            codes = o.short_codes(c["L"])
            if codes is not None:
                out.append((C_I64, c["late"], 0, codes.contiguous(), None, None, None))
                continue
            # a row longer than the program's bound L: the device short_code would map it to the same sentinel as
            # every other long row and merge distinct groups — never launch that (the caller runs the eager atoms)
            raise Unfusable(f"string key longer than the compiled bound {c['L']}")
        if isinstance(o, StringColumn):
            out.append((c["kind"], c["late"], c["L"], None, o.starts.contiguous(), o.ends.contiguous(), o.data))
        else:
            t = o.contiguous()
            out.append((c["kind"], c["late"], c["L"], t, None, None, None))
    return out


# ---------------------------------------------------------------------------------------------- compiled kernels
# Run-time compilation (pipeline_core.h jit_agg_body / jit_mask_body): a program's loads, instructions, keep flag,
# key and values become straight-line C++ on compile-time registers and column kinds, compiled once per program
# shape by hiprtc inside the process (immediates stay kernel arguments: one kernel per query shape, not per literal)
# and cached in memory and on disk. NSDB_PIPE_JIT=0 keeps the interpreter kernels (TILE) for every stage.
JIT = os.environ.get("NSDB_PIPE_JIT", "1") != "0"
# rows per thread per iteration of the compiled kernels (JIT_ROWS_SMALL for programs of at most JIT_SMALL_NREG
# registers); SF 10 launch times by rows 2 / 4 / 8 (profiles/r5_jit/ab_jit_rows.log): Q01 0.96 / 1.00 / 1.22 ms,
# Q06 0.44 / 0.41 / 0.41, the Q14 mask 0.162 / 0.165 / 0.175
JIT_ROWS = 2
JIT_ROWS_SMALL = 4
JIT_SMALL_NREG = 8
# general LIKE in the compiled kernels: the register-window matcher (True), the dword memory scan only (False), or per
# pattern ("auto": the window for a pattern anchored at either end, the scan for floating segments only).
# scripts/ab_like.py, SF 10 (profiles/r6_like): Q13's '%special%requests%' over every order comment 2.87 ms with the
# window vs 2.62 with the scan; Q02's '%BRASS' 4.97 vs 5.11
JIT_LIKE_WINDOW = {"0": False, "1": True}.get(os.environ.get("NSDB_JIT_LIKE_WINDOW", "auto"), "auto")
# the aggregation op compiled into the kernel (True) or read from the launch arguments (False: every accumulate then
# computes sum, min and max and selects; scripts/ab_pipeline_flag.py --flag JIT_FIXED_OP measures both)
JIT_FIXED_OP = os.environ.get("NSDB_JIT_FIXED_OP", "1") != "0"
JIT_STATS = {"compiled": 0, "disk_hits": 0, "launches": 0, "failed": 0}
_JIT_FN: Dict[tuple, Optional[int]] = {}     # (device, generated source) -> kernel handle (None: compile failed)
_JIT_SHAPES: Dict[tuple, tuple] = {}         # program shape -> (kernel handle or None, nreg, rows)
_JIT_HEADER: Optional[str] = None
_FOPS = {OP_ADDF: "+", OP_SUBF: "-", OP_MULF: "*", OP_DIVF: "/"}
_IOPS = {OP_ADDI: "+", OP_SUBI: "-", OP_MULI: "*"}
_FCMPS = {OP_LTF: "<", OP_LEF: "<=", OP_GTF: ">", OP_GEF: ">=", OP_EQF: "==", OP_NEF: "!="}
_ICMPS = {OP_LTI: "<", OP_LEI: "<=", OP_GTI: ">", OP_GEI: ">=", OP_EQI: "==", OP_NEI: "!="}


def _jit_header() -> str:
    global _JIT_HEADER
    if _JIT_HEADER is None:
        path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc", "kernels",
                            "pipeline_core.h")
        with open(path) as f:
            _JIT_HEADER = f.read()
    return _JIT_HEADER


def program_nreg(prog: Program, ncol: int, key_reg: int, val_regs) -> int:
    """Registers the program touches, exactly as the binding's fill_args counts them (the compiled kernel's NR)."""
    n = max(1, ncol, prog.keep_reg + 1, key_reg + 1, getattr(prog, "keep2_reg", -1) + 1, *(v + 1 for v in val_regs))
    for (op, dst, a, b, c, imm, _aux) in prog.ins:
        n = max(n, dst + 1, a + 1, b + 1, c + 1, imm + 1 if op == OP_SEL else 0)
    return n


def _like_window(lit: bytes, imm: int) -> bool:
    if JIT_LIKE_WINDOW != "auto":
        return bool(JIT_LIKE_WINDOW)
    off = int(imm) >> 16
    return bool(lit) and off < len(lit) and (lit[off] & 3) != 0     # anchored start or end


def _jit_ins(pc: int, ins, lit: bytes = b"") -> Optional[str]:
    """One instruction as a C++ statement on the register row r (the interpreter's semantics, pipeline.hip run)."""
    op, dst, a, b, c, imm, aux = ins

    def opnd(k):
        return f"r[{k}]" if k >= 0 else (f"(u64)a.ins[{pc}].imm" if k == IMM else "0ull")

    X, Y = opnd(a), opnd(b)
    if op == OP_NOP:
        return None
    if op == OP_CONST:
        z = f"(u64)a.ins[{pc}].imm"
    elif op in _FOPS:
        z = f"f2u(u2f({X}) {_FOPS[op]} u2f({Y}))"
    elif op == OP_NEGF:
        z = f"f2u(-u2f({X}))"
    elif op in _IOPS:
        z = f"(u64)((long long){X} {_IOPS[op]} (long long){Y})"
    elif op == OP_I2F:
        z = f"f2u((double)(long long){X})"
    elif op in _FCMPS:
        z = f"(u64)(u2f({X}) {_FCMPS[op]} u2f({Y}))"
    elif op in _ICMPS:
        z = f"(u64)((long long){X} {_ICMPS[op]} (long long){Y})"
    elif op == OP_AND:
        z = f"(u64)(({X} != 0ull) & ({Y} != 0ull))"
    elif op == OP_OR:
        z = f"(u64)(({X} != 0ull) | ({Y} != 0ull))"
    elif op == OP_NOT:
        z = f"(u64)({X} == 0ull)"
    elif op == OP_PACK:
        z = f"(({X} << (a.ins[{pc}].imm & 63)) | {Y})"
    elif op == OP_SEL:
        z = f"({X} ? {Y} : r[{int(imm)}])"
    elif op in (OP_RNGF, OP_RNGI):
        k, mode = aux & 0xFF, aux >> 8
        lo_c, hi_c = (">=" if mode & 1 else ">"), ("<=" if mode & 2 else "<")
        if op == OP_RNGF:
            x, lo, hi = f"u2f({X})", f"u2f((u64)a.ins[{pc}].imm)", f"u2f((u64)a.kpool[{k}])"
        else:
            x, lo, hi = f"(long long){X}", f"a.ins[{pc}].imm", f"a.kpool[{k}]"
        z = f"(u64)(({x} {lo_c} {lo}) && ({x} {hi_c} {hi}))"
    elif op in (OP_SEQ, OP_SPRE, OP_SSUF):
        mode = {OP_SEQ: 0, OP_SPRE: 1, OP_SSUF: 2}[op]
        z = f"(u64)str_match(a.col[{b}].dat, {X}, a.lit, a.ins[{pc}].imm, {mode})"
    elif op == OP_SLIKE:
        z = f"(u64)str_like<{'true' if _like_window(lit, imm) else 'false'}>(a.col[{b}].dat, {X}, a.lit, a.ins[{pc}].imm)"
    else:
        z = "0ull"
    if c >= 0:
        z = f"(u64)(({z}) != 0ull && r[{c}] != 0ull)"
    return f"r[{dst}] = {z};"


_LOADS = {C_F64: ("u64", "p[row[j]]"), C_I64: ("u64", "p[row[j]]"), C_I32: ("int", "(u64)(long long)p[row[j]]"),
          C_F32: ("float", "f2u((double)p[row[j]])"), C_U8: ("unsigned char", "(u64)p[row[j]]")}


def _jit_loads(kinds, lates, late) -> List[str]:
    """Load statements of the columns of one pass: ``late`` 0 / False = first pass, 1 / True = the kept rows' late
    probe-side columns, 2 = a fused join's build-side columns at the matched build rows (index ``brow``)."""
    out = []
    which = int(late)
    for c, (kind, lt) in enumerate(zip(kinds, lates)):
        if int(lt) != which:
            continue
        ix = "brow[j]" if which == 2 else "row[j]"
        full = "false" if which == 2 else "FULL"
        if kind in _LOADS:
            t, e = _LOADS[kind]
            e = e.replace("row[j]", ix)
            out.append(f"    {{ const {t}* p = reinterpret_cast<const {t}*>(a.col[{c}].p);\n"
                       f"#pragma unroll\n      for (int j = 0; j < ROWS; ++j) R[j][{c}] = ({full} || m[j]) ? {e} : 0ull; }}")
        elif kind in (C_SCODE, C_SREF):
            v = (f"short_code(a.col[{c}].dat, s, e - s, a.col[{c}].L)" if kind == C_SCODE else
                 "(((u64)s << 24) | (u64)(e - s < 0xFFFFFFll ? e - s : 0xFFFFFFll))")
            out.append(f"    {{ const long long* st = a.col[{c}].st; const long long* en = a.col[{c}].en;\n"
                       f"#pragma unroll\n      for (int j = 0; j < ROWS; ++j) {{\n"
                       f"        const bool mj = {full} || m[j];\n"
                       f"        const long long s = mj ? st[{ix}] : 0ll, e = mj ? en[{ix}] : 0ll;\n"
                       f"        R[j][{c}] = mj ? {v} : 0ull;\n      }} }}")
        else:
            raise Unfusable(f"column kind {kind}")
    return out


def jit_source(prog: Program, kinds, lates, kind: str, key_reg: int = -1, val_regs=(), rows: int = JIT_ROWS,
               agg_op: int = -1) -> str:
    """The C++ source of the compiled kernel of ``prog`` (``kind`` "agg", "emit" or "mask") over columns of these
    kinds. "emit" writes every kept row's key-part registers (prog.emit_keys) and value registers. ``agg_op`` (0 sum,
    1 min, 2 max; -1: the launch's argument) fixes the aggregation op at compile time."""
    nreg = program_nreg(prog, len(kinds), key_reg, val_regs)
    F = max(1, len(val_regs))
    staged = kind in ("agg", "emit", "pairs")        # segment A / late columns / segment B split
    nins_a = prog.nins_a if staged else len(prog.ins)
    emit_regs = [k[0] for k in getattr(prog, "emit_keys", [])] + list(val_regs)   # -1 / -2: the probe / build row

    def seg(lo, hi):
        lit = bytes(prog.lit or b"")
        body = [t for pc in range(lo, hi) if (t := _jit_ins(pc, prog.ins[pc], lit)) is not None]
        if not body:
            return "    (void)a; (void)R;"
        return ("#pragma unroll\n    for (int j = 0; j < ROWS; ++j) {\n      u64* r = R[j];\n"
                + "".join(f"      {t}\n" for t in body) + "    }")

    join = staged and getattr(prog, "jk_reg", -1) >= 0

    def loads(late):
        ls = _jit_loads(kinds, [lt if staged else 0 for lt in lates], late)
        idx = "brow" if late == 2 else "row"
        return "\n".join(ls) if ls else f"    (void)a; (void){idx}; (void)m; (void)R;"

    vals = "".join(f"    v[{f}] = u2f(r[{reg}]);\n" for f, reg in enumerate(val_regs)) or "    v[0] = 0.0; (void)r;\n"
    keep = "true" if prog.keep_reg < 0 else f"r[{prog.keep_reg}] != 0ull"
    keep2 = f"r[{prog.keep2_reg}] != 0ull" if join and getattr(prog, "keep2_reg", -1) >= 0 else "true"
    key = "0ll" if key_reg < 0 else f"(long long)r[{key_reg}]"
    body = "jit_join_agg_body" if join else "jit_agg_body"
    if kind == "agg":
        entry = ("extern \"C\" __global__ void __launch_bounds__(nsdb_pipe::NTHR) nsdb_jit_agg(const nsdb_pipe::PipeArgs a) {\n"
                 f"  nsdb_pipe::{body}<nsdb_pipe::JitProg>(a);\n}}\n")
    elif kind in ("emit", "pairs"):
        entry = ("extern \"C\" __global__ void __launch_bounds__(nsdb_pipe::NTHR) nsdb_jit_emit(const nsdb_pipe::PipeArgs a, "
                 "unsigned long long* out, long long tile_rows, long long cap, long long ostride, unsigned* tile_cnt) {\n"
                 "  nsdb_pipe::jit_emit_body<nsdb_pipe::JitProg>(a, out, tile_rows, cap, ostride, tile_cnt);\n}\n")
    else:
        entry = ("extern \"C\" __global__ void __launch_bounds__(nsdb_pipe::NTHR) nsdb_jit_mask(const nsdb_pipe::PipeArgs a, "
                 "unsigned char* mask) {\n  nsdb_pipe::jit_mask_body<nsdb_pipe::JitProg>(a, mask);\n}\n")
    emit = "".join(f"    w[{i}] = {'(u64)row' if reg == -1 else '(u64)brow' if reg == -2 else f'r[{reg}]'};\n"
                   for i, reg in enumerate(emit_regs)) or "    w[0] = 0ull; (void)r;\n"
    ne = max(1, len(emit_regs))
    if kind == "pairs":                              # a fused filter + probe: (probe row, build row) per match
        emit, ne = "    (void)r;\n    w[0] = (u64)row;\n    w[1] = (u64)brow;\n", 2
    return f"""// generated by netsdb_amd.execution.pipeline.jit_source ({kind})
#include "pipeline_core.h"
namespace nsdb_pipe {{
struct JitProg {{
  static constexpr int F = {F}, NR = {nreg}, ROWS = {rows}, JK = {max(0, getattr(prog, "jk_reg", -1))};
  static constexpr int NE = {ne}, OP = {int(agg_op)};
  static constexpr bool JOIN = {"true" if join else "false"};
  template <bool LATE, bool FULL>
  __device__ static __forceinline__ void load(const PipeArgs& a, const long long (&row)[ROWS], const bool (&m)[ROWS],
                                              u64 (&R)[ROWS][NR]) {{
    if constexpr (!LATE) {{
{loads(False)}
    }} else {{
{loads(True)}
    }}
  }}
  __device__ static __forceinline__ void loadb(const PipeArgs& a, const long long (&brow)[ROWS], const bool (&m)[ROWS],
                                               u64 (&R)[ROWS][NR]) {{
{loads(2) if join else "    (void)a; (void)brow; (void)m; (void)R;"}
  }}
  __device__ static __forceinline__ void run_a(const PipeArgs& a, u64 (&R)[ROWS][NR]) {{
{seg(0, nins_a)}
  }}
  __device__ static __forceinline__ void run_b(const PipeArgs& a, u64 (&R)[ROWS][NR]) {{
{seg(nins_a, len(prog.ins))}
  }}
  __device__ static __forceinline__ bool keep(const u64 (&r)[NR]) {{ (void)r; return {keep}; }}
  __device__ static __forceinline__ bool keep2(const u64 (&r)[NR]) {{ (void)r; return {keep2}; }}
  __device__ static __forceinline__ long long key(const u64 (&r)[NR]) {{ (void)r; return {key}; }}
  __device__ static __forceinline__ void vals(const u64 (&r)[NR], double (&v)[F]) {{
{vals}  }}
  __device__ static __forceinline__ void emit(const u64 (&r)[NR], u64 (&w)[NE], long long row, long long brow) {{
    (void)row; (void)brow;
{emit}  }}
}};
}}  // namespace nsdb_pipe
{entry}"""


def _jit_cache_dir() -> Optional[str]:
    d = os.environ.get("NSDB_JIT_CACHE") or os.path.join(os.path.expanduser("~"), ".cache", "netsdb_amd", "jit")
    try:
        os.makedirs(d, exist_ok=True)
        return d
    except OSError:
        return None


def _dev_index(dev=None) -> int:
    if dev is not None and torch.device(dev).type == "cuda":
        d = torch.device(dev)
        return d.index if d.index is not None else torch.cuda.current_device()
    return torch.cuda.current_device() if torch.cuda.is_available() else -1


def jit_kernel(src: str, name: str, dev=None) -> Optional[int]:
    """The loaded kernel of a generated source on device ``dev`` (default: the current one), compiled once per process,
    code objects cached on disk; or None when compilation fails (the interpreter kernels then run that stage). A
    loaded module belongs to one device's context, so the handle cache is per device; the disk cache digest covers
    the target, the header, the source and the hiprtc version."""
    di = _dev_index(dev)
    if (di, src) in _JIT_FN:
        return _JIT_FN[(di, src)]
    h = _ext.hip()
    fn = None
    try:
        hdr = _jit_header()
        arch = os.environ.get("PYTORCH_ROCM_ARCH") or "gfx950"
        rtc = h.jit_version() if hasattr(h, "jit_version") else "?"
        digest = hashlib.sha256((arch + "\0" + rtc + "\0" + hdr + "\0" + src).encode()).hexdigest()[:32]
        d = _jit_cache_dir()
        path = os.path.join(d, f"{digest}.hsaco") if d else None
        code = None
        if path and os.path.exists(path):
            with open(path, "rb") as f:
                code = f.read()
            JIT_STATS["disk_hits"] += 1
        if not code:
            code = h.jit_compile(src, hdr)
            JIT_STATS["compiled"] += 1
            if path:
                tmp = f"{path}.{os.getpid()}.tmp"
                with open(tmp, "wb") as f:
                    f.write(code)
                os.replace(tmp, path)
        if di >= 0:
            with torch.cuda.device(di):         # the module loads into this device's context
                fn = int(h.jit_load(code, name))
        else:
            fn = int(h.jit_load(code, name))
    except Exception as e:          # noqa: BLE001 - any compiler / loader failure keeps the interpreter path
        JIT_STATS["failed"] += 1
        warnings.warn(f"pipeline kernel compilation failed, interpreting this stage: {e}")
        fn = None
    _JIT_FN[(di, src)] = fn
    return fn


def _jit_for(prog: Program, cargs, kind: str, key_reg: int = -1, val_regs=(), dev=None, agg_op: int = -1):
    """(kernel handle, nreg, rows) of the compiled kernel for this launch on ``dev``, or None (interpreter)."""
    if not JIT or not hasattr(_ext.hip(), "jit_compile"):
        return None
    kinds = tuple(c[0] for c in cargs)
    lates = tuple(c[1] for c in cargs) if kind in ("agg", "emit", "pairs") else ()
    # the kernel of a program shape: generated + compiled once, then found by the shape alone (generating the source
    # costs ~30 us of Python per launch)
    shape = (_dev_index(dev), kind, tuple(prog.ins), kinds, lates, key_reg, tuple(val_regs), prog.keep_reg,
             prog.nins_a, getattr(prog, "jk_reg", -1), getattr(prog, "keep2_reg", -1),
             tuple(k[0] for k in getattr(prog, "emit_keys", [])) if kind == "emit" else (), JIT_ROWS, JIT_ROWS_SMALL,
             JIT_SMALL_NREG, JIT_LIKE_WINDOW, bytes(prog.lit or b"") if JIT_LIKE_WINDOW == "auto" else b"", agg_op)
    hit = _JIT_SHAPES.get(shape)
    if hit is None:
        nreg = program_nreg(prog, len(kinds), key_reg, val_regs)
        rows = JIT_ROWS_SMALL if nreg <= JIT_SMALL_NREG else JIT_ROWS
        try:
            src = jit_source(prog, list(kinds), list(lates) or [0] * len(kinds), kind, key_reg, val_regs, rows=rows,
                             agg_op=agg_op)
        except Unfusable:
            return None
        fn = jit_kernel(src, {"agg": "nsdb_jit_agg", "emit": "nsdb_jit_emit", "pairs": "nsdb_jit_emit"}.get(
            kind, "nsdb_jit_mask"), dev)
        if len(_JIT_SHAPES) >= 4096:          # the shape includes the immediates: bound it for varying literals
            _JIT_SHAPES.clear()
        hit = _JIT_SHAPES[shape] = (fn, nreg, rows)
    if hit[0] is None:
        return None
    JIT_STATS["launches"] += 1
    return hit


_LIT_DEV: Dict[tuple, torch.Tensor] = {}       # (literal bytes, device) -> the pool on the device (read-only)


def _prog_tensors(prog: Program, dev):
    """The program's instruction table (host int64 [nins, 7]) and its literal pool on ``dev``: built once per compiled
    program / literal pool and shared by every launch of it (a cached program's copies share its ``_ins_t``)."""
    ins = prog.__dict__.get("_ins_t")
    if ins is None:
        ins = torch.tensor(prog.ins if prog.ins else [[0, 0, -1, -1, -1, 0, 0]], dtype=torch.int64).reshape(-1, 7)
        if not prog.ins:
            ins = ins[:0]
        prog._ins_t = ins
    key = (bytes(prog.lit or b"\0"), dev)
    lit = _LIT_DEV.get(key)
    if lit is None:
        if len(_LIT_DEV) >= 256:
            _LIT_DEV.clear()
        lit = _LIT_DEV[key] = torch.frombuffer(bytearray(key[0]), dtype=torch.uint8).to(dev)
    return ins, lit


def _join_table(plan: StagePlan, dev):
    """(slots, perm, build rows, probe filter or None) of the fused join's device hash table (relops join_build),
    built on first use."""
    bt = plan.builds[plan.join["name"]]
    if bt.batch is None or bt.batch.n == 0:
        raise Unfusable("empty build side")
    jt = bt.table(dev)
    d = getattr(jt, "_dev", None)
    if d is None:
        raise Unfusable("build side without a device hash table")
    return d[0], d[1], int(bt.batch.n), (d[2] if len(d) > 2 and d[2].numel() else None)


def _launch(prog: Program, n: int, dev, plan: StagePlan):
    h = _ext.hip()
    ins, lit = _prog_tensors(prog, dev)
    cargs = _col_args(prog, dev)
    jtab = jperm = jbloom = None
    bn = -1
    if plan.join is not None:
        jtab, jperm, bn, jbloom = _join_table(plan, dev)
    jit = _jit_for(prog, cargs, "agg", prog.key_reg, prog.val_regs, dev,
                   agg_op=AGG_OPS[plan.op] if JIT_FIXED_OP else -1)
    if jit is None and plan.join is not None:
        raise Unfusable("the fused join probe needs the compiled kernels")
    fn, jnreg, jrows = jit if jit else (0, 0, 0)
    table = h.pipe_agg(ins, prog.nins_a, cargs, lit, n, prog.keep_reg, prog.key_reg, prog.val_regs,
                       AGG_OPS[plan.op], 0, TILE, prog.kpool, fn, jnreg, jrows, jtab, jperm, bn, jbloom)
    host = _read_table(table)                    # the one device -> host read of the launch
    if int(host[0]) != 0:
        return None
    if n:
        _SEL_EST[plan.sig] = int(host[1]) / n
    gcap = (host.size - 2) // (1 + FMAX)
    keys = host[2:2 + gcap]
    occ = np.flatnonzero(keys != _EMPTY)           # a few KB: numpy, not torch CPU-op dispatch
    k = keys[occ]
    order = np.argsort(k, kind="stable")
    vals = host[2 + gcap:].view(np.float64).reshape(gcap, FMAX)
    sel = occ[order]
    return torch.from_numpy(k[order]), torch.from_numpy(np.ascontiguousarray(vals[sel, : prog.nval]))


_TABLE_HOST: Dict[tuple, torch.Tensor] = {}     # (device, words) -> pinned host buffer of the result table


def _read_table(table: torch.Tensor):
    """The launch's result table on the host (numpy int64), through a pinned buffer kept per device: one
    asynchronous copy + one stream sync instead of a pageable copy."""
    if not table.is_cuda:
        return table.numpy()
    key = (table.device, table.numel(), threading.get_ident())     # per thread: concurrent jobs never share one
    buf = _TABLE_HOST.get(key)
    if buf is None:
        if len(_TABLE_HOST) >= 64:
            _TABLE_HOST.clear()
        buf = _TABLE_HOST[key] = torch.empty(table.numel(), dtype=table.dtype, pin_memory=True)
    buf.copy_(table, non_blocking=True)
    torch.cuda.current_stream(table.device).synchronize()
    return buf.numpy()                           # only read before the next launch; results are fancy-indexed copies


def _merge(k: torch.Tensor, v: torch.Tensor, op: str):
    uniq, inv = torch.unique(k, return_inverse=True)
    g = int(uniq.numel())
    if op == "sum":
        out = torch.zeros(g, v.shape[1], dtype=torch.float64, device=v.device).index_add_(0, inv, v)
    else:
        out = torch.zeros(g, v.shape[1], dtype=torch.float64, device=v.device).scatter_reduce_(
            0, inv.unsqueeze(1).expand_as(v), v, "amin" if op == "min" else "amax", include_self=False)
    return uniq, out


def _key_columns(prog: Program, keys: torch.Tensor):
    lay = prog.key_layout
    if lay[0] == "const":
        v = lay[1]
        dt = torch.float64 if isinstance(v, float) else torch.int64
        return torch.full((keys.numel(),), v, dtype=dt, device=keys.device)
    if lay[0] == "int":
        col = keys.to(lay[1])
        return (col,) if lay[2] else col
    Ls = lay[1]
    bits = [8 * L + 3 for L in Ls]
    cols, shift = [], sum(bits)
    for L, b in zip(Ls, bits):
        shift -= b
        code = (keys >> shift) & ((1 << b) - 1)
        cols.append(StringColumn.from_short_codes(code, L))
    return tuple(cols) if lay[2] else cols[0]


def _value_column(prog: Program, vals: torch.Tensor):
    return vals.contiguous() if prog.val_shape == "row" else vals[:, 0].contiguous()


# ---------------------------------------------------------------------------------------------- torch interpreter
def _floating_like(pattern) -> bool:
    """A LIKE pattern of '%'-separated segments only ('%a%b%'), each 2-16 bytes starting with two literal bytes: the
    launch precomputes its match column buffer-parallel (StringColumn.like -> strings.hip like_occ_kernel) instead of a
    per-row search inside the fused kernel. JIT_LIKE_OCC = False keeps every LIKE in the kernel."""
    if not JIT_LIKE_OCC or not isinstance(pattern, str) or not pattern.startswith("%") or not pattern.endswith("%"):
        return False
    from ..objects.strings import _ANY, _compile_like

    buf, st, ln, a0, a1 = _compile_like(pattern)
    return (not a0 and not a1 and 1 <= len(ln) <= 4 and all(2 <= n <= 16 for n in ln)
            and all(buf[s] != _ANY and buf[s + 1] != _ANY for s in st))


JIT_LIKE_OCC = os.environ.get("NSDB_JIT_LIKE_OCC", "1") != "0"


def _like_mask(c: dict) -> torch.Tensor:
    """The 0/1 match column of a precomputed LIKE (uint8, one per row of the string column)."""
    return c["obj"].like(c["like"]).view(torch.uint8)


def _col_values(c: dict) -> torch.Tensor:
    if c.get("like") is not None:
        return _like_mask(c).long()
    o, kind = c["obj"], c["kind"]
    if kind == C_SCODE:
        return o.short_codes(c["L"])
    if kind == C_SREF:
        return torch.stack([o.starts, o.ends], 1)                 # kept as (start, end); string ops read bytes
    if kind in (C_F64, C_F32):
        return o.double().view(torch.int64) if kind == C_F64 else o.double().view(torch.int64)
    return o.long()


def interpret(prog: Program, n: int, op: str):
    """The program evaluated with whole-column torch ops (same semantics as pipeline.hip; the CPU check of the
    compiler). Returns the merged (keys, values)."""
    regs = _run_program(prog, n)
    f = lambda t: t.view(torch.float64)  # noqa: E731
    keep = torch.ones(n, dtype=torch.bool) if prog.keep_reg < 0 else regs[prog.keep_reg] != 0
    key = torch.zeros(n, dtype=torch.int64) if prog.key_reg < 0 else regs[prog.key_reg]
    vals = torch.stack([f(regs[r]) for r in prog.val_regs], 1) if prog.val_regs else torch.zeros(n, 0, dtype=torch.float64)
    idx = keep.nonzero().flatten()
    if torch.unique(key[idx]).numel() > INTERP_CAP:
        return None
    return _merge(key[idx], vals[idx], op)


def interpret_emit(prog: Program, n: int, plan: StagePlan):
    """The emitted form with whole-column torch ops (the CPU model of jit_emit_body): (int64 words [ne, rows], rows)
    of every kept (matched) row, key-part registers first, then the value registers."""
    from . import kernels as KK

    prow = brow = None
    if plan.join is None:
        regs = _run_program(prog, n)
        keep = torch.ones(n, dtype=torch.bool) if prog.keep_reg < 0 else regs[prog.keep_reg] != 0
        prow = torch.arange(n)
    else:
        regs = _run_program(prog, n, hi=prog.nins_a, sides=(0,))
        keep = torch.ones(n, dtype=torch.bool) if prog.keep_reg < 0 else regs[prog.keep_reg] != 0
        kidx = keep.nonzero().flatten()
        bt = plan.builds[plan.join["name"]]
        bi, pi = bt.table(kidx.device).probe(KK.hash_keys(regs[prog.jk_reg][kidx]))
        prow = kidx[pi]
        n = int(prow.numel())
        regs = _run_program(prog, n, lo=prog.nins_a, rowmap={i: (bi if c["late"] == 2 else prow)
                                                             for i, c in enumerate(prog.cols)})
        keep = torch.ones(n, dtype=torch.bool) if prog.keep2_reg < 0 else regs[prog.keep2_reg] != 0
        brow = bi
    idx = keep.nonzero().flatten()
    rs = [k[0] for k in prog.emit_keys] + list(prog.val_regs)
    pick = lambda r: prow.to(torch.int64) if r == -1 else brow.to(torch.int64) if r == -2 else regs[r]  # noqa: E731
    words = torch.stack([pick(r)[idx] for r in rs]) if rs else torch.zeros(1, idx.numel(), dtype=torch.int64)
    return words, int(idx.numel())


def interpret_join(prog: Program, n: int, plan: StagePlan):
    """A fused join program with whole-column torch ops (the CPU model of jit_join_agg_body): segment A over the
    probe rows, the probe against the build side's join hashes (kernels.JoinTable), segment B over every (build row,
    probe row) pair, then the post-join keep flag, key and values merged."""
    from . import kernels as KK

    regs = _run_program(prog, n, hi=prog.nins_a, sides=(0,))
    keep = torch.ones(n, dtype=torch.bool) if prog.keep_reg < 0 else regs[prog.keep_reg] != 0
    kidx = keep.nonzero().flatten()
    bt = plan.builds[plan.join["name"]]
    h = KK.hash_keys(regs[prog.jk_reg][kidx])
    bi, pi = bt.table(h.device).probe(h)
    prow = kidx[pi]
    m = int(prow.numel())
    rowmap = {i: (bi if c["late"] == 2 else prow) for i, c in enumerate(prog.cols)}
    regs = _run_program(prog, m, lo=prog.nins_a, rowmap=rowmap)
    f = lambda t: t.view(torch.float64)  # noqa: E731
    keep2 = torch.ones(m, dtype=torch.bool) if prog.keep2_reg < 0 else regs[prog.keep2_reg] != 0
    key = torch.zeros(m, dtype=torch.int64) if prog.key_reg < 0 else regs[prog.key_reg]
    vals = torch.stack([f(regs[r]) for r in prog.val_regs], 1) if prog.val_regs else torch.zeros(m, 0, dtype=torch.float64)
    idx = keep2.nonzero().flatten()
    if torch.unique(key[idx]).numel() > INTERP_CAP:
        return None
    return _merge(key[idx], vals[idx], plan.op)


def _run_program(prog: Program, n: int, lo: int = 0, hi: Optional[int] = None, sides=(0, 1),
                 rowmap: Optional[dict] = None) -> List[Optional[torch.Tensor]]:
    """Instructions [lo, hi) of the program over whole columns: the final register values. ``rowmap``: column slot ->
    the row of that column each of the n evaluated rows reads (a fused join's expanded pairs); ``sides``: which
    columns to load (0 = the stage's own, build-side columns only with 1 in it)."""
    regs: List[Optional[torch.Tensor]] = [None] * NREG
    for i, c in enumerate(prog.cols):
        if (1 if c["late"] == 2 else 0) not in sides:
            continue
        v = _col_values(c)
        regs[i] = v if rowmap is None else v[rowmap[i]]
    f = lambda t: t.view(torch.float64)  # noqa: E731
    u = lambda t: t.view(torch.int64)    # noqa: E731

    def strmatch(ref, col, imm, mode):
        o = prog.cols[col]["obj"]
        off, ll = imm >> 16, imm & 0xFFFF
        lit = bytes(prog.lit[off: off + ll])
        s = o.tolist()
        if rowmap is not None:
            s = [s[i] for i in rowmap[col].tolist()]
        if mode == 3:                          # general LIKE: decode the pool entry back into a regex
            flags, nseg = lit[0], lit[1]
            lens, body, segs, o = lit[2:2 + nseg], lit[2 + nseg:], [], 0
            for ln_ in lens:
                segs.append(body[o:o + ln_])
                o += ln_
            pieces = [re.escape(g).replace(re.escape(b"\xff"), b".") for g in segs]
            if not pieces:
                rx = re.compile(rb"\A\Z" if flags == 3 else rb"", re.S)
            else:
                rx = re.compile((rb"\A" if flags & 1 else rb".*") + b".*".join(pieces) + (rb"\Z" if flags & 2 else b""),
                                re.S)
            m = [rx.match(x.encode()) is not None for x in s]
        elif mode == 0:
            m = [x.encode() == lit for x in s]
        elif mode == 1:
            m = [x.encode().startswith(lit) for x in s]
        else:
            m = [x.encode().endswith(lit) for x in s]
        return torch.tensor(m, dtype=torch.int64)

    def run(lo, hi):
        for opc, d, a, b, c, imm, aux in prog.ins[lo:hi]:
            x = regs[a] if a >= 0 else (torch.full((n,), imm, dtype=torch.int64) if a == IMM else None)
            y = regs[b] if b >= 0 else (torch.full((n,), imm, dtype=torch.int64) if b == IMM else None)
            if opc == OP_CONST:
                z = torch.full((n,), imm, dtype=torch.int64)
            elif opc in (OP_ADDF, OP_SUBF, OP_MULF, OP_DIVF):
                fx, fy = f(x), f(y)
                z = u({OP_ADDF: fx + fy, OP_SUBF: fx - fy, OP_MULF: fx * fy, OP_DIVF: fx / fy}[opc].contiguous())
            elif opc == OP_NEGF:
                z = u((-f(x)).contiguous())
            elif opc in (OP_ADDI, OP_SUBI, OP_MULI):
                z = {OP_ADDI: x + y, OP_SUBI: x - y, OP_MULI: x * y}[opc]
            elif opc == OP_I2F:
                z = u(x.double())
            elif OP_LTF <= opc <= OP_NEF:
                fx, fy = f(x), f(y)
                z = [fx < fy, fx <= fy, fx > fy, fx >= fy, fx == fy, fx != fy][opc - OP_LTF].long()
            elif OP_LTI <= opc <= OP_NEI:
                z = [x < y, x <= y, x > y, x >= y, x == y, x != y][opc - OP_LTI].long()
            elif opc == OP_AND:
                z = ((x != 0) & (y != 0)).long()
            elif opc == OP_OR:
                z = ((x != 0) | (y != 0)).long()
            elif opc == OP_NOT:
                z = (x == 0).long()
            elif opc == OP_PACK:
                z = (x << (imm & 63)) | y
            elif opc in (OP_SEQ, OP_SPRE, OP_SSUF, OP_SLIKE):
                z = strmatch(x, b, imm, {OP_SEQ: 0, OP_SPRE: 1, OP_SSUF: 2, OP_SLIKE: 3}[opc])
            elif opc == OP_SEL:
                z = torch.where(x != 0, y, regs[imm])
            elif opc in (OP_RNGF, OP_RNGI):
                hi_v, mode = prog.kpool[aux & 0xFF], aux >> 8
                xv, lo_t, hi_t = (f(x), f(torch.tensor([imm])), f(torch.tensor([hi_v]))) if opc == OP_RNGF else \
                    (x, torch.tensor([imm]), torch.tensor([hi_v]))
                z = (((xv >= lo_t) if mode & 1 else (xv > lo_t)) & ((xv <= hi_t) if mode & 2 else (xv < hi_t))).long()
            else:
                z = torch.zeros(n, dtype=torch.int64)
            if c >= 0:                          # compare folded with its conjunction's AND
                z = ((z != 0) & (regs[c] != 0)).long()
            regs[d] = z

    run(lo, len(prog.ins) if hi is None else hi)
    return regs


# ---------------------------------------------------------------------------------------------- fused probe
class ProbePlan(StagePlan):
    """[lambda-tree APPLYs + FILTER] -> HASH -> JOIN probe as ONE compiled launch (the "pairs" emit form): predicate,
    probe of the build side's device hash table and the CSR walk of repeated keys in registers, writing the (probe
    row, build row) of every kept, matched row. The join's output is then two row selections (lazy takes) — no mask,
    compaction, key gather, hash column or probe / expand passes (reference JoinProbe in the pipeline chain,
    src/lambdas/headers/JoinTuple.h:434)."""

    def __init__(self, atoms, conj: List[E], join_atom: dict, key_col: str):
        super().__init__([], atoms, conj, E("const", (), 0), E("vals", ()), "sum", "", "",
                         join={"name": join_atom["output"]["name"], "key": E("src", (), key_col)})
        self.jatom = join_atom
        self.cap_mult = 2


def fuse_probes(ops: List[dict]) -> List[dict]:
    """``ops`` (after fuse_filters) with every [FUSED_FILTER]? HASHLEFT/RIGHT JOIN run whose probe key is one plain
    column of the incoming batch replaced by one FUSED_PROBE op (its atoms kept for the eager fallback)."""
    out: List[dict] = []
    i = 0
    while i < len(ops):
        o = ops[i]
        nxt = ops[i + 1] if i + 1 < len(ops) else None
        if o["type"] in ("HASHLEFT", "HASHRIGHT") and nxt is not None and nxt["type"] == "JOIN" and \
                len(o["input"]["atts"]) == 1 and nxt.get("_strategy") != "partitioned":
            side = nxt.get("_probe_side")
            probe_in = nxt["input"] if side == "left" else nxt["input2"] if side == "right" else None
            if probe_in is not None and probe_in["name"] == o["output"]["name"] and \
                    probe_in["atts"][0] == o["output"]["atts"][-1]:
                key = o["input"]["atts"][0]
                ff = out[-1] if out and out[-1]["type"] == "FUSED_FILTER" else None
                if ff is not None and key not in ff["plan"].proj:
                    ff = None
                if ff is not None:
                    out.pop()
                    atoms, conj = ff["atoms"] + [o, nxt], list(ff["plan"].conj)
                else:
                    atoms, conj = [o, nxt], []
                out.append({"type": "FUSED_PROBE", "plan": ProbePlan(atoms, conj, nxt, key), "atoms": atoms,
                            "join": nxt})
                i += 2
                continue
        out.append(o)
        i += 1
    return out


def run_probe(plan: ProbePlan, batch: RecordBatch):
    """(probe rows, build rows) of every kept, matched row of ``batch`` from one compiled launch, or None (eager atoms:
    no compiled kernels, a column the kernel cannot read, an empty or out-of-core build side, a region overflow)."""
    if plan.disabled or batch.n == 0:
        return None
    dev = batch.device
    on_gpu = dev.type == "cuda" and _ext.hip() is not None and hasattr(_ext.hip(), "pipe_emit")
    if not on_gpu and not (CPU_INTERPRETER and dev.type == "cpu"):
        return None
    try:
        prog = _compile_cached(plan, batch, "pairs")
        got = _launch_emit(prog, batch.n, dev, plan, "pairs") if on_gpu else interpret_pairs(prog, batch.n, plan)
    except Unfusable as e:
        plan.disabled = True
        plan.reason = str(e)
        return None
    if got is None:                      # more matches per probe row than the tile regions hold: wider next time
        plan.cap_mult *= 4
        if plan.cap_mult > 32:
            plan.disabled = True
        return None
    words, m = got
    plan.stats["fused_batches"] += 1
    return words[0], words[1]


def interpret_pairs(prog: Program, n: int, plan: StagePlan):
    """The "pairs" form with whole-column torch ops (CPU model): (int64 [2, m] probe rows / build rows, m)."""
    from . import kernels as KK

    regs = _run_program(prog, n, hi=prog.nins_a, sides=(0,))
    keep = torch.ones(n, dtype=torch.bool) if prog.keep_reg < 0 else regs[prog.keep_reg] != 0
    kidx = keep.nonzero().flatten()
    bt = plan.builds[plan.join["name"]]
    if bt.batch is None or bt.batch.n == 0:
        raise Unfusable("empty build side")
    bi, pi = bt.table(kidx.device).probe(KK.hash_keys(regs[prog.jk_reg][kidx]))
    prow = kidx[pi]
    return torch.stack([prow, bi.to(prow.dtype)]), int(prow.numel())


# ---------------------------------------------------------------------------------------------- fused FILTER
class FilterPlan(StagePlan):
    """A run of lambda-tree APPLY atoms ending in their FILTER: the predicate as one mask launch (pipe_mask)."""

    def __init__(self, atoms, conj: E, proj: List[str]):
        super().__init__([], atoms, [conj], E("const", (), 0), E("vals", ()), "sum", "", "")
        self.proj = proj


def fuse_filters(ops: List[dict], comps: dict) -> List[dict]:
    """``ops`` with every maximal run [lambda-tree APPLYs..., FILTER] whose FILTER keeps only columns that existed
    before the run replaced by one FUSED_FILTER op (its atoms kept for the eager fallback)."""
    out, i = [], 0
    while i < len(ops):
        o = ops[i]
        if o["type"] != "FILTER":
            out.append(o)
            i += 1
            continue
        j = len(out)                                    # walk back over the fusable APPLYs just before it
        while j > 0 and out[j - 1]["type"] == "APPLY" and not out[j - 1]["lambda"].startswith("self_") and \
                _apply_fusable(out[j - 1], comps):
            j -= 1
        run = out[j:]
        fp = _filter_plan(run, o, comps) if run else None
        if fp is None:
            out.append(o)
        else:
            del out[j:]
            out.append({"type": "FUSED_FILTER", "plan": fp, "atoms": run + [o]})
        i += 1
    return out


def _apply_fusable(o, comps) -> bool:
    node = comps[o["comp"]].extract_lambdas().get(o["lambda"])
    if node is None:
        return False
    try:
        _node_expr(node, [E("src", (), a) for a in o["input"]["atts"]])
    except Unfusable:
        return False
    return True


def _filter_plan(run, filt, comps) -> Optional[FilterPlan]:
    env: Dict[str, E] = {}
    col = lambda name: env[name] if name in env else E("src", (), name)  # noqa: E731
    try:
        for o in run:
            node = comps[o["comp"]].extract_lambdas()[o["lambda"]]
            env[o["output"]["atts"][-1]] = _node_expr(node, [col(a) for a in o["input"]["atts"]])
    except (Unfusable, KeyError):
        return None
    conj = col(filt["input"]["atts"][0])
    proj = list(filt["projection"]["atts"])
    if conj.kind == "src" or any(c in env for c in proj):
        return None
    return FilterPlan(run + [filt], conj, proj)


def run_filter(plan: FilterPlan, batch: RecordBatch) -> Optional[RecordBatch]:
    """The FILTER's output (its projection columns, the kept rows) from one mask launch, or None (eager atoms)."""
    if plan.disabled or batch.n == 0:
        return None
    dev = batch.device
    on_gpu = dev.type == "cuda" and _ext.hip() is not None and hasattr(_ext.hip(), "pipe_mask")
    if not on_gpu and not (CPU_INTERPRETER and dev.type == "cpu"):
        return None
    try:
        prog = _compile_cached(plan, batch)
    except Unfusable as e:
        plan.disabled = True
        plan.reason = str(e)
        return None
    if on_gpu:
        ins, lit = _prog_tensors(prog, dev)
        try:
            cargs = _col_args(prog, dev)
        except Unfusable as e:
            plan.disabled = True
            plan.reason = str(e)
            return None
        jit = _jit_for(prog, cargs, "mask", dev=dev)
        fn, jnreg, jrows = jit if jit else (0, 0, 0)
        mask = _ext.hip().pipe_mask(ins, cargs, lit, batch.n, prog.keep_reg, TILE, prog.kpool, fn, jnreg,
                                    jrows).view(torch.bool)      # 0 / 1 bytes: a bool view, no conversion pass
    else:
        mask = interpret_mask(prog, batch.n)
    plan.stats["fused_batches"] += 1
    idx = K.selected_rows(mask)
    keep = RecordBatch({c: batch.columns[c] for c in plan.proj}, batch.n)
    return keep.take(idx)


def interpret_mask(prog: Program, n: int) -> torch.Tensor:
    """The predicate program's keep flags with the torch interpreter (CPU check of the compiler)."""
    regs = _run_program(prog, n)
    return torch.ones(n, dtype=torch.bool) if prog.keep_reg < 0 else regs[prog.keep_reg] != 0


__all__ = ["plan_stage", "run_batch", "StagePlan", "Unfusable", "interpret", "interpret_join", "fuse_filters", "run_filter",
           "FilterPlan", "ProbePlan", "fuse_probes", "run_probe", "interpret_pairs"]
