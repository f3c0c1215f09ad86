"""Compile a computation graph into TCAP — netsDB's tuple-set IR.

Reference: each Computation's ``toTCAPString`` (src/lambdas/headers/*Comp.h) and the grammar in
src/logicalPlan/source/Parser.y.  Every lambda-tree node becomes one APPLY atom; predicates
become FILTER; equality join keys become HASHLEFT/HASHRIGHT + JOIN (HASHONE for cartesian
inputs); aggregations become AGGREGATE; writers become OUTPUT.

A tuple-set column that holds an input object is named ``in<i>_<comp>``; the executor stores a
row-aligned :class:`RecordBatch` there.
"""
from __future__ import annotations

import itertools
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

from ..computations import (AggregateComp, Computation, JoinComp, MultiSelectionComp, PartitionComp, ScanSet,
                            SelectionComp, TopKComp, WriteSet)
from ..lambdas import Arg, Binary, Lambda, Literal


@dataclass
class TupleSpec:
    name: str
    atts: List[str]

    def __str__(self):
        return f"{self.name}({', '.join(self.atts)})"


@dataclass
class CompiledPlan:
    tcap: str
    computations: Dict[str, Computation]      # TCAP computation name -> object
    sinks: List[str]


class _Ctx:
    def __init__(self):
        self.lines: List[str] = []
        self.counter = itertools.count()
        self.comps: Dict[str, Computation] = {}
        self.names: Dict[int, str] = {}
        self.outputs: Dict[int, TupleSpec] = {}
        self.comp_counter = itertools.count()

    def tset(self, base: str) -> str:
        return f"{base}_{next(self.counter)}"

    def emit(self, line: str):
        self.lines.append(line)


def _q(s: str) -> str:
    return "'" + s.replace("'", "") + "'"


def compile_lambda(ctx: _Ctx, lam: Lambda, comp_name: str, cur: TupleSpec, obj_cols: Dict[int, str],
                   keep: Sequence[str], prefix: str) -> Tuple[TupleSpec, str]:
    """Emit APPLYs for every node of ``lam`` (postorder). Returns (tuple set, result column)."""
    result_col: Dict[int, str] = {}
    # intermediate tuple sets carry the kept columns, every input object column and the
    # results computed so far; the root's APPLY keeps only ``keep`` + its result
    avail = [c for c in cur.atts]
    carry = list(keep) + [c for c in obj_cols.values() if c not in keep and c in avail]
    nodes = lam.nodes_postorder()
    for pos, node in enumerate(nodes):
        if node.children:
            args = [result_col[id(c)] for c in node.children]
        elif isinstance(node, Literal):
            args = []
        else:
            args = [obj_cols[i] for i in node.input_indices()]
        col = f"{prefix}{next(ctx.counter)}"
        last = pos == len(nodes) - 1
        this_carry = list(keep) if last else carry
        out = TupleSpec(ctx.tset(f"{node.kind.replace('=', 'eq').replace('&', 'and').replace('|', 'or')}"
                                 f"OutFor_{comp_name}"), this_carry + [col])
        ctx.emit(f"{out} <= APPLY ({TupleSpec(cur.name, args)}, {TupleSpec(cur.name, this_carry)}, "
                 f"{_q(comp_name)}, {_q(node.name)})")
        result_col[id(node)] = col
        cur = out
        carry = carry + [col]
    return cur, result_col[id(lam)]


def _conjuncts(lam: Lambda) -> List[Lambda]:
    if isinstance(lam, Binary) and lam.op == "&&":
        return _conjuncts(lam.children[0]) + _conjuncts(lam.children[1])
    return [lam]


def _equality_keys(sel: Lambda, left: set, right: int):
    """Equality conjuncts usable as hash keys between the input set ``left`` and input ``right``."""
    keys = []
    for c in _conjuncts(sel):
        if isinstance(c, Binary) and c.op == "==":
            a, b = c.children
            ia, ib = set(a.input_indices()), set(b.input_indices())
            if ia and ib and ia <= left and ib == {right}:
                keys.append((a, b, c))
            elif ia and ib and ib <= left and ia == {right}:
                keys.append((b, a, c))
    return keys


class TCAPCompiler:
    def __init__(self):
        self.ctx = _Ctx()

    def compile(self, sinks: Sequence[Computation]) -> CompiledPlan:
        names = []
        for s in sinks:
            self._visit(s)
            names.append(self.ctx.names[id(s)])
        return CompiledPlan("\n".join(self.ctx.lines) + "\n", dict(self.ctx.comps), names)

    # ------------------------------------------------------------------ traversal
    def _visit(self, comp: Computation) -> TupleSpec:
        if id(comp) in self.ctx.outputs:
            return self.ctx.outputs[id(comp)]
        ins = []
        for i, c in enumerate(comp.inputs):
            if c is None:
                raise ValueError(f"{comp!r}: input {i} not set")
            ins.append(self._visit(c))
            if comp.input_types[i] is None:
                comp.input_types[i] = c.output_type
        name = f"{comp.comp_type}_{next(self.ctx.comp_counter)}"
        self.ctx.names[id(comp)] = name
        self.ctx.comps[name] = comp
        comp._tcap_name = name
        comp._lambdas = {}
        out = self._emit(comp, name, ins)
        self.ctx.outputs[id(comp)] = out
        return out

    def _register(self, comp, lam: Lambda, counter):
        lam.assign_names(counter)
        for n in lam.nodes_postorder():
            comp._lambdas[n.name] = n
        return lam

    def _emit(self, comp: Computation, name: str, ins: List[TupleSpec]) -> TupleSpec:
        ctx = self.ctx
        lc = itertools.count()
        args = [Arg(i, t) for i, t in enumerate(comp.input_types)]
        if isinstance(comp, ScanSet):
            out = TupleSpec(ctx.tset(f"inputDataFor{name}"), [f"in0_{name}"])
            ctx.emit(f"{out} <= SCAN ({_q(comp.db)}, {_q(comp.set_name)}, {_q(name)})")
            return out
        if isinstance(comp, WriteSet):
            src = ins[0]
            out = TupleSpec(ctx.tset(f"outFor{name}"), [])
            ctx.emit(f"{out} <= OUTPUT ({TupleSpec(src.name, src.atts[-1:])}, {_q(comp.db)}, "
                     f"{_q(comp.set_name)}, {_q(name)})")
            return out
        if isinstance(comp, (SelectionComp,)):
            src = ins[0]
            obj = src.atts[-1]
            cur = TupleSpec(src.name, [obj])
            sel = self._register(comp, comp.get_selection(args[0]), lc)
            proj = self._register(comp, comp.get_projection(args[0]), lc)
            if not (isinstance(sel, Literal) and sel.value is True):
                cur, bcol = compile_lambda(ctx, sel, name, cur, {0: obj}, [obj], "sel")
                filt = TupleSpec(ctx.tset(f"filteredInputFor{name}"), [obj])
                ctx.emit(f"{filt} <= FILTER ({TupleSpec(cur.name, [bcol])}, {TupleSpec(cur.name, [obj])}, {_q(name)})")
                cur = filt
            cur, pcol = compile_lambda(ctx, proj, name, cur, {0: obj}, [], "proj")
            if isinstance(comp, MultiSelectionComp):
                flat = TupleSpec(ctx.tset(f"flattenedOutFor{name}"), [f"flat_{name}"])
                ctx.emit(f"{flat} <= FLATTEN ({TupleSpec(cur.name, [pcol])}, {TupleSpec(cur.name, [])}, {_q(name)})")
                return flat
            return TupleSpec(cur.name, [pcol])
        if isinstance(comp, JoinComp):
            return self._emit_join(comp, name, ins, args, lc)
        if isinstance(comp, (AggregateComp, TopKComp)):
            src = ins[0]
            obj = src.atts[-1]
            key = self._register(comp, comp.get_key_projection(args[0]), lc)
            val = self._register(comp, comp.get_value_projection(args[0]), lc)
            cur, kcol = compile_lambda(ctx, key, name, TupleSpec(src.name, [obj]), {0: obj}, [obj], "key")
            cur, vcol = compile_lambda(ctx, val, name, cur, {0: obj}, [kcol], "val")
            out = TupleSpec(ctx.tset(f"aggOutFor{name}"), [f"aggOut_{name}"])
            ctx.emit(f"{out} <= AGGREGATE ({TupleSpec(cur.name, [kcol, vcol])}, {_q(name)})")
            return out
        if isinstance(comp, PartitionComp):
            src = ins[0]
            obj = src.atts[-1]
            key = self._register(comp, comp.get_key_projection(args[0]), lc)
            cur, kcol = compile_lambda(ctx, key, name, TupleSpec(src.name, [obj]), {0: obj}, [obj], "key")
            out = TupleSpec(ctx.tset(f"partitionOutFor{name}"), [f"part_{name}"])
            ctx.emit(f"{out} <= PARTITION ({TupleSpec(cur.name, [kcol, obj])}, {_q(name)})")
            return out
        raise TypeError(f"cannot compile {comp!r}")

    def _emit_join(self, comp: JoinComp, name: str, ins: List[TupleSpec], args, lc) -> TupleSpec:
        ctx = self.ctx
        sel = self._register(comp, comp.get_selection(*args), lc)
        proj = self._register(comp, comp.get_projection(*args), lc)
        objs = {}
        # rename every input's object column to in<i>_<name>
        cur_specs = []
        for i, s in enumerate(ins):
            col = f"in{i}_{name}"
            objs[i] = col
            t = TupleSpec(ctx.tset(f"in{i}For{name}"), [col])
            ctx.emit(f"{t} <= APPLY ({TupleSpec(s.name, s.atts[-1:])}, {TupleSpec(s.name, [])}, {_q(name)}, 'self_in{i}')")
            cur_specs.append(t)
        left = cur_specs[0]
        left_inputs = {0}
        left_cols = [objs[0]]
        for r in range(1, len(ins)):
            keys = _equality_keys(sel, left_inputs, r)
            right = cur_specs[r]
            if keys:
                lcur, rcur = TupleSpec(left.name, left_cols), TupleSpec(right.name, [objs[r]])
                lkeys, rkeys = [], []
                for (lk, rk, eq) in keys:
                    lcur, kc = compile_lambda(ctx, lk, name, lcur, objs, left_cols, "lk")
                    lkeys.append(kc)
                    lcur = TupleSpec(lcur.name, left_cols)
                    rcur, kr = compile_lambda(ctx, rk, name, rcur, objs, [objs[r]], "rk")
                    rkeys.append(kr)
                    rcur = TupleSpec(rcur.name, [objs[r]])
                eqname = keys[0][2].name
                lh = TupleSpec(ctx.tset(f"hashLeftFor{name}"), left_cols + [f"lh{r}_{name}"])
                ctx.emit(f"{lh} <= HASHLEFT ({TupleSpec(lcur.name, lkeys)}, {TupleSpec(lcur.name, left_cols)}, "
                         f"{_q(name)}, {_q(eqname)})")
                rh = TupleSpec(ctx.tset(f"hashRightFor{name}"), [objs[r], f"rh{r}_{name}"])
                ctx.emit(f"{rh} <= HASHRIGHT ({TupleSpec(rcur.name, rkeys)}, {TupleSpec(rcur.name, [objs[r]])}, "
                         f"{_q(name)}, {_q(eqname)})")
            else:
                lh = TupleSpec(ctx.tset(f"hashOneLeftFor{name}"), left_cols + [f"lh{r}_{name}"])
                ctx.emit(f"{lh} <= HASHONE ({TupleSpec(left.name, left_cols)}, {TupleSpec(left.name, left_cols)}, {_q(name)})")
                rh = TupleSpec(ctx.tset(f"hashOneRightFor{name}"), [objs[r], f"rh{r}_{name}"])
                ctx.emit(f"{rh} <= HASHONE ({TupleSpec(right.name, [objs[r]])}, {TupleSpec(right.name, [objs[r]])}, {_q(name)})")
            joined_cols = left_cols + [objs[r]]
            j = TupleSpec(ctx.tset(f"joinedFor{name}"), joined_cols)
            ctx.emit(f"{j} <= JOIN ({TupleSpec(lh.name, [lh.atts[-1]])}, {TupleSpec(lh.name, left_cols)}, "
                     f"{TupleSpec(rh.name, [rh.atts[-1]])}, {TupleSpec(rh.name, [objs[r]])}, {_q(name)})")
            left, left_cols = j, joined_cols
            left_inputs.add(r)
        cur = TupleSpec(left.name, left_cols)
        if not (isinstance(sel, Literal) and sel.value is True):
            cur, bcol = compile_lambda(ctx, sel, name, cur, objs, left_cols, "sel")
            filt = TupleSpec(ctx.tset(f"filteredJoinFor{name}"), left_cols)
            ctx.emit(f"{filt} <= FILTER ({TupleSpec(cur.name, [bcol])}, {TupleSpec(cur.name, left_cols)}, {_q(name)})")
            cur = filt
        cur, pcol = compile_lambda(ctx, proj, name, cur, objs, [], "proj")
        return TupleSpec(cur.name, [pcol])


def compile_tcap(sinks: Sequence[Computation]) -> CompiledPlan:
    return TCAPCompiler().compile(list(sinks))


def _lam_tokens(lam: Lambda) -> tuple:
    return tuple((type(n).__name__, n.kind, n.name, getattr(n, "field", None), getattr(n, "method", None),
                  getattr(n, "op", None), tuple(n.input_indices()) if not n.children else len(n.children))
                 for n in lam.nodes_postorder())


_PRIM = (bool, int, float, str, type(None))


def _node_values(n) -> tuple:
    """The constants a lambda node carries (literal value, LIKE pattern, IN list): not part of the graph signature
    but of any plan decision made from the values (execution/pipeline.py's fused stage expressions)."""
    nd = n.__dict__
    if "pattern" not in nd and "values" not in nd and type(nd.get("value")) in _PRIM:
        v = nd.get("value")
        return (type(v), v)                      # a plain literal (the common case); 1, 1.0 and True differ here
    out = []
    for a in ("value", "pattern", "negate", "values"):
        v = getattr(n, a, None)
        if isinstance(v, list):
            v = tuple((type(x), x) if isinstance(x, _PRIM) else ("?", type(x).__name__) for x in v)
        elif isinstance(v, _PRIM):
            v = (type(v), v)
        else:
            v = ("?", type(v).__name__)          # not a fusable constant: its type decides the plan
        out.append(v)
    return tuple(out)


def graph_signature(sinks: Sequence[Computation], values: Optional[list] = None
                    ) -> Tuple[tuple, Dict[str, Computation], Dict[str, Tuple[str, str]]]:
    """Structural key of a computation graph + its TCAP name bindings, WITHOUT emitting TCAP.

    Walks the graph in exactly the compiler's order and binds every computation's name and lambda
    names the same way (so a cached TCAP / parsed atom list can execute against this graph instance):
    two graphs with the same signature compile to the same TCAP text.  Lambda literal values and native
    lambda bodies are looked up on the live objects at run time, so they are not part of the key
    (QuerySchedulerServer's pre-compiled workloads, src/queryPlanning/headers/PreCompiledWorkload.h).
    ``values``, when given, receives every lambda node's constants in the same walk (signature + values key plans
    that depend on the constants)."""
    comps: Dict[str, Computation] = {}
    names: Dict[int, str] = {}
    sets: Dict[str, Tuple[str, str]] = {}
    counter = itertools.count()
    toks: List[tuple] = []

    def reg(comp, lam, lc):
        # assign_names + the name table + _lam_tokens in ONE walk of the tree (this runs on every execution)
        d = comp._lambdas
        out = []
        for n in lam.nodes_postorder():
            if n.name is None:
                n.name = f"{n.kind}_{next(lc)}"
            d[n.name] = n
            if values is not None:
                nd = n.__dict__
                if "value" in nd or "pattern" in nd or "values" in nd:
                    values.append((n.name, _node_values(n)))
            out.append((type(n).__name__, n.kind, n.name, getattr(n, "field", None), getattr(n, "method", None),
                        getattr(n, "op", None), tuple(n.input_indices()) if not n.children else len(n.children)))
        return tuple(out)

    def visit(comp) -> str:
        if id(comp) in names:
            return names[id(comp)]
        ins = []
        for i, c in enumerate(comp.inputs):
            if c is None:
                raise ValueError(f"{comp!r}: input {i} not set")
            ins.append(visit(c))
            if comp.input_types[i] is None:
                comp.input_types[i] = c.output_type
        name = f"{comp.comp_type}_{next(counter)}"
        names[id(comp)] = name
        comps[name] = comp
        comp._tcap_name = name
        comp._lambdas = {}
        lc = itertools.count()
        args = [Arg(i, t) for i, t in enumerate(comp.input_types)]
        tok: list = [type(comp).__module__ + "." + type(comp).__qualname__, comp.comp_type, tuple(ins)]
        if isinstance(comp, (ScanSet, WriteSet)):
            sets[name] = (comp.db, comp.set_name)     # parameters of the workload, not part of its shape
        elif isinstance(comp, SelectionComp):
            tok.append(reg(comp, comp.get_selection(args[0]), lc))
            tok.append(reg(comp, comp.get_projection(args[0]), lc))
        elif isinstance(comp, JoinComp):
            tok.append(reg(comp, comp.get_selection(*args), lc))
            tok.append(reg(comp, comp.get_projection(*args), lc))
        elif isinstance(comp, (AggregateComp, TopKComp)):
            tok.append(reg(comp, comp.get_key_projection(args[0]), lc))
            tok.append(reg(comp, comp.get_value_projection(args[0]), lc))
        elif isinstance(comp, PartitionComp):
            tok.append(reg(comp, comp.get_key_projection(args[0]), lc))
        toks.append(tuple(tok))
        return name

    for s in sinks:
        toks.append(("sink", visit(s)))
    return tuple(toks), comps, sets


def bind_atoms(atoms: List[dict], sets: Dict[str, Tuple[str, str]]) -> List[dict]:
    """A cached (pre-compiled) atom list re-bound to this instance's scanned / written sets."""
    out = []
    for a in atoms:
        if a["type"] in ("SCAN", "OUTPUT") and a.get("comp") in sets:
            db, st = sets[a["comp"]]
            if (a.get("db"), a.get("set")) != (db, st):
                a = dict(a, db=db, set=st)
        out.append(a)
    return out


__all__ = ["TupleSpec", "CompiledPlan", "TCAPCompiler", "compile_tcap", "compile_lambda", "graph_signature", "bind_atoms"]
