"""LA DSL evaluator (reference: src/linearAlgebraDSL/source/LAEvaluateFunctions.cc + LAPDBInstance.h).

Every expression node is evaluated into a matrix set of database ``LA_db``; operators build
the LA UDF computations over ScanSets of their operand sets and run them as one job each.
"""
from __future__ import annotations

import itertools
import time
from typing import Dict

import torch

from ..computations import ScanSet, WriteSet
from ..models import blocks as B
from ..objects.builtin import MatrixBlock
from . import computations as L
from .parser import parse

DB = "LA_db"


class LAInstance:
    def __init__(self, client, dtype=torch.bfloat16, partition_loads: bool = False, verbose: bool = False):
        self.client = client
        self.dtype = dtype
        self.partition_loads = partition_loads
        self.verbose = verbose
        self.vars: Dict[str, str] = {}
        self._ids = itertools.count()
        self.job_stats = []
        client.create_database(DB)
        client.register_type(MatrixBlock)

    # ------------------------------------------------------------------ api
    def run(self, program: str) -> Dict[str, str]:
        for name, expr in parse(program):
            t0 = time.perf_counter()
            sname = self._eval(expr)
            self.vars[name] = sname
            if self.verbose:
                print(f"[LA] {name} = {sname} ({time.perf_counter() - t0:.3f}s)")
        return dict(self.vars)

    def run_file(self, path: str):
        with open(path) as f:
            return self.run(f.read())

    def get(self, name: str) -> torch.Tensor:
        return B.to_tensor(self.client, DB, self.vars[name])

    # ------------------------------------------------------------------ evaluation
    def _new(self) -> str:
        return f"LA_tmp_{next(self._ids)}"

    def _out(self) -> str:
        n = self._new()
        self.client.create_set(DB, n, MatrixBlock, dense=True)
        return n

    def _run(self, comp, job):
        out = self._out()
        st = self.client.execute_computations(WriteSet(DB, out, MatrixBlock).set_input(comp), job_name=job)
        self.job_stats.append(st)
        return out

    def _scan(self, s):
        return ScanSet(DB, s, MatrixBlock)

    def _eval(self, e) -> str:
        kind = e[0]
        if kind == "id":
            if e[1] not in self.vars:
                raise KeyError(f"LA: undefined identifier {e[1]}")
            return self.vars[e[1]]
        if kind == "init":
            return self._init(e[1], e[2])
        if kind == "num":
            raise ValueError("a bare constant is not a matrix")
        if kind == "bin":
            op, lhs, rhs = e[1], e[2], e[3]
            if op == "*" and (lhs[0] == "num" or rhs[0] == "num"):
                scalar = lhs[1] if lhs[0] == "num" else rhs[1]
                m = self._eval(rhs if lhs[0] == "num" else lhs)
                return self._scale(m, scalar)
            a, b = self._eval(lhs), self._eval(rhs)
            if op in ("%*%", "'*"):
                j = L.LAMultiply1Join() if op == "%*%" else L.LATransposeMultiply1Join()
                j.set_input(0, self._scan(a))
                j.set_input(1, self._scan(b))
                return self._run(L.LAMultiply2Aggregate().set_input(j), "la_multiply")
            j = {"+": L.LAAddJoin, "-": L.LASubstractJoin, "*": L.LAScaleMultiplyJoin}[op]()
            j.set_input(0, self._scan(a))
            j.set_input(1, self._scan(b))
            return self._run(j, f"la_{op}")
        if kind == "post":
            a = self._eval(e[2])
            comp = L.LATransposeSelection() if e[1] == "^T" else L.LAInverseAggregate()
            return self._run(comp.set_input(self._scan(a)), "la_post")
        if kind == "func":
            a = self._eval(e[2])
            cls = {"rowMax": L.LARowMaxAggregate, "rowMin": L.LARowMinAggregate, "rowSum": L.LARowSumAggregate,
                   "colMax": L.LAColMaxAggregate, "colMin": L.LAColMinAggregate, "colSum": L.LAColSumAggregate,
                   "max": L.LAMaxElementAggregate, "min": L.LAMinElementAggregate}[e[1]]
            return self._run(cls().set_input(self._scan(a)), f"la_{e[1]}")
        if kind == "dup":
            a = self._eval(e[2])
            cls = L.LADuplicateRowMultiSelection if e[1] == "duplicateRow" else L.LADuplicateColMultiSelection
            return self._run(cls(e[3], e[4]).set_input(self._scan(a)), f"la_{e[1]}")
        raise ValueError(f"LA: cannot evaluate {e}")

    def _init(self, kind, args) -> str:
        name = self._new()
        if kind == "identity":
            bs, nb = args
            n = bs * nb
            B.load_tensor(self.client, DB, name, torch.eye(n, device=self.client.device), bs, bs, dtype=self.dtype)
            return name
        brs, bcs, brn, bcn = args[:4]
        rows, cols = brs * brn, bcs * bcn
        if kind in ("zeros", "ones"):
            B.load_matrix(self.client, DB, name, rows, cols, brs, bcs, dtype=self.dtype,
                          value=1.0 if kind == "ones" else 0.0, partition_rows=self.partition_loads)
            return name
        # load(blockRowSize, blockColSize, blockRowNum, blockColNum, path)
        B.load_block_file(self.client, DB, name, args[4], brs, bcs, brn, bcn, dtype=torch.float32)
        return name

    def _scale(self, m: str, scalar: float) -> str:
        """``c * A``: one distributed selection job (LAScaleSelection), each rank scaling the blocks it holds."""
        return self._run(L.LAScaleSelection(scalar).set_input(self._scan(m)), "la_scale")


__all__ = ["LAInstance", "DB"]
