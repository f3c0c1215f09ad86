"""Tensor-pattern fusion: lower join+aggregate block-matrix chains onto fused MFMA kernels.

netsDB expresses a matrix multiply as JoinComp(A.blockCol == B.blockCol, project A·Bᵀ) +
ClusterAggregateComp(sum by output block) (src/FF/headers/FFTransposeMult.h + FFAggMatrix.h;
src/sharedLibraries/headers/LASillyMultiply1Join.h + LASillyMultiply2Aggregate.h) and an
activation as another join with the bias set (FFReluBiasSum, FFTransposeBiasSum).  Executed
literally that is one small GEMM per block pair, a hash aggregation of partial blocks, and one
more pass per epilogue.

When the computations declare their tensor pattern (``tensor_pattern()``) and the operands are
dense matrix sets, this pass rewrites the chain into :class:`MatmulNode` s that run as ONE split-K
MFMA GEMM each (the split-K slab reducer *is* the block aggregate) with bias/act/dropout fused in
the epilogue, and :class:`SoftmaxNode` s for RowAggregate+OutputLayer.  Operand orientation is
chosen per node so that every GEMM reads both operands K-contiguous with no transposes
(``physical flag`` bookkeeping below).  Everything not matched runs through the generic TCAP
pipeline; fused results feeding generic computations are materialised into temp dense sets.
"""
from __future__ import annotations

import itertools
from typing import Dict, List, Optional, Tuple

import torch

from .. import ops
from ..computations import (AggregateComp, BiasAct, BlockMatmul, BlockSum, Computation, JoinComp, RowSoftmax,
                            ScanSet, WriteSet)
from ..storage.sets import DenseMatrixSet

_tmp_ids = itertools.count()


class Dense:
    """A logical matrix value: physical 2-D tensor + 'transposed' flag (+ block geometry)."""

    def __init__(self, phys: torch.Tensor, rows: int, cols: int, transposed: bool, br: int, bc: int):
        self.phys, self.rows, self.cols, self.transposed = phys, rows, cols, transposed
        self.br, self.bc = br, bc

    def physical(self, want_transposed: bool) -> torch.Tensor:
        """K-contiguous physical layout in the wanted orientation (copy only on mismatch)."""
        if want_transposed == self.transposed:
            p = self.phys
        else:
            # logical L: phys = L if not transposed else L^T; materialise the other orientation
            r, c = (self.cols, self.rows) if self.transposed else (self.rows, self.cols)
            p = self.phys[:r, :c].t().contiguous()
        if p.shape[1] % 8 or p.stride(0) % 8:
            p = ops.pad_k(p.contiguous())
        return p

    def logical(self) -> torch.Tensor:
        if self.transposed:
            return self.phys[: self.cols, : self.rows].t()
        return self.phys[: self.rows, : self.cols]


def _kslice(t: torch.Tensor, rows: int, k8: int) -> torch.Tensor:
    """[rows, k8] view of a zero-padded physical panel (pads with zeros when it is narrower)."""
    t = t[:rows]
    if t.shape[1] < k8:
        t = torch.nn.functional.pad(t, (0, k8 - t.shape[1]))
    return t[:, :k8]


class Node:
    consumers_want_t: Optional[bool] = None
    value: Optional[Dense] = None


class SourceNode(Node):
    def __init__(self, uset: DenseMatrixSet):
        self.set = uset

    def eval(self, engine) -> Dense:
        s = self.set
        if self.value is None:
            phys = s.panel
            rows, cols = (s.local_rows, s.total_cols)
            if s.transposed:
                phys = s.panel
            self.value = Dense(phys, rows, cols, s.transposed, s.block_rows, s.block_cols)
        return self.value


class MatmulNode(Node):
    def __init__(self, a: Node, b: Node, pattern: BlockMatmul):
        self.a, self.b, self.p = a, b, pattern
        self.bias: Optional[Node] = None
        self.bias_along = "row"
        self.act = "none"
        self.dropout = 0.0
        self.seed = 0
        self.transpose_out = False

    def eval(self, engine) -> Dense:
        if self.value is not None:
            return self.value
        A, B = self.a.eval(engine), self.b.eval(engine)
        # effective logical operands: C = opA(A) . opB(B)
        M = A.cols if self.p.transpose_a else A.rows
        K = A.rows if self.p.transpose_a else A.cols
        N = B.rows if self.p.transpose_b else B.cols
        Kb = B.cols if self.p.transpose_b else B.rows
        if K != Kb:
            raise ValueError(f"fused matmul K mismatch {K} vs {Kb}")
        # X = opA(A) as [M,K] K-contig <=> physical(A) with flag == transpose_a
        # Y = opB(B)^T as [N,K] K-contig <=> physical(B) with flag == (not transpose_b)
        K8 = (K + 7) // 8 * 8
        X = _kslice(A.physical(self.p.transpose_a), M, K8)
        Y = _kslice(B.physical(not self.p.transpose_b), N, K8)
        # logical output L = C (or C^T with transpose_out); the consumer asks for a physical
        # orientation relative to L; compute C = X.Y^T or C^T = Y.X^T accordingly (no copies)
        want_t = bool(self.consumers_want_t)
        phys_is_c = self.transpose_out == want_t
        bias_t = None
        mode = ops.BIAS_NONE
        if self.bias is not None:
            bias_t = self.bias.eval(engine).logical().reshape(-1).float().contiguous()
            along_c_rows = self.bias_along == "row"
            mode = (ops.BIAS_ROW if along_c_rows else ops.BIAS_COL) if phys_is_c else \
                (ops.BIAS_COL if along_c_rows else ops.BIAS_ROW)
        act = ops.act_code(self.act)
        # exp'd scores (FFTransposeBiasSum) keep f32 so the later row normalisation is exact
        odt = torch.float32 if act == ops.ACT_EXP else torch.bfloat16
        if phys_is_c:
            phys = ops.gemm_nt(X, Y, bias_t, mode, act, out_dtype=odt, dropout=self.dropout, seed=self.seed)
        else:
            phys = ops.gemm_nt(Y, X, bias_t, mode, act, out_dtype=odt, dropout=self.dropout, seed=self.seed)
        lr, lc = (M, N) if not self.transpose_out else (N, M)
        transposed = want_t
        br = A.bc if self.p.transpose_a else A.br
        bc = B.br if self.p.transpose_b else B.bc
        if self.transpose_out:
            br, bc = bc, br
        self.value = Dense(phys, lr, lc, transposed, br, bc)
        return self.value


class SoftmaxNode(Node):
    def __init__(self, x: Node):
        self.x = x

    def eval(self, engine) -> Dense:
        if self.value is None:
            self.x.consumers_want_t = False
            X = self.x.eval(engine)
            phys = X.physical(False)[:, : X.cols]
            if phys.stride(-1) != 1:
                phys = phys.contiguous()
            # RowAggregate(sum) + OutputLayer(divide) over exp'd scores == row normalisation
            y = ops.row_normalize(phys, out_dtype=torch.float32)
            self.value = Dense(y, X.rows, X.cols, False, X.br, X.bc)
        return self.value


class BiasActNode(Node):
    """Stand-alone epilogue (input not a fresh GEMM)."""

    def __init__(self, x: Node, bias: Node, pat: BiasAct):
        self.x, self.bias, self.p = x, bias, pat

    def eval(self, engine) -> Dense:
        if self.value is None:
            self.x.consumers_want_t = False
            X = self.x.eval(engine)
            b = self.bias.eval(engine).logical().reshape(-1).float().contiguous()
            phys = X.physical(False)[:, : X.cols].contiguous()
            mode = ops.BIAS_ROW if self.p.bias_along == "row" else ops.BIAS_COL
            y = ops.bias_act(phys, b, mode, ops.act_code(self.p.act), self.p.dropout, self.p.seed)
            if self.p.transpose_out:
                self.value = Dense(ops.pad_k(y), X.cols, X.rows, True, X.bc, X.br)
            else:
                self.value = Dense(ops.pad_k(y), X.rows, X.cols, False, X.br, X.bc)
        return self.value


class Fuser:
    def __init__(self, engine):
        self.engine = engine
        self.memo: Dict[int, Optional[Node]] = {}
        self.fused: List[str] = []

    def match(self, c: Computation) -> Optional[Node]:
        if id(c) in self.memo:
            return self.memo[id(c)]
        n = self._match(c)
        self.memo[id(c)] = n
        return n

    def _source(self, c) -> Optional[Node]:
        if isinstance(c, ScanSet):
            st = self.engine.storage
            if st.has_set(c.db, c.set_name):
                s = st.get_set(c.db, c.set_name)
                if isinstance(s, DenseMatrixSet) and s.panel is not None:
                    return SourceNode(s)
        return None

    def _match(self, c: Computation) -> Optional[Node]:
        src = self._source(c)
        if src is not None:
            return src
        pat = c.tensor_pattern()
        if isinstance(c, AggregateComp) and isinstance(pat, BlockSum):
            j = c.inputs[0]
            jp = j.tensor_pattern() if j is not None else None
            if isinstance(j, JoinComp) and isinstance(jp, BlockMatmul):
                a = self.match(j.inputs[jp.a_input])
                b = self.match(j.inputs[jp.b_input])
                if a is not None and b is not None:
                    node = MatmulNode(a, b, jp)
                    # operand orientation requests flow to producers
                    if isinstance(a, (MatmulNode, BiasActNode)):
                        a.consumers_want_t = jp.transpose_a
                    if isinstance(b, (MatmulNode, BiasActNode)):
                        b.consumers_want_t = not jp.transpose_b
                    self.fused.append(f"matmul[{type(j).__name__}+{type(c).__name__}]")
                    return node
            return None
        if isinstance(c, JoinComp) and isinstance(pat, BiasAct):
            x = self.match(c.inputs[pat.data_input])
            b = self.match(c.inputs[pat.bias_input])
            if x is None or not isinstance(b, SourceNode):
                return None
            if isinstance(x, MatmulNode) and x.bias is None and x.act == "none" and not x.transpose_out:
                x.bias, x.bias_along, x.act, x.dropout, x.seed = b, pat.bias_along, pat.act, pat.dropout, pat.seed
                x.transpose_out = pat.transpose_out
                self.fused.append(f"epilogue[{type(c).__name__}]")
                return x
            self.fused.append(f"bias_act[{type(c).__name__}]")
            return BiasActNode(x, b, pat)
        if isinstance(c, JoinComp) and isinstance(pat, RowSoftmax):
            x = self.match(c.inputs[0])
            if x is None:
                return None
            self.fused.append(f"softmax[{type(c).__name__}]")
            return SoftmaxNode(x)
        return None

    # ------------------------------------------------------------------ rewrite
    def run(self, sinks: List[Computation]) -> List[Computation]:
        remaining: List[Computation] = []
        for s in sinks:
            if isinstance(s, WriteSet):
                n = self.match(s.inputs[0])
                if n is not None and not isinstance(n, SourceNode):
                    self._write(n, s.db, s.set_name)
                    continue
            self._replace_inputs(s, set())
            remaining.append(s)
        return remaining

    def _replace_inputs(self, c: Computation, seen):
        if id(c) in seen:
            return
        seen.add(id(c))
        for i, inp in enumerate(c.inputs):
            if inp is None:
                continue
            n = self.match(inp)
            if n is not None and not isinstance(n, SourceNode):
                name = f"__fused_tmp_{next(_tmp_ids)}"
                db = "__tmp"
                self._write(n, db, name, create=True)
                c.inputs[i] = ScanSet(db, name, getattr(inp, "output_type", None))
            else:
                self._replace_inputs(inp, seen)

    def _write(self, n: Node, db: str, name: str, create: bool = False):
        v = n.eval(self.engine)
        st = self.engine.storage
        if create or not st.has_set(db, name):
            st.create_set(db, name, None, dense=True, persistent=False)
        s = st.get_set(db, name)
        if isinstance(s, DenseMatrixSet):
            s.set_panel(v.phys, v.rows if not v.transposed else v.rows, v.cols, max(1, v.br), max(1, v.bc),
                        transposed=v.transposed)
            s.total_rows = v.rows
            s.local_rows = v.rows
        else:
            tmp = DenseMatrixSet(st, db, name, s.type, -1, s.page_size, s.device)
            tmp.set_panel(v.phys, v.rows, v.cols, max(1, v.br), max(1, v.bc), transposed=v.transposed)
            tmp.local_rows = v.rows
            s.add_batch(tmp.to_blocks())


def fuse_tensor_patterns(sinks: List[Computation], engine) -> Tuple[List[Computation], List[str]]:
    f = Fuser(engine)
    rest = f.run(sinks)
    return rest, f.fused


__all__ = ["fuse_tensor_patterns", "Fuser", "MatmulNode", "SoftmaxNode", "BiasActNode", "SourceNode", "Dense"]
