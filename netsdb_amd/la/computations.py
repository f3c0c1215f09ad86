"""Linear-algebra UDFs over MatrixBlock sets (reference: src/sharedLibraries/headers/LASilly*.h,
LAScanMatrixBlockSet.h, LAWriteMatrixBlockSet.h — the computations the linearAlgebraDSL
evaluator instantiates for every operator).

Each class works on the generic engine (blockwise lambdas on MatrixBlock batches) and declares
its tensor pattern so the planner lowers it onto the dense-panel kernels (MFMA GEMM for
multiplies, layout-flag transpose, device reductions).
"""
from __future__ import annotations

import torch

from ..computations import (AggregateComp, BlockMatmul, Duplicate, Elementwise, Inverse, JoinComp, MultiSelectionComp, Reduce, Scale, SelectionComp, Transpose)
from ..lambdas import make_batch_lambda, make_lambda_from_method
from ..models.ff import FFAggMatrix, _bmm_nt, mk_blocks
from ..objects.builtin import MatrixBlock
from ..objects.record import RecordBatch


def _mb(r, c, d, tr, tc):
    return mk_blocks(r, c, d, tr, tc, MatrixBlock)


class LAMultiply1Join(JoinComp):
    """A %*% B partial products: join A.blockCol == B.blockRow."""

    def get_selection(self, a, b):
        return make_lambda_from_method(a, "getBlockColIndex") == make_lambda_from_method(b, "getBlockRowIndex")

    def get_projection(self, a, b):
        def proj(x: RecordBatch, y: RecordBatch):
            d = _bmm_nt(x.columns["data"], y.columns["data"].transpose(-1, -2).contiguous())
            return _mb(x.columns["block_row"], y.columns["block_col"], d, x.columns["total_rows"],
                       y.columns["total_cols"])

        return make_batch_lambda(a, b, proj, tag="block_matmul_nn")

    def tensor_pattern(self):
        return BlockMatmul(transpose_a=False, transpose_b=False)


class LATransposeMultiply1Join(JoinComp):
    """A '* B = A^T B partial products: join A.blockRow == B.blockRow."""

    def get_selection(self, a, b):
        return make_lambda_from_method(a, "getBlockRowIndex") == make_lambda_from_method(b, "getBlockRowIndex")

    def get_projection(self, a, b):
        def proj(x: RecordBatch, y: RecordBatch):
            d = _bmm_nt(x.columns["data"].transpose(-1, -2).contiguous(), y.columns["data"].transpose(-1, -2).contiguous())
            return _mb(x.columns["block_col"], y.columns["block_col"], d, x.columns["total_cols"],
                       y.columns["total_cols"])

        return make_batch_lambda(a, b, proj, tag="block_matmul_tn")

    def tensor_pattern(self):
        return BlockMatmul(transpose_a=True, transpose_b=False)


class LAMultiply2Aggregate(FFAggMatrix):
    """Sum partial products by output block."""

    def make_output(self, keys, values):
        r, c, tr, tc = keys
        return _mb(r, c, values, tr, tc)


MatrixBlock.getFullKey = lambda self: (self.block_row, self.block_col, self.total_rows, self.total_cols)
MatrixBlock.getFullKey.__vectorized__ = lambda b: (b.columns["block_row"], b.columns["block_col"],
                                                   b.columns["total_rows"], b.columns["total_cols"])


class _EwiseJoin(JoinComp):
    op = "add"
    _F = {"add": torch.add, "sub": torch.sub, "mul": torch.mul}

    def get_selection(self, a, b):
        return (make_lambda_from_method(a, "getBlockRowIndex") == make_lambda_from_method(b, "getBlockRowIndex")) & \
               (make_lambda_from_method(a, "getBlockColIndex") == make_lambda_from_method(b, "getBlockColIndex"))

    def get_projection(self, a, b):
        def proj(x: RecordBatch, y: RecordBatch):
            d = self._F[self.op](x.columns["data"].float(), y.columns["data"].float())
            return _mb(x.columns["block_row"], x.columns["block_col"], d, x.columns["total_rows"],
                       x.columns["total_cols"])

        return make_batch_lambda(a, b, proj, tag=f"ewise_{self.op}")

    def tensor_pattern(self):
        return Elementwise(self.op)


class LAAddJoin(_EwiseJoin):
    op = "add"


class LASubstractJoin(_EwiseJoin):
    op = "sub"


class LAScaleMultiplyJoin(_EwiseJoin):
    op = "mul"


class LATransposeSelection(SelectionComp):
    def get_projection(self, a):
        def proj(x: RecordBatch):
            return _mb(x.columns["block_col"], x.columns["block_row"], x.columns["data"].transpose(1, 2).contiguous(),
                       x.columns["total_cols"], x.columns["total_rows"])

        return make_batch_lambda(a, proj, tag="transpose")

    def tensor_pattern(self):
        return Transpose()


class LAScaleSelection(SelectionComp):
    """c * A block by block: a selection, so every rank scales only the blocks (rows) it holds — on dense
    panels the fused lowering keeps A's row partition (no gather), on block records the engine maps each page."""

    def __init__(self, scalar: float):
        super().__init__()
        self.scalar = float(scalar)

    def get_projection(self, a):
        s = self.scalar

        def proj(x: RecordBatch):
            d = x.columns["data"]
            return _mb(x.columns["block_row"], x.columns["block_col"], (d.float() * s).to(d.dtype),
                       x.columns["total_rows"], x.columns["total_cols"])

        return make_batch_lambda(a, proj, tag="scale")

    def tensor_pattern(self):
        return Scale(self.scalar)


class _ReduceAgg(AggregateComp):
    axis = "row"
    op = "sum"

    @property
    def reduce_op(self):
        return self.op

    def get_key_projection(self, a):
        def key(x: RecordBatch):
            z = torch.zeros_like(x.columns["block_row"])
            if self.axis == "row":
                return (x.columns["block_row"], z, x.columns["total_rows"])
            if self.axis == "col":
                return (z, x.columns["block_col"], x.columns["total_cols"])
            return (z, z, z)

        return make_batch_lambda(a, key)

    def get_value_projection(self, a):
        red = {"sum": torch.sum, "max": torch.amax, "min": torch.amin}[self.op]

        def val(x: RecordBatch):
            d = x.columns["data"].float()
            # mask padding of partial edge blocks: rows/cols beyond the totals
            if self.axis == "row":
                return red(d, dim=2)
            if self.axis == "col":
                return red(d, dim=1)
            return red(d.reshape(d.shape[0], -1), dim=1)

        return make_batch_lambda(a, val)

    def make_output(self, keys, values):
        r, c, t = keys
        if self.axis == "row":
            return _mb(r, c, values.unsqueeze(-1), t, 1)
        if self.axis == "col":
            return _mb(r, c, values.unsqueeze(1), 1, t)
        return _mb(r, c, values.reshape(-1, 1, 1), 1, 1)

    def tensor_pattern(self):
        return Reduce(self.axis, self.op)


def _reducer(axis, op):
    return type(f"LA{axis.title()}{op.title()}Aggregate", (_ReduceAgg,), {"axis": axis, "op": op})


LARowMaxAggregate, LARowMinAggregate, LARowSumAggregate = _reducer("row", "max"), _reducer("row", "min"), _reducer("row", "sum")
LAColMaxAggregate, LAColMinAggregate, LAColSumAggregate = _reducer("col", "max"), _reducer("col", "min"), _reducer("col", "sum")
LAMaxElementAggregate, LAMinElementAggregate = _reducer("all", "max"), _reducer("all", "min")


class LAInverseAggregate(AggregateComp):
    """Gather all blocks into one matrix and invert it (reference: Inverse1Aggregate ->
    Inverse2Selection -> Inverse3MultiSelection)."""

    reduce_op = None

    def get_key_projection(self, a):
        return make_batch_lambda(a, lambda x: torch.zeros_like(x.columns["block_row"]))

    def get_value_projection(self, a):
        from ..lambdas import make_lambda_from_self

        return make_lambda_from_self(a)

    def tensor_pattern(self):
        return Inverse()


class _DupSel(MultiSelectionComp):
    axis = "row"

    def __init__(self, block_size: int, num_blocks: int):
        super().__init__()
        self.block_size, self.num_blocks = block_size, num_blocks

    def get_projection(self, a):
        def proj(x):
            return [x] * self.num_blocks

        from ..lambdas import make_lambda

        return make_lambda(a, proj)

    def tensor_pattern(self):
        return Duplicate(self.axis, self.block_size, self.num_blocks)


class LADuplicateRowMultiSelection(_DupSel):
    axis = "row"


class LADuplicateColMultiSelection(_DupSel):
    axis = "col"


__all__ = [n for n in dir() if n.startswith("LA")]
