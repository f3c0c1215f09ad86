"""Feed-forward neural-network inference as netsDB UDFs (reference: src/FF — SimpleFF.cc
inference / inference_unit / inference_compute, FFTransposeMult, FFAggMatrix, FFReluBiasSum,
FFInputLayerJoin, FFTransposeBiasSum, FFTransposeBiasSumSigmoid, FFRowAggregate, FFOutputLayer,
FFMatrixBlockScanner, FFMatrixWriter; driver src/tests/source/FFTest.cc).

Each class is a real JoinComp/AggregateComp whose lambdas work on whole MatrixBlock batches (the
generic engine path: batched MFMA block GEMMs over the join pairs, segment-sum aggregation), and
declares its tensor pattern so the planner can fuse the chain into split-K GEMMs with
bias/ReLU/dropout/exp epilogues over the dense HBM panels (query_planning/fusion.py).

Math (reference semantics, row-major blocks):
    Y1 = relu(W1 . X^T + b1)            [hidden x batch]   (FFTransposeMult + FFAggMatrix + FFReluBiasSum)
    Y2 = relu(W2 . Y1 + b2)             [hidden2 x batch]  (FFInputLayerJoin + FFAggMatrix + FFReluBiasSum)
    YO = exp(Wo . Y + bo)^T             [batch x labels]   (FFInputLayerJoin + FFAggMatrix + FFTransposeBiasSum)
    OUT = YO / rowsum(YO)  = softmax    [batch x labels]   (FFRowAggregate + FFOutputLayer)
"""
from __future__ import annotations

import time
from typing import Optional

import torch

from .. import ops
from ..computations import (AggregateComp, BiasAct, BlockMatmul, BlockSum, JoinComp, MultiSelectionComp,
                            PartitionComp, RowSoftmax, ScanSet, WriteSet)
from ..lambdas import make_batch_lambda, make_lambda_from_method, make_lambda_from_self
from ..objects.builtin import FFMatrixBlock, getter
from ..objects.nested import NestedColumn
from ..objects.record import PDBObject, RecordBatch, Tensor
from . import blocks as B


def mk_blocks(block_row, block_col, data, total_rows, total_cols, type_=FFMatrixBlock) -> RecordBatch:
    n = data.shape[0]
    dev = data.device

    def col(v):
        if isinstance(v, torch.Tensor):
            return v.to(dev).long()
        return torch.full((n,), int(v), dtype=torch.int64, device=dev)

    cols = {"block_row": col(block_row), "block_col": col(block_col),
            "row_nums": col(data.shape[1]), "col_nums": col(data.shape[2]),
            "total_rows": col(total_rows), "total_cols": col(total_cols), "data": data}
    for f in type_.__fields__:
        if f not in cols:
            cols[f] = torch.zeros(n, dtype=torch.int64, device=dev) if f != "partition_by_col" else \
                torch.zeros(n, dtype=torch.bool, device=dev)
    return RecordBatch(cols, n, type_)


def _bmm_nt(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """Batched a[p] @ b[p]^T on the MFMA kernel (f32 out): one launch for all join pairs."""
    if a.shape[0] == 0:
        return torch.empty(0, a.shape[1], b.shape[1], device=a.device)
    K = a.shape[-1]
    if K % 8:
        a, b = ops.pad_k(a), ops.pad_k(b)
    if a.is_cuda:
        return ops.gemm_nt(a.to(torch.bfloat16).contiguous(), b.to(torch.bfloat16).contiguous(),
                           out_dtype=torch.float32)
    return torch.matmul(a.float(), b.float().transpose(-1, -2))


# ------------------------------------------------------------------------------------ joins
class FFTransposeMult(JoinComp):
    """A . B^T block product: join on A.blockCol == B.blockCol (shared K index)."""

    def get_selection(self, in1, in2):
        return make_lambda_from_method(in1, "getBlockColIndex") == make_lambda_from_method(in2, "getBlockColIndex")

    def get_projection(self, in1, in2):
        def proj(a: RecordBatch, b: RecordBatch):
            d = _bmm_nt(a.columns["data"], b.columns["data"])
            return mk_blocks(a.columns["block_row"], b.columns["block_row"], d, a.columns["total_rows"],
                             b.columns["total_rows"])

        return make_batch_lambda(in1, in2, proj, tag="block_matmul_nt")

    def tensor_pattern(self):
        return BlockMatmul(transpose_a=False, transpose_b=True)


class FFInputLayerJoin(JoinComp):
    """A . B block product: join on A.blockCol == B.blockRow."""

    def get_selection(self, in1, in2):
        return make_lambda_from_method(in1, "getBlockColIndex") == make_lambda_from_method(in2, "getBlockRowIndex")

    def get_projection(self, in1, in2):
        def proj(a: RecordBatch, b: RecordBatch):
            d = _bmm_nt(a.columns["data"], b.columns["data"].transpose(-1, -2).contiguous())
            return mk_blocks(a.columns["block_row"], b.columns["block_col"], d, a.columns["total_rows"],
                             b.columns["total_cols"])

        return make_batch_lambda(in1, in2, proj, tag="block_matmul_nn")

    def tensor_pattern(self):
        return BlockMatmul(transpose_a=False, transpose_b=False)


class FFAggMatrix(AggregateComp):
    """Sum partial block products by output block (ClusterAggregateComp)."""

    def get_key_projection(self, blk):
        return make_lambda_from_method(blk, "getFullKey")

    def get_value_projection(self, blk):
        return make_lambda_from_method(blk, "getValue")

    def make_output(self, keys, values):
        r, c, tr, tc = keys
        return mk_blocks(r, c, values, tr, tc)

    def tensor_pattern(self):
        return BlockSum()


def _get_full_key(b: RecordBatch):
    return (b.columns["block_row"], b.columns["block_col"], b.columns["total_rows"], b.columns["total_cols"])


FFMatrixBlock.getFullKey = lambda self: (self.block_row, self.block_col, self.total_rows, self.total_cols)
FFMatrixBlock.getFullKey.__vectorized__ = _get_full_key


class _BiasJoin(JoinComp):
    act = "none"
    transpose_out = False

    def __init__(self, dropout_rate: float = 0.0, seed: int = 0):
        super().__init__()
        self.dropout_rate = dropout_rate
        self.seed = seed

    def get_selection(self, in1, in2):
        return make_lambda_from_method(in1, "getBlockRowIndex") == make_lambda_from_method(in2, "getBlockRowIndex")

    def get_projection(self, in1, in2):
        def proj(x: RecordBatch, bias: RecordBatch):
            d = x.columns["data"].float()
            bv = bias.columns["data"].float()[:, : d.shape[1], :1]
            v = ops._apply_act(d + bv, ops.act_code(self.act))
            if self.dropout_rate > 0:
                v = ops._dropout_ref(v.cpu(), self.dropout_rate, self.seed).to(v.device)
            if self.transpose_out:
                return mk_blocks(x.columns["block_col"], x.columns["block_row"], v.transpose(1, 2).contiguous(),
                                 x.columns["total_cols"], x.columns["total_rows"])
            return mk_blocks(x.columns["block_row"], x.columns["block_col"], v, x.columns["total_rows"],
                             x.columns["total_cols"])

        return make_batch_lambda(in1, in2, proj, tag=f"bias_{self.act}")

    def tensor_pattern(self):
        return BiasAct(act=self.act, dropout=self.dropout_rate, bias_along="row", transpose_out=self.transpose_out,
                       seed=self.seed)


class FFReluBiasSum(_BiasJoin):
    """relu(X + bias) (+ inference-time dropout, as in the reference)."""

    act = "relu"


class FFTransposeBiasSum(_BiasJoin):
    """exp(X + bias), transposed: [labels x batch] -> [batch x labels]."""

    act = "exp"
    transpose_out = True


class FFTransposeBiasSumSigmoid(_BiasJoin):
    """sigmoid(X + bias), transposed (logistic-regression output)."""

    act = "sigmoid"
    transpose_out = True


# ------------------------------------------------------------------------------------ softmax
class FFRowAggregate(AggregateComp):
    """Row sums of exp'd scores keyed by block row."""

    def get_key_projection(self, blk):
        return make_lambda_from_method(blk, "getRowKey2")

    def get_value_projection(self, blk):
        return make_lambda_from_method(blk, "getRowSumValue")

    def make_output(self, keys, values):
        r, tr = keys
        return mk_blocks(r, torch.zeros_like(r), values.unsqueeze(-1), tr, 1)


FFMatrixBlock.getRowKey2 = lambda self: (self.block_row, self.total_rows)
FFMatrixBlock.getRowKey2.__vectorized__ = lambda b: (b.columns["block_row"], b.columns["total_rows"])
FFMatrixBlock.getRowSumValue = lambda self: self.data.float().sum(-1)
FFMatrixBlock.getRowSumValue.__vectorized__ = lambda b: b.columns["data"].float().sum(-1)


class FFOutputLayer(JoinComp):
    """X / rowsum(X) (join on block row)."""

    def get_selection(self, in1, in2):
        return make_lambda_from_method(in1, "getBlockRowIndex") == make_lambda_from_method(in2, "getBlockRowIndex")

    def get_projection(self, in1, in2):
        def proj(x: RecordBatch, s: RecordBatch):
            d = x.columns["data"].float() / s.columns["data"].float()[:, : x.columns["data"].shape[1], :1]
            return mk_blocks(x.columns["block_row"], x.columns["block_col"], d, x.columns["total_rows"],
                             x.columns["total_cols"])

        return make_batch_lambda(in1, in2, proj, tag="row_normalize")

    def tensor_pattern(self):
        return RowSoftmax()


# ------------------------------------------------------------------------------------ helper UDFs
class InferenceResult(PDBObject):
    """One inference row: its global row index, its block row and the first two output scores
    (src/FF/headers/InferenceResult.h; label = 1 if score0 > score1 else -1)."""

    index: int
    block_row_id: int
    inference: Tensor()

    getKey = getter("index")
    getInference = getter("inference")

    def getLabel(self):
        return 1 if float(self.inference[0]) > float(self.inference[1]) else -1

    getLabel.__vectorized__ = lambda b: torch.where(b.columns["inference"][:, 0] > b.columns["inference"][:, 1], 1, -1)


class FFSingleMatrix(FFMatrixBlock):
    """Every block of a matrix assembled into one (src/FF/headers/FFSingleMatrix.h: key 1 + the block)."""

    key: int

    def getKey(self):
        return self.key

    getKey.__vectorized__ = lambda b: b.columns["key"]


class FFMatrixPartitioner(PartitionComp):
    """Store FFMatrixBlocks hash-partitioned across nodes by block row index (src/FF/headers/
    FFMatrixPartitioner.h; the ``enablePartition`` output writer of SimpleFF.cc inference)."""

    def __init__(self, db: str = "", set_name: str = ""):
        super().__init__(db, set_name)

    def get_key_projection(self, blk):
        return make_lambda_from_method(blk, "getBlockRowIndex")


class InferenceResultPartition(PartitionComp):
    """Store InferenceResults partitioned by their row index (src/FF/headers/InferenceResultPartition.h)."""

    def __init__(self, db: str = "", set_name: str = ""):
        super().__init__(db, set_name)

    def get_key_projection(self, r):
        return make_lambda_from_method(r, "getKey")


class FFMatrixMultiSel(MultiSelectionComp):
    """FFMatrixBlock -> one InferenceResult per row (index = blockRow * rowNums + i, the row's first two values;
    src/FF/headers/FFMatrixMultiSel.h). Vectorised: one [rows, 2] slice of the stacked block data per batch."""

    def get_selection(self, blk):
        return make_batch_lambda(blk, lambda b: torch.ones(b.n, dtype=torch.bool, device=b.columns["data"].device))

    def get_projection(self, blk):
        def proj(b: RecordBatch):
            d = b.columns["data"]
            n, rows = b.n, d.shape[1]
            dev = d.device
            br = b.columns["block_row"].to(dev).long()
            rn = b.columns["row_nums"].to(dev).long()
            i = torch.arange(rows, device=dev)
            res = RecordBatch({"index": (br * rn).unsqueeze(1).add(i).reshape(-1),
                               "block_row_id": br.repeat_interleave(rows),
                               "inference": d[:, :, :2].reshape(n * rows, -1).double()}, n * rows, InferenceResult)
            return NestedColumn(torch.arange(n + 1, device=dev) * rows, res)

        return make_batch_lambda(blk, proj, tag="ff_matrix_multisel")


class FFAggMatrixToOneMatrix(AggregateComp):
    """Merge every FFMatrixBlock into one FFSingleMatrix (key 1): each block lands at its (blockRow, blockCol)
    position of the total_rows x total_cols matrix (src/FF/headers/FFAggMatrixToOneMatrix.h + the block-placing
    FFMatrixBlock::operator+). Vectorised: the blocks of a group are scattered into the matrix in one indexed copy
    (engine group_values hook), not merged pairwise."""

    reduce_op = None

    def get_key_projection(self, blk):
        return make_batch_lambda(blk, lambda b: torch.ones(b.n, dtype=torch.int64, device=b.columns["data"].device))

    def get_value_projection(self, blk):
        return make_lambda_from_self(blk)

    def group_values(self, values, inv, ngroups):
        b = values if isinstance(values, RecordBatch) else RecordBatch.concat(values)
        d = b.columns["data"]
        dev = d.device
        inv = inv.to(dev)
        br, bc = d.shape[1], d.shape[2]
        out = []
        for g in range(ngroups):
            sel = torch.nonzero(inv == g).flatten()
            r = b.columns["block_row"].to(dev).index_select(0, sel)
            c = b.columns["block_col"].to(dev).index_select(0, sel)
            tr = int(b.columns["total_rows"][sel[0]])
            tc = int(b.columns["total_cols"][sel[0]])
            nbr, nbc = -(-tr // br), -(-tc // bc)
            full = torch.zeros(nbr, nbc, br, bc, dtype=d.dtype, device=dev)
            full[r, c] = d.index_select(0, sel)
            out.append(full.permute(0, 2, 1, 3).reshape(nbr * br, nbc * bc)[:tr, :tc])
        return out

    def make_output(self, keys, values):
        mats = values
        n = len(mats)
        dev = mats[0].device if n else None
        R = max(m.shape[0] for m in mats) if n else 0
        C = max(m.shape[1] for m in mats) if n else 0
        data = torch.zeros(n, R, C, dtype=mats[0].dtype if n else torch.float32, device=dev)
        for i, m in enumerate(mats):
            data[i, : m.shape[0], : m.shape[1]] = m
        rows = torch.tensor([m.shape[0] for m in mats], dtype=torch.int64, device=dev)
        cols = torch.tensor([m.shape[1] for m in mats], dtype=torch.int64, device=dev)
        blk = mk_blocks(0, 0, data, rows, cols, type_=FFSingleMatrix)
        blk.columns["row_nums"], blk.columns["col_nums"] = rows, cols
        blk.columns["key"] = keys.to(dev) if isinstance(keys, torch.Tensor) else torch.ones(n, dtype=torch.int64,
                                                                                              device=dev)
        return blk


def FFMatrixBlockScanner(db: str, set_name: str):
    return ScanSet(db, set_name, FFMatrixBlock)


def FFMatrixWriter(db: str, set_name: str):
    return WriteSet(db, set_name, FFMatrixBlock)


# ------------------------------------------------------------------------------------ drivers
def setup(client, db: str):
    client.create_database(db)
    client.register_type(FFMatrixBlock)


def create_output_set(client, db: str, name: str):
    if client.storage.has_set(db, name):
        client.remove_set(db, name)
    client.create_set(db, name, FFMatrixBlock, dense=True)


def inference_unit(client, db: str, w1: str, wo: str, inputs: str, b1: str, bo: str, output: str,
                   dropout_rate: float = 0.0, seed: int = 0, single_job: bool = False) -> dict:
    """SimpleFF.cc inference_unit: one hidden layer + softmax output (two jobs, the exp'd scores materialised
    in the intermediate set "yo" between them, as the reference does).

    ``single_job=True`` submits the whole graph as ONE job with no "yo" set (FFOutputLayer and FFRowAggregate
    read the FFTransposeBiasSum result directly): the fuser then lowers the output layer to one GEMM whose
    epilogue computes the max-subtracted softmax (ops.gemm_nt_softmax), with no exp'd round trip through HBM."""
    if not single_job:
        create_output_set(client, db, "yo")
    create_output_set(client, db, output)
    t0 = time.perf_counter()
    readA, readB = FFMatrixBlockScanner(db, w1), FFMatrixBlockScanner(db, inputs)
    join = FFTransposeMult()
    join.set_input(0, readA)
    join.set_input(1, readB)
    agg = FFAggMatrix().set_input(join)
    relu = FFReluBiasSum(dropout_rate, seed)
    relu.set_input(0, agg)
    relu.set_input(1, FFMatrixBlockScanner(db, b1))
    join1 = FFInputLayerJoin()
    join1.set_input(0, FFMatrixBlockScanner(db, wo))
    join1.set_input(1, relu)
    agg1 = FFAggMatrix().set_input(join1)
    bsum = FFTransposeBiasSum()
    bsum.set_input(0, agg1)
    bsum.set_input(1, FFMatrixBlockScanner(db, bo))
    if single_job:
        soft = FFOutputLayer()
        soft.set_input(0, bsum)
        soft.set_input(1, FFRowAggregate().set_input(bsum))
        s = client.execute_computations(FFMatrixWriter(db, output).set_input(soft), job_name="inference-unit-fused")
        return {"seconds": time.perf_counter() - t0, "jobs": [s]}
    s1 = client.execute_computations(FFMatrixWriter(db, "yo").set_input(bsum), job_name="inference-unit-intermediate")
    readF = FFMatrixBlockScanner(db, "yo")
    expsum = FFRowAggregate().set_input(readF)
    soft = FFOutputLayer()
    soft.set_input(0, readF)
    soft.set_input(1, expsum)
    s2 = client.execute_computations(FFMatrixWriter(db, output).set_input(soft), job_name="inference-unit")
    return {"seconds": time.perf_counter() - t0, "jobs": [s1, s2]}


def inference(client, db: str, w1: str, w2: str, wo: str, inputs: str, b1: str, b2: str, bo: str, output: str,
              dropout_rate: float = 0.0, seed: int = 0, enable_partition: bool = False) -> dict:
    """SimpleFF.cc inference / inference_compute: two hidden layers (y1, y2, yo) + softmax.

    ``enable_partition`` (SimpleFF.cc:129-132,194-197): the hidden layers' outputs y1 / y2 are written by
    :class:`FFMatrixPartitioner` — FFMatrixBlock records hash-partitioned across the nodes by block row — instead
    of the dense FFMatrixWriter panels; the next layer reads them as block records (generic join path)."""
    for n in ("yo", output) if enable_partition else ("y1", "y2", "yo", output):
        create_output_set(client, db, n)
    if enable_partition:
        for n in ("y1", "y2"):
            if client.storage.has_set(db, n):
                client.remove_set(db, n)
            client.create_set(db, n, FFMatrixBlock)
    t0 = time.perf_counter()
    stats = []

    def layer(w, x, b, out, first, last):
        j = FFTransposeMult() if first else FFInputLayerJoin()
        j.set_input(0, FFMatrixBlockScanner(db, w))
        j.set_input(1, FFMatrixBlockScanner(db, x))
        a = FFAggMatrix().set_input(j)
        bj = FFTransposeBiasSum() if last else FFReluBiasSum(dropout_rate, seed)
        bj.set_input(0, a)
        bj.set_input(1, FFMatrixBlockScanner(db, b))
        writer = FFMatrixPartitioner(db, out) if (enable_partition and not last) else FFMatrixWriter(db, out)
        stats.append(client.execute_computations(writer.set_input(bj), job_name=f"inference-{out}"))

    layer(w1, inputs, b1, "y1", True, False)
    layer(w2, "y1", b2, "y2", False, False)
    layer(wo, "y2", bo, "yo", False, True)
    readF = FFMatrixBlockScanner(db, "yo")
    soft = FFOutputLayer()
    soft.set_input(0, readF)
    soft.set_input(1, FFRowAggregate().set_input(readF))
    stats.append(client.execute_computations(FFMatrixWriter(db, output).set_input(soft), job_name="inference-out"))
    return {"seconds": time.perf_counter() - t0, "jobs": stats}


def load_model(client, db: str, batch: int, features: int, hidden: int, labels: int, block_x: int, block_y: int,
               seed: int = 0, partition_inputs: bool = True, hidden2: Optional[int] = None, dtype=torch.bfloat16):
    """FFTest.cc data loading: inputs [batch x features], w1 [hidden x features], b1 [hidden x 1],
    (w2 [hidden2 x hidden], b2), wo [labels x hidden(2)], bo [labels x 1] — random init."""
    setup(client, db)
    sc1 = (3.0 / features) ** 0.5
    B.load_matrix(client, db, "inputs", batch, features, block_x, block_y, seed=seed + 1,
                  partition_rows=partition_inputs, dtype=dtype)
    B.load_matrix(client, db, "w1", hidden, features, block_x, block_y, seed=seed + 2, scale=sc1, dtype=dtype)
    B.load_matrix(client, db, "b1", hidden, 1, block_x, 1, seed=seed + 3, scale=0.1, dtype=dtype)
    last_in = hidden
    if hidden2:
        B.load_matrix(client, db, "w2", hidden2, hidden, block_x, block_x, seed=seed + 4, scale=(3.0 / hidden) ** 0.5,
                      dtype=dtype)
        B.load_matrix(client, db, "b2", hidden2, 1, block_x, 1, seed=seed + 5, scale=0.1, dtype=dtype)
        last_in = hidden2
    B.load_matrix(client, db, "wo", labels, last_in, block_x, block_x, seed=seed + 6, scale=(3.0 / last_in) ** 0.5,
                  dtype=dtype)
    B.load_matrix(client, db, "bo", labels, 1, block_x, 1, seed=seed + 7, scale=0.1, dtype=dtype)
    # the weights are re-read by every inference step: "model" locality in the cost-based page cache
    for name in ("w1", "b1", "wo", "bo") + (("w2", "b2") if hidden2 else ()):
        if client.storage.has_set(db, name):
            client.set_locality(db, name, "model")


def reference_inference(x, w1, b1, wo, bo, w2=None, b2=None):
    """Plain fp32 PyTorch reference of the same network (numerics oracle)."""
    y = torch.relu(w1.float() @ x.float().t() + b1.float().reshape(-1, 1))
    if w2 is not None:
        y = torch.relu(w2.float() @ y + b2.float().reshape(-1, 1))
    z = (wo.float() @ y + bo.float().reshape(-1, 1)).t()
    return torch.softmax(z, dim=-1)


__all__ = ["FFTransposeMult", "FFInputLayerJoin", "FFAggMatrix", "FFReluBiasSum", "FFTransposeBiasSum",
           "FFTransposeBiasSumSigmoid", "FFRowAggregate", "FFOutputLayer", "FFMatrixBlockScanner", "FFMatrixWriter",
           "InferenceResult", "FFSingleMatrix", "FFMatrixPartitioner", "InferenceResultPartition", "FFMatrixMultiSel",
           "FFAggMatrixToOneMatrix",
           "inference_unit", "inference", "load_model", "reference_inference", "mk_blocks", "setup"]
