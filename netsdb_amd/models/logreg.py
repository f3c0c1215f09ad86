"""Logistic regression and the FF_proj fully-connected network (reference: src/LogReg/Logistic_Regression.h,
src/FF/source/SimpleFF.cc inference_unit_log_reg / inference_unit_log_reg1 (FFTransposeBiasSumSigmoid),
src/FF_proj/FullyConnectedNetwork.h, drivers src/tests/source/LogisticRegression*.cc, FCProjTest.cc).

``inference_unit_log_reg`` is the reference plan: inputs ⋈ w (FFInputLayerJoin) -> +b, sigmoid
(FFTransposeBiasSumSigmoid) -> output; it is fused onto one GEMM with a sigmoid epilogue.
``FullyConnectedNetwork`` is FF_proj's "projection" formulation: the whole layer stack as one
SelectionComp UDF per input page (each layer = one GEMM with bias/act epilogue).
"""
from __future__ import annotations

import time
from typing import List, Optional

import torch

from .. import ops
from ..computations import SelectionComp
from ..lambdas import make_batch_lambda
from ..objects.record import RecordBatch
from .ff import (FFAggMatrix, FFMatrixBlockScanner, FFMatrixWriter, FFTransposeBiasSumSigmoid,
                 create_output_set)
from . import blocks as B


def load_logreg(client, db: str, batch: int, features: int, block_x: int, block_y: int, seed: int = 0,
                dtype=torch.bfloat16, partition_inputs: bool = True):
    client.create_database(db)
    B.load_matrix(client, db, "inputs", batch, features, block_x, block_y, seed=seed + 1, dtype=dtype,
                  partition_rows=partition_inputs)
    B.load_matrix(client, db, "w", features, 1, block_y, 1, seed=seed + 2, scale=(3.0 / features) ** 0.5, dtype=dtype)
    B.load_matrix(client, db, "b", 1, 1, 1, 1, seed=seed + 3, scale=0.1, dtype=dtype)


class _Bias1(FFTransposeBiasSumSigmoid):
    """bias join for the [1 x batch] logits (bias indexed by the single output row)."""


def inference_unit_log_reg(client, db: str, w: str = "w", inputs: str = "inputs", b: str = "b",
                           output: str = "output") -> dict:
    """sigmoid(X · w + b): FFInputLayerJoin(inputs, w) + FFAggMatrix + FFTransposeBiasSumSigmoid."""
    create_output_set(client, db, output)
    t0 = time.perf_counter()
    # logits^T = w^T X^T  ->  use (w^T) as the row operand so the bias joins on the single row
    from ..la.computations import LATransposeMultiply1Join

    j = LATransposeMultiply1Join()        # w '* X^T  == (w^T)(X^T)
    j.set_input(0, FFMatrixBlockScanner(db, w))
    from ..la.computations import LATransposeSelection

    xt = LATransposeSelection().set_input(FFMatrixBlockScanner(db, inputs))
    j.set_input(1, xt)
    agg = FFAggMatrix().set_input(j)
    sig = _Bias1()
    sig.set_input(0, agg)
    sig.set_input(1, FFMatrixBlockScanner(db, b))
    st = client.execute_computations(FFMatrixWriter(db, output).set_input(sig), job_name="logreg")
    return {"seconds": time.perf_counter() - t0, "job": st}


class FullyConnectedNetwork(SelectionComp):
    """FF_proj: the whole MLP as one projection UDF over pages of input rows (dense features in a
    tensor column 'data')."""

    def __init__(self, weights: List[torch.Tensor], biases: List[torch.Tensor], acts: Optional[List[str]] = None,
                 softmax: bool = True):
        super().__init__()
        self.W = [ops.pad_k(w.to(torch.bfloat16)).contiguous() for w in weights]
        self.b = [b.float() for b in biases]
        self.acts = acts or (["relu"] * (len(weights) - 1) + ["none"])
        self.softmax = softmax

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        h = x
        for w, b, a in zip(self.W, self.b, self.acts):
            h = ops.gemm_nt(ops.pad_k(h.to(torch.bfloat16)).contiguous(), w.to(h.device), b.to(h.device),
                            ops.BIAS_COL, a)
        return ops.softmax_rows(h) if self.softmax else h.float()

    def get_projection(self, row):
        def proj(batch: RecordBatch):
            y = self.forward(batch.columns["data"])
            return RecordBatch({"data": y}, batch.n)

        return make_batch_lambda(row, proj, tag="fc_network")


__all__ = ["load_logreg", "inference_unit_log_reg", "FullyConnectedNetwork"]
