"""Text classification with (heterogeneous-model) deduplication — the drivers of
src/tests/source/heterogeneousModelDeduplication/{TestNNLM50IMDB, TestNNLM128Yelp, TestWiki250Civil,
TestWiki500Yelp, TextClassifierWithoutDeduplication}.cc and HybridTestWithDeduplication.cc.

One workload (per model): embedding weights W [embed x vocab] and a batch of bag-of-words inputs X
[batch x vocab] (blocks 50 x 10000):

    job 1  FFTransposeMult(W, X) + FFAggMatrix          -> "intermediate" = W . X^T   [embed x batch]
    job 2  FFAggMatrixToOneMatrix(intermediate)         -> one FFSingleMatrix (every block placed)
           SemanticClassifierSingleBlock                -> labels [1 x batch] -> "outputs"

Job 1 lowers to one split-K MFMA GEMM over the dense panels (query_planning/fusion.py); job 2 runs on the
generic engine (the aggregate assembles the blocks in one indexed copy, the classifier's two GEMMs run on the
exact-f32 MFMA kernel).

Heterogeneous dedup: several models' embedding matrices share blocks (here: a smaller model's rows are a
prefix of a larger model's, as models fine-tuned from one embedding table are); every distinct block is
stored once in a BlockPool (models/dedup.py) and each model's weight set is linked to it, so the node holds
the union of the models' distinct blocks instead of their sum. Synthetic data and random weights of the
reference geometry (no network: the reference's model files are not available).
"""
from __future__ import annotations

import time
from typing import Dict, Optional, Sequence

import torch

from ..computations import ScanSet, WriteSet
from ..objects.builtin import FFMatrixBlock
from . import blocks as B
from .dedup import BlockPool
from .ff import (FFAggMatrix, FFAggMatrixToOneMatrix, FFMatrixBlockScanner, FFMatrixWriter, FFTransposeMult,
                 create_output_set)
from .word2vec import SemanticClassifierSingleBlock

# (vocab size, embedding dimension) of the reference drivers
MODELS = {"nnlm-50": (963812, 50), "nnlm-128": (963812, 128), "wiki-250": (1009375, 250),
          "wiki-500": (1009375, 500)}
BLOCK_X, BLOCK_Y, BATCH = 50, 10000, 100


def load_workload(client, db: str, vocab: int, embed: int, batch: int = BATCH, block_x: int = BLOCK_X,
                  block_y: int = BLOCK_Y, seed: int = 0, weights: Optional[torch.Tensor] = None,
                  dtype=torch.bfloat16):
    """createData(): inputs [batch x vocab] (bag-of-words counts) and weights [embed x vocab]."""
    client.create_database(db)
    g = torch.Generator().manual_seed(seed)
    x = (torch.rand(batch, vocab, generator=g) < 0.01).float()
    B.load_tensor(client, db, "inputs", x, block_x, block_y, dtype=dtype)
    if weights is None:
        weights = (torch.rand(embed, vocab, generator=g) * 2 - 1) * 0.1
    B.load_tensor(client, db, "weights", weights, block_x, block_y, dtype=dtype)
    client.set_locality(db, "weights", "model")


def run_workload(client, db: str, embed: int, dense0: int = 16, dense1: int = 1, seed: int = 0) -> dict:
    """runWorkload(): the two jobs of the module doc; returns timings and the [dense1 x batch] labels."""
    create_output_set(client, db, "intermediate")
    if client.storage.has_set(db, "outputs"):
        client.remove_set(db, "outputs")
    client.create_set(db, "outputs", FFMatrixBlock)
    t0 = time.perf_counter()
    j = FFTransposeMult()
    j.set_input(0, FFMatrixBlockScanner(db, "weights"))
    j.set_input(1, FFMatrixBlockScanner(db, "inputs"))
    s1 = client.execute_computations(WriteSet(db, "intermediate", FFMatrixBlock).set_input(FFAggMatrix().set_input(j)),
                                     job_name=f"{db}-embed")
    t1 = time.perf_counter()
    one = FFAggMatrixToOneMatrix().set_input(ScanSet(db, "intermediate", FFMatrixBlock))
    clf = SemanticClassifierSingleBlock(embed, dense0, dense1, seed=seed).set_input(one)
    s2 = client.execute_computations(FFMatrixWriter(db, "outputs").set_input(clf), job_name=f"{db}-classify")
    t2 = time.perf_counter()
    out = [b for b in client.get_set_batches(db, "outputs", gather=True) if b.n]
    labels = out[0].columns["data"][0] if out else None
    return {"embed_s": t1 - t0, "classify_s": t2 - t1, "jobs": [s1, s2], "labels": labels}


def reference_labels(W: torch.Tensor, X: torch.Tensor, embed: int, dense0: int = 16, dense1: int = 1,
                     seed: int = 0) -> torch.Tensor:
    """fp32 reference of run_workload on the same (bf16-rounded) operands."""
    x0 = W.float() @ X.float().t()
    return SemanticClassifierSingleBlock(embed, dense0, dense1, seed=seed).classify(x0.cpu())


def heterogeneous_dedup(client, models: Dict[str, tuple], batch: int = BATCH, block_x: int = BLOCK_X,
                        block_y: int = BLOCK_Y, seed: int = 0, run: Sequence[str] = ()) -> dict:
    """HybridTestWithDeduplication / TextClassifierDeduplication: models whose embedding tables share rows
    (every model's rows are a prefix of the largest table of its vocabulary) stored ONCE in a block pool, each
    model's weight set linked to it; then the listed workloads run on the linked sets."""
    by_vocab: Dict[int, torch.Tensor] = {}
    g = torch.Generator().manual_seed(seed)
    for name, (vocab, embed) in models.items():
        top = max(e for v, e in models.values() if v == vocab)
        if vocab not in by_vocab:
            by_vocab[vocab] = ((torch.rand(top, vocab, generator=g) * 2 - 1) * 0.1).to(torch.bfloat16)
    pool = BlockPool(block_x, block_y, device=client.device or "cpu", dtype=torch.bfloat16)
    private = 0
    for name, (vocab, embed) in models.items():
        W = by_vocab[vocab][:embed]
        pool.add_model(name, W.to(pool.device))
        private += W.numel() * W.element_size()
    res = {"models": list(models), "dedup_ratio": pool.dedup_ratio(), "bytes_private": private,
           "bytes_pooled": int(pool.blocks.numel() * pool.blocks.element_size()), "runs": {}}
    for name in run:
        vocab, embed = models[name]
        W = pool.materialize(name)
        db = name.replace("-", "_")
        load_workload(client, db, vocab, embed, batch, block_x, block_y, seed=seed + 1, weights=W.float().cpu())
        r = run_workload(client, db, embed, seed=seed)
        X = B.to_tensor(client, db, "inputs")
        ref = reference_labels(B.to_tensor(client, db, "weights"), X, embed, seed=seed)
        r["match"] = bool(r["labels"] is not None and torch.equal(r["labels"].float().cpu().reshape(ref.shape), ref))
        res["runs"][name] = r
    return res


__all__ = ["MODELS", "load_workload", "run_workload", "reference_labels", "heterogeneous_dedup"]
