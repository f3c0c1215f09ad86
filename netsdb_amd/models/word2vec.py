"""word2vec embedding inference and the semantic (text) classifier (reference: src/word2vec —
Word2Vec.cc (inference as one-hot batch x embedding matrix through FFTransposeMult/FFAggMatrix),
EmbeddingLookupSparse.h (MultiSelection emitting EmbeddingSegments for the requested ids),
EmbeddingSegment.h, SemanticClassifier.h / SemanticClassifierSingleBlock.h, TestSemanticClassifier.cc;
model-inference/word2vec, text-classification).

Three plans over an embedding set (vocab x dim, block-partitioned):
  * matmul plan (reference Word2Vec.cc): one-hot [batch x vocab] · E — fused split-K MFMA GEMM;
  * sparse lookup plan (EmbeddingLookupSparse): MultiSelection over embedding blocks emitting the
    rows of the requested ids (generic engine);
  * fused lookup (MI355X-native): ``embedding_bag`` HIP kernel gathering whole rows from HBM.
"""
from __future__ import annotations

import time
from typing import List

import torch

from .. import ops
from ..computations import MultiSelectionComp, ScanSet, SelectionComp, WriteSet
from ..lambdas import make_batch_lambda
from ..objects.builtin import FFMatrixBlock
from ..objects.record import PDBObject, RecordBatch, Tensor
from . import blocks as B
from .ff import FFAggMatrix, FFMatrixBlockScanner, FFTransposeMult, create_output_set


class EmbeddingSegment(PDBObject):
    """One id's slice of embedding columns held by one block (id, block_col, width, values)."""

    word_id: int
    block_col: int
    width: int
    data: Tensor()


class EmbeddingLookupSparse(MultiSelectionComp):
    def __init__(self, ids: List[int]):
        super().__init__()
        self.ids = torch.tensor(sorted(set(int(i) for i in ids)), dtype=torch.int64)

    def get_selection(self, blk):
        def sel(b: RecordBatch):
            r0 = b.columns["block_row"] * b.columns["row_nums"]
            r1 = r0 + b.columns["row_nums"]
            ids = self.ids.to(r0.device)
            lo = torch.searchsorted(ids, r0)
            hi = torch.searchsorted(ids, r1)
            return hi > lo

        return make_batch_lambda(blk, sel)

    def get_projection(self, blk):
        def proj(b: RecordBatch):
            out = []
            ids = self.ids.to(b.columns["block_row"].device)
            for k in range(b.n):
                rn = int(b.columns["row_nums"][k])
                r0 = int(b.columns["block_row"][k]) * rn
                sel = ids[(ids >= r0) & (ids < r0 + rn)]
                segs = []
                for i in sel.tolist():
                    segs.append(EmbeddingSegment(i, int(b.columns["block_col"][k]), int(b.columns["col_nums"][k]),
                                                 b.columns["data"][k, i - r0].float()))
                out.append(segs)
            return out

        return make_batch_lambda(blk, proj, tag="embedding_lookup_sparse")


def load_embeddings(client, db: str, name: str, vocab: int, dim: int, block_x: int, block_y: int, seed: int = 0,
                    dtype=torch.bfloat16):
    client.create_database(db)
    return B.load_matrix(client, db, name, vocab, dim, block_x, block_y, seed=seed, scale=0.5, dtype=dtype)


def word2vec_matmul(client, db: str, emb: str, ids: torch.Tensor, vocab: int, block_x: int, block_y: int,
                    output: str = "w2v_out") -> dict:
    """Word2Vec.cc plan: one-hot(ids) [batch x vocab] times E [vocab x dim]."""
    dev = client.device
    onehot = torch.zeros(ids.numel(), vocab, dtype=torch.bfloat16, device=dev)
    onehot[torch.arange(ids.numel(), device=dev), ids.to(dev)] = 1
    B.load_tensor(client, db, "w2v_inputs", onehot, block_x, block_y)
    E = client.storage.get_set(db, emb)
    # E^T as the "B" operand of FFTransposeMult: X · (E^T)^T
    from ..la.computations import LATransposeSelection

    create_output_set(client, db, output)
    t0 = time.perf_counter()
    j = FFTransposeMult()
    j.set_input(0, FFMatrixBlockScanner(db, "w2v_inputs"))
    j.set_input(1, LATransposeSelection().set_input(FFMatrixBlockScanner(db, emb)))
    st = client.execute_computations(WriteSet(db, output, FFMatrixBlock).set_input(FFAggMatrix().set_input(j)),
                                     job_name="word2vec")
    _ = E
    return {"seconds": time.perf_counter() - t0, "job": st}


def word2vec_lookup(client, db: str, emb: str, ids: torch.Tensor) -> torch.Tensor:
    """Fused lookup: rows of E for ids via the embedding_bag kernel (one id per bag)."""
    E = client.storage.get_set(db, emb).matrix()
    idx = ids.to(E.device).long()
    offs = torch.arange(idx.numel() + 1, device=E.device)
    return ops.embedding_bag(E.contiguous() if not E.is_contiguous() else E, idx, offs)


def word2vec_sparse(client, db: str, emb: str, ids: List[int], output: str = "w2v_segments") -> dict:
    """EmbeddingLookupSparse plan on the generic engine (segments per block)."""
    if client.storage.has_set(db, output):
        client.remove_set(db, output)
    client.create_set(db, output, EmbeddingSegment)
    t0 = time.perf_counter()
    m = EmbeddingLookupSparse(ids).set_input(ScanSet(db, emb, FFMatrixBlock))
    st = client.execute_computations(WriteSet(db, output, EmbeddingSegment).set_input(m), job_name="w2v_sparse")
    return {"seconds": time.perf_counter() - t0, "job": st}


def assemble_segments(client, db: str, name: str, dim: int) -> dict:
    out = {}
    for s in client.get_set_iterator(db, name, gather=True):
        v = out.setdefault(s.word_id, torch.zeros(dim))
        c0 = s.block_col * s.width
        v[c0:c0 + s.data.numel()] = s.data.float().cpu()[: max(0, min(s.data.numel(), dim - c0))]
    return out


class SemanticClassifier:
    """Text classifier: mean word embedding of each document -> FF layer(s) -> softmax
    (SemanticClassifier.h; model-inference/text-classification)."""

    def __init__(self, E: torch.Tensor, hidden: int, labels: int, seed: int = 0):
        g = torch.Generator(device=E.device).manual_seed(seed)
        d = E.shape[1]
        self.E = E
        self.W1 = ((torch.rand(hidden, d, generator=g, device=E.device) * 2 - 1) * (3.0 / d) ** 0.5)
        self.b1 = torch.zeros(hidden, device=E.device)
        self.W2 = ((torch.rand(labels, hidden, generator=g, device=E.device) * 2 - 1) * (3.0 / hidden) ** 0.5)
        self.b2 = torch.zeros(labels, device=E.device)

    def forward(self, idx: torch.Tensor, offsets: torch.Tensor) -> torch.Tensor:
        emb = ops.embedding_bag(self.E, idx, offsets, mode="mean")                     # [docs, d] f32
        h = ops.gemm_nt(ops.pad_k(emb.to(torch.bfloat16)), ops.pad_k(self.W1.to(torch.bfloat16)), self.b1,
                        ops.BIAS_COL, "relu")
        z = ops.gemm_nt(ops.pad_k(h), ops.pad_k(self.W2.to(torch.bfloat16)), self.b2, ops.BIAS_COL,
                        out_dtype=torch.float32)
        return ops.softmax_rows(z)

    def reference(self, idx, offsets):
        E = self.E.float().cpu()
        docs = []
        for b in range(offsets.numel() - 1):
            s, e = int(offsets[b]), int(offsets[b + 1])
            docs.append(E[idx[s:e].cpu()].mean(0) if e > s else torch.zeros(E.shape[1]))
        x = torch.stack(docs)
        h = torch.relu(x @ self.W1.float().cpu().t() + self.b1.cpu())
        return torch.softmax(h @ self.W2.float().cpu().t() + self.b2.cpu(), -1)


class SemanticClassifierSingleBlock(SelectionComp):
    """Text classifier over the whole embedded batch as ONE matrix (src/word2vec/headers/
    SemanticClassifierSingleBlock.h): x0 [sizeEmbed x batch] (an FFSingleMatrix from FFAggMatrixToOneMatrix) ->
    relu(W0 x0 + b0) [sizeDense0 x batch] -> sigmoid(W1 y0 + b1) [sizeDense1 x batch] -> label (> 0.5 -> 1 else 0),
    written as one FFMatrixBlock. The reference's dense weights are placeholder constants; here they are
    seeded random weights of the same geometry (``weights()``), evaluated with exact-f32 GEMMs."""

    def __init__(self, size_embed: int = 500, size_dense0: int = 16, size_dense1: int = 1, seed: int = 0):
        super().__init__()
        self.size_embed, self.size_dense0, self.size_dense1, self.seed = size_embed, size_dense0, size_dense1, seed

    def weights(self, device=None):
        g = torch.Generator().manual_seed(self.seed)
        w0 = (torch.rand(self.size_dense0, self.size_embed, generator=g) * 2 - 1) * (3.0 / self.size_embed) ** 0.5
        b0 = (torch.rand(self.size_dense0, generator=g) * 2 - 1) * 0.1
        w1 = (torch.rand(self.size_dense1, self.size_dense0, generator=g) * 2 - 1) * (3.0 / self.size_dense0) ** 0.5
        b1 = (torch.rand(self.size_dense1, generator=g) * 2 - 1) * 0.1
        return [t.to(device) for t in (w0, b0, w1, b1)]

    def classify(self, x0: torch.Tensor) -> torch.Tensor:
        """x0 [sizeEmbed, batch] -> labels [sizeDense1, batch] (float 0 / 1)."""
        w0, b0, w1, b1 = self.weights(x0.device)
        x0 = x0.float()
        if x0.is_cuda:
            y0 = torch.relu(ops.gemm_nt_f32(w0.contiguous(), x0.t().contiguous()) + b0[:, None])
            y1 = torch.sigmoid(ops.gemm_nt_f32(w1.contiguous(), y0.t().contiguous()) + b1[:, None])
        else:
            y0 = torch.relu(w0 @ x0 + b0[:, None])
            y1 = torch.sigmoid(w1 @ y0 + b1[:, None])
        return (y1 > 0.5).float()

    def get_selection(self, m):
        return make_batch_lambda(m, lambda b: torch.ones(b.n, dtype=torch.bool, device=b.columns["data"].device))

    def get_projection(self, m):
        from .ff import mk_blocks

        def proj(b: RecordBatch):
            outs = []
            for k in range(b.n):
                r, c = int(b.columns["row_nums"][k]), int(b.columns["col_nums"][k])
                outs.append(self.classify(b.columns["data"][k, :r, :c]))
            d = torch.stack(outs)
            return mk_blocks(b.columns["block_row"], b.columns["block_col"], d, self.size_dense1, d.shape[2])

        return make_batch_lambda(m, proj, tag="semantic_classifier_single_block")


__all__ = ["EmbeddingSegment", "EmbeddingLookupSparse", "load_embeddings", "word2vec_matmul", "word2vec_lookup",
           "word2vec_sparse", "assemble_segments", "SemanticClassifier", "SemanticClassifierSingleBlock"]
