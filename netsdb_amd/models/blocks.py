"""Block-matrix helpers shared by the model libraries (reference: src/FF/source/FFMatrixUtil.cc —
loadMatrix / load_matrix_data / print_stats; src/linearAlgebraDSL LAPDBInstance loading).

Matrices are created as DenseMatrixSets (one HBM panel per rank, block geometry recorded) and
filled from synthetic random data, a text file in the reference's block format, or a tensor.
"""
from __future__ import annotations

import math
from typing import Optional

import torch

from ..objects.builtin import FFMatrixBlock, MatrixBlock
from ..storage.sets import DenseMatrixSet


def create_matrix_set(client, db: str, name: str, rows: int, cols: int, block_rows: int, block_cols: int,
                      dtype=torch.bfloat16, replicated: bool = True, partition_rows: bool = False,
                      type_=FFMatrixBlock) -> DenseMatrixSet:
    """Create (or reset) a dense matrix set. ``partition_rows``: each rank holds a contiguous
    block-row range (row-partitioned data set); otherwise every rank holds the full matrix."""
    if client.storage.has_set(db, name):
        client.remove_set(db, name)
    client.create_set(db, name, type_, dense=True)
    s: DenseMatrixSet = client.storage.get_set(db, name)
    ws, rank = client.ctx.world_size, client.ctx.rank
    if partition_rows and client.ctx.distributed:
        nbr = math.ceil(rows / block_rows)
        per = math.ceil(nbr / ws)
        r0 = min(rows, rank * per * block_rows)
        r1 = min(rows, (rank + 1) * per * block_rows)
        s.define(rows, cols, block_rows, block_cols, row_offset=r0, local_rows=r1 - r0, dtype=dtype)
        s.replicated = False
    else:
        s.define(rows, cols, block_rows, block_cols, dtype=dtype)
        s.replicated = True
    return s


def fill_random(s: DenseMatrixSet, seed: int = 0, scale: Optional[float] = None, low: float = -1.0,
                high: float = 1.0):
    """Uniform random fill (deterministic per (seed, global row) so partitions are consistent)."""
    g = torch.Generator(device=s.panel.device).manual_seed(seed + s.row_offset * 7919)
    view = s.panel[: s.local_rows, : s.total_cols]
    tmp = torch.empty(view.shape, dtype=torch.float32, device=s.panel.device)
    tmp.uniform_(low, high, generator=g)
    if scale is not None:
        tmp.mul_(scale)
    view.copy_(tmp)
    return s


def load_matrix(client, db: str, name: str, rows: int, cols: int, block_rows: int, block_cols: int,
                seed: int = 0, scale: Optional[float] = None, dtype=torch.bfloat16, partition_rows: bool = False,
                value: Optional[float] = None) -> DenseMatrixSet:
    """ff::loadMatrix equivalent: a random (or constant) matrix as a block-partitioned set."""
    s = create_matrix_set(client, db, name, rows, cols, block_rows, block_cols, dtype, partition_rows=partition_rows)
    if value is not None:
        s.panel[: s.local_rows, : s.total_cols].fill_(value)
    else:
        fill_random(s, seed, scale)
    return s


def load_tensor(client, db: str, name: str, t: torch.Tensor, block_rows: int, block_cols: int,
                dtype=torch.bfloat16, partition_rows: bool = False) -> DenseMatrixSet:
    rows, cols = t.shape
    s = create_matrix_set(client, db, name, rows, cols, block_rows, block_cols, dtype, partition_rows=partition_rows)
    s.panel[: s.local_rows, :cols].copy_(t[s.row_offset: s.row_offset + s.local_rows].to(s.panel.device, dtype))
    return s


def load_block_file(client, db: str, name: str, path: str, block_rows: int, block_cols: int, nbr: int, nbc: int,
                    dtype=torch.float32) -> DenseMatrixSet:
    """Reference text block format ('i j v00 v01 ...' per block; LAEvaluateFunctions 'load')."""
    rows, cols = nbr * block_rows, nbc * block_cols
    s = create_matrix_set(client, db, name, rows, cols, block_rows, block_cols, dtype, type_=MatrixBlock)
    with open(path) as f:
        toks = f.read().split()
    pos = 0
    for _ in range(nbr * nbc):
        i, j = int(toks[pos]), int(toks[pos + 1])
        pos += 2
        vals = torch.tensor([float(x) for x in toks[pos: pos + block_rows * block_cols]], dtype=torch.float32)
        pos += block_rows * block_cols
        s.panel[i * block_rows:(i + 1) * block_rows, j * block_cols:(j + 1) * block_cols] = \
            vals.reshape(block_rows, block_cols).to(s.panel.device, dtype)
    return s


def to_tensor(client, db: str, name: str, gather: bool = True) -> torch.Tensor:
    """The logical matrix of a dense set (all-gathered over row-partitioned ranks)."""
    s = client.storage.get_set(db, name)
    if isinstance(s, DenseMatrixSet):
        m = s.matrix()[: s.local_rows] if not s.transposed else s.matrix()
        if gather and client.ctx.distributed and not s.replicated:
            parts = client.ctx.all_gather_tensor(m.contiguous())
            m = torch.cat(parts)
        return m
    # generic MatrixBlock set: assemble from blocks
    batches = client.get_set_batches(db, name, gather=gather)
    if not batches:
        return torch.empty(0)
    from ..objects.record import RecordBatch

    b = RecordBatch.concat(batches)
    keep = (b.columns["block_row"] >= 0) & (b.columns["block_col"] >= 0)     # unmapped shared blocks
    if not bool(keep.all()):
        b = b.take(keep.nonzero().flatten())
    if b.n == 0:
        return torch.empty(0)
    tr, tc = int(b.columns["total_rows"][0]), int(b.columns["total_cols"][0])
    data = b.columns["data"]
    br, bc = data.shape[1], data.shape[2]
    nbr, nbc = -(-tr // br), -(-tc // bc)
    # one scatter of every block into the padded [nbr, br, nbc, bc] view (no per-block host loop)
    out = torch.zeros(nbr, br, nbc, bc, dtype=torch.float32, device=data.device)
    r = b.columns["block_row"].to(data.device)
    c = b.columns["block_col"].to(data.device)
    out[r, :, c, :] = data.float()
    return out.reshape(nbr * br, nbc * bc)[:tr, :tc]


__all__ = ["create_matrix_set", "fill_random", "load_matrix", "load_tensor", "load_block_file", "to_tensor"]
