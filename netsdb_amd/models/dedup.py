"""Model deduplication: share identical / near-identical tensor blocks across models.

Reference: src/deduplication (TensorBlockIndex — map persisted deduplicated source blocks to the
runtime blocks of each target set; SharedFFMatrixBlockSet / SharedTensorBlockSet — sets whose pages
are shared; PartitionTensorBlockSharedPageIterator), PDBClient::addSharedMapping / addSharedPage,
model-inference/deduplication (LSH block matching in indexing/, page packing in page-packing/),
drivers FFTestWithDeduplication.cc, TestWord2VecWithDeduplication.cc, TextClassifierDeduplication.cc.

MI355X-native design: all models' blocks live ONCE in an HBM block pool [n_unique, br, bc]; each
model is a block-index table (TensorBlockIndex).  Dedup detection hashes blocks on the GPU
(exact) or compares random-projection LSH signatures + an L-inf tolerance (approximate).  A model
is materialised for inference by one gather (index_select) into its dense panel, or page-packed:
blocks are ordered so models that share blocks share pages (greedy packing, page_packing.py's
bin-packing idea).  Across GPUs, :class:`DistributedBlockPool` stores every distinct block once in the
cluster (hash-owner placement, RCCL all-to-all).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import torch

from ..execution.kernels import mix64


@dataclass
class TensorBlockIndex:
    """model name -> [nbr, nbc] table of pool block ids (+ geometry)."""

    block_rows: int
    block_cols: int
    tables: Dict[str, torch.Tensor] = field(default_factory=dict)
    shapes: Dict[str, Tuple[int, int]] = field(default_factory=dict)

    # --- FFMatrixBlockIndex parity (src/deduplication/headers/FFMatrixBlockIndex.h): per target set,
    # distinct (shared) block id -> target block metadata (block_row, block_col, total_rows, total_cols)
    targets: Dict[int, Dict[int, Tuple[int, int, int, int]]] = field(default_factory=dict)

    @staticmethod
    def set_key(db_id: int, type_id: int, set_id: int) -> int:
        return int(type_id) + int(set_id) * 100000 + int(db_id) * 100000000

    def insert_index(self, set_key: int, block_key: int, meta: Tuple[int, int, int, int]) -> bool:
        self.targets.setdefault(int(set_key), {})[int(block_key)] = tuple(int(x) for x in meta)
        return True

    def remove_index(self, set_key: int, block_key: int) -> bool:
        m = self.targets.get(int(set_key))
        if m is None:
            return False
        m.pop(int(block_key), None)
        return True

    def get_target_metadata(self, set_key: int, block_key: int) -> Optional[Tuple[int, int, int, int]]:
        return self.targets.get(int(set_key), {}).get(int(block_key))

    def load_index_file(self, set_key: int, path: str, total_rows: int, total_cols: int,
                        transpose: bool = False) -> Dict[int, Tuple[int, int, int, int]]:
        """SharedFFMatrixBlockSet::loadIndexFromFile: lines 'blockKey,blockRow,blockCol' (transpose swaps
        the target row/col), every target sized total_rows x total_cols."""
        with open(path) as f:
            for line in f:
                parts = [x.strip() for x in line.replace(",", " ").split()]
                if len(parts) < 3:
                    continue
                key, r, c = int(parts[0]), int(parts[1]), int(parts[2])
                if transpose:
                    r, c = c, r
                self.insert_index(set_key, key, (r, c, total_rows, total_cols))
        return dict(self.targets.get(int(set_key), {}))

    def to_json(self) -> dict:
        return {"block_rows": self.block_rows, "block_cols": self.block_cols,
                "tables": {k: v.cpu().tolist() for k, v in self.tables.items()},
                "shapes": {k: list(v) for k, v in self.shapes.items()},
                "targets": {str(k): {str(b): list(m) for b, m in v.items()} for k, v in self.targets.items()}}

    @staticmethod
    def from_json(d: dict) -> "TensorBlockIndex":
        idx = TensorBlockIndex(d["block_rows"], d["block_cols"])
        idx.tables = {k: torch.tensor(v, dtype=torch.int64) for k, v in d["tables"].items()}
        idx.shapes = {k: tuple(v) for k, v in d["shapes"].items()}
        idx.targets = {int(k): {int(b): tuple(m) for b, m in v.items()} for k, v in d.get("targets", {}).items()}
        return idx


def to_blocks(m: torch.Tensor, br: int, bc: int) -> torch.Tensor:
    R, C = m.shape
    nbr, nbc = math.ceil(R / br), math.ceil(C / bc)
    m = torch.nn.functional.pad(m, (0, nbc * bc - C, 0, nbr * br - R))
    return m.reshape(nbr, br, nbc, bc).permute(0, 2, 1, 3).reshape(nbr * nbc, br, bc)


def from_blocks(blocks: torch.Tensor, nbr: int, nbc: int, R: int, C: int) -> torch.Tensor:
    br, bc = blocks.shape[1], blocks.shape[2]
    return blocks.reshape(nbr, nbc, br, bc).permute(0, 2, 1, 3).reshape(nbr * br, nbc * bc)[:R, :C]


def block_hashes(blocks: torch.Tensor) -> torch.Tensor:
    """Exact content hash per block (on device): mix64 over the raw 16-bit/32-bit words."""
    flat = blocks.reshape(blocks.shape[0], -1)
    if flat.dtype in (torch.bfloat16, torch.float16):
        words = flat.view(torch.int16).to(torch.int64) & 0xFFFF
    else:
        words = flat.float().view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    pos = torch.arange(words.shape[1], device=words.device, dtype=torch.int64)
    h = mix64(words * 0x100000001B3 + pos)
    return mix64(h.sum(1))   # order-aware (pos mixed in), commutative sum is fine after mixing


def lsh_signatures(blocks: torch.Tensor, bits: int = 64, seed: int = 0) -> torch.Tensor:
    """Random-hyperplane LSH signature per block (similar blocks -> equal signatures)."""
    flat = blocks.reshape(blocks.shape[0], -1).float()
    g = torch.Generator(device=flat.device).manual_seed(seed)
    planes = torch.randn(flat.shape[1], bits, generator=g, device=flat.device)
    s = (flat @ planes) > 0
    w = (1 << torch.arange(bits - 1, device=flat.device, dtype=torch.int64))
    return (s[:, : bits - 1].long() * w).sum(1)


class BlockPool:
    """Deduplicated block storage shared by many models (SharedFFMatrixBlockSet analogue)."""

    def __init__(self, block_rows: int, block_cols: int, device="cpu", dtype=torch.bfloat16, tolerance: float = 0.0):
        self.br, self.bc = block_rows, block_cols
        self.device, self.dtype = device, dtype
        self.tolerance = tolerance
        self.blocks = torch.empty(0, block_rows, block_cols, dtype=dtype, device=device)
        self.keys = torch.empty(0, dtype=torch.int64, device=device)
        self.index = TensorBlockIndex(block_rows, block_cols)
        self.stats = {"blocks_in": 0, "blocks_stored": 0}

    def add_model(self, name: str, m: torch.Tensor) -> torch.Tensor:
        m = m.to(self.device, self.dtype)
        R, C = m.shape
        nbr, nbc = math.ceil(R / self.br), math.ceil(C / self.bc)
        ids = self.insert_blocks(to_blocks(m, self.br, self.bc))
        self.index.tables[name] = ids.reshape(nbr, nbc)
        self.index.shapes[name] = (R, C)
        return ids

    def insert_blocks(self, blks: torch.Tensor, keys: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Pool ids of ``blks`` [n, br, bc]: a block equal (within tolerance) to a stored one reuses its
        id; new distinct blocks are appended (deduplicated among themselves too)."""
        blks = blks.to(self.device, self.dtype)
        if keys is None:
            keys = block_hashes(blks) if self.tolerance == 0 else lsh_signatures(blks)
        ids = torch.empty(blks.shape[0], dtype=torch.int64, device=self.device)
        # match against the pool (sorted-key binary search), verify content within tolerance
        if self.keys.numel():
            order = torch.argsort(self.keys)
            sk = self.keys[order]
            pos = torch.searchsorted(sk, keys).clamp(max=sk.numel() - 1)
            cand = order[pos]
            hit = sk[pos] == keys
            if hit.any():
                diff = (self.blocks[cand].float() - blks.float()).abs().amax(dim=(1, 2))
                hit &= diff <= self.tolerance
        else:
            cand = torch.zeros_like(ids)
            hit = torch.zeros(blks.shape[0], dtype=torch.bool, device=self.device)
        ids[hit] = cand[hit]
        new = (~hit).nonzero().flatten()
        if new.numel():
            # dedup within the incoming blocks themselves
            nk = keys[new]
            uk, inv = torch.unique(nk, return_inverse=True)
            first = torch.full((uk.numel(),), new.numel(), dtype=torch.int64, device=self.device)
            first.scatter_reduce_(0, inv, torch.arange(new.numel(), device=self.device), reduce="amin")
            base = self.blocks.shape[0]
            self.blocks = torch.cat([self.blocks, blks[new[first]]])
            self.keys = torch.cat([self.keys, uk if self.tolerance == 0 else nk[first]])
            ids[new] = base + inv
        self.stats["blocks_in"] += blks.shape[0]
        self.stats["blocks_stored"] = self.blocks.shape[0]
        return ids

    def materialize(self, name: str) -> torch.Tensor:
        t = self.index.tables[name]
        R, C = self.index.shapes[name]
        blks = self.blocks.index_select(0, t.flatten().to(self.blocks.device))
        return from_blocks(blks, t.shape[0], t.shape[1], R, C)

    def dedup_ratio(self) -> float:
        return self.stats["blocks_stored"] / max(1, self.stats["blocks_in"])

    def pack_pages(self, blocks_per_page: int, algorithm: str = "greedy1") -> List[List[int]]:
        """Page packing: blocks shared by the same set of models go to the same pages, so a model
        touches as few pages as possible (model-inference/deduplication/page-packing).  ``algorithm``:
        greedy1 (equivalence classes, default), two_stage, greedy2, baseline (models/page_packing.py)."""
        if algorithm != "greedy1":
            from .page_packing import pack

            models = [set(t.flatten().tolist()) for t in self.index.tables.values()]
            return pack(models, blocks_per_page, algorithm).pages
        owners: Dict[int, set] = {}
        for name, t in self.index.tables.items():
            for b in t.flatten().tolist():
                owners.setdefault(b, set()).add(name)
        groups: Dict[frozenset, List[int]] = {}
        for b, o in owners.items():
            groups.setdefault(frozenset(o), []).append(b)
        pages: List[List[int]] = []
        for key in sorted(groups, key=lambda k: (-len(k), sorted(k))):
            blks = sorted(groups[key])
            for s in range(0, len(blks), blocks_per_page):
                pages.append(blks[s:s + blocks_per_page])
        return pages


class DistributedBlockPool:
    """Cluster-wide model deduplication (one process per GPU): every distinct block is stored ONCE in
    the cluster, on the rank that owns its content hash, so identical blocks of models held by
    different GPUs (fine-tuned word2vec / classifier embedding tables) share one copy.

    ``add_model`` (collective): block hashes on the device -> RCCL all-to-all of (hash, payload) to the
    hash owners -> owners deduplicate against their pool (content-verified, :meth:`BlockPool.insert_blocks`)
    -> global ids (owner << 40 | owner-local id) all-to-all'd back.  ``materialize`` (collective) fetches
    a model's blocks from their owners with a second all-to-all pair.  The reference shares blocks through
    TensorBlockIndex + SharedFFMatrixBlockSet pages over its socket dispatcher (src/deduplication,
    TestWord2VecWithDeduplication.cc)."""

    SHIFT = 40

    def __init__(self, ctx, block_rows: int, block_cols: int, device=None, dtype=torch.bfloat16,
                 tolerance: float = 0.0):
        self.ctx = ctx
        self.br, self.bc = block_rows, block_cols
        self.device = torch.device(device) if device is not None else ctx.device
        self.dtype = dtype
        self.local = BlockPool(block_rows, block_cols, device=self.device, dtype=dtype, tolerance=tolerance)
        self.tables: Dict[str, torch.Tensor] = {}
        self.shapes: Dict[str, Tuple[int, int]] = {}
        self.stats = {"blocks_in": 0}

    def _ship(self, rows: torch.Tensor, dest: torch.Tensor):
        """Group rows by destination rank and all-to-all them: (received rows, recv counts, send order)."""
        order = torch.argsort(dest, stable=True)
        counts = torch.bincount(dest, minlength=self.ctx.world_size).tolist()
        got, recv = self.ctx.all_to_all_rows(rows[order], counts)
        return got, recv, order

    def _payload(self, blks: torch.Tensor) -> torch.Tensor:
        return blks.reshape(blks.shape[0], self.br * self.bc).contiguous().view(torch.uint8)

    def add_model(self, name: str, m: Optional[torch.Tensor]) -> torch.Tensor:
        ws, rank = self.ctx.world_size, self.ctx.rank
        m = torch.empty(0, self.bc, dtype=self.dtype, device=self.device) if m is None else m.to(self.device, self.dtype)
        R, C = m.shape
        nbr, nbc = math.ceil(R / self.br), math.ceil(C / self.bc)
        if m.numel():
            blks = to_blocks(m, self.br, self.bc)
            h = block_hashes(blks)
        else:
            blks = torch.empty(0, self.br, self.bc, dtype=self.dtype, device=self.device)
            h = torch.empty(0, dtype=torch.int64, device=self.device)
        owner = (mix64(h) & 0x7FFFFFFFFFFFFFFF) % ws
        got_h, recv, order = self._ship(h, owner)
        got_b, _, _ = self._ship(self._payload(blks), owner)
        got_b = got_b.to(self.device).view(self.dtype).reshape(-1, self.br, self.bc)
        if got_b.shape[0]:
            local_ids = self.local.insert_blocks(got_b, got_h.to(self.device))
        else:
            local_ids = torch.empty(0, dtype=torch.int64, device=self.device)
        back, _ = self.ctx.all_to_all_rows((rank << self.SHIFT) | local_ids, recv)
        ids = torch.empty_like(h)
        ids[order] = back.to(ids.device)
        self.tables[name] = ids.reshape(nbr, nbc)
        self.shapes[name] = (R, C)
        self.stats["blocks_in"] += int(blks.shape[0])
        return ids

    def materialize(self, name: Optional[str]) -> Optional[torch.Tensor]:
        """Collective: rebuild this rank's model ``name`` (None: only serve the other ranks' requests)."""
        if name is not None:
            ids = self.tables[name].flatten()
        else:
            ids = torch.empty(0, dtype=torch.int64, device=self.device)
        req, recv, order = self._ship(ids & ((1 << self.SHIFT) - 1), ids >> self.SHIFT)
        payload = self._payload(self.local.blocks.index_select(0, req.to(self.device)))
        got, _ = self.ctx.all_to_all_rows(payload, recv)
        if name is None:
            return None
        blks = torch.empty(ids.numel(), self.br, self.bc, dtype=self.dtype, device=self.device)
        blks[order] = got.to(self.device).view(self.dtype).reshape(-1, self.br, self.bc)
        t = self.tables[name]
        R, C = self.shapes[name]
        return from_blocks(blks, t.shape[0], t.shape[1], R, C)

    def stored_blocks(self) -> int:
        """Distinct blocks stored on this rank (the sum over ranks = cluster-wide distinct blocks)."""
        return int(self.local.blocks.shape[0])


def pages_touched(pool: BlockPool, pages: List[List[int]], name: str) -> int:
    page_of = {b: i for i, p in enumerate(pages) for b in p}
    return len({page_of[b] for b in pool.index.tables[name].flatten().tolist()})


__all__ = ["TensorBlockIndex", "BlockPool", "DistributedBlockPool", "block_hashes", "lsh_signatures", "to_blocks", "from_blocks",
           "pages_touched"]
