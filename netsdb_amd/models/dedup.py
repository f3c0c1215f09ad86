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


_FNV = 0x100000001B3


def _words32(blocks: torch.Tensor) -> torch.Tensor:
    """Each block's raw bytes as u32 words (int64 holding 0..2^32-1), zero-padded to a whole word."""
    flat = blocks.reshape(blocks.shape[0], -1).contiguous()
    raw = flat.view(torch.uint8)
    pad = (-raw.shape[1]) % 4
    if pad:
        raw = torch.nn.functional.pad(raw, (0, pad))
    return raw.view(torch.int32).to(torch.int64) & 0xFFFFFFFF


def block_hashes_reference(blocks: torch.Tensor, chunk_words: int = 1 << 24) -> torch.Tensor:
    """Canonical block content hash in torch (any device):
    ``mix64(sum_j mix64(w_j * 0x100000001B3 + j))`` over the block's 32-bit words, wrapping int64.
    Processed in bounded chunks of blocks so a 2-MB-block model never materialises 8 B per element."""
    n = blocks.shape[0]
    out = torch.empty(n, dtype=torch.int64, device=blocks.device)
    if n == 0:
        return out
    per = max(1, (blocks[0].numel() * blocks.element_size() + 3) // 4)
    step = max(1, chunk_words // per)
    for b0 in range(0, n, step):
        w = _words32(blocks[b0: b0 + step])
        pos = torch.arange(w.shape[1], device=w.device, dtype=torch.int64)
        out[b0: b0 + step] = mix64(mix64(w * _FNV + pos).sum(1))
    return out


def _native_ok(blocks: torch.Tensor) -> bool:
    if not blocks.is_cuda or blocks.shape[0] == 0:
        return False
    return (blocks[0].numel() * blocks.element_size()) % 16 == 0 and blocks.is_contiguous() and \
        blocks.data_ptr() % 16 == 0


def block_hashes(blocks: torch.Tensor) -> torch.Tensor:
    """Exact content hash per block: one HBM pass of the ``block_hash`` HIP kernel on a GPU (partial sums
    per split, finished here), the chunked torch reference elsewhere — bit-identical results."""
    if _native_ok(blocks):
        from .. import _ext

        return mix64(_ext.hip().block_hash_partial(blocks).sum(1))
    return block_hashes_reference(blocks)


def block_maxdiff(pool: torch.Tensor, cand: torch.Tensor, blks: torch.Tensor) -> torch.Tensor:
    """max |pool[cand[i]] - blks[i]| per block (content verification of hash hits); the HIP kernel reads
    both operands once without gathering the candidates."""
    if blks.shape[0] == 0:
        return torch.empty(0, dtype=torch.float32, device=blks.device)
    if _native_ok(blks) and pool.is_contiguous() and pool.dtype in (torch.float32, torch.bfloat16):
        from .. import _ext

        return _ext.hip().block_maxdiff_partial(pool, cand.contiguous(), blks).amax(1)
    return (pool.index_select(0, cand).float() - blks.float()).abs().flatten(1).amax(1)


def lsh_signatures(blocks: torch.Tensor, bits: int = 64, seed: int = 0) -> torch.Tensor:
    """Random-hyperplane LSH signature per block (similar blocks -> equal signatures)."""
    flat = blocks.reshape(blocks.shape[0], -1).float()
    g = torch.Generator(device=flat.device).manual_seed(seed)
    planes = torch.randn(flat.shape[1], bits, generator=g, device=flat.device)
    s = (flat @ planes) > 0
    w = (1 << torch.arange(bits - 1, device=flat.device, dtype=torch.int64))
    return (s[:, : bits - 1].long() * w).sum(1)


class BlockPool:
    """Deduplicated block storage shared by many models (SharedFFMatrixBlockSet analogue).

    The pool is one capacity-doubling device buffer [cap, br, bc] (amortised O(1) appends, no
    re-concatenation of the whole pool per insert) plus its keys kept sorted for the hash-hit
    search; stored blocks never move, so pool ids stay valid."""

    def __init__(self, block_rows: int, block_cols: int, device="cpu", dtype=torch.bfloat16, tolerance: float = 0.0):
        self.br, self.bc = block_rows, block_cols
        self.device, self.dtype = device, dtype
        self.tolerance = tolerance
        self._buf = torch.empty(0, block_rows, block_cols, dtype=dtype, device=device)
        self._n = 0
        self.keys = torch.empty(0, dtype=torch.int64, device=device)        # key of pool id i
        self._sorted_keys = self.keys
        self._sorted_ids = torch.empty(0, dtype=torch.int64, device=device)
        self.index = TensorBlockIndex(block_rows, block_cols)
        self.stats = {"blocks_in": 0, "blocks_stored": 0, "grows": 0}

    @property
    def blocks(self) -> torch.Tensor:
        return self._buf[: self._n]

    def _reserve(self, n: int):
        if n <= self._buf.shape[0]:
            return
        cap = max(n, 2 * self._buf.shape[0], 16)
        buf = torch.empty(cap, self.br, self.bc, dtype=self.dtype, device=self.device)
        if self._n:
            buf[: self._n].copy_(self._buf[: self._n])
        self._buf = buf
        self.stats["grows"] += 1

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
        blks = blks.to(self.device, self.dtype).contiguous()
        if keys is None:
            keys = block_hashes(blks) if self.tolerance == 0 else lsh_signatures(blks)
        keys = keys.to(self.device)
        ids = torch.empty(blks.shape[0], dtype=torch.int64, device=self.device)
        # match against the pool (binary search in the sorted keys), verify content within tolerance
        if self._n:
            sk = self._sorted_keys
            pos = torch.searchsorted(sk, keys).clamp(max=sk.numel() - 1)
            cand = self._sorted_ids[pos]
            hit = sk[pos] == keys
            if bool(hit.any()):
                hi = hit.nonzero().flatten()
                ok = block_maxdiff(self.blocks, cand[hi], blks[hi]) <= self.tolerance
                hit[hi] = ok
        else:
            cand = torch.zeros_like(ids)
            hit = torch.zeros(blks.shape[0], dtype=torch.bool, device=self.device)
        ids[hit] = cand[hit]
        new = (~hit).nonzero().flatten()
        if new.numel():
            # dedup within the incoming blocks themselves (equal keys -> the first occurrence)
            nk = keys[new]
            uk, inv = torch.unique(nk, return_inverse=True)
            first = torch.full((uk.numel(),), new.numel(), dtype=torch.int64, device=self.device)
            first.scatter_reduce_(0, inv, torch.arange(new.numel(), device=self.device), reduce="amin")
            base, k = self._n, uk.numel()
            self._reserve(base + k)
            self._buf[base: base + k].copy_(blks[new[first]])
            self._n = base + k
            new_keys = uk if self.tolerance == 0 else nk[first]
            self.keys = torch.cat([self.keys, new_keys])
            sk, order = torch.sort(torch.cat([self._sorted_keys, new_keys]), stable=True)
            self._sorted_keys = sk
            self._sorted_ids = torch.cat([self._sorted_ids,
                                          torch.arange(base, base + k, device=self.device)])[order]
            ids[new] = base + inv
        self.stats["blocks_in"] += blks.shape[0]
        self.stats["blocks_stored"] = self._n
        return ids

    def materialize(self, name: str) -> torch.Tensor:
        t = self.index.tables[name]
        R, C = self.index.shapes[name]
        blks = self.blocks.index_select(0, t.flatten().to(self.blocks.device))
        return from_blocks(blks, t.shape[0], t.shape[1], R, C)

    # ------------------------------------------------------------------ storage integration
    def store(self, client, db: str, set_name: str, blocks_per_page: int = 64, algorithm: str = "greedy1") -> Dict[int, int]:
        """Persist the distinct blocks as an FFMatrixBlock set whose pages follow the page packing (blocks
        shared by the same models land on the same pages), so each model links only the pages it uses.
        Returns {pool block id: page number}.  The set's pages go through the node's buffer pool like any
        other set (budgeted, spillable, flushed)."""
        from ..objects.builtin import FFMatrixBlock
        from ..objects.record import RecordBatch

        pages = self.pack_pages(blocks_per_page, algorithm)
        blk_bytes = self.br * self.bc * torch.empty(0, dtype=self.dtype).element_size() + 80
        big = max((len(p) for p in pages), default=1)
        page_size = int(big * blk_bytes * 16 // 15) + 8192
        if client.storage.has_set(db, set_name):
            client.remove_set(db, set_name)
        client.create_database(db)
        client.create_set(db, set_name, FFMatrixBlock, page_size=page_size)
        st = client.storage.get_set(db, set_name)
        page_of: Dict[int, int] = {}
        for pg in pages:
            ids = torch.tensor(pg, dtype=torch.int64, device=self.blocks.device)
            n = ids.numel()
            z = torch.zeros(n, dtype=torch.int64, device=ids.device)
            cols = {"block_row": z, "block_col": z.clone(),
                    "row_nums": torch.full((n,), self.br, dtype=torch.int64, device=ids.device),
                    "col_nums": torch.full((n,), self.bc, dtype=torch.int64, device=ids.device),
                    "total_rows": z.clone(), "total_cols": z.clone(), "data": self.blocks.index_select(0, ids),
                    "distinct_block_id": ids, "partition_by_col": torch.zeros(n, dtype=torch.bool, device=ids.device)}
            before = len(st.pages)
            st.add_batch(RecordBatch(cols, n, FFMatrixBlock))
            assert len(st.pages) == before + 1, "a packed page must map to exactly one storage page"
            for b in pg:
                page_of[int(b)] = before
        self.stored_pages = page_of
        return page_of

    def link_model(self, client, db: str, model_set: str, pool_set: str, name: str) -> int:
        """Make ``model_set`` read model ``name`` from the stored pool set: link exactly the pages holding
        its blocks (addSharedPage) and map each distinct block to its place(s) in the model
        (addSharedMapping).  Returns the number of pages linked."""
        from ..objects.builtin import FFMatrixBlock

        t = self.index.tables[name].cpu()
        R, C = self.index.shapes[name]
        if not client.storage.has_set(db, model_set):
            client.create_set(db, model_set, FFMatrixBlock)
        places: Dict[int, list] = {}
        for (r, c), b in zip(torch.cartesian_prod(torch.arange(t.shape[0]), torch.arange(t.shape[1])).tolist(),
                             t.flatten().tolist()):
            places.setdefault(int(b), []).append((r, c))
        pages = sorted({self.stored_pages[b] for b in places})
        for p in pages:
            client.add_shared_page(db, model_set, FFMatrixBlock, db, pool_set, FFMatrixBlock, p)
        client.add_shared_mapping(db, model_set, FFMatrixBlock, db, pool_set, FFMatrixBlock,
                                  mapping={b: v if len(v) > 1 else v[0] for b, v in places.items()},
                                  total_rows=R, total_cols=C)
        return len(pages)

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


class SharedInference:
    """Batched inference of many deduplicated models, computing each shared column block ONCE:
    ``y_m = W_m @ X^T`` for models m with identical geometry.  Column blocks whose pool ids agree across
    every model (the word2vec/text-classifier case: fine-tuned copies of one embedding table) form one
    common panel; ``P = W_common @ X_common^T`` is one MFMA GEMM for all models, and each model adds only
    its private columns' GEMM on top (``accumulate`` epilogue), so the work and the HBM traffic scale with
    the DISTINCT bytes, not with models x model size.  The reference runs FFTransposeMult + FFAggMatrix
    per model over shared pages (TestWord2VecWithDeduplication.cc:96-152) and re-reads the shared blocks
    every time."""

    def __init__(self, tables: Dict[str, torch.Tensor], shapes: Dict[str, Tuple[int, int]], fetch, br: int, bc: int):
        self.names = list(tables)
        T = torch.stack([tables[n].cpu() for n in self.names])          # [M, nbr, nbc]
        assert len({shapes[n] for n in self.names}) == 1, "SharedInference needs models of one shape"
        self.R, self.C = shapes[self.names[0]]
        self.br, self.bc = br, bc
        self.nbr, self.nbc = T.shape[1], T.shape[2]
        common = (T == T[0:1]).all(0).all(0)                              # [nbc]
        self.common_cols = common.nonzero().flatten()
        self.priv_cols = (~common).nonzero().flatten()

        def panel(t: torch.Tensor, cols: torch.Tensor) -> torch.Tensor:
            ids = t[:, cols].flatten()
            blks = fetch(ids)                                              # [nbr*len(cols), br, bc]
            return from_blocks(blks, self.nbr, cols.numel(), self.nbr * br, cols.numel() * bc).contiguous()

        self.w_common = panel(T[0], self.common_cols) if self.common_cols.numel() else None
        # private panels stacked [M, R, kp]: every model's private columns scored by ONE batched GEMM
        self.w_priv = torch.stack([panel(T[i], self.priv_cols) for i in range(len(self.names))]) \
            if self.priv_cols.numel() else None
        dev = (self.w_common if self.w_common is not None else self.w_priv).device
        self.common_runs = _runs(self.common_cols.tolist())
        self.priv_runs = _runs(self.priv_cols.tolist())
        self.common_cols, self.priv_cols = self.common_cols.to(dev), self.priv_cols.to(dev)

    def panel_bytes(self) -> int:
        ps = [p for p in (self.w_common, self.w_priv) if p is not None]
        return sum(p.numel() * p.element_size() for p in ps)

    def _xpart(self, X: torch.Tensor, cols: torch.Tensor, runs) -> list:
        """(panel column offset, X column block view) per contiguous run of column blocks: zero-copy strided
        views of X (the GEMM takes any K-contiguous row stride); many short runs fall back to one gather."""
        if len(runs) <= 4:
            out, off = [], 0
            for c0, c1 in runs:
                out.append((off, X[:, c0 * self.bc: c1 * self.bc]))
                off += (c1 - c0) * self.bc
            return out
        g = X.reshape(X.shape[0], self.nbc, self.bc).index_select(1, cols).reshape(X.shape[0], -1).contiguous()
        return [(0, g)]

    def run(self, X: torch.Tensor) -> Dict[str, torch.Tensor]:
        """X [B, C] -> {model: [R, B] f32} (rows beyond R of the padded row blocks dropped)."""
        from .. import ops

        ref = self.w_common if self.w_common is not None else self.w_priv
        X = X.to(ref.dtype)
        if X.shape[1] != self.nbc * self.bc:
            X = torch.nn.functional.pad(X, (0, self.nbc * self.bc - X.shape[1]))
        side = None
        if self.overlap and X.is_cuda and self.w_common is not None and self.w_priv is not None:
            # private panels on a second HIP stream, launched first: it waits only for X (an event on the main
            # stream), so it runs concurrently with the common panel's GEMM enqueued next on the main stream
            main = torch.cuda.current_stream(X.device)
            side = SharedInference._side.get(X.device)
            if side is None:
                side = SharedInference._side[X.device] = torch.cuda.Stream(X.device)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                Yp = self._private(X, None)
            X.record_stream(side)
        xp = ps = None
        if (side is None and self.prefetch_x and X.is_cuda and self.w_common is not None
                and self.w_priv is not None):
            # the private columns of X compacted on a second stream while the common panel's GEMM streams its
            # weights on the main one (a 20 MB copy next to a 900 MB stream, instead of serialised between them)
            main = torch.cuda.current_stream(X.device)
            ps = SharedInference._side.get(X.device)
            if ps is None:
                ps = SharedInference._side[X.device] = torch.cuda.Stream(X.device)
            ps.wait_stream(main)
            with torch.cuda.stream(ps):
                xp = [(off, self._compact(xv)) for off, xv in self._xpart(X, self.priv_cols, self.priv_runs)]
            X.record_stream(ps)
        P = None
        if self.w_common is not None:
            for off, xv in self._xpart(X, self.common_cols, self.common_runs):
                wv = self.w_common[:, off: off + xv.shape[1]]
                P = ops.gemm_nt(wv, xv, P, ops.BIAS_MAT if P is not None else ops.BIAS_NONE, out_dtype=torch.float32)
        if self.w_priv is None:
            return {n: P[: self.R] for n in self.names}
        if side is not None:
            main.wait_stream(side)
            Yp.record_stream(main)
            Y = Yp.add_(P.unsqueeze(0))
        else:
            if xp is not None:
                main.wait_stream(ps)
                for _, xv in xp:
                    xv.record_stream(main)
            Y = self._private(X, P, xp)
        return {n: Y[i, : self.R] for i, n in enumerate(self.names)}

    # Private panels concurrent with the common panel (run(): two HIP streams), the private result joined by one
    # broadcast add instead of accumulating onto P in its epilogue. Measured slower at config 5 (interleaved, 5 x 20
    # runs: 0.492 vs 0.480 ms, profiles/r6_dedup/dedup_overlap_ab.json: both GEMMs already stream HBM with the whole
    # GPU, so running them side by side only splits the bandwidth), so it is off by default.
    overlap = False
    prefetch_x = False   # compact X's private columns on a second stream during the common GEMM (A/B: bench_dedup)
    _side: Dict[torch.device, "torch.cuda.Stream"] = {}

    @staticmethod
    def _compact(xv: torch.Tensor) -> torch.Tensor:
        # a narrow private slice of X is compacted first (a 20 MB copy; the GEMM then streams B rows 200 KB apart
        # instead of 2 MB apart: 266 vs 296 us at 12 x 500 x 100 x 100k)
        return xv.contiguous() if xv.stride(0) > 2 * xv.shape[1] else xv

    def _private(self, X: torch.Tensor, Y: Optional[torch.Tensor], parts=None) -> torch.Tensor:
        from .. import ops

        M = self.w_priv.shape[0]
        for off, xv in (parts if parts is not None else self._xpart(X, self.priv_cols, self.priv_runs)):
            wv = self.w_priv[:, :, off: off + xv.shape[1]]
            xv = self._compact(xv)
            xb = xv.unsqueeze(0).expand(M, -1, -1)            # batch stride 0: one X panel for every model
            Y = ops.gemm_nt(wv, xb, Y, ops.BIAS_MAT if Y is not None else ops.BIAS_NONE, out_dtype=torch.float32)
        return Y


def _runs(cols) -> list:
    """Sorted column-block ids -> [(start, end)) contiguous runs."""
    out = []
    for c in cols:
        if out and out[-1][1] == c:
            out[-1][1] = c + 1
        else:
            out.append([c, c + 1])
    return [tuple(r) for r in out]


def pages_touched(pool: BlockPool, pages: List[List[int]], name: str) -> int:
    page_of = {b: i for i, p in enumerate(pages) for b in p}
    return len({page_of[b] for b in pool.index.tables[name].flatten().tolist()})


__all__ = ["TensorBlockIndex", "BlockPool", "DistributedBlockPool", "block_hashes", "block_hashes_reference",
           "block_maxdiff", "SharedInference", "lsh_signatures", "to_blocks", "from_blocks", "pages_touched"]
