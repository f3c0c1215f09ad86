"""Accuracy-guarded approximate model deduplication — the detector that decides WHICH tensor blocks of a
model may be replaced by a similar block already stored for another model.

Reference: model-inference/deduplication/indexing — ``blocker.py`` (block a model's weights layer by layer,
zero-pad the edges, per-block magnitude = a quantile of the block normalised by the layer's range, larger layers
first), ``indexer.py`` (the store of candidate blocks, ``build_index`` / ``update_index``), ``lsh/l2lsh.py``
(p-stable L2 LSH for candidate retrieval) and ``deduplicator.py::deduplicate_model`` (greedy magnitude-ordered
replacement: a block's similarity to a candidate is the fraction of elements within ``fp`` of it, the best
candidate with similarity >= ``sim`` replaces it, the model is evaluated every ``eval_step`` replacements and the
pass stops once the accuracy drop exceeds ``stop_acc_drop``; optional fine-tuning of the replaced blocks).

MI355X-native design: every candidate block lives in ONE device pool ``[n, br, bc]``; the similarity of a query
block to all candidates is one HIP streaming kernel (``block_simcount``: per-candidate count of elements within
``fp`` over the query's real ``h x w`` corner, 16-B loads, many workgroups per candidate) instead of a Python loop
of numpy diffs; LSH signatures of all blocks are one GEMM against the projection matrix. The detector's output
(``report``) feeds the storage-side deduplication (``dedup.BlockPool`` / shared pages).

Unlike the reference (which only truncates its result lists), a pass that ends above the accuracy budget really
restores the blocks replaced since the last evaluation that was within budget.
"""
from __future__ import annotations

import json
import math
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import torch

Key = Tuple[int, int, int]          # (weight index, block row, block column)

_MAGNITUDE_Q = {"q1": 0.25, "q2": 0.5, "q3": 0.75, "p90": 0.90}


def _block_magnitude(blocks: torch.Tensor, how: str) -> torch.Tensor:
    """blocks: [n, elems] (real elements only) -> [n] magnitude (blocker.py compute_* functions)."""
    if how == "none":
        return torch.zeros(blocks.shape[0], dtype=torch.float64, device=blocks.device)
    x = blocks.float()
    if how == "avg":
        return x.mean(1).double()
    if how == "max":
        return x.amax(1).double()
    q = _MAGNITUDE_Q[how]
    # torch.quantile refuses very large inputs: rank-select per row instead (same linear interpolation)
    n = x.shape[1]
    pos = q * (n - 1)
    lo, hi = int(math.floor(pos)), int(math.ceil(pos))
    out = []
    for c in range(0, x.shape[0], max(1, (1 << 24) // max(1, n))):
        srt = x[c: c + max(1, (1 << 24) // max(1, n))].sort(dim=1).values
        v = srt[:, lo] + (srt[:, hi] - srt[:, lo]) * (pos - lo)
        out.append(v.double())
    return torch.cat(out)


@dataclass
class ModelStorage:
    """blocker.py's ``model_storage``: zero-padded 2-D weights + shapes, block grids and block magnitudes."""
    weights: List[torch.Tensor]
    shapes: List[Tuple[int, ...]]
    block_num: List[Tuple[int, int]]
    magnitude: Dict[Key, float]
    br: int
    bc: int

    def block(self, key: Key) -> torch.Tensor:
        w, i, j = key
        return self.weights[w][i * self.br:(i + 1) * self.br, j * self.bc:(j + 1) * self.bc]

    def real_extent(self, key: Key) -> Tuple[int, int]:
        """Rows x columns of the block's real (unpadded) part; a bias vector counts one column."""
        w, i, j = key
        shp = self.shapes[w]
        rows = shp[0]
        cols = 1 if len(shp) == 1 else shp[1]
        return min(self.br, rows - i * self.br), min(self.bc, cols - j * self.bc)

    def is_padded(self, key: Key) -> bool:
        h, w = self.real_extent(key)
        return len(self.shapes[key[0]]) == 1 and self.br * self.bc > 1 or (h, w) != (self.br, self.bc)

    def keys(self) -> List[Key]:
        return [(w, i, j) for w, (nx, ny) in enumerate(self.block_num) for i in range(nx) for j in range(ny)]


def block_model(weights: Sequence[torch.Tensor], block_rows: int, block_cols: Optional[int] = None,
                magnitude: str = "q3", norm_by_layer: bool = True, dedup_by_layer: bool = True,
                device=None) -> ModelStorage:
    """blocker.py ``block_model_2d``: every weight (1-D biases as a column) zero-padded to whole blocks; the
    block magnitude is computed on the real part, normalised by the layer's [min, max] range and, with
    ``dedup_by_layer``, shifted by -(layer size) so that sorting ascending visits the largest layer first."""
    br = block_rows
    bc = block_cols if block_cols is not None else block_rows
    out_w, shapes, nums, mags = [], [], [], {}
    for idx, w in enumerate(weights):
        w = w.detach().to(device) if device is not None else w.detach()
        shapes.append(tuple(w.shape))
        m = w.reshape(-1, 1) if w.dim() == 1 else w
        assert m.dim() == 2, "2-D weights (or 1-D biases)"
        rows, cols = m.shape
        nx, ny = math.ceil(rows / br), math.ceil(cols / bc)
        wmin, wmax = float(m.min()), float(m.max())
        rng = (wmax - wmin) or 1.0
        padded = torch.zeros(nx * br, ny * bc, dtype=m.dtype, device=m.device)
        padded[:rows, :cols] = m
        # interior blocks in one batch, edge blocks one by one (their real parts differ in size)
        fx, fy = rows // br, cols // bc
        keys_int, vals = [], []
        if fx and fy:
            blk = padded[:fx * br, :fy * bc].reshape(fx, br, fy, bc).permute(0, 2, 1, 3).reshape(fx * fy, br * bc)
            mv = _block_magnitude(blk, magnitude).tolist()
            keys_int = [(idx, i, j) for i in range(fx) for j in range(fy)]
            vals = mv
        for i in range(nx):
            for j in range(ny):
                if i < fx and j < fy:
                    continue
                real = m[i * br:(i + 1) * br, j * bc:(j + 1) * bc].reshape(1, -1)
                keys_int.append((idx, i, j))
                vals.append(float(_block_magnitude(real, magnitude)[0]))
        for k, v in zip(keys_int, vals):
            if norm_by_layer and magnitude != "none":
                v = (v - wmin) / rng
            if dedup_by_layer:
                v += -(rows * cols)
            mags[k] = v
        out_w.append(padded)
        nums.append((nx, ny))
    return ModelStorage(out_w, shapes, nums, mags, br, bc)


def reconstruct(storage: ModelStorage) -> List[torch.Tensor]:
    """blocker.py ``reconstruct_weight_2d``: the unpadded weights (biases back to 1-D)."""
    out = []
    for w, shp in zip(storage.weights, storage.shapes):
        out.append(w[:shp[0], 0].clone() if len(shp) == 1 else w[:shp[0], :shp[1]].clone())
    return out


class BlockIndexer:
    """indexer.py ``Indexer``: the candidate blocks of every indexed model in one device pool
    ``[n, br, bc]`` (capacity doubles), with (model, weight, block row, block column) ids."""

    def __init__(self, block_rows: int, block_cols: Optional[int] = None, device=None, dtype=None):
        self.br = block_rows
        self.bc = block_cols if block_cols is not None else block_rows
        self.device = device
        self.dtype = dtype
        self._pool: Optional[torch.Tensor] = None
        self.n = 0
        self.ids: List[Tuple[str, int, int, int]] = []
        self.model_names: set = set()

    @property
    def blocks(self) -> torch.Tensor:
        if self._pool is None:
            return torch.empty(0, self.br, self.bc, device=self.device, dtype=self.dtype or torch.float32)
        return self._pool[: self.n]

    def _append(self, blk: torch.Tensor, ident):
        if self._pool is None:
            dt = self.dtype or blk.dtype
            dev = self.device if self.device is not None else blk.device
            self._pool = torch.empty(16, self.br, self.bc, dtype=dt, device=dev)
        if self.n == self._pool.shape[0]:
            grown = torch.empty(2 * self.n, self.br, self.bc, dtype=self._pool.dtype, device=self._pool.device)
            grown[: self.n] = self._pool
            self._pool = grown
        self._pool[self.n] = blk
        self.ids.append(ident)
        self.n += 1

    def build_index(self, storage: ModelStorage, model_name: str) -> Dict[Key, int]:
        """Add every block of ``storage``; returns (weight, i, j) -> pool index (to exclude self matches)."""
        if model_name in self.model_names:
            raise ValueError(f"model {model_name!r} already indexed")
        assert (storage.br, storage.bc) == (self.br, self.bc), "block size mismatch"
        self.model_names.add(model_name)
        finder = {}
        for k in storage.keys():
            finder[k] = self.n
            self._append(storage.block(k), (model_name,) + k)
        return finder

    def update_index(self, storage: ModelStorage, report: List[dict], model_name: str) -> int:
        """Add the blocks of a deduplicated model that were NOT replaced (indexer.py ``update_index``)."""
        dedup = {r["duplicate_block_idx"] for r in report if r["is_deduplicated"]}
        added = 0
        for k in storage.keys():
            if k not in dedup:
                self._append(storage.block(k), (model_name,) + k)
                added += 1
        self.model_names.add(model_name)
        return added

    def save(self, path: str):
        """Blocks as safetensors + ids as JSON (no pickle)."""
        from safetensors.torch import save_file

        save_file({"blocks": self.blocks.contiguous().cpu()}, path)
        with open(path + ".json", "w") as f:
            json.dump({"br": self.br, "bc": self.bc, "ids": self.ids, "models": sorted(self.model_names)}, f)

    @staticmethod
    def load(path: str, device=None) -> "BlockIndexer":
        from safetensors.torch import load_file

        with open(path + ".json") as f:
            meta = json.load(f)
        ix = BlockIndexer(meta["br"], meta["bc"], device=device)
        blocks = load_file(path)["blocks"]
        ix._pool = blocks.to(device) if device is not None else blocks
        ix.n = blocks.shape[0]
        ix.ids = [tuple(x) for x in meta["ids"]]
        ix.model_names = set(meta["models"])
        return ix


class L2LSH:
    """lsh/l2lsh.py: p-stable LSH for the L2 distance, h(v) = floor((a . v + b) / r) with a ~ N(0, I),
    b ~ U[0, r); ``num_k`` codes concatenated per table, ``num_l`` tables. All signatures of a block set are one
    GEMM against the [num_l * num_k, dim] projection; a query's candidates are the blocks that share a bucket
    with it in at least one table."""

    def __init__(self, dim: int, r: float = 0.09, num_k: int = 1, num_l: int = 90, seed: int = 0, device=None):
        g = torch.Generator().manual_seed(seed)
        self.r, self.k, self.l = float(r), int(num_k), int(num_l)
        self.A = torch.randn(self.l * self.k, dim, generator=g).to(device)
        self.b = (torch.rand(self.l * self.k, generator=g) * self.r).to(device)
        self.sigs: Optional[torch.Tensor] = None      # [n, L] int64
        self.ids: Optional[torch.Tensor] = None

    def signatures(self, blocks: torch.Tensor) -> torch.Tensor:
        x = blocks.reshape(blocks.shape[0], -1).to(self.A.device, torch.float32)
        codes = torch.floor((x @ self.A.t() + self.b) / self.r).to(torch.int64).reshape(-1, self.l, self.k)
        h = torch.zeros(codes.shape[:2], dtype=torch.int64, device=codes.device)
        for kk in range(self.k):                       # order-aware combine of the k codes of a table
            h = h * 1000003 + codes[:, :, kk]
        return h

    def insert(self, blocks: torch.Tensor, ids: Optional[torch.Tensor] = None):
        s = self.signatures(blocks)
        i = ids if ids is not None else torch.arange(s.shape[0], device=s.device)
        self.sigs = s if self.sigs is None else torch.cat([self.sigs, s])
        self.ids = i.to(s.device) if self.ids is None else torch.cat([self.ids, i.to(s.device)])

    def query(self, block: torch.Tensor) -> torch.Tensor:
        if self.sigs is None:
            return torch.empty(0, dtype=torch.int64)
        q = self.signatures(block.reshape(1, -1))
        hit = (self.sigs == q).any(1)
        return self.ids[hit]


def similarity(pool: torch.Tensor, cand: torch.Tensor, query: torch.Tensor, h: int, w: int, fp: float) -> torch.Tensor:
    """Fraction of the query's real ``h x w`` corner within ``fp`` of each candidate block ``pool[cand]``
    (deduplicator.py's ``np.sum(|b1 - b2| <= fp) / block_cap``). GPU: the ``block_simcount`` HIP kernel."""
    if cand.numel() == 0:
        return torch.empty(0, dtype=torch.float32, device=pool.device)
    br, bc = query.shape
    if pool.is_cuda:
        from .. import _ext

        q = query.to(pool.dtype).contiguous()
        if (br * bc * pool.element_size()) % 16 == 0 and pool.dtype in (torch.float32, torch.bfloat16):
            part = _ext.hip().block_simcount_partial(pool.reshape(pool.shape[0], -1).contiguous(),
                                                     cand.to(pool.device, torch.int64).contiguous(), q.reshape(-1),
                                                     bc, h, w, float(fp))
            return part.sum(1).float() / float(max(1, h * w))
    c = pool[cand.to(pool.device)][:, :h, :w].float()
    return ((c - query[:h, :w].float()).abs() <= fp).float().mean((1, 2))


def deduplicate_model(storage: ModelStorage, indexer: BlockIndexer,
                      evaluate: Optional[Callable[[List[torch.Tensor]], float]] = None,
                      fp: float = 0.01, sim: float = 0.7, stop_acc_drop: float = 0.04, eval_step: int = 5,
                      use_lsh: bool = False, lsh: Optional[L2LSH] = None,
                      finetune: Optional[Callable[[ModelStorage, List[Key]], None]] = None, ft_step: int = 5,
                      self_index: Optional[Dict[Key, int]] = None) -> List[dict]:
    """deduplicator.py ``deduplicate_model`` on the device pool. Visits blocks by ascending magnitude (largest
    layer first with ``dedup_by_layer`` magnitudes), skips layers that are a single block, replaces a block by
    its most similar candidate when the similarity reaches ``sim``, evaluates ``evaluate(weights) -> accuracy``
    every ``eval_step`` replacements and stops once ``original - accuracy > stop_acc_drop``; a final evaluation
    above budget restores the blocks replaced after the last in-budget evaluation. ``finetune(storage, keys)``
    (optional) is called every ``ft_step`` steps with the replaced blocks. Mutates ``storage``; returns one
    report row per block (replaced or not), as deduplicator.py's result frame."""
    if use_lsh and lsh is None:
        lsh = L2LSH(indexer.br * indexer.bc, device=indexer.blocks.device)
        lsh.insert(indexer.blocks)
    pool = indexer.blocks
    all_ids = torch.arange(indexer.n, device=pool.device)
    ori_acc = evaluate(reconstruct(storage)) if evaluate is not None else None
    acc = ori_acc
    report: List[dict] = []
    replaced: List[Tuple[Key, torch.Tensor]] = []      # (key, old block) since the last in-budget evaluation
    dedup_keys: List[Key] = []
    step, last_eval_row = 1, 0
    for key, mag in sorted(storage.magnitude.items(), key=lambda kv: kv[1]):
        t0 = time.perf_counter()
        w = key[0]
        nx, ny = storage.block_num[w]
        h, wd = storage.real_extent(key)
        best, best_sim, t_search = None, 0.0, None
        if nx * ny > 1:
            ts = time.perf_counter()
            b1 = storage.block(key)
            cand = lsh.query(b1) if use_lsh else all_ids
            if self_index is not None and key in self_index:
                cand = cand[cand != self_index[key]]
            if cand.numel():
                sims = similarity(pool, cand, b1, h, wd, fp)
                i = int(torch.argmax(sims))
                s = float(sims[i])
                if s >= sim:
                    best, best_sim = int(cand[i]), s
            t_search = time.perf_counter() - ts
        t_eval = None
        if best is not None:
            blk = storage.block(key)
            replaced.append((key, blk.clone()))
            blk.copy_(pool[best].to(blk.dtype))
            dedup_keys.append(key)
            step += 1
            if evaluate is not None and step % eval_step == 0:
                te = time.perf_counter()
                acc = evaluate(reconstruct(storage))
                t_eval = time.perf_counter() - te
                step += 1
                if ori_acc - acc <= stop_acc_drop:
                    replaced.clear()
                    last_eval_row = len(report) + 1
        if finetune is not None and best is not None and step % ft_step == 0:
            finetune(storage, list(dedup_keys))
            if evaluate is not None:
                acc = evaluate(reconstruct(storage))
        report.append({"duplicate_block_idx": key, "deduplicate_block_idx": best, "block_similarity": best_sim,
                       "model_accuracy": acc, "is_padded_block": storage.is_padded(key),
                       "is_deduplicated": best is not None, "block_magnitude": mag, "search_time": t_search,
                       "eval_time": t_eval, "total_time": time.perf_counter() - t0})
        if evaluate is not None and ori_acc - acc > stop_acc_drop:
            break
    if evaluate is not None:
        acc = evaluate(reconstruct(storage))
        if ori_acc - acc > stop_acc_drop:
            for key, old in reversed(replaced):          # restore the blocks past the last in-budget state
                storage.block(key).copy_(old)
            report = report[:last_eval_row]
            for r in report[last_eval_row - 1:] if last_eval_row else []:
                r["model_accuracy"] = evaluate(reconstruct(storage))
        elif report:
            report[-1]["model_accuracy"] = acc
    seen = {r["duplicate_block_idx"] for r in report}
    for key in storage.keys():
        if key not in seen:
            report.append({"duplicate_block_idx": key, "deduplicate_block_idx": None, "block_similarity": None,
                           "model_accuracy": None, "is_padded_block": storage.is_padded(key),
                           "is_deduplicated": False, "block_magnitude": storage.magnitude.get(key),
                           "search_time": None, "eval_time": None, "total_time": None})
    return report


def dedup_summary(report: List[dict]) -> dict:
    n = len(report)
    d = sum(1 for r in report if r["is_deduplicated"])
    return {"blocks": n, "deduplicated": d, "ratio": d / n if n else 0.0}
