"""Tensor-pattern fusion: lower join+aggregate block-matrix chains onto fused MFMA kernels.

netsDB expresses a matrix multiply as JoinComp(A.blockCol == B.blockCol, project A·Bᵀ) +
ClusterAggregateComp(sum by output block) (src/FF/headers/FFTransposeMult.h + FFAggMatrix.h;
src/sharedLibraries/headers/LASillyMultiply1Join.h + LASillyMultiply2Aggregate.h) and an
activation as another join with the bias set (FFReluBiasSum, FFTransposeBiasSum).  Executed
literally that is one small GEMM per block pair, a hash aggregation of partial blocks, and one
more pass per epilogue.

When the computations declare their tensor pattern (``tensor_pattern()``) and the operands are
dense matrix sets, this pass rewrites the chain into nodes evaluated on the dense HBM panels:
:class:`MatmulNode` = ONE split-K MFMA GEMM (the split-K slab reducer *is* the block aggregate)
with bias/act/dropout fused in the epilogue; softmax/row-normalise, elementwise, transpose
(a layout flag flip, no data movement), reductions, inverse and duplication nodes.  Operand
orientation is chosen per node so every GEMM reads both operands K-contiguous with no transposes.

Distribution (one rank per GPU): a matrix value is replicated or partitioned by logical rows or
columns.  Row-split A against K-split B (both sets row-partitioned, the LA DSL's ``A %*% B``) runs
as an N-chunked pipeline: B^T chunks are all-gathered over RCCL (all xGMI links) while the previous
chunk's full-K GEMM writes its column block of C in place.  A K-split product (``A '* B``, or one
side replicated) multiplies each rank's K range into an f32 partial and reduce-scatters it —
netsDB's hash-partitioned join + shuffle-aggregate of partial blocks, as collectives.

Everything not matched runs through the generic TCAP pipeline; fused results feeding generic
computations are materialised into temp dense sets.
"""
from __future__ import annotations

import itertools
from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist

from .. import ops
from ..computations import (AggregateComp, BiasAct, BlockMatmul, BlockSum, CellUpdate, Computation, Duplicate,
                            Elementwise, GateSum, HiddenOut, Inverse, JoinComp, MultiSelectionComp, Reduce, RowSoftmax,
                            ScanSet, Scale, SelectionComp, Transpose, WriteSet)
from ..storage.sets import DenseMatrixSet

_tmp_ids = itertools.count()


class Dense:
    """A logical matrix value: physical 2-D tensor + 'transposed' flag + distribution.

    ``rows``/``cols`` are the LOCAL logical extents; ``part`` is None (replicated), 'rows' or 'cols'
    (the logical dimension split over ranks, ``offset`` = first global index held here,
    ``total`` = global extent of that dimension)."""

    def __init__(self, phys: Optional[torch.Tensor], rows: int, cols: int, transposed: bool, br: int, bc: int,
                 part: Optional[str] = None, offset: int = 0, total: Optional[int] = None, src=None):
        self._phys, self.rows, self.cols, self.transposed = phys, rows, cols, transposed
        self.br, self.bc = br, bc
        self.part, self.offset = part, offset
        self.total = total if total is not None else (rows if part == "rows" else cols if part == "cols" else 0)
        self.src = src            # the DenseMatrixSet behind a scanned value (panel fetched on first use)

    @property
    def phys(self) -> torch.Tensor:
        if self._phys is None and self.src is not None:
            return self.src.panel          # reloads a spilled panel; not cached: the set may evict it again
        return self._phys

    @phys.setter
    def phys(self, t):
        self._phys = t

    def physical(self, want_transposed: bool) -> torch.Tensor:
        """K-contiguous physical layout in the wanted orientation (copy only on mismatch)."""
        if want_transposed == self.transposed:
            p = self.phys
        else:
            r, c = (self.cols, self.rows) if self.transposed else (self.rows, self.cols)
            p = self.phys[:r, :c].t().contiguous()
        if p.shape[1] % 8 or p.stride(0) % 8 or p.stride(1) != 1:
            p = ops.pad_k(p.contiguous())
        return p

    def logical(self) -> torch.Tensor:
        if self.transposed:
            return self.phys[: self.cols, : self.rows].t()
        return self.phys[: self.rows, : self.cols]

    def t(self) -> "Dense":
        part = {"rows": "cols", "cols": "rows"}.get(self.part) if self.part else None
        return Dense(self._phys, self.cols, self.rows, not self.transposed, self.bc, self.br, part, self.offset,
                     self.total, self.src)

    @staticmethod
    def of(t: torch.Tensor, br: int, bc: int, part=None, offset=0, total=None) -> "Dense":
        phys = t if (t.shape[1] % 8 == 0 and t.stride(1) == 1) else ops.pad_k(t.contiguous())
        return Dense(phys, t.shape[0], t.shape[1], False, br, bc, part, offset, total)


def _kslice(t: torch.Tensor, rows: int, k8: int) -> torch.Tensor:
    """[rows, k8] view of a zero-padded physical panel (pads with zeros when it is narrower)."""
    t = t[:rows]
    if t.shape[1] < k8:
        t = torch.nn.functional.pad(t, (0, k8 - t.shape[1]))
    return t[:, :k8]


def _replicate(engine, d: Dense) -> Dense:
    """All-gather a partitioned value along its split dimension (broadcast-join build side)."""
    ctx = engine.ctx
    if d.part is None or not ctx.distributed:
        return d
    L = d.logical()
    if d.part == "rows":
        full = torch.cat(ctx.all_gather_tensor(L.contiguous()))
    else:
        full = torch.cat(ctx.all_gather_tensor(L.t().contiguous())).t()
    return Dense.of(full.contiguous(), d.br, d.bc)


class Node:
    consumers_want_t: Optional[bool] = None
    value: Optional[Dense] = None
    uses: int = 0              # graph consumers (the fused softmax needs its GEMM to have exactly one)


class SourceNode(Node):
    def __init__(self, uset: DenseMatrixSet):
        self.set = uset

    def eval(self, engine) -> Dense:
        s = self.set
        if self.value is None:
            part = None if (s.replicated or not engine.ctx.distributed) else "rows"
            self.value = Dense(None, s.local_rows, s.total_cols, s.transposed, s.block_rows, s.block_cols,
                               part, s.row_offset, s.total_rows, src=s)
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
        self.fuse_softmax = False      # set by the only consumer, a SoftmaxNode: normalise in the epilogue
        self.softmax_fused = False     # the value holds softmax(scores), not exp(scores)

    def eval(self, engine) -> Dense:
        if self.value is not None:
            return self.value
        armed = self._arm_operand_prefetch(engine)
        try:
            A, B = self.a.eval(engine), self.b.eval(engine)
        finally:
            if armed is not None:
                from ..execution.streams import disarm_operand_prefetch

                disarm_operand_prefetch(armed)
        return self._eval(engine, A, B)

    def _prefetch_weight(self, engine):
        """The stored weight operand of a GEMM whose other operand comes out of a GEMM evaluated first (the FF
        output layer after layer 1), when it is worth warming (on the GPU, >= 4 MiB); else None."""
        srcs = [c for c in (self.a, self.b) if isinstance(c, SourceNode)]
        heavy = [c for c in (self.a, self.b) if isinstance(c, (MatmulNode, BiasActNode, EwiseNode))]
        if len(srcs) != 1 or len(heavy) != 1 or heavy[0].value is not None:
            return None
        try:
            w = srcs[0].eval(engine).phys
        except Exception:
            return None
        if not isinstance(w, torch.Tensor) or not w.is_cuda or w.numel() * w.element_size() < (4 << 20):
            return None
        return w

    def _arm_operand_prefetch(self, engine):
        """In-kernel operand prefetch (engine option ``operand_prefetch``, default on): the weight is armed on the
        current stream, and the first long 8-phase GEMM launched while the children are evaluated (layer 1)
        reads it into the Infinity Cache with its workgroups as they finish (ops.gemm_nt). Returns the device to
        disarm, or None."""
        if not getattr(engine, "operand_prefetch", False):
            return None
        w = self._prefetch_weight(engine)
        if w is None:
            return None
        from ..execution.streams import arm_operand_prefetch

        return w.device if arm_operand_prefetch(w) else None

    def _eval(self, engine, A: Dense, B: Dense) -> Dense:
        opA = A.t() if self.p.transpose_a else A           # [M, K]
        opB = B.t() if self.p.transpose_b else B           # [K, N]
        # distribution (one rank per GPU): M-split A / N-split B are local; a K-split of B against
        # row-split A runs the N-chunked all-gather pipeline; K-split partial products are
        # reduce-scattered (netsDB's shuffle aggregation of partial blocks)
        dist_mode = "local"
        if engine.ctx.distributed:
            if opA.part == "cols" and opB.part == "cols":
                opA = _replicate(engine, opA)
            if opA.part == "rows" and opB.part == "cols":
                opB = _replicate(engine, opB)
            if opA.part == "rows" and opB.part == "rows":
                dist_mode = "allgather_n"
            elif opA.part == "cols" or opB.part == "rows":
                dist_mode = "kpartial"
        if dist_mode != "local":
            ds = engine.__dict__.setdefault("dist_stats", {})
            ds[dist_mode] = ds.get(dist_mode, 0) + 1
        M, K, N = opA.rows, opA.cols, opB.cols
        if dist_mode == "local" and K != opB.rows:
            raise ValueError(f"fused matmul K mismatch {K} vs {opB.rows}")
        want_t = bool(self.consumers_want_t)
        phys_is_c = self.transpose_out == want_t
        bias_t, mode = None, ops.BIAS_NONE
        if self.bias is not None:
            bias_t = ops.derived(_replicate(engine, self.bias.eval(engine)).logical(), "bias_f32",
                                 lambda t: t.reshape(-1).float().contiguous())
            along_c_rows = self.bias_along == "row"
            if opA.part == "rows" and along_c_rows:
                bias_t = bias_t[opA.offset: opA.offset + M]
            if opB.part == "cols" and not along_c_rows:
                bias_t = bias_t[opB.offset: opB.offset + N]
            mode = (ops.BIAS_ROW if along_c_rows else ops.BIAS_COL) if phys_is_c else \
                (ops.BIAS_COL if along_c_rows else ops.BIAS_ROW)
        act = ops.act_code(self.act)
        # exp'd scores keep f32 (exact row normalisation); f32 operands keep an f32 result
        odt = torch.float32 if (act == ops.ACT_EXP or opA.phys.dtype == torch.float32
                                or opB.phys.dtype == torch.float32) else torch.bfloat16
        if dist_mode == "allgather_n":
            phys = self._allgather_n(engine, opA, opB, M, N, phys_is_c, bias_t, mode, act, odt)
        elif dist_mode == "kpartial":
            value = self._kpartial(engine, opA, opB, M, N, phys_is_c, bias_t, act, odt)
            self.value = value
            return value
        elif self._out_of_core(engine, opA, opB, M, N, K, odt):
            phys = self._ooc_matmul(engine, opA, opB, M, N, K, phys_is_c, bias_t, mode, act, odt)
        else:
            K8 = (K + 7) // 8 * 8
            # X = opA as [M,K] K-contig <=> opA physical not transposed; Y = opB^T as [N,K]
            X = _kslice(opA.physical(False), M, K8)
            Y = _kslice(opB.physical(True), N, K8)
            # result rows padded to 64 elements (128-B aligned for bf16): a consumer GEMM's LDS-DMA then
            # moves whole cache lines per row segment (1000-wide bf16 rows straddle lines: +12% on the FF
            # output layer); consumers read the [rows, cols] view, the padding is never touched
            pr, pc = (M, N) if phys_is_c else (N, M)
            out = None
            if X.is_cuda and pc % 64 and pc >= 64:
                out = torch.empty(pr, (pc + 63) // 64 * 64, dtype=odt, device=X.device)[:, :pc]
            if self.fuse_softmax and act == ops.ACT_EXP and self.dropout == 0.0 and mode != ops.BIAS_MAT \
                    and X.is_cuda:
                # exp(scores + b) / rowsum over the rows of this node's LOGICAL value (C, or C^T when
                # transpose_out): the rows of phys when phys holds that value, else its columns
                axis = 1 if phys_is_c != self.transpose_out else 2
                phys = ops.gemm_nt_softmax(X, Y, bias_t, mode, axis=axis, out=out) if phys_is_c else \
                    ops.gemm_nt_softmax(Y, X, bias_t, mode, axis=axis, out=out)
                self.softmax_fused = True
            elif phys_is_c:
                phys = ops.gemm_nt(X, Y, bias_t, mode, act, out_dtype=odt, dropout=self.dropout, seed=self.seed,
                                   out=out)
            else:
                phys = ops.gemm_nt(Y, X, bias_t, mode, act, out_dtype=odt, dropout=self.dropout, seed=self.seed,
                                   out=out)
        part, offset, total = None, 0, None
        if opA.part == "rows":
            part, offset, total = "rows", opA.offset, opA.total
        elif opB.part == "cols":
            part, offset, total = "cols", opB.offset, opB.total
        br, bc = opA.br, opB.bc
        if self.transpose_out:
            value = Dense(phys, N, M, want_t, bc, br, {"rows": "cols", "cols": "rows"}.get(part), offset, total)
        else:
            value = Dense(phys, M, N, want_t, br, bc, part, offset, total)
        self.value = value
        return value

    # ---------------------------------------------------------------- out-of-core block GEMM
    @staticmethod
    def _out_of_core(engine, opA: Dense, opB: Dense, M, N, K, odt) -> bool:
        """Both operands are stored dense sets whose panels are the GEMM's [rows, K] operands and they do
        not fit the device budget together with the result: run the block GEMM slab by slab."""
        sa, sb = opA.src, opB.src
        if sa is None or sb is None or opA.transposed or not opB.transposed or sa is sb:
            return False
        mgr = engine.storage
        out_b = M * N * torch.empty(0, dtype=odt).element_size()
        return sa.panel_nbytes() + sb.panel_nbytes() + out_b > mgr.device_budget

    def _ooc_matmul(self, engine, opA: Dense, opB: Dense, M, N, K, phys_is_c, bias_t, mode, act, odt):
        """netsDB's block-matmul join executed out of core: row slabs of the two operand panels are loaded
        (from HBM when resident, else from the pinned host tier / page pool they were evicted to) so that
        two slabs + the result stay within the device budget; each slab pair is one fused MFMA GEMM
        writing its block of C in place (PipelineStage over spilled pages, PartitionedHashSet-style
        bounded working set). Dropout masks are drawn per slab pair (seeded by its position)."""
        sa, sb = opA.src, opB.src
        mgr = engine.storage
        dev = mgr.home
        K8 = (K + 7) // 8 * 8
        pr, pc = (M, N) if phys_is_c else (N, M)
        out = torch.empty(pr, pc, dtype=odt, device=dev)
        out_b = out.numel() * out.element_size()
        mgr.account_bytes(out_b, dev)
        # make room: spill every evictable panel/page (the operands included: their slabs stream back)
        mgr.evict(mgr.device_bytes)
        row_b = max(sa.row_bytes(), sb.row_bytes())
        avail = max(mgr.available(), 2 * 16 * row_b)
        slab = max(16, min(max(M, N), avail // (2 * row_b)))
        slab = slab // 16 * 16 if slab >= 32 else slab
        sa_rows = min(M, slab)
        sb_rows = min(N, slab)
        nblk = 0
        for a0 in range(0, M, sa_rows):
            a1 = min(M, a0 + sa_rows)
            Xa = sa.load_rows(a0, a1, dev)
            xb = Xa.numel() * Xa.element_size()
            mgr.account_bytes(xb, dev)
            Xa = _kslice(Xa, a1 - a0, K8)
            for b0 in range(0, N, sb_rows):
                b1 = min(N, b0 + sb_rows)
                Yb = sb.load_rows(b0, b1, dev)
                yb = Yb.numel() * Yb.element_size()
                mgr.account_bytes(yb, dev)
                Yb = _kslice(Yb, b1 - b0, K8)
                seed = self.seed + 0x9E3779B1 * (nblk + 1)
                if phys_is_c:
                    b = None if bias_t is None else (bias_t[a0:a1] if mode == ops.BIAS_ROW else bias_t[b0:b1])
                    ops.gemm_nt(Xa, Yb, b, mode, act, out_dtype=odt, dropout=self.dropout, seed=seed,
                                out=out[a0:a1, b0:b1])
                else:
                    b = None if bias_t is None else (bias_t[b0:b1] if mode == ops.BIAS_ROW else bias_t[a0:a1])
                    ops.gemm_nt(Yb, Xa, b, mode, act, out_dtype=odt, dropout=self.dropout, seed=seed,
                                out=out[b0:b1, a0:a1])
                del Yb
                mgr.release_bytes(yb, dev)
                nblk += 1
            del Xa
            mgr.release_bytes(xb, dev)
        mgr.release_bytes(out_b, dev)          # re-charged when the result is installed in its set
        st = getattr(engine, "ooc_stats", None)
        if st is not None:
            st["ooc_matmuls"] = st.get("ooc_matmuls", 0) + 1
            st["ooc_slab_pairs"] = st.get("ooc_slab_pairs", 0) + nblk
        return out

    def _allgather_n(self, engine, opA: Dense, opB: Dense, M, N, phys_is_c, bias_t, mode, act, odt):
        """Row-split A [M_r, K] x K-split B (rank s holds rows K_s of B): every rank needs all of B.

        B^T is all-gathered in N-chunks over RCCL (one collective per chunk uses every xGMI link of
        the node, unlike a neighbour ring that is bound by one link) on the communication stream while
        the previous chunk's full-K MFMA GEMM runs: C_r[:, n0:n1] = epi(A_r . B[:, n0:n1]) written in
        place.  The gathered chunk [ws, nc, kseg] is consumed IN PLACE by the K-segmented GEMM (each
        rank's K slab is one segment; no permute/reshape copy), and A's columns are laid out once as
        the matching [M, ws * kseg] panel (cached).  The ranks' K ranges are plan metadata: gathered
        once per (set, geometry) over the host metadata group and cached — no per-call collective and
        no device->host sync."""
        ctx = engine.ctx
        ws = ctx.world_size
        cd = ctx._comm_device()
        key = ("kranges", id(opB.src) if opB.src is not None else None, opB.offset, opB.rows, ws)
        cache = engine.__dict__.setdefault("meta_cache", {})
        ranges = cache.get(key) if opB.src is not None else None
        if ranges is None:
            ranges = [tuple(r) for r in ctx.all_gather_ints([opB.offset, opB.rows])]
            if opB.src is not None:
                cache[key] = ranges
        kseg = max(64, (max(k for _, k in ranges) + 63) // 64 * 64)
        A_full = opA.physical(False)                         # [M, >= K_total]: local rows, all K
        dev = A_full.device

        def lay_out(a):
            out = torch.zeros(M, ws * kseg, dtype=a.dtype, device=a.device)
            for s_, (off, k) in enumerate(ranges):
                out[:, s_ * kseg: s_ * kseg + k] = a[:M, off: off + k]
            return out

        A_use = ops.derived(A_full, f"kseg_layout:{kseg}:{ranges}", lay_out)
        Bt = opB.physical(True)[:N, : opB.rows]               # [N, K_r] K-contiguous
        if Bt.shape[1] != kseg or not Bt.is_contiguous():
            Bt = torch.nn.functional.pad(Bt, (0, kseg - Bt.shape[1])).contiguous()
        # chunk N: ~8 chunks of >= 1024 columns (multiples of 256 = whole GEMM tiles)
        nchunks = max(1, min(8, N // 1024))
        step = (N + nchunks - 1) // nchunks
        step = (step + 255) // 256 * 256
        bounds = [(n0, min(N, n0 + step)) for n0 in range(0, N, step)]
        out = torch.empty((M, N) if phys_is_c else (N, M), dtype=odt, device=dev)
        nccl = ctx.tensor_collectives            # one [ws, nc, kseg] buffer (RCCL's form; gloo too)

        def start(c):
            n0, n1 = bounds[c]
            src = Bt[n0:n1].to(cd).contiguous()
            if ctx.health is not None:
                ctx.health.check()
            ctx.stats["collectives"] += 1
            ctx._account("all_gather", src)
            if nccl:
                # concatenated form [ws * nc, kseg] (every backend accepts it; viewed as [ws, nc, kseg] below)
                dst = torch.empty(ws * (n1 - n0), kseg, dtype=src.dtype, device=cd)
                return dst, dist.all_gather_into_tensor(dst, src, async_op=True)
            parts = [torch.empty_like(src) for _ in range(ws)]
            return parts, dist.all_gather(parts, src, async_op=True)

        pending = start(0)
        for c, (n0, n1) in enumerate(bounds):
            got, work = pending
            if c + 1 < len(bounds):
                pending = start(c + 1)        # next chunk's collective overlaps this chunk's GEMM
            ctx._wait(work)
            g = got.view(ws, n1 - n0, kseg) if nccl else torch.stack(got)   # [ws, nc, kseg]: rank s's K slab
            g = g.to(dev)
            b = None
            if bias_t is not None:
                b = bias_t[n0:n1] if (mode == ops.BIAS_COL) == phys_is_c else bias_t
            seed = self.seed + c * 0x9E3779B1
            if phys_is_c:
                ops.gemm_nt_segmented(A_use, g, b, mode, act, out_dtype=odt, dropout=self.dropout, seed=seed,
                                      out=out[:, n0:n1])
            else:
                # C^T chunk = (A . Bchunk^T)^T: the segmented operand must be B, so transpose the small result
                mode_t = {ops.BIAS_ROW: ops.BIAS_COL, ops.BIAS_COL: ops.BIAS_ROW}.get(mode, mode)
                r = ops.gemm_nt_segmented(A_use, g, b, mode_t, act, out_dtype=odt, dropout=self.dropout, seed=seed)
                out[n0:n1].copy_(r.t())
        return out

    def _kpartial_overlapped(self, engine, X, Y, phys_is_c, R, Ccols, counts, eq):
        """Σ_ranks (X . Y^T) (or Y . X^T), reduce-scattered by rows, in column chunks: the chunk-c partial
        [ws * eq, cw] f32 is written by the MFMA GEMM straight into the collective's send buffer (rows past R
        zeroed once), its reduce-scatter is issued asynchronously (RCCL runs it on its own stream) and the
        GEMM of chunk c+1 runs meanwhile. At most two chunk partials are alive at any time (the one reducing
        and the one being computed) instead of one f32 partial of the whole [R, Ccols] output (the LA
        DSL's 64k x 64k K-split product: 16 GiB per rank before). Reference pattern:
        src/sharedLibraries/headers/LASillyMultiply1Join.h + LASillyMultiply2Aggregate.h (per-block partial
        products aggregated by key), realised as GEMM + reduce-scatter on the node's xGMI links."""
        ctx = engine.ctx
        ws, r = ctx.world_size, ctx.rank
        dev = X.device
        cd = ctx._comm_device()
        loc = torch.empty(counts[r], Ccols, dtype=torch.float32, device=dev)
        chunks = _kpartial_chunks(Ccols)
        st = engine.__dict__.setdefault("ooc_stats", {})
        live = {"bytes": 0, "peak": 0}

        def alloc(nbytes):
            live["bytes"] += nbytes
            live["peak"] = max(live["peak"], live["bytes"])

        def start(c0, c1):
            cw = c1 - c0
            P = torch.empty(ws * eq, cw, dtype=torch.float32, device=dev)
            alloc(P.numel() * 4)
            if ws * eq > R:
                P[R:].zero_()
            if phys_is_c:
                ops.gemm_nt(X, Y[c0:c1], out_dtype=torch.float32, out=P[:R])
            else:
                ops.gemm_nt(Y, X[c0:c1], out_dtype=torch.float32, out=P[:R])
            src = P.to(cd)
            if ctx.health is not None:
                ctx.health.check()
                ctx.health.mark_progress()
            ctx.stats["collectives"] += 1
            ctx._account("reduce_scatter" if ctx.tensor_collectives else "all_reduce", src)
            if ctx.tensor_collectives:
                out = torch.empty(eq, cw, dtype=torch.float32, device=cd)
                work = dist.reduce_scatter_tensor(out, src, op=dist.ReduceOp.SUM, async_op=True)
            else:
                out = src
                work = dist.all_reduce(src, async_op=True)
            return P, out, work

        def finish(c0, c1, P, out, work):
            ctx._wait(work)
            got = out[: counts[r]] if ctx.tensor_collectives else out[r * eq: r * eq + counts[r]]
            loc[:, c0:c1].copy_(got.to(dev))
            live["bytes"] -= P.numel() * 4

        pending = None
        for c0, c1 in chunks:
            nxt = (c0, c1) + start(c0, c1)          # this chunk's GEMM overlaps the previous reduce-scatter
            if pending is not None:
                finish(*pending)
            pending = nxt
        if pending is not None:
            finish(*pending)
        st["kpartial_chunks"] = st.get("kpartial_chunks", 0) + len(chunks)
        st["kpartial_peak_partial_bytes"] = max(st.get("kpartial_peak_partial_bytes", 0), live["peak"])
        st["kpartial_full_partial_bytes"] = max(st.get("kpartial_full_partial_bytes", 0), ws * eq * Ccols * 4)
        return loc

    def _kpartial(self, engine, opA: Dense, opB: Dense, M, N, phys_is_c, bias_t, act, odt) -> Dense:
        """K-split product: each rank multiplies the K range it holds (A's column slab and/or B's row
        slab, slicing the replicated operand to that range) into f32 partials of the output, and
        reduce-scatter sums them so each rank keeps its block-row range of C (C^T when the consumer wants
        the transposed layout) — then the epilogue runs on the local slice. The partial is produced and
        reduced in column chunks, pipelined (:meth:`_kpartial_overlapped`). The K-range agreement is cached
        plan metadata."""
        ctx = engine.ctx
        ws, r = ctx.world_size, ctx.rank
        if opA.part == "cols" and opB.part == "rows":
            cache = engine.__dict__.setdefault("meta_cache", {})
            key = ("kpart", id(opA.src), id(opB.src), opA.offset, opA.cols, opB.offset, opB.rows, ws)
            same = cache.get(key) if (opA.src is not None and opB.src is not None) else None
            if same is None:
                rows = ctx.all_gather_ints([opA.offset, opA.cols, opB.offset, opB.rows])
                same = all(x[0] == x[2] and x[1] == x[3] for x in rows)
                if opA.src is not None and opB.src is not None:
                    cache[key] = same
            if not same:
                opA = _replicate(engine, opA)
        if opA.part == "cols":
            k0, kn = opA.offset, opA.cols
        else:
            k0, kn = opB.offset, opB.rows
        kn8 = (kn + 7) // 8 * 8
        A_loc = opA.physical(False)
        Bt_loc = opB.physical(True)
        a0 = 0 if opA.part == "cols" else k0
        b0 = 0 if opB.part == "rows" else k0
        X = A_loc[:M, a0: a0 + kn]
        Y = Bt_loc[:N, b0: b0 + kn]
        if kn8 != kn or a0 % 8 or b0 % 8:
            X = torch.nn.functional.pad(X, (0, kn8 - kn)).contiguous()
            Y = torch.nn.functional.pad(Y, (0, kn8 - kn)).contiguous()
        R, Ccols = (M, N) if phys_is_c else (N, M)
        blk = max(1, opA.br if phys_is_c else opB.bc)
        nb = (R + blk - 1) // blk
        per = (nb + ws - 1) // ws
        counts = [max(0, min(R, (s + 1) * per * blk) - min(R, s * per * blk)) for s in range(ws)]
        off = min(R, r * per * blk)
        loc = self._kpartial_overlapped(engine, X, Y, phys_is_c, R, Ccols, counts, per * blk)
        # epilogue on the local rows: bias along C rows (phys rows when phys_is_c) is sliced by offset
        along_phys_rows = (self.bias_along == "row") == phys_is_c
        b = None
        if bias_t is not None:
            b = bias_t[off: off + counts[r]] if along_phys_rows else bias_t
        y = ops.bias_act(loc.contiguous(), b, ops.BIAS_ROW if along_phys_rows else ops.BIAS_COL, act, self.dropout,
                         self.seed + r, out_dtype=odt)
        br, bc = opA.br, opB.bc
        total = R
        if phys_is_c:      # phys = C rows [off, off+cnt) -> logical C row-partitioned
            part = "rows"
            if self.transpose_out:
                return Dense(y, N, counts[r], True, bc, br, "cols", off, total)
            return Dense(y, counts[r], N, False, br, bc, part, off, total)
        # phys = C^T rows = C columns [off, off+cnt)
        if self.transpose_out:
            return Dense(y, counts[r], M, False, bc, br, "rows", off, total)
        return Dense(y, M, counts[r], True, br, bc, "cols", off, total)


def _kpartial_chunks(ccols: int, target: int = 8):
    """Column chunks of the K-split partial: ~``target`` chunks of whole 256-column GEMM tiles."""
    if ccols <= 256:
        return [(0, ccols)]
    step = max(256, ((ccols + target - 1) // target + 255) // 256 * 256)
    return [(c0, min(ccols, c0 + step)) for c0 in range(0, ccols, step)]


class SoftmaxNode(Node):
    """RowAggregate(sum) + OutputLayer(divide) over exp'd scores == row normalisation."""

    def __init__(self, x: Node):
        self.x = x
        self.notes: Optional[List[str]] = None     # the fuser's fused-op list (records the epilogue fusion)

    def eval(self, engine) -> Dense:
        if self.value is None:
            self.x.consumers_want_t = False
            if isinstance(self.x, MatmulNode) and self.x.value is None and self.x.uses == 1 and self.x.act == "exp":
                self.x.fuse_softmax = True
            X = self.x.eval(engine)
            if getattr(self.x, "softmax_fused", False):
                self.value = X                      # normalised inside the GEMM epilogue
                if self.notes is not None:
                    self.notes.append("softmax_epilogue[gemm]")
                return self.value
            if X.part == "cols":
                X = _replicate(engine, X)
            # row-normalise reads any row stride: no K-padding copy of the [rows, labels] scores
            phys = X.phys[: X.rows, : X.cols] if not X.transposed else X.logical().contiguous()
            if phys.stride(-1) != 1:
                phys = phys.contiguous()
            y = ops.row_normalize(phys, out_dtype=torch.float32)
            self.value = Dense(y, X.rows, X.cols, False, X.br, X.bc, X.part, X.offset, X.total)
        return self.value


class BiasActNode(Node):
    """Stand-alone epilogue (input not a fresh GEMM)."""

    def __init__(self, x: Node, bias: Node, pat: BiasAct):
        self.x, self.bias, self.p = x, bias, pat

    def eval(self, engine) -> Dense:
        if self.value is None:
            self.x.consumers_want_t = False
            X = self.x.eval(engine)
            b = _replicate(engine, self.bias.eval(engine)).logical().reshape(-1).float().contiguous()
            if X.part == "rows" and self.p.bias_along == "row":
                b = b[X.offset: X.offset + X.rows]
            if X.part == "cols" and self.p.bias_along != "row":
                b = b[X.offset: X.offset + X.cols]
            phys = X.physical(False)[: X.rows, : X.cols].contiguous()
            mode = ops.BIAS_ROW if self.p.bias_along == "row" else ops.BIAS_COL
            y = ops.bias_act(phys, b, mode, ops.act_code(self.p.act), self.p.dropout, self.p.seed)
            v = Dense.of(y, X.br, X.bc, X.part, X.offset, X.total)
            self.value = v.t() if self.p.transpose_out else v
        return self.value


class EwiseNode(Node):
    _OPS = {"add": torch.add, "sub": torch.sub, "mul": torch.mul, "div": torch.div}

    def __init__(self, a: Node, b: Node, op: str):
        self.a, self.b, self.op = a, b, op

    def eval(self, engine) -> Dense:
        if self.value is None:
            A, B = self.a.eval(engine), self.b.eval(engine)
            if A.part != B.part or A.offset != B.offset:
                A, B = _replicate(engine, A), _replicate(engine, B)
            y = self._OPS[self.op](A.logical().float(), B.logical().float()).to(torch.bfloat16)
            self.value = Dense.of(y.contiguous(), A.br, A.bc, A.part, A.offset, A.total)
        return self.value


# --------------------------------------------------------------------------------------- LSTM (src/LSTM)
_KCAT: Dict[tuple, torch.Tensor] = {}


def _kcat(parts: List[torch.Tensor], cache: bool) -> torch.Tensor:
    """Concatenate K-contiguous [rows, K_i] operands along K (each K_i padded to 8). Weight panels are
    concatenated once and reused while none of them is written (keyed by storage + version)."""
    key = tuple((p.data_ptr(), p._version, tuple(p.shape), tuple(p.stride())) for p in parts) if cache else None
    if key is not None and key in _KCAT:
        return _KCAT[key]
    out = torch.cat([ops.pad_k(p) for p in parts], 1).contiguous()
    if key is not None:
        if len(_KCAT) > 64:
            _KCAT.clear()
        _KCAT[key] = out
    return out


def _is_plain_matmul(n) -> bool:
    return isinstance(n, MatmulNode) and n.bias is None and n.act == "none" and not n.transpose_out \
        and n.value is None


def _local(engine, node) -> Dense:
    v = node.eval(engine)
    return _replicate(engine, v) if v.part is not None and engine.ctx.distributed else v


class GateSumNode(Node):
    """LSTMThreeWaySum: act(W.x + U.h + B).  The block-matmul inputs become ONE GEMM over the
    K-concatenation [W | U] . [x ; h] (the sum of the products IS the product of the concatenations),
    the remaining (dense) inputs are summed into a full-matrix bias added in the GEMM epilogue, and the
    sigmoid/tanh is applied there too (no separate elementwise passes)."""

    def __init__(self, ins: List[Node], act: str):
        self.ins, self.act = ins, act

    def parts(self, engine):
        mms = [n for n in self.ins if _is_plain_matmul(n)]
        rest = [n for n in self.ins if not _is_plain_matmul(n)]
        ops_ = []
        for m in mms:
            A, B = _local(engine, m.a), _local(engine, m.b)
            opA = A.t() if m.p.transpose_a else A
            opB = B.t() if m.p.transpose_b else B
            ops_.append((opA, opB))
        return ops_, rest

    def eval(self, engine) -> Dense:
        if self.value is not None:
            return self.value
        ops_, rest = self.parts(engine)
        bias = None
        for n in rest:
            t = _local(engine, n).logical().float()
            bias = t.clone() if bias is None else bias + t
        act = ops.act_code(self.act)
        if ops_:
            M, N = ops_[0][0].rows, ops_[0][1].cols
            if any(a.rows != M or b.cols != N or a.cols != b.rows for a, b in ops_):
                raise ValueError("LSTM gate products of different shapes")
            X = _kcat([_kslice(a.physical(False), M, a.cols) for a, _ in ops_], cache=True)
            Y = _kcat([_kslice(b.physical(True), N, b.rows) for _, b in ops_], cache=False)
            if X.shape[1] != Y.shape[1]:
                raise ValueError("K mismatch in the gate GEMM")
            b = bias.contiguous() if bias is not None else None
            y = ops.gemm_nt(X, Y, b, ops.BIAS_MAT if b is not None else ops.BIAS_NONE, act,
                            out_dtype=torch.float32)
        else:
            y = ops.bias_act(bias.contiguous(), None, ops.BIAS_NONE, act, out_dtype=torch.float32)
        first = ops_[0][0] if ops_ else _local(engine, rest[0])
        self.value = Dense.of(y, first.br, (ops_[0][1].bc if ops_ else first.bc))
        return self.value


class CellUpdateNode(Node):
    """LSTMTwoSum: c = f * c_prev + i * g (one elementwise HIP pass)."""

    def __init__(self, f, cp, i, g):
        self.f, self.cp, self.i, self.g = f, cp, i, g
        self.fused_step = None       # set when HiddenOutNode lowered the whole step

    def eval(self, engine) -> Dense:
        if self.value is None:
            vs = [_local(engine, n) for n in (self.f, self.cp, self.i, self.g)]
            t = [v.logical().float().contiguous() for v in vs]
            y = ops.lstm_two_sum(*t)
            self.value = Dense.of(y, vs[0].br, vs[0].bc)
        return self.value


class HiddenOutNode(Node):
    """LSTMHiddenState: h = o * tanh(c).

    When the whole time step is in the graph — h = HiddenState(o, TwoSum(f, c_prev, i, g)) with the four
    gates ThreeWaySums of W.x + U.h + B over the SAME x and h — it lowers to ONE stacked gate GEMM
    (all four gates' [W | U] rows, bias matrices in the epilogue, gates laid out [batch, 4H]) followed by
    the fused ``lstm_cell`` kernel, which also yields c_t for the TwoSum's writer."""

    def __init__(self, o, c):
        self.o, self.c = o, c

    def _step_pattern(self):
        c = self.c
        if not isinstance(c, CellUpdateNode):
            return None
        gates = {"i": c.i, "f": c.f, "g": c.g, "o": self.o}
        want = {"i": "sigmoid", "f": "sigmoid", "g": "tanh", "o": "sigmoid"}
        for k, n in gates.items():
            if not isinstance(n, GateSumNode) or n.act != want[k] or n.value is not None:
                return None
            mms = [x for x in n.ins if _is_plain_matmul(x)]
            if len(mms) != 2 or len(n.ins) != 3:
                return None
        return gates

    def eval(self, engine) -> Dense:
        if self.value is not None:
            return self.value
        gates = self._step_pattern()
        if gates is not None:
            try:
                self.value = self._fused_step(engine, gates)
                return self.value
            except ValueError:
                pass
        O, C = _local(engine, self.o), _local(engine, self.c)
        y = ops.lstm_hidden(O.logical().float().contiguous(), C.logical().float().contiguous())
        self.value = Dense.of(y, O.br, O.bc)
        return self.value

    def _fused_step(self, engine, gates) -> Dense:
        order = ("i", "f", "g", "o")            # lstm_cell's gate layout
        xs, ys, biases = [], None, []
        shape = None
        for k in order:
            ops_, rest = gates[k].parts(engine)
            (a0, b0), (a1, b1) = ops_
            M, N = a0.rows, b0.cols
            if shape is None:
                shape = (M, N, a0.br, b0.bc)
                ys = [b0, b1]
            elif (M, N) != shape[:2] or b0.src is not ys[0].src or b1.src is not ys[1].src:
                raise ValueError("gates do not share x / h")
            if (b0.src is None and b0._phys is not ys[0]._phys) or (b1.src is None and b1._phys is not ys[1]._phys):
                raise ValueError("gates do not share x / h")
            xs.append(_kcat([_kslice(a0.physical(False), M, a0.cols), _kslice(a1.physical(False), M, a1.cols)],
                            cache=True))
            bm = None
            for n in rest:
                t = _local(engine, n).logical().float()
                bm = t if bm is None else bm + t
            biases.append(bm)
        M, N, br, bc = shape
        W = _kcat_rows(xs)                                   # [4H, D + H]  (cached while weights unchanged)
        Y = _kcat([_kslice(ys[0].physical(True), N, ys[0].rows), _kslice(ys[1].physical(True), N, ys[1].rows)],
                  cache=False)                              # [batch, D + H] = [x ; h]^T
        bias_t = torch.cat([(b if b is not None else torch.zeros(M, N, device=W.device)).t() for b in biases],
                           1).contiguous()                  # [batch, 4H]
        g = ops.gemm_nt(Y, W, bias_t, ops.BIAS_MAT, ops.ACT_NONE, out_dtype=torch.float32)   # [batch, 4H]
        cprev = _local(engine, self.c.cp).logical().float().t().contiguous()               # [batch, H]
        h, c = ops.lstm_cell(g, cprev)
        self.c.value = Dense.of(c.t().contiguous(), br, bc)
        self.c.fused_step = True
        st = getattr(engine, "ooc_stats", None)
        if st is not None:
            st["lstm_fused_steps"] = st.get("lstm_fused_steps", 0) + 1
        return Dense.of(h.t().contiguous(), br, bc)


_ROWCAT: Dict[tuple, torch.Tensor] = {}


def _kcat_rows(parts: List[torch.Tensor]) -> torch.Tensor:
    key = tuple((p.data_ptr(), tuple(p.shape)) for p in parts)
    hit = _ROWCAT.get(key)
    if hit is not None and hit[1] == tuple(p._version for p in parts):
        return hit[0]
    out = torch.cat(parts, 0).contiguous()
    if len(_ROWCAT) > 32:
        _ROWCAT.clear()
    _ROWCAT[key] = (out, tuple(p._version for p in parts))
    return out


class TransposeNode(Node):
    def __init__(self, x: Node):
        self.x = x

    def eval(self, engine) -> Dense:
        if self.value is None:
            self.value = self.x.eval(engine).t()      # metadata only: flip the layout flag
        return self.value


class ScaleNode(Node):
    """c * X on the value as it is laid out and distributed: each rank scales its own rows / columns."""

    def __init__(self, x: Node, scalar: float):
        self.x, self.scalar = x, scalar

    def eval(self, engine) -> Dense:
        if self.value is None:
            X = self.x.eval(engine)
            p = X.phys
            y = (p.float() * self.scalar).to(p.dtype)
            self.value = Dense(y, X.rows, X.cols, X.transposed, X.br, X.bc, X.part, X.offset, X.total)
        return self.value


def _dop(op):
    return {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}[op]


class ReduceNode(Node):
    def __init__(self, x: Node, axis: str, op: str):
        self.x, self.axis, self.op = x, axis, op

    def eval(self, engine) -> Dense:
        if self.value is None:
            X = self.x.eval(engine)
            L = X.logical().float()
            red = {"sum": torch.sum, "max": torch.amax, "min": torch.amin}[self.op]
            ctx = engine.ctx
            if self.axis == "row":          # -> column vector [rows, 1]
                y = red(L, dim=1, keepdim=True)
                if X.part == "cols":
                    y = ctx.all_reduce(y.contiguous(), _dop(self.op))
                v = Dense.of(y, X.br, 1, "rows" if X.part == "rows" else None, X.offset, X.total)
            elif self.axis == "col":        # -> row vector [1, cols]
                y = red(L, dim=0, keepdim=True)
                if X.part == "rows":
                    y = ctx.all_reduce(y.contiguous(), _dop(self.op))
                v = Dense.of(y, 1, X.bc, "cols" if X.part == "cols" else None, X.offset, X.total)
            else:
                y = red(L).reshape(1, 1)
                if X.part is not None:
                    y = ctx.all_reduce(y.contiguous(), _dop(self.op))
                v = Dense.of(y, 1, 1)
            self.value = v
        return self.value


class InverseNode(Node):
    def __init__(self, x: Node):
        self.x = x

    def eval(self, engine) -> Dense:
        if self.value is None:
            X = _replicate(engine, self.x.eval(engine))
            inv = torch.linalg.inv(X.logical().double()).float()
            self.value = Dense.of(inv.contiguous(), X.br, X.bc)
        return self.value


class DuplicateNode(Node):
    def __init__(self, x: Node, pat: Duplicate):
        self.x, self.p = x, pat

    def eval(self, engine) -> Dense:
        if self.value is None:
            X = _replicate(engine, self.x.eval(engine))
            L = X.logical()
            n = self.p.block_size * self.p.num_blocks
            if self.p.axis == "row":
                y = L[:1].expand(n, L.shape[1]).contiguous()
                self.value = Dense.of(y, self.p.block_size, X.bc)
            else:
                y = L[:, :1].expand(L.shape[0], n).contiguous()
                self.value = Dense.of(y, X.br, self.p.block_size)
        return self.value


class Fuser:
    def __init__(self, engine):
        self.engine = engine
        self.memo: Dict[int, Optional[Node]] = {}
        self.fused: List[str] = []

    def match(self, c: Computation) -> Optional[Node]:
        if id(c) in self.memo:
            n = self.memo[id(c)]
            if n is not None:
                n.uses += 1
            return n
        n = self._match(c)
        if n is not None:
            n.uses += 1
        self.memo[id(c)] = n
        return n

    def _source(self, c) -> Optional[Node]:
        if isinstance(c, ScanSet):
            st = self.engine.storage
            if st.has_set(c.db, c.set_name):
                s = st.get_set(c.db, c.set_name)
                if isinstance(s, DenseMatrixSet):
                    s.resolve_shared()         # dedup: linked shared blocks -> the dense panel
                if isinstance(s, DenseMatrixSet) and s.has_data():
                    return SourceNode(s)
        return None

    def _match(self, c: Computation) -> Optional[Node]:
        src = self._source(c)
        if src is not None:
            return src
        pat = c.tensor_pattern()
        if pat is None:
            return None
        name = type(c).__name__
        if isinstance(c, AggregateComp) and isinstance(pat, BlockSum):
            j = c.inputs[0]
            jp = j.tensor_pattern() if j is not None else None
            if isinstance(j, JoinComp) and isinstance(jp, BlockMatmul):
                a = self.match(j.inputs[jp.a_input])
                b = self.match(j.inputs[jp.b_input])
                if a is not None and b is not None:
                    node = MatmulNode(a, b, jp)
                    if isinstance(a, MatmulNode):
                        a.consumers_want_t = jp.transpose_a
                    if isinstance(b, MatmulNode):
                        b.consumers_want_t = not jp.transpose_b
                    self.fused.append(f"matmul[{type(j).__name__}+{name}]")
                    return node
            return None
        if isinstance(c, JoinComp) and isinstance(pat, BiasAct):
            x = self.match(c.inputs[pat.data_input])
            b = self.match(c.inputs[pat.bias_input])
            if x is None or b is None:
                return None
            if isinstance(x, MatmulNode) and x.bias is None and x.act == "none" and not x.transpose_out \
                    and x.value is None:
                x.bias, x.bias_along, x.act, x.dropout, x.seed = b, pat.bias_along, pat.act, pat.dropout, pat.seed
                x.transpose_out = pat.transpose_out
                x.uses -= 1                     # the epilogue join is absorbed into the GEMM, not a consumer
                self.fused.append(f"epilogue[{name}]")
                return x
            self.fused.append(f"bias_act[{name}]")
            return BiasActNode(x, b, pat)
        if isinstance(c, JoinComp) and isinstance(pat, RowSoftmax):
            x = self.match(c.inputs[0])
            if x is None:
                return None
            self.fused.append(f"softmax[{name}]")
            node = SoftmaxNode(x)
            node.notes = self.fused
            return node
        if isinstance(c, JoinComp) and isinstance(pat, GateSum):
            ins = [self.match(x) for x in c.inputs]
            if any(x is None for x in ins):
                return None
            self.fused.append(f"gate_gemm[{name}:{sum(_is_plain_matmul(x) for x in ins)}x]")
            return GateSumNode(ins, pat.act)
        if isinstance(c, JoinComp) and isinstance(pat, CellUpdate):
            ins = [self.match(x) for x in c.inputs]
            if any(x is None for x in ins):
                return None
            self.fused.append(f"lstm_two_sum[{name}]")
            return CellUpdateNode(*ins)
        if isinstance(c, JoinComp) and isinstance(pat, HiddenOut):
            ins = [self.match(x) for x in c.inputs]
            if any(x is None for x in ins):
                return None
            node = HiddenOutNode(*ins)
            self.fused.append("lstm_step[stacked gate GEMM + lstm_cell]" if node._step_pattern() is not None
                              else f"lstm_hidden[{name}]")
            return node
        if isinstance(c, JoinComp) and isinstance(pat, Elementwise):
            a, b = self.match(c.inputs[0]), self.match(c.inputs[1])
            if a is None or b is None:
                return None
            self.fused.append(f"ewise_{pat.op}[{name}]")
            return EwiseNode(a, b, pat.op)
        if isinstance(c, SelectionComp) and isinstance(pat, Transpose):
            x = self.match(c.inputs[0])
            if x is None:
                return None
            self.fused.append(f"transpose[{name}]")
            return TransposeNode(x)
        if isinstance(c, SelectionComp) and isinstance(pat, Scale):
            x = self.match(c.inputs[0])
            if x is None:
                return None
            self.fused.append(f"scale[{name}]")
            return ScaleNode(x, pat.scalar)
        if isinstance(c, AggregateComp) and isinstance(pat, Reduce):
            x = self.match(c.inputs[0])
            if x is None:
                return None
            self.fused.append(f"reduce_{pat.axis}_{pat.op}[{name}]")
            return ReduceNode(x, pat.axis, pat.op)
        if isinstance(pat, Inverse):
            x = self.match(c.inputs[0])
            if x is None:
                return None
            self.fused.append(f"inverse[{name}]")
            return InverseNode(x)
        if isinstance(c, MultiSelectionComp) and isinstance(pat, Duplicate):
            x = self.match(c.inputs[0])
            if x is None:
                return None
            self.fused.append(f"duplicate_{pat.axis}[{name}]")
            return DuplicateNode(x, pat)
        return None

    # ------------------------------------------------------------------ rewrite
    def run(self, sinks: List[Computation]) -> List[Computation]:
        remaining: List[Computation] = []
        # writers of a whole LSTM step (h_t) first: their stacked-gate lowering also produces c_t
        sinks = sorted(sinks, key=lambda s: 0 if (isinstance(s, WriteSet) and s.inputs and
                                                  isinstance(self.match(s.inputs[0]), HiddenOutNode)) else 1)
        # match every sink's inputs before anything is evaluated, so Node.uses counts all consumers (a GEMM
        # whose exp'd scores are also read elsewhere must not normalise them in its epilogue)
        for s in sinks:
            if not isinstance(s, WriteSet):
                for inp in s.inputs:
                    if inp is not None:
                        self.match(inp)
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
        ctx = self.engine.ctx
        if v.part == "cols":
            v = _replicate(self.engine, v)
        st = self.engine.storage
        if create or not st.has_set(db, name):
            st.create_set(db, name, None, dense=True, persistent=False)
        s = st.get_set(db, name)
        replicated = v.part is None
        row_off = v.offset if v.part == "rows" else 0
        total_rows = v.total if v.part == "rows" else v.rows
        if isinstance(s, DenseMatrixSet):
            s.set_panel(v.phys, total_rows, v.cols, max(1, v.br), max(1, v.bc), row_offset=row_off,
                        transposed=v.transposed, replicated=replicated or not ctx.distributed)
            s.local_rows = v.rows
        else:
            tmp = DenseMatrixSet(st, db, name, s.type, -1, s.page_size, s.device)
            tmp.set_panel(v.phys, total_rows, v.cols, max(1, v.br), max(1, v.bc), row_offset=row_off,
                          transposed=v.transposed)
            tmp.local_rows = v.rows
            s.add_batch(tmp.to_blocks())


def fuse_tensor_patterns(sinks: List[Computation], engine) -> Tuple[List[Computation], List[str]]:
    f = Fuser(engine)
    rest = f.run(sinks)
    return rest, f.fused


__all__ = ["fuse_tensor_patterns", "Fuser", "MatmulNode", "SoftmaxNode", "BiasActNode", "SourceNode", "Dense",
           "EwiseNode", "TransposeNode", "ReduceNode", "InverseNode", "DuplicateNode", "GateSumNode", "CellUpdateNode",
           "HiddenOutNode"]
