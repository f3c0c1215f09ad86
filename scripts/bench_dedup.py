"""Model-deduplication benchmark (BASELINE.json config "Model-deduplication over word2vec embedding tables
across 8 GPUs (hash-join + RCCL all-to-all, 288 GB HBM page-pool sizing)"), modelled on
src/tests/source/TestWord2VecWithDeduplication.cc: ``--models`` word2vec weight matrices of
``rows x cols`` (500 x 1,000,000 = 5 x 100 FFMatrixBlocks of 100 x 10000) whose first ``shared`` column
blocks (90 of 100) are identical across models and whose remaining columns are private; a batch of
``batch`` (100) one-hot-sized input rows is scored against every model (FFTransposeMult + FFAggMatrix:
``y = W @ X^T``).

    python scripts/bench_dedup.py [--models 12] [--steps 5 --warmup 2] [--gpus N] [--small]
    torchrun --nproc-per-node N --master-addr 127.0.0.1 scripts/bench_dedup.py

``--gpus N`` without torchrun starts its own N ranks (netsdb_amd.parallel.launch: the parent makes no GPU call).
The collective phases report the payload bytes each rank hands to RCCL and the xGMI time the node model predicts
for them (parallel/comm.py xgmi_seconds) next to their measured time.

Models are assigned round-robin to ranks; every phase is collective (ranks with no model that round take
part with None).  Timed phases (each bracketed by barrier + synchronize, max over ranks):

* add         — DistributedBlockPool.add_model: device block hashing (HIP ``block_hash`` kernel), RCCL
                all-to-all of (hash, payload) to the hash owners, content-verified dedup insert;
* materialize — fetch every model's blocks back from their owners (all-to-all pair) into dense panels;
* infer_naive — per model ``W_m @ X^T`` on the MFMA GEMM (what the reference does per model);
* infer_dedup — SharedInference: the common column panel's GEMM once per batch, plus each model's private
                columns accumulated on top.

Rank 0 prints ONE JSON line (whole-job numbers: rows/s = models x batch / time).  Synthetic random
weights of the reference geometry (no checkpoints are available offline).
"""
import argparse
import json
import math
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", type=int, default=12)
    ap.add_argument("--rows", type=int, default=500)
    ap.add_argument("--cols", type=int, default=1_000_000)
    ap.add_argument("--block-rows", type=int, default=100)
    ap.add_argument("--block-cols", type=int, default=10_000)
    ap.add_argument("--shared-blocks", type=int, default=90, help="column blocks shared by every model")
    ap.add_argument("--batch", type=int, default=100)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--check", type=int, default=1, help="compare model 0's scores with an fp32 reference")
    ap.add_argument("--gpus", type=int, default=1, help="ranks to start when not under torchrun (one per GPU)")
    ap.add_argument("--small", action="store_true", help="CPU / contract size (8 models of 20 x 4000, blocks 10 x 400)")
    ap.add_argument("--overlap", type=int, default=0,
                    help="1: the private panels' GEMM on a second stream, concurrent with the common panel's")
    ap.add_argument("--prefetch-x", type=int, default=-1,
                    help="1 / 0: compact X's private columns on a second stream during the common GEMM (-1: default)")
    ap.add_argument("--ab-prefetch", type=int, default=0,
                    help="N > 0: also time N interleaved rounds of prefetch-x off / on (ab_prefetch in the JSON)")
    ap.add_argument("--ab-overlap", type=int, default=0,
                    help="N > 0: also time N interleaved rounds of overlap off / on (ab_overlap in the JSON)")
    a = ap.parse_args()
    if a.small:
        a.models, a.rows, a.cols, a.block_rows, a.block_cols, a.shared_blocks, a.batch = 8, 20, 4000, 10, 400, 9, 16
        a.steps, a.warmup = 1, 0
    from netsdb_amd.parallel import launch

    if launch.should_launch(a.gpus):
        sys.exit(launch.launch_ranks(__file__, a.gpus, sys.argv[1:]))

    from netsdb_amd.models.dedup import DistributedBlockPool, SharedInference
    from netsdb_amd import ops
    from netsdb_amd.parallel.comm import ClusterContext

    ctx = ClusterContext.from_env()
    dev = ctx.device
    ws, rank = ctx.world_size, ctx.rank
    R, C, br, bc = a.rows, a.cols, a.block_rows, a.block_cols
    nbc = math.ceil(C / bc)
    shared_c = min(a.shared_blocks, nbc) * bc
    rounds = math.ceil(a.models / ws)
    mine = [m for m in range(a.models) if m % ws == rank]
    dt_ = torch.bfloat16

    g = torch.Generator(device=dev).manual_seed(1234)                       # same shared part on every rank
    shared = (torch.randn(R, shared_c, device=dev, generator=g) * 0.05).to(dt_)

    def model(m):
        gm = torch.Generator(device=dev).manual_seed(10_000 + m)
        w = torch.empty(R, C, dtype=dt_, device=dev)
        w[:, :shared_c] = shared
        w[:, shared_c:] = (torch.randn(R, C - shared_c, device=dev, generator=gm) * 0.05).to(dt_)
        return w

    X = (torch.randn(a.batch, C, device=dev, generator=torch.Generator(device=dev).manual_seed(7)) * 0.05).to(dt_)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        ctx.barrier()
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    comm = {}

    def comm_mark():
        return ctx.stats["coll_bytes"], ctx.stats["xgmi_pred_s"]

    def comm_record(tag, mark, steps=1):
        b = ctx.all_reduce_scalar(float(ctx.stats["coll_bytes"] - mark[0]), "max") / steps
        x = ctx.all_reduce_scalar(ctx.stats["xgmi_pred_s"] - mark[1], "max") / steps
        comm[f"{tag}_coll_MB_per_rank"] = round(b / 1e6, 3)
        comm[f"{tag}_xgmi_pred_ms"] = round(x * 1e3, 3)

    def timed(fn, steps, tag=None):
        sync()
        mk = comm_mark()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        sync()
        dt = ctx.all_reduce_scalar((time.perf_counter() - t0) / steps, "max")
        if tag:
            comm_record(tag, mk, steps)
        return dt

    # ---------------------------------------------------------------- add (timed once per pool build)
    def build_pool():
        pool = DistributedBlockPool(ctx, br, bc, device=dev, dtype=dt_)
        add_t = 0.0
        for r in range(rounds):
            m = r * ws + rank
            w = model(m) if m < a.models else None
            sync()
            t0 = time.perf_counter()
            pool.add_model(f"w{m}" if w is not None else "__none", w)
            sync()
            add_t += time.perf_counter() - t0
            del w
        return pool, ctx.all_reduce_scalar(add_t, "max")

    for _ in range(max(1, a.warmup // 2)):
        build_pool()                                   # warm the hash / all-to-all paths
    mk = comm_mark()
    pool, t_add = build_pool()
    comm_record("add", mk)
    model_bytes = a.models * R * C * 2
    stored = ctx.all_reduce_scalar(float(pool.stored_blocks()), "sum")
    blocks_in = a.models * math.ceil(R / br) * nbc

    # ---------------------------------------------------------------- materialize
    dense = {}

    def materialize():
        for r in range(rounds):
            m = r * ws + rank
            out = pool.materialize(f"w{m}" if m < a.models else None)
            if out is not None:
                dense[m] = out

    for _ in range(a.warmup):
        materialize()
    t_mat = timed(materialize, a.steps, "materialize")

    # ---------------------------------------------------------------- inference
    def infer_naive():
        for m in mine:
            ops.gemm_nt(dense[m], X, out_dtype=torch.float32)

    si = None
    if mine:
        local = {f"w{m}": pool.tables[f"w{m}"] for m in mine}
        shapes = {n: pool.shapes[n] for n in local}
        cache = {}

        def fetch(ids):
            # blocks of this rank's models, cut from the materialized panels (ids -> first occurrence)
            out = torch.empty(ids.numel(), br, bc, dtype=dt_, device=dev)
            for j, gid in enumerate(ids.tolist()):
                out[j] = cache[gid]
            return out

        from netsdb_amd.models.dedup import to_blocks
        for m in mine:
            blks = to_blocks(dense[m], br, bc)
            for j, gid in enumerate(pool.tables[f"w{m}"].flatten().tolist()):
                cache.setdefault(gid, blks[j])
        si = SharedInference(local, shapes, fetch, br, bc)
        cache.clear()

    def infer_dedup():
        if si is not None:
            si.run(X)

    if si is not None:
        si.overlap = bool(a.overlap)
        if a.prefetch_x >= 0:
            si.prefetch_x = bool(a.prefetch_x)
    for _ in range(a.warmup):
        infer_naive()
        infer_dedup()
    t_naive = timed(infer_naive, a.steps)
    t_dedup = timed(infer_dedup, a.steps)
    ab = None
    if a.ab_overlap > 0 and si is not None:
        ab = {"off_ms": [], "on_ms": []}
        for _ in range(a.ab_overlap):
            for flag, k in ((False, "off_ms"), (True, "on_ms")):
                si.overlap = flag
                infer_dedup()
                ab[k].append(round(timed(infer_dedup, max(a.steps, 20)) * 1e3, 4))
        si.overlap = bool(a.overlap)
    abp = None
    if a.ab_prefetch > 0 and si is not None:
        keep = si.prefetch_x
        abp = {"off_ms": [], "on_ms": []}
        for _ in range(a.ab_prefetch):
            for flag, k in ((False, "off_ms"), (True, "on_ms")):
                si.prefetch_x = flag
                infer_dedup()
                abp[k].append(round(timed(infer_dedup, max(a.steps, 20)) * 1e3, 4))
        si.prefetch_x = keep

    err = None
    if a.check and 0 in mine:
        y = si.run(X)["w0"]
        w0 = model(0).float()
        ref = w0 @ X.float().t()
        err = float((y - ref).abs().max() / ref.abs().max())
    err = ctx.all_reduce_scalar(err if err is not None else 0.0, "max") if a.check else None

    rows = a.models * a.batch
    if rank == 0:
        print(json.dumps({
            "metric": "word2vec dedup inference rows/s (SharedInference)", "value": round(rows / t_dedup, 1),
            "unit": "rows/s", "n_gpus": ws, "steps": a.steps, "warmup": a.warmup, "higher_is_better": True,
            "vs_baseline": None, "dtype": "bf16", "data": "synthetic random weights of the reference geometry",
            "config": {"models": a.models, "rows": R, "cols": C, "block": [br, bc], "shared_col_blocks": a.shared_blocks,
                       "batch": a.batch},
            "dedup_ratio": round(stored / blocks_in, 4), "blocks_in": blocks_in, "blocks_stored": int(stored),
            "add_GBps": round(model_bytes / t_add / 1e9, 1), "add_ms": round(t_add * 1e3, 2),
            "materialize_GBps": round(model_bytes / t_mat / 1e9, 1), "materialize_ms": round(t_mat * 1e3, 2),
            "infer_naive_rows_per_s": round(rows / t_naive, 1), "infer_naive_ms": round(t_naive * 1e3, 3),
            "infer_dedup_ms": round(t_dedup * 1e3, 3), "dedup_speedup": round(t_naive / t_dedup, 2),
            "panel_GB_dedup": round((si.panel_bytes() if si else 0) / 1e9, 3),
            "panel_GB_naive": round(len(mine) * R * C * 2 / 1e9, 3), "rel_err_model0": err,
            "overlap": bool(a.overlap), "ab_overlap": ab,
            "prefetch_x": bool(si.prefetch_x) if si is not None else None, "ab_prefetch": abp, **comm}), flush=True)
    if ctx.distributed:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
