"""linearAlgebraDSL distributed dense matmul benchmark (BASELINE.json config "linearAlgebraDSL 64k x 64k
dense matmul on 8 x MI355X (join+aggregate shuffle as RCCL collectives)").

    python scripts/bench_la_matmul.py [--size 65536] [--steps 3 --warmup 1] [--gpus N]
    torchrun --nproc-per-node N --master-addr 127.0.0.1 scripts/bench_la_matmul.py --size 65536

``--gpus N`` without torchrun starts its own N ranks (netsdb_amd.parallel.launch: the parent makes no GPU call).

The program is the DSL text ``C = A %*% B`` evaluated by LAInstance (src/linearAlgebraDSL): A and B
are loaded row-partitioned over the ranks (random data, bf16), and ``%*%`` is LAMultiply1Join +
LAMultiply2Aggregate, which the planner fuses into the row-split x K-split distributed matmul
(query_planning/fusion.py ``MatmulNode._allgather_n``: B^T N-chunks all-gathered over RCCL while
the previous chunk's full-K MFMA GEMM runs).  Rank 0 prints one JSON line: whole-job TFLOP/s,
ms per multiply, the max relative error on sampled output rows vs an fp32 reference, and the communication
budget of one multiply next to its compute: payload bytes each rank hands to RCCL per multiply, the xGMI time
those collectives take under the node model (parallel/comm.py xgmi_seconds: one 153 GB/s link per peer), and the
time of the rank's own GEMM of the same shape with no communication (so the three can be compared directly).
"""
import argparse
import json
import os
import sys
import tempfile
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def local_gemm_seconds(c, ctx, n, op, reps=2):
    """One rank's GEMM of the multiply with no communication: ``mul`` is [rows, n] x [n, n]^T (row split), ``tmul``
    the [n, rows] x [rows, n] K-split partial; random bf16 operands, max over ranks."""
    from netsdb_amd import ops

    dev = ctx.device
    rows = -(-n // ctx.world_size)
    g = torch.Generator(device=dev).manual_seed(3)
    if op == "mul":
        A = torch.rand(rows, n, device=dev, generator=g).to(torch.bfloat16)
        Bt = torch.rand(n, n, device=dev, generator=g).to(torch.bfloat16)
    else:
        A = torch.rand(n, rows + (-rows) % 8, device=dev, generator=g).to(torch.bfloat16)
        Bt = torch.rand(n, rows + (-rows) % 8, device=dev, generator=g).to(torch.bfloat16)
    out = ops.gemm_nt(A, Bt, out_dtype=torch.bfloat16)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(reps):
        ops.gemm_nt(A, Bt, out_dtype=torch.bfloat16, out=out)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    dt = (time.perf_counter() - t0) / reps
    del A, Bt, out
    return ctx.all_reduce_scalar(dt, "max")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=65536)
    ap.add_argument("--block", type=int, default=8192, help="DSL block size (blockRowSize = blockColSize)")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--check", type=int, default=32, help="output rows checked against an fp32 reference")
    ap.add_argument("--op", choices=["mul", "tmul"], default="mul",
                    help="mul: C = A %%*%% B (row x K split, all-gather pipeline); tmul: C = A '* B (K x K split, "
                         "overlapped chunked reduce-scatter)")
    ap.add_argument("--small", action="store_true", help="CPU/contract size: 320 x 320 in blocks of 64, 1 step")
    ap.add_argument("--gpus", type=int, default=1, help="ranks to start when not under torchrun (one per GPU)")
    a = ap.parse_args()
    from netsdb_amd.parallel import launch

    if launch.should_launch(a.gpus):
        sys.exit(launch.launch_ranks(__file__, a.gpus, sys.argv[1:]))
    if a.small:
        a.size, a.block, a.steps, a.warmup = 320, 64, 1, 0

    from netsdb_amd.client import PDBClient
    from netsdb_amd.la import LAInstance
    from netsdb_amd.models import blocks as B
    from netsdb_amd.parallel.comm import ClusterContext

    ctx = ClusterContext.from_env()
    c = PDBClient(ctx=ctx, root=tempfile.mkdtemp(prefix=f"nsdb_la_r{ctx.rank}_"), device=ctx.device)
    la = LAInstance(c, partition_loads=True)
    n, bs = a.size, a.block
    nb = (n + bs - 1) // bs
    # random operands (the DSL's load() reads text block files; synthetic data of that shape here)
    B.load_matrix(c, "LA_db", "A_in", n, n, bs, bs, seed=11, partition_rows=True)
    B.load_matrix(c, "LA_db", "B_in", n, n, bs, bs, seed=12, partition_rows=True)
    la.vars.update({"A": "A_in", "B": "B_in"})
    prog = "C = A %*% B" if a.op == "mul" else "C = A '* B"

    def sync():
        if ctx.device.type == "cuda":
            torch.cuda.synchronize(ctx.device)
        ctx.barrier()
        if ctx.device.type == "cuda":
            torch.cuda.synchronize(ctx.device)

    def step():
        old = la.vars.get("C")
        if old is not None:
            c.remove_set("LA_db", old)
        la.run(prog)

    for _ in range(a.warmup):
        step()
    sync()
    b0, x0, c0 = ctx.stats["coll_bytes"], ctx.stats["xgmi_pred_s"], ctx.stats["data_collectives"]
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    sync()
    dt = ctx.all_reduce_scalar(time.perf_counter() - t0, "max") / a.steps
    coll_b = ctx.all_reduce_scalar(float(ctx.stats["coll_bytes"] - b0), "max") / a.steps
    xgmi_s = ctx.all_reduce_scalar(ctx.stats["xgmi_pred_s"] - x0, "max") / a.steps
    ncoll = ctx.all_reduce_scalar(float(ctx.stats["data_collectives"] - c0), "max") / a.steps
    gemm_s = local_gemm_seconds(c, ctx, n, a.op)

    err = 0.0
    if a.check > 0:
        sa, sb, sc = (c.storage.get_set("LA_db", x) for x in ("A_in", "B_in", la.vars["C"]))
        rows = min(a.check, sc.local_rows)
        Cl = sc.matrix()[:rows, :n].float()
        Al = sa.matrix()[:rows, :n].float()
        ref = torch.zeros_like(Cl)
        rng = torch.tensor([[sb.row_offset, sb.local_rows]], device=ctx.device)
        ranges = [(int(pr[0, 0]), int(pr[0, 1])) for pr in ctx.all_gather_tensor(rng)]

        def full(st, s, k0, kn):
            M = st.matrix()[:kn, :n].contiguous() if s == ctx.rank else torch.empty(kn, n, dtype=st.panel.dtype,
                                                                                    device=ctx.device)
            if ctx.distributed:
                torch.distributed.broadcast(M, src=s)
            return M.float()

        if a.op == "mul":
            for s, (k0, kn) in enumerate(ranges):
                ref += Al[:, k0:k0 + kn] @ full(sb, s, k0, kn)
        else:
            # C = A^T B: this rank's output rows are columns [c0, c0 + rows) of A
            c0 = sc.row_offset
            for s, (k0, kn) in enumerate(ranges):
                As = full(sa, s, k0, kn)
                ref += As[:, c0:c0 + rows].t() @ full(sb, s, k0, kn)
        err = float((Cl - ref).abs().max() / ref.abs().max().clamp(min=1e-6)) if Cl.numel() else 0.0   # empty rank
        err = ctx.all_reduce_scalar(err, "max")
    flops = 2.0 * n * n * n
    if ctx.rank == 0:
        st = la.job_stats[-1] if la.job_stats else {}
        print(json.dumps({"metric": f"LA DSL {prog} dense matmul", "n": n, "block": bs, "blocks_per_dim": nb,
                          "n_gpus": ctx.world_size, "ms_per_multiply": round(dt * 1e3, 3),
                          "tflops_total": round(flops / dt / 1e12, 1),
                          "tflops_per_gpu": round(flops / dt / 1e12 / ctx.world_size, 1), "dtype": "bf16",
                          "data": "synthetic random", "rel_err_sampled": err,
                          "fused": st.get("fused_ops"), "out_of_core": st.get("out_of_core"),
                          "coll_MB_per_multiply_per_rank": round(coll_b / 1e6, 3),
                          "data_collectives_per_multiply": ncoll,
                          "xgmi_pred_ms_per_multiply": round(xgmi_s * 1e3, 3),
                          "local_gemm_ms": round(gemm_s * 1e3, 3)}), flush=True)
    if ctx.distributed:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
