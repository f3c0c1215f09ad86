"""Headline benchmark: whole-node inference rows/sec for netsDB's FF-NN + conv2d block.

One step (per GPU, weak scaling; every rank holds its own partition of the inference inputs and
the model is replicated — netsDB's broadcast join of the weight sets, "materializeModel"):
  1. FF-NN inference_unit on AmazonCat-14k dims (reference src/tests/source/FFTestWithDeduplication.cc:
     batch 1000, features 597540, hidden 1000, labels 14588; blocks 50x10000; dropout 0.5 as FFTest.cc)
     = the reference's 2 jobs (W1·Xᵀ -> +b1, relu, dropout -> Wo·Y -> +bo, exp, ᵀ  |  row softmax) submitted as ONE
     engine job: the planner lowers the output layer + row softmax to one GEMM with the normalisation in its
     epilogue (--two-job keeps the materialised "yo" set and the separate row-normalise job)
  2. conv2d_memory_fusion block (reference src/tests/source/PipelinedConv2dMemFuseTest.cc: 100 images
     3x112x112, 64 filters 7x7x3, stride 1, no padding) = 1 job, fused implicit-GEMM conv + bias.
The conv2d job is independent of the FF jobs (resident images, own weights); --overlap before|after submits
it on a second HIP stream (PDBClient.submit_job) next to the FF kernels.  Default: serial — once the clocks
have ramped (warmup 10) the overlap measures no gain (1.037-1.043M vs 1.034-1.045M rows/s, profiles/r1_overlap).
The default warmup of 10 steps keeps the GPU clock ramp out of the timed window (10 timed steps after 2
warmups measured 0.85-0.89M rows/s on the same box that gives 1.03-1.07M after 10).
rows/step/GPU = FF input rows + images.  Synthetic data, random-init weights, bf16 compute.

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...

Without torchrun (WORLD_SIZE unset) and N > 1, bench.py launches its own ranks: N child processes, one per GPU
(LOCAL_RANK = GPU index, RCCL; gloo on a CPU-only host), started as ordinary subprocesses BEFORE this process makes
any GPU call (it never re-execs itself), rendezvous on 127.0.0.1. Rank 0's JSON line is the result.
"""
import argparse
import json
import os
import sys
import tempfile
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

FULL = dict(batch=1000, features=597540, hidden=1000, labels=14588, block_x=50, block_y=10000,
            images=100, channels=3, height=112, width=112, filters=64, ksize=7)
SMALL = dict(batch=64, features=4096, hidden=256, labels=512, block_x=32, block_y=512,
             images=4, channels=3, height=32, width=32, filters=16, ksize=7)


def verify(client, cv, ff, w, b, dev, nrows=16, nimg=2, single_job=False):
    """Untimed correctness check after the timed steps: one more FF inference_unit with dropout 0,
    sampled output rows vs the fp32 network (hidden activations rounded to bf16 as the plan stores
    them), and sampled conv2d images vs F.conv2d in fp32. Returns max relative errors."""
    from netsdb_amd.models.blocks import to_tensor

    ff.inference_unit(client, "ff", "w1", "wo", "inputs", "b1", "bo", "output", dropout_rate=0.0, seed=0,
                      single_job=single_job)
    out = to_tensor(client, "ff", "output", gather=False).float()
    x_all = to_tensor(client, "ff", "inputs", gather=False)
    n = min(nrows, out.shape[0])
    rows = torch.linspace(0, out.shape[0] - 1, n, device=out.device).long()
    x = x_all[rows].float()
    w1, b1 = to_tensor(client, "ff", "w1").float(), to_tensor(client, "ff", "b1").float().reshape(-1)
    wo, bo = to_tensor(client, "ff", "wo").float(), to_tensor(client, "ff", "bo").float().reshape(-1)
    y = torch.relu(x @ w1.t() + b1).to(torch.bfloat16).float()
    ref = torch.softmax(y @ wo.t() + bo, dim=-1)
    ff_err = ((out[rows] - ref).abs().max() / ref.abs().max()).item()
    row_sum_err = (out[rows].sum(-1) - 1).abs().max().item()
    imgs = client.storage.get_set("conv2d", "img").all().columns["data"][:nimg]
    got = client.storage.get_set("conv2d", "conv_out").all().columns["data"][:nimg].float()
    cref = torch.nn.functional.conv2d(imgs.float(), w.to(torch.bfloat16).float(), b.float())
    conv_err = ((got - cref).abs().max() / cref.abs().max()).item()
    ok = ff_err < 1e-2 and row_sum_err < 1e-2 and conv_err < 1e-2
    return {"ff_sampled_rows": n, "ff_max_rel_err": ff_err, "ff_row_sum_err": row_sum_err,
            "conv_images": nimg, "conv_max_rel_err": conv_err, "ok": bool(ok)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--small", action="store_true", help="tiny shapes (CPU smoke only; not a valid measurement)")
    ap.add_argument("--dropout", type=float, default=0.5)
    ap.add_argument("--settle-ms", type=float, default=400.0,
                    help="untimed steps run before the W warmup steps until this much wall time has passed: "
                         "the chip's clock dips for ~10-20 ms after the GEMMs start and then settles "
                         "(profiles/r2_clock_settle); the timed window should see the settled clock")
    ap.add_argument("--overlap", choices=["none", "after", "before"], default="none",
                    help="conv2d job on its own HIP stream (PDBClient.submit_job), submitted after/before the FF jobs "
                         "(independent inputs); default serial: no gain once the clocks have ramped (profiles/r1_overlap)")
    ap.add_argument("--two-job", action="store_true",
                    help="submit inference_unit as the reference's two jobs (output layer exp -> 'yo' set, then the row "
                         "normalise); default: ONE job, whose output layer is one GEMM with the max-subtracted softmax "
                         "in its epilogue (55-59 us vs 66-70 + 18 us in-bench, profiles/r3_s3/softmax)")
    ap.add_argument("--single-job", action="store_true", help=argparse.SUPPRESS)   # the default; kept for old scripts
    ap.add_argument("--mfma", type=int, choices=[0, 16, 32], default=0,
                    help="8-phase GEMM main-loop MFMA shape for this run (0 = the library default; A/B arm)")
    ap.add_argument("--fixup", type=int, choices=[-1, 0, 1], default=-1,
                    help="layer-1 split-K reduction inside the GEMM launch (1) or the separate reducer (0); "
                         "-1 = the library default")
    args = ap.parse_args()
    args.single_job = not args.two_job
    from netsdb_amd.parallel import launch

    if launch.should_launch(args.gpus):
        sys.exit(launch.launch_ranks(__file__, args.gpus, sys.argv[1:]))

    from netsdb_amd.client import PDBClient
    from netsdb_amd.models import conv2d as cv
    from netsdb_amd.models import ff
    from netsdb_amd.parallel.comm import ClusterContext

    from netsdb_amd import ops

    if args.mfma:
        ops.set_kernel_options(gemm_mfma=args.mfma)
    if args.fixup >= 0:
        ops.set_kernel_options(gemm_fixup=args.fixup)
    cfg = SMALL if args.small else FULL
    ctx = ClusterContext.from_env()
    if ctx.world_size != args.gpus and ctx.rank == 0:
        print(f"[bench] note: --gpus {args.gpus} but WORLD_SIZE={ctx.world_size}", file=sys.stderr)
    root = tempfile.mkdtemp(prefix=f"nsdb_bench_r{ctx.rank}_")
    client = PDBClient(ctx=ctx, root=root, device=ctx.device)
    dev = ctx.device

    # ---- data (per-rank partition of the inputs, replicated model) ----
    ff.load_model(client, "ff", cfg["batch"] * ctx.world_size, cfg["features"], cfg["hidden"], cfg["labels"],
                  cfg["block_x"], cfg["block_y"], seed=1234, partition_inputs=True)
    client.create_database("conv2d")
    cv.load_images(client, "conv2d", "img", cfg["images"], cfg["channels"], cfg["height"], cfg["width"], seed=99)
    w, b = cv.random_kernel(cfg["filters"], cfg["channels"], cfg["ksize"], cfg["ksize"], seed=7, device=dev)
    local_rows = client.storage.get_set("ff", "inputs").local_rows
    client.job_lanes = 1
    client.job_lane_priority = {0: -1}

    def conv():
        cv.conv2d_memfuse_inference(client, "conv2d", "img", "conv_out", w, b)

    def ffjobs(i):
        ff.inference_unit(client, "ff", "w1", "wo", "inputs", "b1", "bo", "output", dropout_rate=args.dropout,
                          seed=i, single_job=args.single_job)

    def step(i):
        if args.overlap == "before":
            client.submit_job(conv, independent=True)
        ffjobs(i)
        if args.overlap == "none":
            conv()
        elif args.overlap == "after":
            client.submit_job(conv, independent=True)
        if args.overlap != "none":
            client.wait_jobs()   # the step ends when both jobs have (stream-ordered join)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        ctx.barrier()
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    if args.warmup > 0:
        # first step serially: derived weights / plans are materialised once, before any lane reads them
        ffjobs(0)
        conv()
        sync()
    settle_steps = 0
    if args.warmup > 0 and args.settle_ms > 0 and dev.type == "cuda":
        t_s = time.perf_counter()
        more = True
        while more:
            for _ in range(5):
                step(args.warmup)
                settle_steps += 1
            torch.cuda.synchronize(dev)
            # every rank runs the same number of settle steps (the conv job's planner does collectives)
            more = ctx.all_reduce_scalar(float((time.perf_counter() - t_s) * 1e3 < args.settle_ms), "max") > 0
    for i in range(1, args.warmup):
        step(i)
    client.wait_jobs()
    sync()
    coll0 = ctx.stats.get("collectives", 0)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i)
    client.wait_jobs()
    sync()
    dt = time.perf_counter() - t0
    coll_per_step = (ctx.stats.get("collectives", 0) - coll0 - (1 if ctx.distributed else 0)) / max(1, args.steps)  # minus sync()'s barrier
    dt = ctx.all_reduce_scalar(dt, "max")
    rows_local = local_rows + cfg["images"]
    rows_total = ctx.all_reduce_scalar(float(rows_local), "sum") * args.steps
    value = rows_total / dt
    check = verify(client, cv, ff, w, b, dev, single_job=args.single_job)
    if ctx.rank == 0:
        res = {
            "metric": "inference rows/sec (whole node), FF-NN + conv2d block",
            "value": round(value, 2),
            "unit": "rows/s",
            "n_gpus": ctx.world_size,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (random inputs/images, random-init weights)",
            "config": {
                "model": "FF-NN AmazonCat-14k (597540-1000-14588, relu+dropout0.5, softmax) + conv2d 7x7x3->64 block",
                "global_batch": int(rows_total / args.steps),
                "ff_rows_per_gpu": local_rows,
                "conv_images_per_gpu": cfg["images"],
                "image": [cfg["channels"], cfg["height"], cfg["width"]],
                "seq_len": None,
                "parallelism": f"dp{ctx.world_size} (row-partitioned inputs, broadcast model)",
                "small": bool(args.small),
                "check": check,
                "settle_steps_untimed": settle_steps,
                "conv_overlap": args.overlap,
                "collectives_per_step": round(coll_per_step, 2),
                "single_job": bool(args.single_job),
                "gemm_mfma": args.mfma or "default",
                "gemm_fixup": args.fixup if args.fixup >= 0 else "default",
            },
        }
        print(json.dumps(res), flush=True)
    if ctx.distributed:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
