"""Our layer-1 GEMM vs hipBLASLt on the SAME work and the SAME data (round-4 ceiling measurement).

FF layer 1 is W1 . X^T with W1 [1000, 597568] (U(-1,1) * sqrt(3/597540), as models/ff.load_model) and X
[1000, 597568] U(-1,1). Our production launch splits K 16 ways inside one kernel. hipBLASLt gets the same
split as a plain contiguous batched GEMM: both operands re-laid out ONCE (untimed) as [16, 1000, 37348], then
torch.bmm -> [16, 1000, 1000] partials (+ the 16-way sum, timed separately). Also the un-split library call
and 8192^3 U(-1,1), in interleaved rounds in one process (methodology rule 24).

    python scripts/ab_vendor_split.py [--rounds 5] [--only ff|8k]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from netsdb_amd import ops  # noqa: E402


def timeit(fn, iters):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def run(fns, flops, rounds, iters):
    res = {k: [] for k in fns}
    for _ in range(rounds):
        for k, f in fns.items():
            res[k].append(timeit(f, iters))
    out = {}
    for k, v in res.items():
        med = statistics.median(v)
        out[k] = {"ms_median": round(med, 4), "ms_min": round(min(v), 4),
                  "tflops_median": round(flops.get(k, 0) / med / 1e9, 1)}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--only", choices=["ff", "8k", "all"], default="all")
    a = ap.parse_args()
    dev = "cuda:0"
    torch.manual_seed(0)
    if a.only in ("ff", "all"):
        M = N = 1000
        K, S = 597568, 16
        ks = K // S
        w1 = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
        x = torch.empty(N, K, device=dev, dtype=torch.bfloat16)
        w1.copy_(torch.empty(M, K, device=dev).uniform_(-1, 1).mul_((3.0 / 597540) ** 0.5))
        x.copy_(torch.empty(N, K, device=dev).uniform_(-1, 1))
        w1[:, 597540:] = 0
        x[:, 597540:] = 0
        w1s = w1.view(M, S, ks).transpose(0, 1).contiguous()
        xs = x.view(N, S, ks).transpose(0, 1).contiguous()
        part = torch.empty(S, M, N, device=dev, dtype=torch.bfloat16)
        ref = (w1.float() @ x.float().t())
        ours = ops.gemm_nt(w1, x, out_dtype=torch.float32)
        blas = torch.bmm(w1s, xs.transpose(1, 2)).float().sum(0)
        err = lambda t: ((t - ref).abs().max() / ref.abs().max()).item()  # noqa: E731
        print(json.dumps({"check": {"ours_rel_err": err(ours), "hipblaslt_split_rel_err": err(blas)}}), flush=True)
        fl = 2.0 * M * N * K
        fns = {
            "ours_splitk16": lambda: ops.gemm_nt(w1, x, out_dtype=torch.float32),
            "hipblaslt_bmm16": lambda: torch.bmm(w1s, xs.transpose(1, 2), out=part),
            "hipblaslt_bmm16_plus_sum": lambda: torch.bmm(w1s, xs.transpose(1, 2), out=part).float().sum(0),
            "hipblaslt_unsplit": lambda: torch.matmul(w1, x.t()),
        }
        flops = {k: fl for k in fns}
        print(json.dumps({"shape": "ff_layer1 1000x1000x597568", **run(fns, flops, a.rounds, 10)}), flush=True)
        del w1, x, w1s, xs, part, ref
        torch.cuda.empty_cache()
    if a.only in ("8k", "all"):
        n = 8192
        A = torch.empty(n, n, device=dev, dtype=torch.bfloat16).uniform_(-1, 1)
        B = torch.empty(n, n, device=dev, dtype=torch.bfloat16).uniform_(-1, 1)
        fns = {"ours": lambda: ops.gemm_nt(A, B), "hipblaslt": lambda: torch.matmul(A, B.t())}
        flops = {k: 2.0 * n ** 3 for k in fns}
        print(json.dumps({"shape": "8192^3", **run(fns, flops, a.rounds, 20)}), flush=True)


if __name__ == "__main__":
    main()
