"""FF output layer on the PRODUCTION kernels (not the study build), the bench's shapes and data scales:
the output GEMM 1000 x 14588 x 1000 with the f32 exp + per-label bias epilogue into a 64-padded ldc (what the
two-job FFOutputLayer path runs), the row normaliser after it, the fused max-subtracted softmax GEMM (the
single-job path), and a plain bf16 GEMM of the same shape.
Interleaved rounds in one process, CUDA-event timing; correctness of both output paths vs an fp32 softmax.

    python scripts/ab_ff_tail.py [--rounds 5] [--iters 20]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from netsdb_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = "cuda:0"
    M, N, K = 1000, 14588, 1000
    g = torch.Generator(device=dev).manual_seed(0)
    H = torch.empty(M, K, device=dev).uniform_(0, 1, generator=g).to(torch.bfloat16)          # relu'd hidden
    W = (torch.empty(N, K, device=dev).uniform_(-1, 1, generator=g) * (3.0 / K) ** 0.5).to(torch.bfloat16)
    bias = torch.empty(N, device=dev).uniform_(-0.1, 0.1, generator=g)
    outp = torch.empty(M, (N + 63) // 64 * 64, device=dev)[:, :N]
    sm_out = torch.empty(M, N, device=dev)

    ref = torch.softmax(H.float() @ W.float().t() + bias, dim=1)
    e = ops.gemm_nt(H, W, bias, ops.BIAS_COL, ops.ACT_EXP, out_dtype=torch.float32, out=outp)
    y2 = ops.row_normalize(e, out_dtype=torch.float32)
    y1 = ops.gemm_nt_softmax(H, W, bias, ops.BIAS_COL, axis=1, out=sm_out)
    e0_ = ops.gemm_nt(H, W, bias, ops.BIAS_COL, ops.ACT_EXP, out_dtype=torch.float32, epi=0)
    e1_ = ops.gemm_nt(H, W, bias, ops.BIAS_COL, ops.ACT_EXP, out_dtype=torch.float32, epi=1)
    torch.cuda.synchronize()
    err = {"two_job_max_abs": (y2 - ref).abs().max().item(), "fused_max_abs": (y1 - ref).abs().max().item(),
           "ref_max": ref.max().item(), "direct_vs_lds_epi_max_abs": (e0_ - e1_).abs().max().item()}
    print(json.dumps(err), flush=True)

    fns = {
        "gemm2_exp_f32": lambda: ops.gemm_nt(H, W, bias, ops.BIAS_COL, ops.ACT_EXP, out_dtype=torch.float32, out=outp),
        "gemm2_exp_f32_ldsepi": lambda: ops.gemm_nt(H, W, bias, ops.BIAS_COL, ops.ACT_EXP, out_dtype=torch.float32,
                                                    out=outp, epi=0),
        "row_normalize": lambda: ops.row_normalize(outp, out_dtype=torch.float32),
        "two_job_total": lambda: ops.row_normalize(
            ops.gemm_nt(H, W, bias, ops.BIAS_COL, ops.ACT_EXP, out_dtype=torch.float32, out=outp), out_dtype=torch.float32),
        "fused_softmax_gemm": lambda: ops.gemm_nt_softmax(H, W, bias, ops.BIAS_COL, axis=1, out=sm_out),
        "fused_softmax_gemm_ldsepi": lambda: ops.gemm_nt_softmax(H, W, bias, ops.BIAS_COL, axis=1, out=sm_out, epi=0),
        "gemm2_bf16_nobias": lambda: ops.gemm_nt(H, W),
    }
    ts = {k: [] for k in fns}
    for _ in range(a.rounds):
        for k, fn in fns.items():
            for _ in range(3):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            ts[k].append(e0.elapsed_time(e1) / a.iters * 1000)
    print(json.dumps({f"{k}_us_min": round(min(v), 1) for k, v in ts.items()} |
                     {f"{k}_us_med": round(sorted(v)[len(v) // 2], 1) for k, v in ts.items()}), flush=True)


if __name__ == "__main__":
    main()
