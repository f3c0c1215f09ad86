"""A/B timing of the FF output-layer GEMM (short K, wide N) across tile configs and epilogues.

    python scripts/ab_gemm2.py [--cfgs 0,1,2] [--rounds 5]

Shape of netsDB's FFTransposeBiasSum input product on AmazonCat-14k: Y [1000 batch, 1000 hidden]
times Wo [14588 labels, 1000 hidden]^T, + bias per label, exp, f32 out (then row-normalised).
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from netsdb_amd import study, _ext, ops  # noqa: E402


def timeit(fn, iters, rounds):
    best = 1e9
    for _ in range(rounds):
        for _ in range(2):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / iters)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfgs", default="0,1,2")
    ap.add_argument("--shapes", default="1000x14588x1000,14588x1000x1000,1000x1000x597568")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--out-ld-align", type=int, default=1, help="C row stride alignment (elements)")
    ap.add_argument("--splits", type=int, default=0, help="force split-K (0 = launcher's choice)")
    ap.add_argument("--epis", default="plain_bf16,bias_exp_f32")
    ap.add_argument("--ld-align", type=int, default=8, help="operand row stride alignment (elements)")
    a = ap.parse_args()
    cfgs = [int(c) for c in a.cfgs.split(",")]
    for sh in a.shapes.split(","):
        M, N, K = (int(x) for x in sh.split("x"))
        ld = (K + a.ld_align - 1) // a.ld_align * a.ld_align
        A = torch.empty(M, ld, device="cuda:0", dtype=torch.bfloat16).uniform_(-0.05, 0.05)[:, :K]
        B = torch.empty(N, ld, device="cuda:0", dtype=torch.bfloat16).uniform_(-0.05, 0.05)[:, :K]
        bias = torch.zeros(N, device="cuda:0")
        ref = None
        res = {"shape": sh, "ld": ld}
        ldc = (N + a.out_ld_align - 1) // a.out_ld_align * a.out_ld_align
        Cb = torch.empty(M, ldc, device="cuda:0", dtype=torch.bfloat16)[:, :N]
        Cf = torch.empty(M, ldc, device="cuda:0", dtype=torch.float32)[:, :N]
        res["ldc"] = ldc
        for c in cfgs:
            if c < 0:   # hipBLASLt reference (torch.matmul, bf16 out, no epilogue)
                ms = timeit(lambda: torch.matmul(A, B.t()), a.iters, a.rounds)
                res["hipblaslt_bf16_us"] = round(ms * 1e3, 1)
                continue
            study.ext().gemm_force_config(c)
            for epi in a.epis.split(","):
                if epi == "plain_bf16":
                    fn = lambda: study.gemm_nt(A, B, out=Cb, splits=a.splits)  # noqa: E731
                else:
                    fn = lambda: study.gemm_nt(A, B, bias, ops.BIAS_COL, ops.ACT_EXP, out_dtype=torch.float32, out=Cf,
                                               splits=a.splits)  # noqa: E731
                ms = timeit(fn, a.iters, a.rounds)
                res[f"cfg{c}_{epi}_us"] = round(ms * 1e3, 1)
                res[f"cfg{c}_{epi}_tflops"] = round(2.0 * M * N * K / ms / 1e9, 1)
            out = study.gemm_nt(A, B, bias, ops.BIAS_COL, ops.ACT_EXP, out_dtype=torch.float32)
            if ref is None and M * N * K < 2e11:
                ref = torch.exp(A.float() @ B.float().t())
            if ref is not None:
                res[f"cfg{c}_maxrel"] = float(((out - ref).abs() / ref.abs().clamp_min(1e-3)).max())
        study.ext().gemm_force_config(-1)
        print(json.dumps(res), flush=True)
        del A, B


if __name__ == "__main__":
    main()
