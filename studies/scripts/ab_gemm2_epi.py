"""FF output-layer GEMM (1000 x 14588 x 1000) epilogue cost breakdown, interleaved rounds in one process:
bf16 out / f32 out / f32 + bias + exp (the in-bench softmax numerator, 64-padded ldc) / the same with the
epilogue's global stores skipped (diag 1), the row normaliser that follows it, the two together, and the
softmax fused into the GEMM epilogue (ops.gemm_nt_softmax).

    python scripts/ab_gemm2_epi.py [--rounds 5] [--cfg 2]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from netsdb_amd import study, _ext, ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--cfg", type=int, default=2)
    ap.add_argument("--M", type=int, default=1000)
    ap.add_argument("--N", type=int, default=14588)
    ap.add_argument("--K", type=int, default=1000)
    a = ap.parse_args()
    h = study.ext()
    M, N, K = a.M, a.N, a.K
    dev = "cuda:0"
    X = (torch.rand(M, K, device=dev) * 0.1).to(torch.bfloat16)
    W = (torch.randn(N, K, device=dev) * (1.0 / K ** 0.5)).to(torch.bfloat16)
    bias = torch.randn(N, device=dev) * 0.1
    outp = torch.empty(M, (N + 63) // 64 * 64, device=dev)[:, :N]
    variants = {
        "bf16_noepi": lambda: study.gemm_nt(X, W),
        "f32_noepi": lambda: study.gemm_nt(X, W, out_dtype=torch.float32, out=outp),
        "f32_bias_exp": lambda: study.gemm_nt(X, W, bias, ops.BIAS_COL, ops.ACT_EXP, out_dtype=torch.float32, out=outp),
        "f32_bias_exp_nostore": "diag",
        "rownorm": lambda: ops.row_normalize(outp, out_dtype=torch.float32),
        "exp_then_rownorm": lambda: ops.row_normalize(
            study.gemm_nt(X, W, bias, ops.BIAS_COL, ops.ACT_EXP, out_dtype=torch.float32, out=outp), out_dtype=torch.float32),
        "fused_softmax": lambda: ops.gemm_nt_softmax(X, W, bias, ops.BIAS_COL, axis=1, out=outp),
    }
    res = {k: [] for k in variants}
    for _ in range(a.rounds):
        for name, fn in variants.items():
            if fn == "diag":
                h.gemm_force_config(100 + a.cfg)
                fn = variants["f32_bias_exp"]
            else:
                h.gemm_force_config(a.cfg)
            for _ in range(3):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            res[name].append(e0.elapsed_time(e1) / a.iters * 1000)
    h.gemm_force_config(-1)
    print(json.dumps({"shape": f"{M}x{N}x{K}", "cfg": a.cfg,
                      **{k: {"us_min": round(min(v), 1), "us_med": round(sorted(v)[len(v) // 2], 1)} for k, v in res.items()}}))


if __name__ == "__main__":
    main()
