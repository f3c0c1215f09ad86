"""A/B: 8-phase GEMM on row-major operands vs the same kernel on K-tiled [K/64][rows][64] panels
(DRAM page locality of the 128-B-per-row k-step reads; guide §5.4 rule 24: interleaved rounds, one process).

    python scripts/ab_ktiled.py --shapes 1000x1000x597568,8192x8192x8192 [--rounds 5] [--scale-b 0.0022]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from netsdb_amd import study, _ext, ops  # noqa: E402


def ktile(t: torch.Tensor, ld: int) -> torch.Tensor:
    rows, K = t.shape
    p = torch.zeros(K // 64, ld, 64, dtype=t.dtype, device=t.device)
    p[:, :rows].copy_(t.view(rows, K // 64, 64).permute(1, 0, 2))
    return p


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="1000x1000x597568,8192x8192x8192")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--scale-b", type=float, default=1.0, help="scale of B (FF W1 init: sqrt(3/features))")
    a = ap.parse_args()
    h = study.ext()
    for sh in a.shapes.split(","):
        M, N, K = (int(x) for x in sh.split("x"))
        A = torch.empty(M, K, device="cuda:0", dtype=torch.bfloat16).uniform_(-1, 1)
        B = (torch.empty(N, K, device="cuda:0").uniform_(-1, 1) * a.scale_b).to(torch.bfloat16)
        ldA, ldB = (M + 255) // 256 * 256, (N + 255) // 256 * 256
        Ap, Bp = ktile(A, ldA), ktile(B, ldB)
        h.gemm_force_config(2)
        ref = study.gemm_nt(A, B, out_dtype=torch.float32)
        h.gemm_force_config(-1)
        got = h.gemm_nt_ktiled(Ap, Bp, M, N, K, True)
        err = ((got - ref).abs().max() / ref.abs().max().clamp(min=1e-6)).item()
        fns = {"rowmajor_8ph": lambda: study.gemm_nt(A, B), "ktiled_8ph": lambda: h.gemm_nt_ktiled(Ap, Bp, M, N, K, False)}
        best = {k: 1e9 for k in fns}
        for _ in range(a.rounds):
            for k, fn in fns.items():
                if k == "rowmajor_8ph":
                    h.gemm_force_config(2)
                for _ in range(3):
                    fn()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                h.gemm_force_config(-1)
                best[k] = min(best[k], e0.elapsed_time(e1) / a.iters)
        fl = 2.0 * M * N * K
        print(json.dumps({"shape": sh, "scale_b": a.scale_b, "rel_err_vs_rowmajor": err,
                          **{f"{k}_ms": round(v, 4) for k, v in best.items()},
                          **{f"{k}_tflops": round(fl / v / 1e9, 1) for k, v in best.items()}}), flush=True)
        del A, B, Ap, Bp, ref, got
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
