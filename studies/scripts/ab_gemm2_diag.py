"""Where the FF output GEMM's time goes (study build, 8-phase kernel, 1000 x 14588 x 1000, f32 exp + bias into
a 64-padded ldc): forced study configs / diagnostics timed in interleaved rounds —
  2: production structure; 102: no epilogue global stores; 9: DMA on zero-record descriptors (no operand memory
  traffic, LDS writes still happen); 109: both. Diagnostics compute wrong results (timing only).

    python scripts/ab_gemm2_diag.py [--rounds 5] [--cfgs 2,102,9,109]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from netsdb_amd import study, ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--cfgs", default="2,102,9,109")
    ap.add_argument("--K", type=int, default=1000)
    a = ap.parse_args()
    h = study.ext()
    M, N, K = 1000, 14588, a.K
    dev = "cuda:0"
    X = (torch.rand(M, K, device=dev) * 0.1).to(torch.bfloat16)
    W = (torch.randn(N, K, device=dev) * (1.0 / K ** 0.5)).to(torch.bfloat16)
    bias = torch.randn(N, device=dev) * 0.1
    outp = torch.empty(M, (N + 63) // 64 * 64, device=dev)[:, :N]
    fn = lambda: study.gemm_nt(X, W, bias, ops.BIAS_COL, ops.ACT_EXP, out_dtype=torch.float32, out=outp)  # noqa
    cfgs = [int(c) for c in a.cfgs.split(",")]
    res = {c: [] for c in cfgs}
    for _ in range(a.rounds):
        for c in cfgs:
            h.gemm_force_config(c)
            for _ in range(3):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            res[c].append(e0.elapsed_time(e1) / a.iters * 1000)
    h.gemm_force_config(-1)
    print(json.dumps({"shape": f"{M}x{N}x{K}", **{f"cfg{c}": {"us_min": round(min(v), 1),
                                                             "us_med": round(sorted(v)[len(v) // 2], 1)}
                                                  for c, v in res.items()}}), flush=True)


if __name__ == "__main__":
    main()
