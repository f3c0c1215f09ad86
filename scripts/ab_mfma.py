"""In-process interleaved A/B of the 8-phase GEMM main loop's MFMA shape (16x16x32 vs 32x32x16) on the FF layer-1
shape of the headline bench (W1 [1000, 597540] . X [1000, 597540]^T, split-K as the launcher picks it), random
bf16 operands as in bench.py. cdna_hip_programming.md rule 24: variants x rounds in ONE process, distribution
reported; a >= 2 s settle of back-to-back launches first (the chip's clock under load, MI355X_MICROARCH 'DVFS').

    python scripts/ab_mfma.py [--rounds 8 --iters 20 --k 597540]
"""
import argparse
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from netsdb_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--m", type=int, default=1000)
    ap.add_argument("--n", type=int, default=1000)
    ap.add_argument("--k", type=int, default=597544)
    ap.add_argument("--settle-s", type=float, default=2.0)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    A = (torch.rand(a.m, a.k, device=dev, generator=g) - 0.5).to(torch.bfloat16)
    B = (torch.rand(a.n, a.k, device=dev, generator=g) - 0.5).to(torch.bfloat16)
    kw = dict(out_dtype=torch.float32, cfg=2)
    ref = ops.gemm_nt(A, B, mfma=16, **kw)
    got = ops.gemm_nt(A, B, mfma=32, **kw)
    rel = ((got - ref).abs().max() / ref.abs().max()).item()
    flop = 2.0 * a.m * a.n * a.k
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < a.settle_s:
        for mf in (16, 32):
            for _ in range(5):
                ops.gemm_nt(A, B, mfma=mf, **kw)
        torch.cuda.synchronize()
    res = {16: [], 32: []}
    for r in range(a.rounds):
        order = (16, 32) if r % 2 == 0 else (32, 16)
        for mf in order:
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(a.iters):
                ops.gemm_nt(A, B, mfma=mf, **kw)
            e.record()
            torch.cuda.synchronize()
            res[mf].append(s.elapsed_time(e) / a.iters)
    out = {"shape": [a.m, a.n, a.k], "splits": int(ops.gemm_splits(a.m, a.n, a.k)), "rel_err_32_vs_16": rel,
           "rounds": a.rounds, "iters": a.iters}
    for mf, v in res.items():
        out[f"mfma{mf}"] = {"median_ms": round(statistics.median(v), 4), "min_ms": round(min(v), 4),
                            "max_ms": round(max(v), 4), "median_tflops": round(flop / statistics.median(v) / 1e9, 1),
                            "per_round_ms": [round(x, 4) for x in v]}
    out["speedup_32_over_16"] = round(statistics.median(res[16]) / statistics.median(res[32]), 4)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
