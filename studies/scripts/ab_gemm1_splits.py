"""Interleaved timing of the FF layer-1 GEMM (1000x1000x597568, 8-phase 256^2) over split-K factors:
fewer splits = fewer busy CUs (16 tiles x splits workgroups) but less slab traffic; under the power cap the
clock may rise.  python studies/scripts/ab_gemm1_splits.py [--splits 16,15,14,12] [--rounds 4] [--iters 10]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from netsdb_amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--splits", default="16,15,14,12,8")
ap.add_argument("--rounds", type=int, default=4)
ap.add_argument("--iters", type=int, default=10)
a = ap.parse_args()
M, N, K = 1000, 1000, 597568
A = torch.empty(M, K, device="cuda:0", dtype=torch.bfloat16).uniform_(-1, 1)
B = torch.empty(N, K, device="cuda:0", dtype=torch.bfloat16).uniform_(-1, 1)
cands = [int(s) for s in a.splits.split(",")]
ref = ops.gemm_nt(A, B, out_dtype=torch.float32, splits=16)
for s in cands:  # every split factor computes the same product
    d = (ops.gemm_nt(A, B, out_dtype=torch.float32, splits=s) - ref).abs().max().item()
    assert d < 1e-2 * ref.abs().max().item(), (s, d)
for _ in range(3):
    ops.gemm_nt(A, B, splits=16)
best = {s: 1e9 for s in cands}
for r in range(a.rounds):
    for s in cands:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            ops.gemm_nt(A, B, splits=s)
        e1.record()
        e1.synchronize()
        best[s] = min(best[s], e0.elapsed_time(e1) / a.iters)
    print(json.dumps({"round": r, "ms": {s: round(best[s], 4) for s in cands}}), flush=True)
print(json.dumps({"shape": f"{M}x{N}x{K}", "best_ms": best,
                  "tflops": {s: round(2 * M * N * K / best[s] / 1e9, 1) for s in cands}}))
