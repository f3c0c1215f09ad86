"""Is the FF layer-1 GEMM power-limited or CU-limited? Layer 1 (1000 x 1000 x 597568, bench data) with fewer
split-K slices, i.e. fewer workgroups (one per CU) than the 256 CUs: if the time grows much less than 256 / WGs,
the chip's power budget, not its CU count, sets the rate (then CUs can be given to another job for free).
Interleaved rounds, CUDA events, GEMM + reducer.

    python scripts/ab_gemm1_splits_power.py [--rounds 4]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from netsdb_amd import _ext, ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--iters", type=int, default=8)
    ap.add_argument("--splits", default="16,15,14,12,8")
    a = ap.parse_args()
    dev = "cuda:0"
    M, N, K = 1000, 1000, 597568
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.empty(M, K, device=dev).uniform_(-1, 1, generator=g).to(torch.bfloat16)
    W = (torch.empty(N, K, device=dev).uniform_(-1, 1, generator=g) * (3.0 / K) ** 0.5).to(torch.bfloat16)
    sp = [int(s) for s in a.splits.split(",")]
    ts = {s: [] for s in sp}
    for _ in range(a.rounds):
        for s in sp:
            for _ in range(2):
                ops.gemm_nt(W, X, splits=s)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                ops.gemm_nt(W, X, splits=s)
            e1.record()
            torch.cuda.synchronize()
            ts[s].append(e0.elapsed_time(e1) / a.iters * 1000)
    base = sorted(ts[sp[0]])[len(ts[sp[0]]) // 2]
    print(json.dumps({f"splits{s}_wgs{16 * s}": {"us_med": round(sorted(v)[len(v) // 2], 1),
                                                 "time_ratio": round(sorted(v)[len(v) // 2] / base, 3),
                                                 "cu_ratio": round(16 * sp[0] / (16 * s), 3)} for s, v in ts.items()}),
          flush=True)


if __name__ == "__main__":
    main()
