"""Data dependence of the FF layer-1 GEMM time (power-limited clock): the same 1000x1000x597568 split-K GEMM on
operands with different bit activity, interleaved rounds, CUDA events.

    python scripts/ab_data_power.py [--rounds 5]
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
    a = ap.parse_args()
    study.ext().gemm_set_adapt(0)
    M, N, K = 1000, 1000, 597568
    g = torch.Generator(device="cuda:0").manual_seed(0)
    X = torch.empty(M, K, device="cuda:0").uniform_(-1, 1, generator=g).to(torch.bfloat16)
    W = torch.empty(N, K, device="cuda:0").uniform_(-1, 1, generator=g).to(torch.bfloat16)
    Ws = (W.float() * 0.00224).to(torch.bfloat16)
    Z = torch.zeros_like(W)
    O = torch.ones_like(W)
    cases = {"uniform x uniform": (X, W), "uniform x scaled (bench W1)": (X, Ws), "uniform x ones": (X, O),
             "uniform x zeros": (X, Z)}
    ts = {k: [] for k in cases}
    for _ in range(a.rounds):
        for k, (A, B) in cases.items():
            for _ in range(3):
                study.gemm_nt(A, B)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                study.gemm_nt(A, B)
            e1.record()
            torch.cuda.synchronize()
            ts[k].append(e0.elapsed_time(e1) / a.iters)
    print(json.dumps({k: {"ms_min": round(min(v), 4), "ms_med": round(sorted(v)[len(v) // 2], 4)} for k, v in ts.items()}))


if __name__ == "__main__":
    main()
