"""Sweep of the K-tail stealing geometry (cfg 24: tail chunks per split x k-tiles per chunk) against the
static split-K partition (cfg 2) on the FF layer-1 GEMM, interleaved rounds, B scaled like W1.

    python scripts/ab_steal.py [--geoms 4x16,8x16,8x8,16x8,2x16] [--rounds 5]
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
    ap.add_argument("--shape", default="1000x1000x597568")
    ap.add_argument("--geoms", default="4x16,8x16,8x8,16x8,2x16,4x8")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    h = study.ext()
    M, N, K = (int(x) for x in a.shape.split("x"))
    g = torch.Generator(device="cuda:0").manual_seed(0)
    A = torch.empty(M, K, device="cuda:0").uniform_(-1, 1, generator=g).to(torch.bfloat16)
    B = (torch.empty(N, K, device="cuda:0").uniform_(-1, 1, generator=g) * 0.00224).to(torch.bfloat16)
    confs = [("static", 2, None)] + [(f"steal{gm}", 24, tuple(int(x) for x in gm.split("x")))
                                     for gm in a.geoms.split(",")]
    ts = {n: [] for n, _, _ in confs}
    for _ in range(a.rounds):
        for n, cfg, geom in confs:
            h.gemm_force_config(cfg)
            if geom:
                h.gemm_steal(*geom)
            for _ in range(3):
                study.gemm_nt(A, B)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                study.gemm_nt(A, B)
            e1.record()
            torch.cuda.synchronize()
            ts[n].append(e0.elapsed_time(e1) / a.iters)
    h.gemm_force_config(-1)
    h.gemm_steal(4, 16)
    print(json.dumps({n: {"ms_min": round(min(v), 4), "ms_med": round(sorted(v)[len(v) // 2], 4)} for n, v in ts.items()}))


if __name__ == "__main__":
    main()
