"""Does a deeper LDS prefetch help the FF output layer when its weight is cold (as in the bench, after layer 1)?
Output GEMM 1000 x 14588 x 1000 (f32 exp + bias epilogue) under the study launcher: the 8-phase kernel (cfg 2,
3 half-tiles in flight) vs the 10-slot half-tile ring (cfg 14, 5 in flight), each hot (back to back) and cold (a
512 MB write in between). Interleaved rounds, CUDA events per call.

    python scripts/ab_out_ring_cold.py [--rounds 6]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from netsdb_amd import ops, study  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--iters", type=int, default=6)
    a = ap.parse_args()
    dev = "cuda:0"
    M, N, K = 1000, 14588, 1000
    g = torch.Generator(device=dev).manual_seed(0)
    H = torch.empty(M, K, device=dev).uniform_(0, 1, generator=g).to(torch.bfloat16)
    W = (torch.empty(N, K, device=dev).uniform_(-1, 1, generator=g) * (3.0 / K) ** 0.5).to(torch.bfloat16)
    bias = torch.empty(N, device=dev).uniform_(-0.1, 0.1, generator=g)
    flush = torch.empty(512 << 20, dtype=torch.uint8, device=dev)
    run = lambda cfg: study.gemm_nt(H, W, bias, ops.BIAS_COL, ops.ACT_EXP, out_dtype=torch.float32, cfg=cfg)  # noqa
    r2, r14 = run(2), run(14)
    torch.cuda.synchronize()
    print(json.dumps({"cfg14_vs_cfg2_max_abs": (r2 - r14).abs().max().item()}), flush=True)
    ts = {f"cfg{c}_{m}": [] for c in (2, 14) for m in ("hot", "cold")}
    for _ in range(a.rounds):
        for c in (2, 14):
            for mode in ("hot", "cold"):
                for _ in range(a.iters):
                    if mode == "cold":
                        flush.fill_(1)
                    else:
                        run(c)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    run(c)
                    e1.record()
                    torch.cuda.synchronize()
                    ts[f"cfg{c}_{mode}"].append(e0.elapsed_time(e1) * 1000)
    print(json.dumps({k: {"us_min": round(min(v), 1), "us_med": round(sorted(v)[len(v) // 2], 1)} for k, v in ts.items()}),
          flush=True)


if __name__ == "__main__":
    main()
