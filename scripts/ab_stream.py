"""A/B of the skinny long-K GEMM tiles: the 8-phase 256x256 kernel (cfg 2), the 256x128 / 128x256 stream tiles
(cfg 3 / 4: contiguous K chunk per split, cfg 5 / 6: k-interleaved splits) and the 128x128 tile (cfg 0) on the dedup scoring shapes and neighbours. Interleaved rounds, CUDA-event
timing of GEMM + split-K reduce, median / min over rounds; also the HBM bytes of the big operands -> TB/s.

    python scripts/ab_stream.py [--rounds 7] [--iters 10]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [  # (M, N, K, batch)
    (500, 100, 900000, 1),      # dedup common panel
    (500, 100, 100000, 12),     # dedup private panels (batched)
    (100, 500, 900000, 1),      # the same, operands swapped
    (6000, 100, 100000, 1),
    (1000, 128, 600000, 1),
    (1000, 64, 600000, 1),
    (4096, 128, 16384, 1),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    from netsdb_amd import ops
    dev = "cuda:0"
    for (M, N, K, b) in SHAPES:
        shp = (b,) if b > 1 else ()
        torch.manual_seed(0)
        A = (torch.randn(*shp, M, K, device=dev) * 0.05).to(torch.bfloat16)
        B = (torch.randn(*shp, N, K, device=dev) * 0.05).to(torch.bfloat16)
        ref = None
        cfgs = [2, 3 if M >= N else 4, 5 if M >= N else 6, 0]
        times = {c: [] for c in cfgs}
        errs = {}
        for c in cfgs:      # warm + check
            C = ops.gemm_nt(A, B, out_dtype=torch.float32, cfg=c)
            if ref is None:
                ref = C
            errs[c] = ((C - ref).abs().max() / (ref.abs().max() + 1e-9)).item()
        torch.cuda.synchronize()
        for _ in range(a.rounds):
            for c in cfgs:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    ops.gemm_nt(A, B, out_dtype=torch.float32, cfg=c)
                e1.record()
                torch.cuda.synchronize()
                times[c].append(e0.elapsed_time(e1) * 1e3 / a.iters)
        gb = (A.numel() + B.numel()) * 2 / 1e9
        row = {"M": M, "N": N, "K": K, "batch": b, "GB": round(gb, 3)}
        for c in cfgs:
            t = sorted(times[c])
            row[f"cfg{c}_us_med"] = round(t[len(t) // 2], 1)
            row[f"cfg{c}_us_min"] = round(t[0], 1)
            row[f"cfg{c}_TBps"] = round(gb / (t[len(t) // 2] * 1e-6) / 1e3, 2)
            row[f"cfg{c}_rel_vs_cfg2"] = errs[c]
        print(json.dumps(row), flush=True)
        del A, B, ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
