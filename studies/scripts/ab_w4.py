"""A/B of the 8-phase 8-wave GEMM (cfg 2) vs the 4-wave 128x128-per-wave kernel (cfg 12) in one process,
interleaved rounds (guide §5.4 rule 24), uniform random bf16 operands, plus a correctness check of each
config against an fp32 matmul on sampled rows.

    python scripts/ab_w4.py --shapes 1000x1000x597568,8192x8192x8192 [--cfgs 2,12] [--rounds 5]
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
    ap.add_argument("--shapes", default="1000x1000x597568,8192x8192x8192")
    ap.add_argument("--cfgs", default="2,12")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--check-only", action="store_true")
    ap.add_argument("--scale-b", type=float, default=1.0, help="B ~ U(-1,1) * scale (FF W1 init: sqrt(3/features))")
    a = ap.parse_args()
    h = study.ext()
    cfgs = [int(c) for c in a.cfgs.split(",")]
    for sh in a.shapes.split(","):
        M, N, K = (int(x) for x in sh.split("x"))
        g = torch.Generator(device="cuda:0").manual_seed(0)
        A = torch.empty(M, K, device="cuda:0", dtype=torch.bfloat16).uniform_(-1, 1, generator=g)
        B = (torch.empty(N, K, device="cuda:0").uniform_(-1, 1, generator=g) * a.scale_b).to(torch.bfloat16)
        rows = torch.randperm(M, device="cuda:0", generator=g)[:24].sort().values
        rows[-1] = M - 1
        ref = A[rows].float() @ B.float().t()
        res = {"shape": sh, "splits": ops.gemm_splits(M, N, K)}
        for c in cfgs:
            h.gemm_force_config(c)
            out = study.gemm_nt(A, B, out_dtype=torch.float32)
            torch.cuda.synchronize()
            err = ((out[rows] - ref).abs().max() / ref.abs().max()).item()
            res[f"cfg{c}_rel_err"] = err
            del out
        h.gemm_force_config(-1)
        print(json.dumps(res), flush=True)
        if a.check_only:
            continue
        best = {c: [] for c in cfgs}
        for _ in range(a.rounds):
            for c in cfgs:
                h.gemm_force_config(c)
                for _ in range(3):
                    study.gemm_nt(A, B)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    study.gemm_nt(A, B)
                e1.record()
                torch.cuda.synchronize()
                best[c].append(e0.elapsed_time(e1) / a.iters)
        h.gemm_force_config(-1)
        fl = 2.0 * M * N * K
        out = {"shape": sh}
        for c in cfgs:
            ts = sorted(best[c])
            out[f"cfg{c}_ms_min"] = round(ts[0], 4)
            out[f"cfg{c}_ms_med"] = round(ts[len(ts) // 2], 4)
            out[f"cfg{c}_tflops_min_t"] = round(fl / ts[0] / 1e9, 1)
        print(json.dumps(out), flush=True)
        del A, B


if __name__ == "__main__":
    main()
