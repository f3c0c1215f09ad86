"""Interleaved A/B timing of GEMM tile configs / kernel variants in one process (guide §5.4 rule 24).

    python scripts/ab_gemm.py --cfgs 1,2,3 --shapes 8192x8192x8192,1000x1000x597568 [--rounds 5]
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
    ap.add_argument("--cfgs", default="0,1,2")
    ap.add_argument("--shapes", default="8192x8192x8192,4096x4096x4096,1000x1000x597568")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    cfgs = [int(c) for c in a.cfgs.split(",")]
    for sh in a.shapes.split(","):
        M, N, K = (int(x) for x in sh.split("x"))
        A = torch.empty(M, K, device="cuda:0", dtype=torch.bfloat16).uniform_(-1, 1)
        B = torch.empty(N, K, device="cuda:0", dtype=torch.bfloat16).uniform_(-1, 1)
        best = {c: 1e9 for c in cfgs}
        for _ in range(a.rounds):
            for c in cfgs:
                study.ext().gemm_force_config(c)
                for _ in range(3):
                    study.gemm_nt(A, B)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    study.gemm_nt(A, B)
                e1.record()
                torch.cuda.synchronize()
                best[c] = min(best[c], e0.elapsed_time(e1) / a.iters)
        study.ext().gemm_force_config(-1)
        fl = 2.0 * M * N * K
        print(json.dumps({"shape": sh, **{f"cfg{c}_tflops": round(fl / best[c] / 1e9, 1) for c in cfgs}}), flush=True)
        del A, B


if __name__ == "__main__":
    main()
