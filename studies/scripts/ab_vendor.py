"""Our GEMM vs hipBLASLt (torch.matmul / torch.bmm) on the same random operands, interleaved rounds in one
process: square shapes and the FF layer shapes. (A 16-way strided-batched torch.bmm over the FF layer-1 K
slices, lda 597568, hung and faulted the GPU inside the vendor library: not run again.)

    python scripts/ab_vendor.py [--rounds 4]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from netsdb_amd import ops  # noqa: E402


def timeit(fn, iters=10):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=4)
    a = ap.parse_args()
    dev = "cuda:0"
    res = {}
    for (M, N, K) in [(8192, 8192, 8192), (4096, 4096, 4096), (1000, 14588, 1000), (1000, 1000, 597568)]:
        A = torch.empty(M, K, device=dev, dtype=torch.bfloat16).uniform_(-1, 1)
        B = torch.empty(N, K, device=dev, dtype=torch.bfloat16).uniform_(-1, 1)
        fns = {"ours": lambda: ops.gemm_nt(A, B), "hipblaslt": lambda: torch.matmul(A, B.t())}
        best = {k: 1e9 for k in fns}
        for _ in range(a.rounds):
            for k, f in fns.items():
                best[k] = min(best[k], timeit(f))
        fl = 2.0 * M * N * K
        res = {"shape": f"{M}x{N}x{K}", **{f"{k}_ms": round(v, 4) for k, v in best.items()},
               **{f"{k}_tflops": round(fl / v / 1e9, 1) for k, v in best.items()}}
        print(json.dumps(res), flush=True)
        del A, B


if __name__ == "__main__":
    main()
