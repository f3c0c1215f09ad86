"""A/B of the adaptive split-K K partition (8-phase kernel, cfg 2) on vs off, interleaved rounds in one process.

The adaptive state learns per-split rates launch to launch, so each "on" round first runs a few launches
(the state persists across rounds: it converges once) and the per-launch times of the very first launches
are printed to show the convergence. Correctness: sampled rows vs an fp32 matmul, both settings.

    python scripts/ab_adapt.py --shapes 1000x1000x597568 --scale-b 0.0022 [--rounds 8]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from netsdb_amd import study, _ext, ops  # noqa: E402


def timed(A, B, n):
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
    evs[0].record()
    for i in range(n):
        study.gemm_nt(A, B)
        evs[i + 1].record()
    torch.cuda.synchronize()
    return [evs[i].elapsed_time(evs[i + 1]) for i in range(n)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="1000x1000x597568")
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--scale-b", type=float, default=1.0)
    ap.add_argument("--trace", type=int, default=12, help="launches timed one by one from a fresh state")
    a = ap.parse_args()
    h = study.ext()
    h.gemm_force_config(-1)
    for sh in a.shapes.split(","):
        M, N, K = (int(x) for x in sh.split("x"))
        g = torch.Generator(device="cuda:0").manual_seed(0)
        A = torch.empty(M, K, device="cuda:0", dtype=torch.bfloat16).uniform_(-1, 1, generator=g)
        B = (torch.empty(N, K, device="cuda:0").uniform_(-1, 1, generator=g) * a.scale_b).to(torch.bfloat16)
        rows = torch.randperm(M, device="cuda:0", generator=g)[:24].sort().values
        ref = A[rows].float() @ B.float().t()
        h.gemm_set_adapt(1)
        first = timed(A, B, a.trace)             # fresh state: the convergence
        res = {"shape": sh, "splits": ops.gemm_splits(M, N, K), "adapt_first_launches_ms": [round(t, 4) for t in first]}
        sh_, rt_ = h.gemm_adapt_state(M, N, K)
        res["shares_x_splits"] = [round(x * len(sh_), 3) for x in sh_]
        res["rates"] = [round(x, 4) for x in rt_]
        for on in (0, 1):
            h.gemm_set_adapt(on)
            out = study.gemm_nt(A, B, out_dtype=torch.float32)
            torch.cuda.synchronize()
            res[f"adapt{on}_rel_err"] = ((out[rows] - ref).abs().max() / ref.abs().max()).item()
            del out
        print(json.dumps(res), flush=True)
        per = {0: [], 1: []}
        for _ in range(a.rounds):
            for on in (0, 1):
                h.gemm_set_adapt(on)
                timed(A, B, 3)
                per[on] += timed(A, B, a.iters)
        fl = 2.0 * M * N * K
        out = {"shape": sh}
        for on in (0, 1):
            ts = sorted(per[on])
            out[f"adapt{on}_ms_min"] = round(ts[0], 4)
            out[f"adapt{on}_ms_med"] = round(ts[len(ts) // 2], 4)
            out[f"adapt{on}_ms_p90"] = round(ts[int(len(ts) * 0.9)], 4)
            out[f"adapt{on}_tflops_med"] = round(fl / ts[len(ts) // 2] / 1e9, 1)
        sh_, rt_ = h.gemm_adapt_state(M, N, K)
        out["final_shares_x_splits"] = [round(x * len(sh_), 3) for x in sh_]
        print(json.dumps(out), flush=True)
        h.gemm_set_adapt(0)
        del A, B


if __name__ == "__main__":
    main()
