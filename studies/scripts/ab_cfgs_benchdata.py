"""FF layer-1 GEMM tile configs on the bench's operand data (inputs uniform(-1,1), W1 scaled by sqrt(3/K) as
ff.load_model initialises it) — the clock is power-limited, so config A/Bs must use the data the bench runs.
Interleaved rounds, CUDA events; GEMM + split-K reducer.

    python scripts/ab_cfgs_benchdata.py [--cfgs 2,12,16,14] [--rounds 5]
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
    ap.add_argument("--cfgs", default="2,12,16,14")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    h = study.ext()
    h.gemm_set_adapt(0)
    M, N, K = 1000, 1000, 597568
    g = torch.Generator(device="cuda:0").manual_seed(0)
    X = torch.empty(M, K, device="cuda:0").uniform_(-1, 1, generator=g).to(torch.bfloat16)
    W = (torch.empty(N, K, device="cuda:0").uniform_(-1, 1, generator=g) * (3.0 / K) ** 0.5).to(torch.bfloat16)
    cfgs = [int(c) for c in a.cfgs.split(",")]
    ts = {c: [] for c in cfgs}
    for _ in range(a.rounds):
        for c in cfgs:
            h.gemm_force_config(c)
            for _ in range(3):
                study.gemm_nt(W, X)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                study.gemm_nt(W, X)
            e1.record()
            torch.cuda.synchronize()
            ts[c].append(e0.elapsed_time(e1) / a.iters)
    h.gemm_force_config(-1)
    print(json.dumps({f"cfg{c}": {"ms_min": round(min(v), 4), "ms_med": round(sorted(v)[len(v) // 2], 4)}
                      for c, v in ts.items()}))


if __name__ == "__main__":
    main()
