"""Split-K fix-up by each tile's last-arriving workgroup inside the GEMM launch (cfg 26) vs the 8-phase GEMM +
separate slab reducer (cfg 2) on the FF layer-1 GEMM with its real epilogue (bias per row, relu, dropout, bf16
out): bit-exactness check, then interleaved timing rounds (GEMM + reduce together, CUDA events).

    python scripts/ab_fixup.py [--rounds 5] [--iters 10]
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
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    h = study.ext()
    h.gemm_set_adapt(0)
    M, N, K = (int(x) for x in a.shape.split("x"))
    g = torch.Generator(device="cuda:0").manual_seed(0)
    A = torch.empty(M, K, device="cuda:0").uniform_(-1, 1, generator=g).to(torch.bfloat16)
    B = (torch.empty(N, K, device="cuda:0").uniform_(-1, 1, generator=g) * 0.00224).to(torch.bfloat16)
    bias = torch.randn(M, device="cuda:0", generator=g) * 0.1

    def run():
        return study.gemm_nt(A, B, bias, ops.BIAS_ROW, ops.ACT_RELU, dropout=0.5, seed=7)

    outs = {}
    for cfg in (2, 26, 26):
        h.gemm_force_config(cfg)
        outs.setdefault(cfg, []).append(run())
    torch.cuda.synchronize()
    exact = all(torch.equal(o, outs[2][0]) for o in outs[26])
    ts = {2: [], 26: []}
    for _ in range(a.rounds):
        for cfg in (2, 26):
            h.gemm_force_config(cfg)
            for _ in range(3):
                run()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                run()
            e1.record()
            torch.cuda.synchronize()
            ts[cfg].append(e0.elapsed_time(e1) / a.iters)
    h.gemm_force_config(-1)
    print(json.dumps({"bit_exact_vs_reducer": exact,
                      **{("gemm+reduce" if c == 2 else "gemm_fixup"): {"ms_min": round(min(v), 4),
                                                                      "ms_med": round(sorted(v)[len(v) // 2], 4)}
                         for c, v in ts.items()}}))


if __name__ == "__main__":
    main()
