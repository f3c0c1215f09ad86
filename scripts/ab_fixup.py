"""In-process interleaved A/B of the layer-1 GEMM's split-K reduction: the separate reducer launch vs the reduction
inside the 8-phase launch (gemm.hip splitk_fixup_8ph: the splits of a tile meet, each reduces 1/splits of the tile's
rows). FF layer-1 shape and epilogue of the headline bench (bias per column, relu, dropout 0.5, bf16 out), random
bf16 operands; bit-exactness against the reducer checked first. cdna_hip_programming.md rule 24: variants x rounds
in ONE process, a >= 2 s settle of back-to-back launches first.

    python scripts/ab_fixup.py [--rounds 8 --iters 20 --k 597544]
"""
import argparse
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from netsdb_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--m", type=int, default=1000)
    ap.add_argument("--n", type=int, default=1000)
    ap.add_argument("--k", type=int, default=597544)
    ap.add_argument("--settle-s", type=float, default=2.0)
    ap.add_argument("--plain", action="store_true", help="f32 output, no bias / activation / dropout")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    A = (torch.rand(a.m, a.k, device=dev, generator=g) - 0.5).to(torch.bfloat16)
    B = (torch.rand(a.n, a.k, device=dev, generator=g) - 0.5).to(torch.bfloat16)
    bias = torch.rand(a.n, device=dev, generator=g) - 0.5
    kw = dict(bias=bias, bias_mode=ops.BIAS_COL, act="relu", dropout=0.5, seed=7, cfg=2)
    if a.plain:
        kw = dict(out_dtype=torch.float32, cfg=2)
    ref = ops.gemm_nt(A, B, fixup=0, **kw)
    got = ops.gemm_nt(A, B, fixup=1, **kw)
    got2 = ops.gemm_nt(A, B, fixup=1, **kw)       # counters re-zeroed by the previous launch
    exact = bool(torch.equal(ref, got) and torch.equal(ref, got2))
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < a.settle_s:
        for fx in (0, 1):
            for _ in range(5):
                ops.gemm_nt(A, B, fixup=fx, **kw)
        torch.cuda.synchronize()
    res = {0: [], 1: []}
    for r in range(a.rounds):
        for fx in ((0, 1) if r % 2 == 0 else (1, 0)):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(a.iters):
                ops.gemm_nt(A, B, fixup=fx, **kw)
            e.record()
            torch.cuda.synchronize()
            res[fx].append(s.elapsed_time(e) / a.iters)
    out = {"shape": [a.m, a.n, a.k], "splits": int(ops.gemm_splits(a.m, a.n, a.k)), "bit_exact": exact,
           "rounds": a.rounds, "iters": a.iters}
    for fx, v in res.items():
        out["fixup" if fx else "reducer"] = {"median_ms": round(statistics.median(v), 4), "min_ms": round(min(v), 4),
                                             "max_ms": round(max(v), 4), "per_round_ms": [round(x, 4) for x in v]}
    out["saved_us_median"] = round((statistics.median(res[0]) - statistics.median(res[1])) * 1e3, 1)
    print(json.dumps(out), flush=True)
    if not exact:
        sys.exit(1)


if __name__ == "__main__":
    main()
