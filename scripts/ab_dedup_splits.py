"""A/B of the split-K count on the dedup harness's skinny long-K GEMMs (config 5: 12 models x 500 rows, batch 100):
the launcher's one-wave choice against split counts that fill a second / third wave of workgroups.

    python scripts/ab_dedup_splits.py [--iters 20]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from netsdb_amd import ops  # noqa: E402
from netsdb_amd import _ext  # noqa: E402


def timed(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    h = _ext.hip()
    out = {}
    shapes = {"private_12x500x100x100k": (12, 500, 100, 100_000), "common_500x100x900k": (1, 500, 100, 900_000)}
    for name, (bt, M, N, K) in shapes.items():
        A = torch.randn((bt, M, K) if bt > 1 else (M, K), device=dev, generator=g).to(torch.bfloat16)
        B = torch.randn(N, K, device=dev, generator=g).to(torch.bfloat16)
        Bv = B.unsqueeze(0).expand(bt, -1, -1) if bt > 1 else B
        auto = h.gemm_splits(M, N, K, bt)
        ref = ops.gemm_nt(A, Bv, out_dtype=torch.float32)
        res = {"auto_splits": auto}
        for s in sorted({auto, 21, 32, 2 * auto, 3 * auto} if bt > 1 else {auto, 2 * auto}):
            got = ops.gemm_nt(A, Bv, out_dtype=torch.float32, splits=s)
            err = ((got - ref).abs().max() / ref.abs().max()).item()
            res[f"s{s}"] = {"us": round(timed(lambda: ops.gemm_nt(A, Bv, out_dtype=torch.float32, splits=s), a.iters), 1),
                            "rel_err": err}
        # interleaved second pass of the auto choice (clock drift check)
        res["auto_again_us"] = round(timed(lambda: ops.gemm_nt(A, Bv, out_dtype=torch.float32), a.iters), 1)
        out[name] = res
        print(json.dumps({name: res}), flush=True)
        del A, B, Bv, ref


if __name__ == "__main__":
    main()
