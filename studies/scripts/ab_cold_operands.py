"""Cold vs MALL-warm operands for the FF output GEMM (1000 x 14588 x 1000, f32 exp + bias) and the conv2d block
(100 x 3 x 112^2, 64 filters 7x7): in the bench both run right after the layer-1 GEMM has streamed 2.4 GB
through the Infinity Cache, so their operands come from HBM; in isolated A/B loops they are cache-hot. Each
timed call here follows (a) a 1 GiB read that evicts the cache ('cold'), (b) the same read and then a plain
ops.prefetch of just the call's operands ('prefetched'), (c) nothing ('hot'). Event timing of the call alone.

    python scripts/ab_cold_operands.py [--rounds 5]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from netsdb_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    dev = "cuda:0"
    g = torch.Generator(device=dev).manual_seed(0)
    M, N, K = 1000, 14588, 1000
    H = torch.empty(M, K, device=dev).uniform_(0, 1, generator=g).to(torch.bfloat16)
    W = (torch.empty(N, K, device=dev).uniform_(-1, 1, generator=g) * (3.0 / K) ** 0.5).to(torch.bfloat16)
    bias = torch.empty(N, device=dev).uniform_(-0.1, 0.1, generator=g)
    outp = torch.empty(M, (N + 63) // 64 * 64, device=dev)[:, :N]
    X = torch.empty(100, 3, 112, 112, device=dev).uniform_(-1, 1, generator=g).to(torch.bfloat16)
    Wf = ops.pad_k(torch.empty(64, 147, device=dev).uniform_(-0.1, 0.1, generator=g)).to(torch.bfloat16).contiguous()
    cb = torch.randn(64, device=dev, generator=g)
    big = torch.empty(512 << 20, device=dev, dtype=torch.bfloat16).uniform_(-1, 1, generator=g)   # 1 GiB

    calls = {
        "gemm2": (lambda: ops.gemm_nt(H, W, bias, ops.BIAS_COL, ops.ACT_EXP, out_dtype=torch.float32, out=outp),
                  lambda: ops.prefetch([W, H, bias])),
        "conv": (lambda: ops.conv2d(X, Wf, cb, 7, 7, 1, 0, nchw_out=True), lambda: ops.prefetch([X])),
    }
    modes = ("cold", "prefetched", "hot", "after_write")
    res = {f"{k}_{m}": [] for k in calls for m in modes}
    for _ in range(a.rounds):
        for k, (fn, pre) in calls.items():
            for mode in modes:
                for _ in range(3):
                    fn()
                ts = []
                for _ in range(5):
                    if mode in ("cold", "prefetched"):
                        big.sum()          # result discarded: the read is the point
                    if mode == "after_write":
                        ops.row_normalize(outp, out_dtype=torch.float32)   # 58 MB read + 58 MB written just before
                    if mode == "prefetched":
                        pre()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    fn()
                    e1.record()
                    torch.cuda.synchronize()
                    ts.append(e0.elapsed_time(e1) * 1000)
                res[f"{k}_{mode}"].append(sorted(ts)[len(ts) // 2])
    print(json.dumps({f"{k}_us_med": round(sorted(v)[len(v) // 2], 1) for k, v in res.items()} |
                     {f"{k}_us_min": round(min(v), 1) for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
