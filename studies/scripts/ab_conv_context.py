"""The headline conv2d (100 x 3 x 112 x 112, 64 filters 7x7) timed in the contexts it runs in: back to back (hot
input), after a 512 MB write (cold caches), after the fused softmax output layer (what precedes it in the bench),
and after layer 1 + the output layer (the whole FF job). CUDA events around the conv only.

    python scripts/ab_conv_context.py [--reps 10]
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
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dev = "cuda:0"
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.empty(100, 3, 112, 112, device=dev).uniform_(-1, 1, generator=g).to(torch.bfloat16)
    Wf = ops.pad_k(torch.empty(64, 147, device=dev).uniform_(-0.1, 0.1, generator=g)).to(torch.bfloat16).contiguous()
    bias = torch.randn(64, device=dev, generator=g)
    H = torch.empty(1000, 1000, device=dev).uniform_(0, 1, generator=g).to(torch.bfloat16)
    W2 = (torch.empty(14588, 1000, device=dev).uniform_(-1, 1, generator=g) * 0.055).to(torch.bfloat16)
    b2 = torch.empty(14588, device=dev).uniform_(-0.1, 0.1, generator=g)
    Xl = torch.empty(1000, 597568, device=dev).uniform_(-1, 1, generator=g).to(torch.bfloat16)
    W1 = (torch.empty(1000, 597568, device=dev).uniform_(-1, 1, generator=g) * 0.00224).to(torch.bfloat16)
    out = torch.empty(1000, 14588, device=dev)
    flush = torch.empty(512 << 20, dtype=torch.uint8, device=dev)
    conv = lambda: ops.conv2d(X, Wf, bias, 7, 7, 1, 0, nchw_out=True)  # noqa: E731
    pre = {
        "hot": lambda: conv(),
        "cold_flush": lambda: flush.fill_(1),
        "after_softmax_gemm": lambda: ops.gemm_nt_softmax(H, W2, b2, ops.BIAS_COL, axis=1, out=out),
        "after_ff_job": lambda: ops.gemm_nt_softmax(ops.gemm_nt(Xl, W1, act=ops.ACT_RELU), W2, b2, ops.BIAS_COL,
                                                    axis=1, out=out),
    }
    res = {k: [] for k in pre}
    for _ in range(a.reps):
        for k, fn in pre.items():
            fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            conv()
            e1.record()
            torch.cuda.synchronize()
            res[k].append(e0.elapsed_time(e1) * 1000)
    print(json.dumps({k: {"us_min": round(min(v), 1), "us_med": round(sorted(v)[len(v) // 2], 1)} for k, v in res.items()}),
          flush=True)


if __name__ == "__main__":
    main()
