"""A/B of the skinny huge-K GEMM shapes of the dedup scoring path (scripts/bench_dedup.py):
common panel 500 x 100 x 900k, batched private panels 12 x 500 x 100 x 100k (B broadcast), per model
500 x 100 x 1M, under different split / batching / layout choices.  Prints one line per variant."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from netsdb_amd import ops  # noqa: E402


def t(fn, it=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


def main():
    dev = "cuda:0"
    g = torch.Generator(device=dev).manual_seed(1)
    X = (torch.randn(100, 1_000_000, device=dev, generator=g) * 0.05).to(torch.bfloat16)
    Wc = (torch.randn(500, 900_000, device=dev, generator=g) * 0.05).to(torch.bfloat16)
    Wp = (torch.randn(12, 500, 100_000, device=dev, generator=g) * 0.05).to(torch.bfloat16)
    P = torch.randn(500, 100, device=dev)
    Xc, Xp = X[:, :900_000], X[:, 900_000:]
    Xpc = Xp.contiguous()
    gb = lambda b, us: f"{b / us / 1e3:.2f} TB/s"
    us = t(lambda: ops.gemm_nt(Wc, Xc, out_dtype=torch.float32))
    print(f"common 500x100x900k view      {us:8.1f} us  {gb(0.9e9, us)}  splits={ops.gemm_splits(500, 100, 900000)}")
    for cfg, sp in ((0, 64), (0, 256), (2, 128), (2, 64)):
        us = t(lambda: ops.gemm_nt(Wc, Xc, out_dtype=torch.float32, cfg=cfg, splits=sp))
        print(f"common cfg={cfg} splits={sp:3d}         {us:8.1f} us  {gb(0.9e9, us)}")
    for sp in (0, 16, 24, 32, 48, 64):
        xb = Xp.unsqueeze(0).expand(12, -1, -1)
        us = t(lambda: ops.gemm_nt(Wp, xb, P, ops.BIAS_MAT, out_dtype=torch.float32, splits=sp))
        print(f"private batched splits={sp:3d}     {us:8.1f} us  {gb(1.2e9, us)}  auto={ops.gemm_splits(500, 100, 100000, 12)}")
    xb = Xpc.unsqueeze(0).expand(12, -1, -1)
    us = t(lambda: ops.gemm_nt(Wp, xb, P, ops.BIAS_MAT, out_dtype=torch.float32))
    print(f"private batched contiguous X   {us:8.1f} us  {gb(1.2e9, us)}")
    for cfg, sp in ((2, 0), (2, 10), (2, 16), (2, 21)):
        us = t(lambda: ops.gemm_nt(Wp, xb, P, ops.BIAS_MAT, out_dtype=torch.float32, cfg=cfg, splits=sp))
        print(f"private batched cfg={cfg} splits={sp:3d} {us:8.1f} us  {gb(1.2e9, us)}")
    us = t(lambda: [ops.gemm_nt(Wp[i], Xp, P, ops.BIAS_MAT, out_dtype=torch.float32) for i in range(12)])
    print(f"private loop of 12            {us:8.1f} us  {gb(1.2e9, us)}  splits={ops.gemm_splits(500, 100, 100000)}")
    Wflat = Wp.reshape(6000, 100_000)
    us = t(lambda: ops.gemm_nt(Wflat, Xp, out_dtype=torch.float32))
    print(f"private as one 6000x100x100k  {us:8.1f} us  {gb(1.2e9, us)}  splits={ops.gemm_splits(6000, 100, 100000)}")
    us = t(lambda: ops.gemm_nt(Xp, Wflat, out_dtype=torch.float32))
    print(f"private as 100x6000x100k (T)  {us:8.1f} us  {gb(1.2e9, us)}  splits={ops.gemm_splits(100, 6000, 100000)}")
    Wm = (torch.randn(500, 1_000_000, device=dev, generator=g) * 0.05).to(torch.bfloat16)
    us = t(lambda: ops.gemm_nt(Wm, X, out_dtype=torch.float32))
    print(f"naive 500x100x1M              {us:8.1f} us  {gb(1.0e9, us)}")
    us = t(lambda: torch.matmul(Wm, X.t()))
    print(f"torch.matmul 500x100x1M       {us:8.1f} us  {gb(1.0e9, us)}")
    us = t(lambda: Wm.sum())
    print(f"read-only sum of 1 GB         {us:8.1f} us  {gb(1.0e9, us)}")


if __name__ == "__main__":
    main()
