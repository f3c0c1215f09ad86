"""Micro-benchmarks of the CDNA4 kernels vs the vendor-library path (torch.matmul -> hipBLASLt,
torch conv2d -> MIOpen) on the netsDB headline shapes. Random data (never zeros: DVFS, guide §5.4 r25).

    python scripts/bench_kernels.py [--json out.json]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from netsdb_amd import study, ops  # noqa: E402


def timeit(fn, iters=20, warmup=5):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(iters):
        fn()
    ev1.record()
    torch.cuda.synchronize()
    return ev0.elapsed_time(ev1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    ap.add_argument("--quick", action="store_true")
    a = ap.parse_args()
    dev = "cuda:0"
    res = []
    shapes = [
        ("ff_layer1_amazoncat14k_b1000", 1000, 1000, 597568),   # X[1000,597540->pad64] . W1[1000,..]^T
        ("ff_layer2_amazoncat14k_b1000", 1000, 14588, 1000),
        ("square_4096", 4096, 4096, 4096),
        ("square_8192", 8192, 8192, 8192),
        ("la_block_1000", 1000, 1000, 1000),
    ]
    if a.quick:
        shapes = shapes[:3]
    for name, M, N, K in shapes:
        Kp = (K + 7) // 8 * 8
        A = torch.empty(M, Kp, device=dev, dtype=torch.bfloat16).uniform_(-1, 1)
        B = torch.empty(N, Kp, device=dev, dtype=torch.bfloat16).uniform_(-1, 1)
        from netsdb_amd import _ext

        cfg_ms = {}
        for cfg in (0, 1, 2):
            study.ext().gemm_force_config(cfg)
            cfg_ms[cfg] = timeit(lambda: study.gemm_nt(A, B))
        study.ext().gemm_force_config(-1)
        t_ours = timeit(lambda: study.gemm_nt(A, B))
        t_lib = timeit(lambda: torch.matmul(A, B.t()))
        fl = 2.0 * M * N * Kp
        r = dict(op="gemm_nt", shape=name, M=M, N=N, K=Kp, ms=t_ours, tflops=fl / t_ours / 1e9,
                 tile128_tflops=fl / cfg_ms[0] / 1e9, tile256_tflops=fl / cfg_ms[1] / 1e9,
                 tile256_8ph_tflops=fl / cfg_ms[2] / 1e9,
                 lib_ms=t_lib, lib_tflops=fl / t_lib / 1e9, splits=ops.gemm_splits(M, N, Kp))
        print(json.dumps(r), flush=True)
        res.append(r)
        del A, B
    # conv2d_memory_fusion headline: 100 images 3x112x112, 64 filters 7x7, stride 1, pad 0
    X = torch.empty(100, 3, 112, 112, device=dev, dtype=torch.bfloat16).uniform_(-1, 1)
    Wf = ops.pad_k(torch.empty(64, 147, device=dev).uniform_(-0.1, 0.1)).to(torch.bfloat16).contiguous()
    bias = torch.randn(64, device=dev)
    t_ours = timeit(lambda: ops.conv2d(X, Wf, bias, 7, 7, 1, 0))
    from netsdb_amd import _ext as _e

    ops.set_kernel_options(conv_generic=bool(1))
    t_generic = timeit(lambda: ops.conv2d(X, Wf, bias, 7, 7, 1, 0))
    ops.set_kernel_options(conv_generic=bool(0))
    w4 = Wf[:, :147].reshape(64, 3, 7, 7).contiguous()
    t_lib = timeit(lambda: torch.nn.functional.conv2d(X, w4, bias.to(torch.bfloat16)))
    t_mat = timeit(lambda: study.gemm_nt(ops.im2col(X, 7, 7, 1, 0), Wf, bias, ops.BIAS_COL))
    fl = 2.0 * 100 * 106 * 106 * 64 * 147
    r = dict(op="conv2d_7x7x3_64_100img", ms=t_ours, tflops=fl / t_ours / 1e9, generic_gather_ms=t_generic,
             lib_ms=t_lib,
             materialized_im2col_gemm_ms=t_mat, out_GBps=100 * 106 * 106 * 64 * 2 / t_ours / 1e6)
    print(json.dumps(r), flush=True)
    res.append(r)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
