"""A/B of the conv row kernels — warp-specialised (conv2d_ws_kernel, mode 5), full-row (conv2d_rowfull_kernel,
mode 1), two-pass row kernel (mode 0) — and MIOpen on the
memfuse headline shape (100 x 3 x 112 x 112, 64 filters 7x7): correctness vs fp32 F.conv2d, then interleaved
event timing.

    python scripts/ab_conv_full.py [--rounds 5]
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from netsdb_amd import _ext, ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--stamps", action="store_true", help="also the full-row kernel's phase stamps")
    a = ap.parse_args()
    h = _ext.hip()
    dev = "cuda:0"
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.empty(100, 3, 112, 112, device=dev).uniform_(-1, 1, generator=g).to(torch.bfloat16)
    W = torch.empty(64, 3, 7, 7, device=dev).uniform_(-0.1, 0.1, generator=g)
    Wf = ops.pad_k(W.reshape(64, 147)).to(torch.bfloat16).contiguous()
    bias = torch.randn(64, device=dev, generator=g)
    ref = F.conv2d(X.float(), W.to(torch.bfloat16).float(), bias)
    variants = {"warpspec": 5, "rowfull": 1, "rows": 0}
    out = {}
    for name, v in variants.items():
        ops.set_kernel_options(conv_kernel=v)
        for act, fn in ((ops.ACT_NONE, lambda t: t), (ops.ACT_RELU, torch.relu)):
            y = ops.conv2d(X, Wf, bias, 7, 7, 1, 0, act=act, nchw_out=True).float()
            out[f"{name}_act{act}_rel_err"] = ((y - fn(ref)).abs().max() / ref.abs().max()).item()
    ops.set_kernel_options(conv_kernel=5)
    ops.set_kernel_options(conv_contig=0)
    print(json.dumps(out), flush=True)
    Xm, Wm = X.clone(), W.to(torch.bfloat16)
    ours = lambda: ops.conv2d(X, Wf, bias, 7, 7, 1, 0, nchw_out=True)  # noqa: E731
    fns = {k: ours for k in variants} | {"miopen": lambda: F.conv2d(Xm, Wm, bias.to(torch.bfloat16))}
    ts = {k: [] for k in fns}
    for _ in range(a.rounds):
        for k, fn in fns.items():
            ops.set_kernel_options(conv_kernel=variants.get(k, 5))
            for _ in range(3):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            ts[k].append(e0.elapsed_time(e1) / a.iters * 1000)
    ops.set_kernel_options(conv_kernel=5)
    ops.set_kernel_options(conv_contig=0)
    print(json.dumps({f"{k}_us_min": round(min(v), 1) for k, v in ts.items()} |
                     {f"{k}_us_med": round(sorted(v)[len(v) // 2], 1) for k, v in ts.items()}), flush=True)




def stamps(mode=2):
    """Phase stamps of the full-row kernel (kernel option conv_kernel=2): s_memtime cycles per wave."""
    h = _ext.hip()
    dev = "cuda:0"
    X = torch.empty(100, 3, 112, 112, device=dev).uniform_(-1, 1).to(torch.bfloat16)
    Wf = ops.pad_k(torch.empty(64, 147, device=dev).uniform_(-0.1, 0.1)).to(torch.bfloat16).contiguous()
    bias = torch.randn(64, device=dev)
    ops.set_kernel_options(conv_kernel=mode)
    for _ in range(3):
        y = ops.conv2d(X, Wf, bias, 7, 7, 1, 0, nchw_out=True)
    torch.cuda.synchronize()
    st = y.reshape(-1).view(torch.int64)[: 256 * 4 * 8].reshape(256 * 4, 8)[:, :6].double()
    ops.set_kernel_options(conv_kernel=5)
    names = ["total", "mfma", "epilogue", "mid_barrier", "stores", "rows+top_barrier"]
    print(json.dumps({"mode": mode, "stamps_mean": dict(zip(names, [round(float(v)) for v in st.mean(0)])),
                      "stamps_max": dict(zip(names, [round(float(v)) for v in st.max(0).values]))}), flush=True)


def stamps_ws():
    """Phase stamps of the warp-specialised kernel (kernel option conv_kernel=6): s_memtime cycles per wave, compute waves
    (0-3) and store waves (4-7) separately."""
    h = _ext.hip()
    dev = "cuda:0"
    X = torch.empty(100, 3, 112, 112, device=dev).uniform_(-1, 1).to(torch.bfloat16)
    Wf = ops.pad_k(torch.empty(64, 147, device=dev).uniform_(-0.1, 0.1)).to(torch.bfloat16).contiguous()
    bias = torch.randn(64, device=dev)
    ops.set_kernel_options(conv_kernel=6)
    for _ in range(3):
        y = ops.conv2d(X, Wf, bias, 7, 7, 1, 0, nchw_out=True)
    torch.cuda.synchronize()
    st = y.reshape(-1).view(torch.int64)[: 256 * 8 * 8].reshape(256, 8, 8)[:, :, :6].double()
    ops.set_kernel_options(conv_kernel=5)
    names = {"compute": ["total", "tiles_0_1", "wait_S", "tiles_2_6_epilogues", "prologue", "wait_top"],
             "store": ["total", "stage_reads", "wait_S", "store_issue", "row_staging_and_prologue", "wait_top"]}
    out = {}
    for role, sl in (("compute", slice(0, 4)), ("store", slice(4, 8))):
        r = st[:, sl].reshape(-1, 6)
        out[role] = {"mean": dict(zip(names[role], [round(float(v)) for v in r.mean(0)])),
                     "max": dict(zip(names[role], [round(float(v)) for v in r.max(0).values]))}
    print(json.dumps({"ws_stamps": out}), flush=True)


if __name__ == "__main__":
    main()
    stamps_ws()
    if "--stamps" in sys.argv:
        stamps(2)
        stamps(3)
