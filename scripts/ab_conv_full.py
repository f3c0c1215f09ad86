"""A/B of the full-row conv kernel (conv2d_rowfull_kernel) vs the two-pass row kernel and MIOpen on the
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
    a = ap.parse_args()
    h = _ext.hip()
    dev = "cuda:0"
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.empty(100, 3, 112, 112, device=dev).uniform_(-1, 1, generator=g).to(torch.bfloat16)
    W = torch.empty(64, 3, 7, 7, device=dev).uniform_(-0.1, 0.1, generator=g)
    Wf = ops.pad_k(W.reshape(64, 147)).to(torch.bfloat16).contiguous()
    bias = torch.randn(64, device=dev, generator=g)
    ref = F.conv2d(X.float(), W.to(torch.bfloat16).float(), bias)
    variants = {"rowfull": 1, "rowfull_nopipe": 4, "rows": 0, "rowfull_contig": 1}
    out = {}
    for name, v in variants.items():
        h.conv2d_rowfull(v)
        h.conv2d_contig(1 if name == "rowfull_contig" else 0)
        for act, fn in ((ops.ACT_NONE, lambda t: t), (ops.ACT_RELU, torch.relu)):
            y = ops.conv2d(X, Wf, bias, 7, 7, 1, 0, act=act, nchw_out=True).float()
            out[f"{name}_act{act}_rel_err"] = ((y - fn(ref)).abs().max() / ref.abs().max()).item()
    h.conv2d_rowfull(1)
    h.conv2d_contig(0)
    print(json.dumps(out), flush=True)
    Xm, Wm = X.clone(), W.to(torch.bfloat16)
    fns = {
        "rowfull": lambda: ops.conv2d(X, Wf, bias, 7, 7, 1, 0, nchw_out=True),
        "rowfull_nopipe": lambda: ops.conv2d(X, Wf, bias, 7, 7, 1, 0, nchw_out=True),
        "rowfull_contig": lambda: ops.conv2d(X, Wf, bias, 7, 7, 1, 0, nchw_out=True),
        "rows": lambda: ops.conv2d(X, Wf, bias, 7, 7, 1, 0, nchw_out=True),
        "miopen": lambda: F.conv2d(Xm, Wm, bias.to(torch.bfloat16)),
    }
    ts = {k: [] for k in fns}
    for _ in range(a.rounds):
        for k, fn in fns.items():
            h.conv2d_rowfull({"rowfull": 1, "rowfull_nopipe": 4, "rowfull_contig": 1}.get(k, 0))
            h.conv2d_contig(1 if k == "rowfull_contig" else 0)
            for _ in range(3):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            ts[k].append(e0.elapsed_time(e1) / a.iters * 1000)
    h.conv2d_rowfull(1)
    h.conv2d_contig(0)
    print(json.dumps({f"{k}_us_min": round(min(v), 1) for k, v in ts.items()} |
                     {f"{k}_us_med": round(sorted(v)[len(v) // 2], 1) for k, v in ts.items()}), flush=True)




def stamps(mode=2):
    """Phase stamps of the full-row kernel (conv2d_rowfull(2)): s_memtime cycles per wave."""
    h = _ext.hip()
    dev = "cuda:0"
    X = torch.empty(100, 3, 112, 112, device=dev).uniform_(-1, 1).to(torch.bfloat16)
    Wf = ops.pad_k(torch.empty(64, 147, device=dev).uniform_(-0.1, 0.1)).to(torch.bfloat16).contiguous()
    bias = torch.randn(64, device=dev)
    h.conv2d_rowfull(mode)
    for _ in range(3):
        y = ops.conv2d(X, Wf, bias, 7, 7, 1, 0, nchw_out=True)
    torch.cuda.synchronize()
    st = y.reshape(-1).view(torch.int64)[: 256 * 4 * 8].reshape(256 * 4, 8)[:, :6].double()
    h.conv2d_rowfull(1)
    names = ["total", "mfma", "epilogue", "mid_barrier", "stores", "rows+top_barrier"]
    print(json.dumps({"mode": mode, "stamps_mean": dict(zip(names, [round(float(v)) for v in st.mean(0)])),
                      "stamps_max": dict(zip(names, [round(float(v)) for v in st.max(0).values]))}), flush=True)


if __name__ == "__main__":
    main()
    stamps(2)
    stamps(3)
