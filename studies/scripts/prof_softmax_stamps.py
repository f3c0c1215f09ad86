"""Phase stamps of the fused softmax GEMM (FF output layer 1000 x 14588 x 1000, the bench's scales).

Each workgroup (tile) records on the 100 MHz real-time clock: entry, main loop done, partial published,
row-block complete (poll done), statistics combined, stores issued, stores complete, and its XCC/CU id.
Prints, per phase, the median / max over tiles of the time since the launch's first entry (us), for a
cache-cold call (a 512 MB buffer written in between) and a hot one, plus the event-timed kernel.

    python scripts/prof_softmax_stamps.py [--reps 5]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from netsdb_amd import _ext, ops  # noqa: E402

NAMES = ["entry", "mainloop", "published", "rowblock_done", "combined", "stores_issued", "stores_done"]


def summarise(st):
    st = st.view(-1, 8).cpu()
    t0 = st[:, 0].min().item()
    out = {}
    for i, n in enumerate(NAMES):
        v = (st[:, i] - t0).double() / 100.0       # 100 MHz -> us
        s = v.sort().values
        out[n] = {"min": round(s[0].item(), 2), "med": round(s[len(s) // 2].item(), 2), "max": round(s[-1].item(), 2)}
    xcc = (st[:, 7] >> 32).tolist()
    out["tiles_per_xcc"] = {int(x): xcc.count(x) for x in sorted(set(xcc))}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    dev = "cuda:0"
    M, N, K = 1000, 14588, 1000
    g = torch.Generator(device=dev).manual_seed(0)
    H = torch.empty(M, K, device=dev).uniform_(0, 1, generator=g).to(torch.bfloat16)
    W = (torch.empty(N, K, device=dev).uniform_(-1, 1, generator=g) * (3.0 / K) ** 0.5).to(torch.bfloat16)
    bias = torch.empty(N, device=dev).uniform_(-0.1, 0.1, generator=g)
    out = torch.empty(M, N, device=dev)
    tiles = ((M + 255) // 256) * ((N + 255) // 256)
    st = torch.zeros(tiles * 8, dtype=torch.int64, device=dev)
    flush = torch.empty(512 << 20, dtype=torch.uint8, device=dev)
    hip = _ext.hip()
    ref = torch.softmax(H.float() @ W.float().t() + bias, dim=1)
    hip.gemm_nt_softmax(H, W, bias, ops.BIAS_COL, 1, out, 1.0, False, -1, st)
    torch.cuda.synchronize()
    print(json.dumps({"max_abs_err": (out - ref).abs().max().item()}), flush=True)
    res = {}
    for mode in ("cold", "hot"):
        times, summ = [], None
        for _ in range(a.reps):
            if mode == "cold":
                flush.fill_(1)
            else:
                hip.gemm_nt_softmax(H, W, bias, ops.BIAS_COL, 1, out, 1.0, False, -1, None)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            hip.gemm_nt_softmax(H, W, bias, ops.BIAS_COL, 1, out, 1.0, False, -1, st)
            e1.record()
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1) * 1000)
            summ = summarise(st)
        res[mode] = {"event_us": sorted(times)[len(times) // 2], "phases_last_rep": summ}
    print(json.dumps(res, indent=1), flush=True)


if __name__ == "__main__":
    main()
