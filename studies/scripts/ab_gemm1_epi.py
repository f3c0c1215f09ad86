"""FF layer-1 GEMM (1000 x 1000 x 597568, split-K 16) on the PRODUCTION kernels with the bench's operand data:
split-K slab epilogue LDS-staged (epi=0) vs direct register stores (default), each with and without the operand
prefetch of the output layer's weight (14588 x 1000 bf16). Then the output layer (fused softmax GEMM) right
after layer 1 as in the bench, with / without that prefetch. Interleaved rounds, CUDA events, relu + bias +
dropout epilogue through the reducer as the bench runs it.

    python scripts/ab_gemm1_epi.py [--rounds 5] [--iters 10]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from netsdb_amd import _ext, ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    dev = "cuda:0"
    M, N, K, L = 1000, 1000, 597568, 14588
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.empty(M, K, device=dev).uniform_(-1, 1, generator=g).to(torch.bfloat16)
    W = (torch.empty(N, K, device=dev).uniform_(-1, 1, generator=g) * (3.0 / K) ** 0.5).to(torch.bfloat16)
    b1 = torch.empty(N, device=dev).uniform_(-0.1, 0.1, generator=g)
    W2 = (torch.empty(L, N, device=dev).uniform_(-1, 1, generator=g) * (3.0 / N) ** 0.5).to(torch.bfloat16)
    b2 = torch.empty(L, device=dev).uniform_(-0.1, 0.1, generator=g)
    h = _ext.hip()
    out = torch.empty(M, L, device=dev)

    def layer1(epi, pf):
        return h.gemm_nt(X, W, b1, ops.BIAS_COL, ops.ACT_RELU, False, 1.0, 0.5, 7, 0, None, False, -1, None, 0, epi,
                         W2 if pf else None)

    y0 = layer1(0, False)
    y1 = layer1(-1, True)
    torch.cuda.synchronize()
    print(json.dumps({"direct_vs_lds_max_abs": (y0.float() - y1.float()).abs().max().item()}), flush=True)
    cases = {"l1_lds": (0, False), "l1_direct": (-1, False), "l1_direct_pf": (-1, True), "l1_lds_pf": (0, True)}
    ts = {k: [] for k in cases}
    ts.update({"l1+out_nopf": [], "l1+out_pf": [], "out_after_l1_nopf": [], "out_after_l1_pf": []})
    for _ in range(a.rounds):
        for k, (epi, pf) in cases.items():
            for _ in range(2):
                layer1(epi, pf)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                layer1(epi, pf)
            e1.record()
            torch.cuda.synchronize()
            ts[k].append(e0.elapsed_time(e1) / a.iters * 1000)
        for pf in (False, True):
            tot, tail = 0.0, 0.0
            for _ in range(a.iters):
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
                ev[0].record()
                y = layer1(-1, pf)
                ev[1].record()
                ops.gemm_nt_softmax(y, W2, b2, ops.BIAS_COL, axis=1, out=out)
                ev[2].record()
                torch.cuda.synchronize()
                tot += ev[0].elapsed_time(ev[2]) * 1000
                tail += ev[1].elapsed_time(ev[2]) * 1000
            sfx = "pf" if pf else "nopf"
            ts[f"l1+out_{sfx}"].append(tot / a.iters)
            ts[f"out_after_l1_{sfx}"].append(tail / a.iters)
    print(json.dumps({k: {"us_min": round(min(v), 1), "us_med": round(sorted(v)[len(v) // 2], 1)} for k, v in ts.items()}),
          flush=True)


if __name__ == "__main__":
    main()
