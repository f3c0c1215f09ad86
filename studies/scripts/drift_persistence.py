"""Do the FF layer-1 GEMM's per-split (per-XCD) finish times persist from launch to launch? cfg-17 stamps of
N consecutive launches; prints each split's finish lag (k-tiles behind the earliest split) per launch and the
rank correlation between consecutive launches. Persistent per-XCD rates could be balanced by a launch-to-
launch adaptive K partition; random stragglers could not.

    python scripts/drift_persistence.py [--launches 6] [--scale-b 0.0022]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from netsdb_amd import study, _ext, ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--launches", type=int, default=6)
    ap.add_argument("--scale-b", type=float, default=0.0022)
    a = ap.parse_args()
    M, N, K = 1000, 1000, 597568
    h = study.ext()
    A = torch.empty(M, K, device="cuda:0", dtype=torch.bfloat16).uniform_(-1, 1)
    B = (torch.empty(N, K, device="cuda:0").uniform_(-1, 1) * a.scale_b).to(torch.bfloat16)
    st = torch.zeros(256 * 64, dtype=torch.int64, device="cuda:0")
    h.gemm_set_stamps(st.data_ptr())
    h.gemm_force_config(17)
    for _ in range(3):
        study.gemm_nt(A, B)
    lags = []
    for _ in range(a.launches):
        st.zero_()
        study.gemm_nt(A, B)
        torch.cuda.synchronize()
        s = st.view(256, 64).cpu().double()
        last = s[:, 18]
        per_k = ((s[:, 18] - s[:, 0]) / (18 * 32)).mean().item()
        fin = [last[g * 16:(g + 1) * 16].max().item() for g in range(16)]
        mean_fin = [last[g * 16:(g + 1) * 16].median().item() for g in range(16)]
        lo = min(fin)
        lags.append({"max": [round((f - lo) / per_k, 1) for f in fin],
                     "median": [round((f - min(mean_fin)) / per_k, 1) for f in mean_fin]})
    h.gemm_force_config(-1)
    h.gemm_set_stamps(0)

    def ranks(v):
        order = sorted(range(len(v)), key=lambda i: v[i])
        r = [0] * len(v)
        for k, i in enumerate(order):
            r[i] = k
        return r

    def spearman(x, y):
        rx, ry = ranks(x), ranks(y)
        n = len(x)
        return 1 - 6 * sum((p - q) ** 2 for p, q in zip(rx, ry)) / (n * (n * n - 1))

    corr_max = [round(spearman(lags[i]["max"], lags[i + 1]["max"]), 2) for i in range(len(lags) - 1)]
    corr_med = [round(spearman(lags[i]["median"], lags[i + 1]["median"]), 2) for i in range(len(lags) - 1)]
    print(json.dumps({"lags": lags, "spearman_max_consecutive": corr_max, "spearman_median_consecutive": corr_med}))


if __name__ == "__main__":
    main()
