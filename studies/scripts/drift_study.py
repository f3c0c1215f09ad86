"""Workgroup drift within a split-K group of the FF layer-1 GEMM: the 8-phase kernel's diagnostic variant
(cfg 17) stamps the 100 MHz real-time clock every 32 k-tiles per workgroup; for each split (the 16 tiles that
share its A/B panels through one XCD's L2) report how far apart (in k-tiles) its workgroups run.

    python scripts/drift_study.py [--scale-b 0.0022]
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
    ap.add_argument("--scale-b", type=float, default=0.0022)
    a = ap.parse_args()
    M, N, K = 1000, 1000, 597568
    h = study.ext()
    A = torch.empty(M, K, device="cuda:0", dtype=torch.bfloat16).uniform_(-1, 1)
    B = (torch.empty(N, K, device="cuda:0").uniform_(-1, 1) * a.scale_b).to(torch.bfloat16)
    st = torch.zeros(256 * 64, dtype=torch.int64, device="cuda:0")
    h.gemm_set_stamps(st.data_ptr())
    h.gemm_force_config(17)
    for _ in range(5):
        study.gemm_nt(A, B, out_dtype=torch.float32)
    torch.cuda.synchronize()
    h.gemm_force_config(-1)
    h.gemm_set_stamps(0)
    raw = st.view(256, 64).cpu()
    xcc = (raw[:, 63] >> 32).tolist()
    hw_id = (raw[:, 63] & 0xffffffff).tolist()
    groups_xcc = [sorted(set(xcc[g * 16:(g + 1) * 16])) for g in range(16)]
    s = raw.double()
    nslots = 18                          # 292 iterations of 2 k-tiles: stamps at it = 0, 16, ..., 288
    s = s[:, :nslots]
    t0 = s[:, 0].min()
    per_ktile = ((s[:, nslots - 1] - s[:, 0]) / ((nslots - 1) * 32)).mean().item()   # ticks per k-tile
    spreads = []
    for grp in range(16):
        g = s[grp * 16:(grp + 1) * 16]
        spreads.append(((g.max(0).values - g.min(0).values) / per_ktile).tolist())
    worst = max(max(x) for x in spreads)
    mean_last = sum(x[-1] for x in spreads) / 16
    chip = ((s.max(0).values - s.min(0).values) / per_ktile).tolist()
    print(json.dumps({"us_per_ktile": per_ktile / 100.0, "group_spread_ktiles_first": [round(x[0], 2) for x in spreads],
                      "group_spread_ktiles_last": [round(x[-1], 2) for x in spreads], "worst_group_spread_ktiles": round(worst, 2),
                      "mean_group_spread_last": round(mean_last, 2), "chip_spread_ktiles": [round(c, 1) for c in chip],
                      "start_skew_us": round(float((s[:, 0].max() - t0) / 100.0), 2),
                      "xcc_of_each_group": groups_xcc,
                      "group_finish_ktiles_behind_first": [round(float((s[g * 16:(g + 1) * 16, nslots - 1].max()
                                                                         - s[:, nslots - 1].min()) / per_ktile), 1)
                                                           for g in range(16)],
                      "hw_id_sample": hw_id[:4]}))


if __name__ == "__main__":
    main()
