"""A/B: tile config (128^2 2-stage / 256^2 2-stage / 256^2 8-phase) x splits for the skinny dedup GEMMs."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from netsdb_amd import study, _ext, ops  # noqa: E402
from scripts.ab_dedup_gemm import t  # noqa: E402


def main():
    dev = "cuda:0"
    g = torch.Generator(device=dev).manual_seed(1)
    X = (torch.randn(100, 1_000_000, device=dev, generator=g) * 0.05).to(torch.bfloat16)
    Wp = (torch.randn(6000, 100_000, device=dev, generator=g) * 0.05).to(torch.bfloat16)
    Wm = (torch.randn(500, 1_000_000, device=dev, generator=g) * 0.05).to(torch.bfloat16)
    Xp = X[:, 900_000:]
    for cfg in (0, 1, 2):
        study.ext().gemm_force_config(cfg)
        for sp in (0, 8, 16, 32, 64, 128, 256):
            a = t(lambda: study.gemm_nt(Wp, Xp, out_dtype=torch.float32, splits=sp))
            b = t(lambda: study.gemm_nt(Wm, X, out_dtype=torch.float32, splits=sp))
            print(f"cfg={cfg} splits={sp:3d}  6000x100x100k {a:7.1f} us ({1.2e9 / a / 1e6:5.2f} TB/s)   "
                  f"500x100x1M {b:7.1f} us ({1.0e9 / b / 1e6:5.2f} TB/s)", flush=True)
    study.ext().gemm_force_config(-1)


if __name__ == "__main__":
    main()
