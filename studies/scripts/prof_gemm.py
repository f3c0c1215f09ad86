"""Run one GEMM shape under a forced tile config (for rocprofv3 counter runs).

    python scripts/prof_gemm.py M N K CFG [ITERS]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from netsdb_amd import study, _ext, ops  # noqa: E402

M, N, K, cfg = (int(x) for x in sys.argv[1:5])
iters = int(sys.argv[5]) if len(sys.argv) > 5 else 10
A = torch.empty(M, K, device="cuda:0", dtype=torch.bfloat16).uniform_(-1, 1)
B = torch.empty(N, K, device="cuda:0", dtype=torch.bfloat16).uniform_(-1, 1)
study.ext().gemm_force_config(cfg)
for _ in range(iters):
    study.gemm_nt(A, B)
torch.cuda.synchronize()
print("done", M, N, K, cfg)
