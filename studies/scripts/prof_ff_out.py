"""Run the FF output-layer GEMM (1000 x 14588 x 1000, f32 exp + per-label bias into a 64-padded ldc) on the
PRODUCTION kernel for rocprofv3 counter / trace runs.

    python scripts/prof_ff_out.py [ITERS] [EPI]      # EPI: -1 auto, 0 LDS-staged, 1 direct
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from netsdb_amd import ops  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 10
epi = int(sys.argv[2]) if len(sys.argv) > 2 else -1
M, N, K = 1000, 14588, 1000
H = torch.empty(M, K, device="cuda:0").uniform_(0, 1).to(torch.bfloat16)
W = (torch.empty(N, K, device="cuda:0").uniform_(-1, 1) * (3.0 / K) ** 0.5).to(torch.bfloat16)
bias = torch.empty(N, device="cuda:0").uniform_(-0.1, 0.1)
out = torch.empty(M, (N + 63) // 64 * 64, device="cuda:0")[:, :N]
for _ in range(iters):
    ops.gemm_nt(H, W, bias, ops.BIAS_COL, ops.ACT_EXP, out_dtype=torch.float32, out=out, epi=None if epi < 0 else epi)
torch.cuda.synchronize()
print("done", iters, epi)
