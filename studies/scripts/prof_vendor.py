"""One GEMM, repeated, for rocprofv3 counter passes: ours (cfg auto) or hipBLASLt on the same operands.

    python scripts/prof_vendor.py ours|blas 8k|ff [ITERS]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from netsdb_amd import ops  # noqa: E402

who, shape = sys.argv[1], sys.argv[2]
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 5
dev = "cuda:0"
if shape == "8k":
    A = torch.empty(8192, 8192, device=dev, dtype=torch.bfloat16).uniform_(-1, 1)
    B = torch.empty(8192, 8192, device=dev, dtype=torch.bfloat16).uniform_(-1, 1)
    f = (lambda: ops.gemm_nt(A, B)) if who == "ours" else (lambda: torch.matmul(A, B.t()))
else:
    K, S = 597568, 16
    A = torch.empty(1000, K, device=dev, dtype=torch.bfloat16).uniform_(-1, 1).mul_((3.0 / 597540) ** 0.5)
    B = torch.empty(1000, K, device=dev, dtype=torch.bfloat16).uniform_(-1, 1)
    if who == "ours":
        f = lambda: ops.gemm_nt(A, B, out_dtype=torch.float32)  # noqa: E731
    else:
        As = A.view(1000, S, K // S).transpose(0, 1).contiguous()
        Bs = B.view(1000, S, K // S).transpose(0, 1).contiguous()
        del A, B
        f = lambda: torch.bmm(As, Bs.transpose(1, 2))  # noqa: E731
for _ in range(iters):
    f()
torch.cuda.synchronize()
print("done", who, shape)
