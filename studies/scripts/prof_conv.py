"""Run the memfuse headline conv (100 x 3x112x112, 64 filters 7x7) N times (rocprofv3 counter runs)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from netsdb_amd import ops  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 5
X = torch.empty(100, 3, 112, 112, device="cuda:0", dtype=torch.bfloat16).uniform_(-1, 1)
Wf = ops.pad_k(torch.empty(64, 147, device="cuda:0").uniform_(-0.1, 0.1)).to(torch.bfloat16).contiguous()
bias = torch.randn(64, device="cuda:0")
for _ in range(iters):
    ops.conv2d(X, Wf, bias, 7, 7, 1, 0, nchw_out=True)
torch.cuda.synchronize()
print("done")
