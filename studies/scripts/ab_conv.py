"""Timing of the conv2d kernels / diagnostic variants on the memfuse headline shape."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from netsdb_amd import _ext, ops  # noqa: E402
from scripts.bench_kernels import timeit  # noqa: E402

X = torch.empty(100, 3, 112, 112, device="cuda:0", dtype=torch.bfloat16).uniform_(-1, 1)
Wf = ops.pad_k(torch.empty(64, 147, device="cuda:0").uniform_(-0.1, 0.1)).to(torch.bfloat16).contiguous()
bias = torch.randn(64, device="cuda:0")
res = {}
for name, gen, var in (("generic", 1, 0), ("rows", 0, 0), ("rows_nostore", 0, 1), ("rows_nomfma", 0, 2),
                       ("rows_nostage", 0, 4), ("rows_prologue_only", 0, 8), ("rows_nocompute", 0, 16),
                       ("rows_nocompute_nostore", 0, 17), ("rows_nomfma_nostage_nostore", 0, 7)):
    ops.set_kernel_options(conv_generic=bool(gen))
    ops.set_kernel_options(conv_variant=var)
    res[name] = round(timeit(lambda: ops.conv2d(X, Wf, bias, 7, 7, 1, 0, nchw_out=True)) * 1000, 1)
ops.set_kernel_options(conv_generic=bool(0))
ops.set_kernel_options(conv_variant=0)
print(json.dumps({"conv_us": res}))

# stamps (flag 32): per wave [total, stage+barriers, compute(+staging), barrier after compute] s_memtime cycles
for name, var in (("full", 32), ("nocompute_nostore", 32 | 17), ("nocompute", 32 | 16)):
    ops.set_kernel_options(conv_variant=var)
    y = ops.conv2d(X, Wf, bias, 7, 7, 1, 0, nchw_out=True)
    torch.cuda.synchronize()
    st = y.reshape(-1).view(torch.int64)[: 512 * 4 * 4].reshape(512 * 4, 4).double()
    print(json.dumps({"stamps": name, "mean": [round(float(v)) for v in st.mean(0)],
                      "max": [round(float(v)) for v in st.max(0).values]}))
ops.set_kernel_options(conv_variant=0)
