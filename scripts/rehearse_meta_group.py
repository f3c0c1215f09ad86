"""Two ranks on one GPU: RCCL data group + gloo metadata group (the bench's N>1 setup, rehearsed on a
1-GPU box).  Prints whether a metadata all-reduce returns while a long GPU kernel is still running."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from netsdb_amd.parallel.comm import ClusterContext  # noqa: E402

# RCCL refuses two ranks on one GPU at communicator creation ("Duplicate GPU detected"), so the default
# group is created lazily (no device_id) and never used for data here; the gloo metadata group is real
torch.distributed.init_process_group("nccl")
ctx = ClusterContext(int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"]), torch.device("cuda:0"), "nccl")
ctx.attach_meta_group()
a = torch.randn(8192, 8192, device="cuda:0")
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    a = a @ a * 1e-4                     # ~20 GEMMs queued on the GPU
t_enq = time.perf_counter() - t0
v = ctx.all_reduce_scalar(1.0 + ctx.rank, "sum")
t_meta = time.perf_counter() - t0
torch.cuda.synchronize()
t_all = time.perf_counter() - t0
print(f"rank {ctx.rank}: meta_group={'gloo' if ctx.meta_group is not None else None} sum={v} "
      f"enqueue_ms={t_enq*1e3:.2f} meta_ms={t_meta*1e3:.2f} gpu_ms={t_all*1e3:.2f}", flush=True)
torch.distributed.destroy_process_group()
