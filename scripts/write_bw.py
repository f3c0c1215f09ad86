"""Write-bandwidth ceiling of the box (for the store-bound conv2d / output-GEMM epilogues): torch fill_ and
copy_ over buffers the size of the conv output (144 MB) and the exp'd FF scores (58 MB), plus 1 GiB, CUDA events,
min over rounds. Prints one JSON line (TB/s of bytes written; copy_ also reads the same amount)."""
import json

import torch


def bw(fn, nbytes, iters=20, rounds=5):
    for _ in range(3):
        fn()
    best = 1e9
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / iters)
    return round(nbytes / (best * 1e-3) / 1e12, 2), round(best * 1e3, 1)


out = {}
for name, n in (("58MB", 58 << 20), ("144MB", 144 << 20), ("1GiB", 1 << 30)):
    a = torch.empty(n // 2, dtype=torch.bfloat16, device="cuda:0")
    b = torch.empty_like(a)
    out[f"fill_{name}"] = bw(lambda: a.fill_(1.0), n)
    out[f"copy_{name}"] = bw(lambda: b.copy_(a), n)
print(json.dumps({k: {"TBps_written": v[0], "us": v[1]} for k, v in out.items()}))
