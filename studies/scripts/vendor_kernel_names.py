"""Run hipBLASLt (torch.matmul) on square bf16 shapes a few times (for rocprofv3 --kernel-trace: which
Tensile kernel / macro tile the vendor library picks)."""
import torch

for n in (4096, 8192):
    A = torch.empty(n, n, device="cuda:0", dtype=torch.bfloat16).uniform_(-1, 1)
    B = torch.empty(n, n, device="cuda:0", dtype=torch.bfloat16).uniform_(-1, 1)
    for _ in range(3):
        torch.matmul(A, B.t())
    torch.cuda.synchronize()
print("done")
