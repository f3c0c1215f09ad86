"""One hash-aggregation shape run N times (for rocprofv3 kernel traces / PMC passes of the relops kernels).

    python scripts/prof_relops_case.py DISTINCT [N] [ROWS] [F] [nofirst]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from netsdb_amd import _ext  # noqa: E402


def main():
    distinct = int(sys.argv[1])
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 16_000_000
    F = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    first = not (len(sys.argv) > 5 and sys.argv[5] == "nofirst")
    g = torch.Generator(device="cuda").manual_seed(1)
    keys = torch.randint(0, distinct, (n,), device="cuda", generator=g) * 2654435761
    vals = torch.rand(n, F, device="cuda", dtype=torch.float64, generator=g)
    h = _ext.hip()
    for _ in range(reps):
        r = h.hash_aggregate(keys, vals, "sum", False, 0, first)
    torch.cuda.synchronize()
    print(int(r[5][0]), int(r[5][1]))


if __name__ == "__main__":
    main()
