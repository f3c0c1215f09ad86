"""Join build alone (unique int64 keys, sizes from --rows), timed with events; run it under rocprofv3 for the per-kernel
breakdown of the partitioned (>= 1 M rows) and global-insert paths."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from netsdb_amd import _ext  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default="2000000,16000000")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    h = _ext.hip()
    for n in [int(x) for x in a.rows.split(",")]:
        g = torch.Generator(device="cuda").manual_seed(1)
        keys = torch.randperm(n, device="cuda", generator=g) * 7 + 11
        h.join_build(keys)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            h.join_build(keys)
        e1.record()
        torch.cuda.synchronize()
        print(json.dumps({"build_rows": n, "ms": round(e0.elapsed_time(e1) / a.reps, 4)}), flush=True)


if __name__ == "__main__":
    main()
