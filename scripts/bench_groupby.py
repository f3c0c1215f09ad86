"""Group-id micro-benchmark: device hash table (hashagg.hip via ops hash_group_ids) vs torch.unique(sorted,
return_inverse) on int64 key columns of several sizes and cardinalities. CUDA events, median of --reps.

    python scripts/bench_groupby.py [--reps 10]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from netsdb_amd import _ext  # noqa: E402


def timed(fn, reps):
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dev = "cuda:0"
    g = torch.Generator(device=dev).manual_seed(0)
    hk = _ext.hip()
    for n in (1 << 20, 1 << 24):
        for card in (8, 10_000, n):
            keys = torch.randint(0, card, (n,), device=dev, generator=g) * 1_000_003 - 7
            inv, uniq = hk.hash_group_ids(keys)
            ru, ri = torch.unique(keys, sorted=True, return_inverse=True)
            ok = bool(torch.equal(uniq, ru) and torch.equal(inv, ri))
            t_hash = timed(lambda: hk.hash_group_ids(keys), a.reps)
            t_uniq = timed(lambda: torch.unique(keys, sorted=True, return_inverse=True), a.reps)
            print(json.dumps({"n": n, "cardinality": card, "groups": int(ru.numel()), "hash_us": round(t_hash, 1),
                              "torch_unique_us": round(t_uniq, 1), "speedup": round(t_uniq / t_hash, 2),
                              "exact": ok}), flush=True)


if __name__ == "__main__":
    main()
