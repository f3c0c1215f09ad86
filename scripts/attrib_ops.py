"""Which Python call sites launch given ATen ops in TPC-H queries (torch.profiler with stacks, one warm run each).

    python scripts/attrib_ops.py [--sf 1] [--queries q03,q17] [--ops gather,scatter]
"""
import argparse
import collections
import os
import sys
import tempfile

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=1.0)
    ap.add_argument("--queries", default="q03,q12,q14,q17")
    ap.add_argument("--ops", default="gather,scatter")
    a = ap.parse_args()
    from netsdb_amd.client import PDBClient
    from netsdb_amd.models import tpch, tpch_gen

    t = tpch_gen.generate_fast(a.sf, seed=1)
    c = PDBClient(root=tempfile.mkdtemp(), device="cuda:0")
    tpch.load(c, "tpch", t, device="cuda:0")
    del t
    keys = a.ops.split(",")
    for q in a.queries.split(","):
        fn = tpch.QUERIES[q]
        fn(c, "tpch")
        torch.cuda.synchronize()
        with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU], with_stack=True) as prof:
            fn(c, "tpch")
            torch.cuda.synchronize()
        print(f"== {q}", flush=True)
        for e in prof.key_averages(group_by_stack_n=12):
            if any(k in e.key for k in keys) and not e.key.startswith("aten::_"):
                st = [f for f in (e.stack or []) if "netsdb_amd" in f or "models" in f][:4]
                print(f"  {e.count:4d}  {e.key}  {' <- '.join(st) or list(e.stack or [])[:4]}", flush=True)


if __name__ == "__main__":
    main()
