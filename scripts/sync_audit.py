"""Host-synchronisation audit of TPC-H queries: runs each query once under torch.cuda.set_sync_debug_mode("warn")
and prints, per query, how many device->host synchronisations it makes and from which engine lines (the innermost
netsdb_amd frame of each warning's stack). Every sync drains the stream, so their count sets the host floor of a
query's latency.

    python scripts/sync_audit.py [--sf 1] [--queries q01,q06]
"""
import argparse
import collections
import json
import os
import sys
import tempfile
import traceback
import warnings

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=1.0)
    ap.add_argument("--queries", default="q01,q06,q12,q14")
    ap.add_argument("--top", type=int, default=12)
    a = ap.parse_args()
    from netsdb_amd.client import PDBClient
    from netsdb_amd.models import tpch, tpch_gen

    t = tpch_gen.generate_fast(a.sf, seed=1)
    c = PDBClient(root=tempfile.mkdtemp(), device="cuda:0")
    tpch.load(c, "tpch", t, device="cuda:0")
    del t
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for q in a.queries.split(","):
        tpch.QUERIES[q](c, "tpch")                     # warm: compile / allocate outside the audit
        torch.cuda.synchronize()
        sites = collections.Counter()

        def hook(message, category, filename, lineno, file=None, line=None):
            stack = traceback.extract_stack()
            ours = [f for f in stack if f.filename.startswith(os.path.join(root, "netsdb_amd"))]
            f = ours[-1] if ours else stack[-3]
            sites[f"{os.path.relpath(f.filename, root)}:{f.lineno} {f.name}"] += 1

        old = warnings.showwarning
        warnings.showwarning = hook
        with warnings.catch_warnings():
            warnings.simplefilter("always")
            torch.cuda.set_sync_debug_mode("warn")
            try:
                tpch.QUERIES[q](c, "tpch")
            finally:
                torch.cuda.set_sync_debug_mode("default")
                warnings.showwarning = old
        print(json.dumps({"sf": a.sf, "query": q, "syncs": sum(sites.values()),
                          "sites": dict(sites.most_common(a.top))}), flush=True)


if __name__ == "__main__":
    main()
