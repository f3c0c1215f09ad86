"""A/B of the folded join-probe hash (engine.FOLD_HASH_PROBE) on TPC-H join queries at one scale factor: interleaved
rounds in one process, median / min ms per query and setting.

    python scripts/ab_fold_probe.py [--sf 10] [--queries q17,q03,q12,q14] [--rounds 7]
"""
import argparse
import json
import os
import sys
import tempfile
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=10.0)
    ap.add_argument("--queries", default="q17,q03,q12,q14")
    ap.add_argument("--rounds", type=int, default=7)
    a = ap.parse_args()
    from netsdb_amd.client import PDBClient
    from netsdb_amd.execution import engine as EN
    from netsdb_amd.models import tpch, tpch_gen

    t = tpch_gen.generate_fast(a.sf, seed=1)
    c = PDBClient(root=tempfile.mkdtemp(), device="cuda:0")
    tpch.load(c, "tpch", t, device="cuda:0")
    del t
    for q in a.queries.split(","):
        ts = {True: [], False: []}
        res = {}
        for on in (True, False):
            EN.FOLD_HASH_PROBE = on
            res[on] = tpch.QUERIES[q](c, "tpch")
        for _ in range(a.rounds):
            for on in (True, False):
                EN.FOLD_HASH_PROBE = on
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                tpch.QUERIES[q](c, "tpch")
                torch.cuda.synchronize()
                ts[on].append((time.perf_counter() - t0) * 1e3)
        EN.FOLD_HASH_PROBE = True
        out = {"sf": a.sf, "query": q, "same_result": res[True] == res[False]}
        for on in (True, False):
            v = sorted(ts[on])
            out["folded" if on else "hash_atom"] = {"median_ms": round(v[len(v) // 2], 3), "min_ms": round(v[0], 3)}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
