"""A/B of the compiled pipeline kernels' rows per thread (execution/pipeline.py JIT_ROWS / JIT_ROWS_SMALL) on TPC-H
Q01 / Q06 / Q14 at one scale factor: the fused launch's own time (CUDA events around _launch), median of rounds.

    python scripts/ab_jit_rows.py [--sf 10] [--rows 2,4,8] [--rounds 7]
"""
import argparse
import json
import os
import sys
import tempfile

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=10.0)
    ap.add_argument("--rows", default="2,4,8,12")
    ap.add_argument("--queries", default="q01,q06")
    ap.add_argument("--rounds", type=int, default=7)
    a = ap.parse_args()
    from netsdb_amd.client import PDBClient
    from netsdb_amd.execution import pipeline as PL
    from netsdb_amd.models import tpch, tpch_gen

    t = tpch_gen.generate_fast(a.sf, seed=1)
    c = PDBClient(root=tempfile.mkdtemp(), device="cuda:0")
    tpch.load(c, "tpch", t, device="cuda:0")
    del t
    orig = PL._launch
    kt = []

    def timed(prog, n, d, plan):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        r = orig(prog, n, d, plan)
        e1.record()
        torch.cuda.synchronize()
        kt.append(e0.elapsed_time(e1))
        return r

    PL._launch = timed
    rows = [int(x) for x in a.rows.split(",")]
    for q in a.queries.split(","):
        res = {r: [] for r in rows}
        for r in rows:                          # compile every shape first
            PL.JIT_ROWS = PL.JIT_ROWS_SMALL = r
            tpch.QUERIES[q](c, "tpch")
        for _ in range(a.rounds):
            for r in rows:
                PL.JIT_ROWS = PL.JIT_ROWS_SMALL = r
                kt.clear()
                tpch.QUERIES[q](c, "tpch")
                res[r].append(sum(kt))
        print(json.dumps({"sf": a.sf, "query": q, **{f"rows{r}_ms": round(sorted(v)[len(v) // 2], 3)
                                                       for r, v in res.items()}}), flush=True)


if __name__ == "__main__":
    main()
