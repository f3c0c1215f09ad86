"""A/B of the compiled kernels' general LIKE matcher: the register-window search vs the dword memory scan
(pipeline.py JIT_LIKE_WINDOW), on the TPC-H queries whose fused stages carry a general LIKE (Q13's NOT LIKE
'%special%requests%' over every order comment, Q02's '%BRASS' part types). Interleaved rounds, each query run checked
equal between the arms.

    python scripts/ab_like.py [--sf 10] [--rounds 5] [--queries q13,q02]
"""
import argparse
import json
import os
import statistics
import sys
import tempfile
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=10.0)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--queries", default="q13,q02")
    a = ap.parse_args()
    from netsdb_amd.client import PDBClient
    from netsdb_amd.execution import pipeline as PL
    from netsdb_amd.models import tpch, tpch_gen

    t = tpch_gen.generate_fast(a.sf, seed=1)
    c = PDBClient(root=tempfile.mkdtemp(), device="cuda:0")
    tpch.load(c, "tpch", t, device="cuda:0")
    del t
    out = {"sf": a.sf}
    for q in a.queries.split(","):
        fn = tpch.QUERIES[q]
        res, ts = {}, {True: [], False: []}
        for win in (True, False):
            PL.JIT_LIKE_WINDOW = win
            res[win] = fn(c, "tpch")
            fn(c, "tpch")
        for _ in range(a.rounds):
            for win in (True, False):
                PL.JIT_LIKE_WINDOW = win
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                fn(c, "tpch")
                torch.cuda.synchronize()
                ts[win].append((time.perf_counter() - t0) * 1e3)
        out[q] = {"equal": res[True] == res[False],
                  "window_ms": round(statistics.median(ts[True]), 3), "scan_ms": round(statistics.median(ts[False]), 3),
                  "window_all": [round(x, 3) for x in ts[True]], "scan_all": [round(x, 3) for x in ts[False]]}
        print(json.dumps({q: out[q]}), flush=True)
    PL.JIT_LIKE_WINDOW = True
    print(json.dumps(out))


if __name__ == "__main__":
    main()
