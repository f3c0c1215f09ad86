"""TPC-H Q04 plans A/B: the EXISTS as distinct late order keys joined with the quarter (group-by first) vs the quarter's
orders as the join build side probed by every late lineitem (join first). Interleaved rounds, both checked equal.

    python scripts/ab_q04.py [--sf 10] [--rounds 5]
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
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    from netsdb_amd.client import PDBClient
    from netsdb_amd.models import tpch, tpch_gen

    t = tpch_gen.generate_fast(a.sf, seed=1)
    c = PDBClient(root=tempfile.mkdtemp(), device="cuda:0")
    tpch.load(c, "tpch", t, device="cuda:0")
    ref = tpch.reference("q04", t, f=tpch.frames(t))
    del t
    res = {}
    for jf in (False, True):
        got = tpch.q04(c, "tpch", join_first=jf)
        res[f"equal_{jf}"] = sorted(got, key=lambda x: x["o_orderpriority"]) == \
            sorted(ref, key=lambda x: x["o_orderpriority"])
    ts = {False: [], True: []}
    for _ in range(a.rounds):
        for jf in (False, True):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            tpch.q04(c, "tpch", join_first=jf)
            torch.cuda.synchronize()
            ts[jf].append((time.perf_counter() - t0) * 1e3)
    for jf in (False, True):
        v = sorted(ts[jf])
        res["join_first" if jf else "group_first"] = {"median_ms": round(v[len(v) // 2], 3), "min_ms": round(v[0], 3)}
    print(json.dumps({"sf": a.sf, **res}), flush=True)


if __name__ == "__main__":
    main()
