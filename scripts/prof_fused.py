"""Fused scan-filter-aggregate stages: TPC-H Q01 / Q06 (and the fused-FILTER queries) with the fused pipeline on and
off, per-query wall time, the fused launch's own device time, and a host profile of one fused run.

    python scripts/prof_fused.py [--sf 1,10] [--queries q01,q06] [--profile]
"""
import argparse
import cProfile
import io
import json
import os
import pstats
import sys
import tempfile
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", default="1,10")
    ap.add_argument("--queries", default="q01,q06")
    ap.add_argument("--runs", type=int, default=5)
    ap.add_argument("--profile", action="store_true")
    ap.add_argument("--profile-runs", type=int, default=1)
    ap.add_argument("--profile-sort", default="tottime")
    ap.add_argument("--no-eager", action="store_true")
    a = ap.parse_args()
    from netsdb_amd.client import PDBClient
    from netsdb_amd.execution import pipeline as PL
    from netsdb_amd.models import tpch, tpch_gen

    dev = "cuda:0"
    orig_launch = PL._launch
    kt = []

    def timed_launch(prog, n, d, op):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        r = orig_launch(prog, n, d, op)
        e1.record()
        torch.cuda.synchronize()
        kt.append(e0.elapsed_time(e1))
        return r

    for sf in [float(x) for x in a.sf.split(",")]:
        t = tpch_gen.generate_fast(sf, seed=1)
        c = PDBClient(root=tempfile.mkdtemp(), device=dev)
        tpch.load(c, "tpch", t, device=dev)
        del t
        for q in a.queries.split(","):
            res = {"sf": sf, "query": q}
            for fused in ((True,) if a.no_eager else (True, False)):
                c.engine.fused_pipelines = fused
                tpch.QUERIES[q](c, "tpch")
                torch.cuda.synchronize()
                ts = []
                for _ in range(a.runs):
                    t0 = time.perf_counter()
                    tpch.QUERIES[q](c, "tpch")
                    torch.cuda.synchronize()
                    ts.append((time.perf_counter() - t0) * 1e3)
                res["fused_ms" if fused else "eager_ms"] = round(sorted(ts)[len(ts) // 2], 3)
            c.engine.fused_pipelines = True
            PL._launch = timed_launch
            kt.clear()
            tpch.QUERIES[q](c, "tpch")
            PL._launch = orig_launch
            res["pipe_agg_launch_ms"] = [round(x, 3) for x in kt]
            res["stats"] = dict(c.engine.pipeline_stats)
            print(json.dumps(res), flush=True)
            if a.profile:
                pr = cProfile.Profile()
                pr.enable()
                for _ in range(a.profile_runs):
                    tpch.QUERIES[q](c, "tpch")
                    torch.cuda.synchronize()
                pr.disable()
                s = io.StringIO()
                pstats.Stats(pr, stream=s).sort_stats(a.profile_sort).print_stats(45)
                print(s.getvalue()[:12000], flush=True)


if __name__ == "__main__":
    main()
