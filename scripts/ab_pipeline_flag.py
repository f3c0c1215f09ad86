"""A/B of a fused-pipeline switch (a module attribute of netsdb_amd.execution.pipeline, e.g. JIT_FIXED_OP,
JIT_LIKE_WINDOW, JIT_ROWS; or hip:<setter> of the HIP extension, e.g. hip:join_set_part) on TPC-H queries:
interleaved rounds, every arm's answer checked equal to the first arm's.

    python scripts/ab_pipeline_flag.py --flag JIT_FIXED_OP --values True,False [--sf 10] [--rounds 5] [--queries q01,q06]
    python scripts/ab_pipeline_flag.py --flag hip:join_set_part --values True,False --queries q03,q22
    python scripts/ab_pipeline_flag.py --flag objects.record:GROUP_TAKE_MAX_ROWS --values 262144,0 --queries q02
"""
import argparse
import ast
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
    ap.add_argument("--flag", required=True)
    ap.add_argument("--values", required=True, help="comma-separated Python literals")
    ap.add_argument("--sf", type=float, default=10.0)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--queries", default="q01,q06,q12,q14")
    a = ap.parse_args()
    from netsdb_amd.client import PDBClient
    from netsdb_amd.execution import pipeline as PL
    from netsdb_amd.models import tpch, tpch_gen

    vals = [ast.literal_eval(v) for v in a.values.split(",")]
    t = tpch_gen.generate_fast(a.sf, seed=1)
    c = PDBClient(root=tempfile.mkdtemp(), device="cuda:0")
    tpch.load(c, "tpch", t, device="cuda:0")
    del t
    from netsdb_amd import _ext

    if a.flag.startswith("hip:"):                 # a setter of the HIP extension (its default is the first value)
        setter = getattr(_ext.hip(), a.flag[4:])
        setf = lambda v: setter(v)  # noqa: E731
        orig = vals[0]
    elif ":" in a.flag:                           # module:ATTR of another netsdb_amd module
        import importlib

        mname, attr = a.flag.split(":", 1)
        mod = importlib.import_module(f"netsdb_amd.{mname}")
        setf = lambda v: setattr(mod, attr, v)  # noqa: E731
        orig = getattr(mod, attr)
    else:
        setf = lambda v: setattr(PL, a.flag, v)  # noqa: E731
        orig = getattr(PL, a.flag)
    out = {"flag": a.flag, "sf": a.sf}
    for q in a.queries.split(","):
        fn = tpch.QUERIES[q]
        res, ts = [], {str(v): [] for v in vals}
        for v in vals:
            setf(v)
            res.append(fn(c, "tpch"))
            fn(c, "tpch")
        for _ in range(a.rounds):
            for v in vals:
                setf(v)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                fn(c, "tpch")
                torch.cuda.synchronize()
                ts[str(v)].append((time.perf_counter() - t0) * 1e3)
        out[q] = {"equal": all(r == res[0] for r in res),
                  **{f"{k}_ms": round(statistics.median(x), 3) for k, x in ts.items()},
                  **{f"{k}_all": [round(y, 3) for y in x] for k, x in ts.items()}}
        print(json.dumps({q: out[q]}), flush=True)
    setf(orig)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
