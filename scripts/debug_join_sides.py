"""Fused join stages with the build side flipped (the adaptive planner measuring a FILTERed side first, as at SF 10
for Q14): run the join queries on the GPU with AdaptivePlanner.MEASURE_BUILD_MIN lowered, and on a launch failure
dump every program column (expression, pass, object type, rows) against the probe / build row counts.

    python scripts/debug_join_sides.py [--sf 0.05] [--min-bytes 1]
"""
import argparse
import os
import sys
import tempfile

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from netsdb_amd.client import PDBClient  # noqa: E402
from netsdb_amd.execution import pipeline as PL  # noqa: E402
from netsdb_amd.models import tpch, tpch_gen  # noqa: E402
from netsdb_amd.query_planning import planner as P  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=0.05)
    ap.add_argument("--min-bytes", type=int, default=1)
    ap.add_argument("--queries", default="q14,q12,q03,q17,q04,q02")
    ap.add_argument("--clear", action="store_true", help="clear the in-process caches before each query (cold runs)")
    a = ap.parse_args()
    P.AdaptivePlanner.MEASURE_BUILD_MIN = a.min_bytes
    orig = PL._launch

    def launch(prog, n, dev, plan):
        try:
            return orig(prog, n, dev, plan)
        except RuntimeError as e:
            bt = plan.builds[plan.join["name"]] if plan.join else None
            print("LAUNCH FAILED:", e, "n =", n, "bn =", None if bt is None else bt.batch.n, flush=True)
            for c in prog.cols:
                o = c["obj"]
                ln = o.numel() if isinstance(o, torch.Tensor) else len(o)
                print("  col", PL._path(c["expr"]), "late", c["late"], "kind", c["kind"], type(o).__name__, "rows", ln,
                      "shape", tuple(o.shape) if isinstance(o, torch.Tensor) else None, flush=True)
            raise

    PL._launch = launch
    t = tpch_gen.generate_fast(a.sf, seed=1)
    f = tpch.frames(t)
    c = PDBClient(root=tempfile.mkdtemp(), device="cuda:0")
    tpch.load(c, "tpch", t, device="cuda:0")
    for q in a.queries.split(","):
        if a.clear:
            c.engine._plan_cache.clear()
            for d in (PL._STAGE_CACHE, PL._PROG_CACHE, PL._JIT_FN, PL._JIT_SHAPES, PL._LIT_DEV):
                d.clear()
        try:
            got = tpch.QUERIES[q](c, "tpch")
        except RuntimeError as e:           # reported above with the columns; the next query still runs
            print(q, "FAILED", e, flush=True)
            continue
        ref = tpch.reference(q, t, f=f)
        print(q, "ok", (got[:1] if isinstance(got, list) else got), (ref[:1] if isinstance(ref, list) else ref),
              flush=True)
    print(c.engine.pipeline_stats, flush=True)


if __name__ == "__main__":
    main()
