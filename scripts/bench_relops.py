"""Device relational operators vs the PyTorch composites they replace, interleaved rounds in one process.

  * group-by + sum of 16 M rows (int64 key, one f64 value) at 8, 10 k and 10 M distinct keys:
    hash_aggregate (relops.hip) vs torch.unique(return_inverse) + index_add_;
  * hash join: build 2 M rows, probe 16 M rows (PK-FK, ~1 match per probe) via JoinTable vs sort + searchsorted;
    and a build-size sweep (2 / 16 / 64 M unique build keys, 16 M probes): build, probe, build + probe;
  * partition permutation of 16 M rows over 8 destinations: partition_perm vs argsort(stable) + bincount.

    python scripts/bench_relops.py [--rows 16000000] [--rounds 5] [--json out.json]
"""
import argparse
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from netsdb_amd import _ext  # noqa: E402
from netsdb_amd.execution import kernels as K  # noqa: E402


def wall(fn, iters=3):
    """Host wall time per call incl. the call's own host syncs (the result sizes are read back)."""
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e3


def run(fns, rounds):
    res = {k: [] for k in fns}
    for _ in range(rounds):
        for k, f in fns.items():
            res[k].append(wall(f))
    return {k: {"ms_median": round(statistics.median(v), 4), "ms_min": round(min(v), 4)} for k, v in res.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=16_000_000)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    dev = "cuda:0"
    n = a.rows
    g = torch.Generator(device=dev).manual_seed(0)
    h = _ext.hip()
    out = {"rows": n, "groupby": {}, "join": {}, "partition": {}}
    vals = torch.rand(n, device=dev, dtype=torch.float64, generator=g)
    for distinct in (8, 1000, 3000, 5000, 10_000, 10_000_000):
        keys = torch.randint(0, distinct, (n,), device=dev, generator=g) * 2654435761
        ref_u, ref_inv = torch.unique(keys, return_inverse=True)
        ref = torch.zeros(ref_u.numel(), device=dev, dtype=torch.float64).index_add_(0, ref_inv, vals)
        r = h.hash_aggregate(keys, vals, "sum", False, 0)
        order = torch.argsort(r[0])
        assert torch.equal(r[0][order], ref_u), "group keys differ"
        err = ((r[1][order, 0] - ref).abs().max() / ref.abs().max()).item()

        def dev_agg():
            return h.hash_aggregate(keys, vals, "sum", False, 0)

        def dev_agg_inv():
            return h.hash_aggregate(keys, vals, "sum", True, 0)

        def dev_agg_nofirst():   # the engine's numeric-key group-by: no representative rows needed
            return h.hash_aggregate(keys, vals, "sum", False, 0, False)

        r2 = dev_agg_nofirst()
        o2 = torch.argsort(r2[0])
        assert torch.equal(r2[0][o2], ref_u) and torch.allclose(r2[1][o2, 0], ref, rtol=1e-9), "no-first path differs"

        def torch_agg():
            u, inv = torch.unique(keys, return_inverse=True)
            return torch.zeros(u.numel(), device=dev, dtype=torch.float64).index_add_(0, inv, vals)

        def dev_agg_part():      # the same call with the MID path off (A/B: MID vs PART)
            h.agg_set_mid(False)
            try:
                return h.hash_aggregate(keys, vals, "sum", False, 0)
            finally:
                h.agg_set_mid(True)

        arms = {"hash_aggregate": dev_agg, "hash_aggregate_no_first": dev_agg_nofirst,
                "hash_aggregate_with_inverse": dev_agg_inv, "torch_unique_index_add": torch_agg}
        if 8 < distinct < 1_000_000:
            arms["hash_aggregate_mid_off"] = dev_agg_part
        t = run(arms, a.rounds)
        t["groups"] = int(ref_u.numel())
        t["path"] = ("LOW/MID", "PART")[int(r[5][1])]
        t["sample_distinct"] = int(r[5][3])
        t["max_rel_err"] = err
        out["groupby"][str(distinct)] = t
        print(json.dumps({"groupby": distinct, **t}), flush=True)
        del keys, ref_u, ref_inv, ref, r
    # join: build = 2M distinct keys (PK side), probe = 16M FK keys
    nb = max(1, n // 8)
    build = torch.randperm(nb, device=dev, generator=g) * 7 + 1
    probe = (torch.randint(0, nb, (n,), device=dev, generator=g) * 7 + 1)
    probe[::10] = -5   # 10 % without a match

    def dev_join():
        return K.JoinTable(build).probe(probe)

    def torch_join():
        sh, order = torch.sort(build)
        lo = torch.searchsorted(sh, probe)
        hi = torch.searchsorted(sh, probe, right=True)
        cnt = hi - lo
        pi = torch.repeat_interleave(torch.arange(n, device=dev), cnt)
        starts = torch.repeat_interleave(lo, cnt)
        csum = torch.cumsum(cnt, 0)
        offs = torch.arange(pi.numel(), device=dev) - torch.repeat_interleave(csum - cnt, cnt)
        return order[starts + offs], pi

    bi, pi = dev_join()
    assert torch.equal(build[bi], probe[pi]) and pi.numel() == int((probe > 0).sum())
    jt = K.JoinTable(build)
    t = run({"join_table_build_probe": dev_join, "join_probe_only": lambda: jt.probe(probe),
             "torch_sort_searchsorted": torch_join}, a.rounds)
    t["build_rows"], t["probe_rows"], t["matches"] = nb, n, int(pi.numel())
    out["join"] = t
    print(json.dumps({"join": t}), flush=True)
    del jt, bi, pi
    # build-size sweep: unique-key builds of 2 / 16 / 64 M rows, each probed by 16 M keys (~90 % matching)
    out["join_sweep"] = {}
    for nb2 in (2_000_000, 16_000_000, 64_000_000):
        b2 = torch.randperm(nb2, device=dev, generator=g) * 7 + 1
        p2 = torch.randint(0, nb2, (n,), device=dev, generator=g) * 7 + 1
        p2[::10] = -5
        jt2 = K.JoinTable(b2)
        bi2, pi2 = jt2.probe(p2)
        assert torch.equal(b2[bi2], p2[pi2]) and pi2.numel() == int((p2 > 0).sum())
        t = run({"build": lambda: K.JoinTable(b2), "probe": lambda: jt2.probe(p2),
                 "build_probe": lambda: K.JoinTable(b2).probe(p2)}, a.rounds)
        # the same probe against a table built without its probe filter (~90 % of the probes match: the filter
        # word is a second dependent read for most rows)
        _ext.hip().join_set_bloom(False)
        try:
            jt3 = K.JoinTable(b2)
        finally:
            _ext.hip().join_set_bloom(True)
        t.update({"probe_no_filter": run({"p": lambda: jt3.probe(p2)}, a.rounds)["p"]})
        del jt3
        t["build_rows"], t["probe_rows"], t["matches"] = nb2, n, int(pi2.numel())
        out["join_sweep"][str(nb2)] = t
        print(json.dumps({"join_sweep": nb2, **t}), flush=True)
        del b2, p2, jt2, bi2, pi2
    dest = torch.randint(0, 8, (n,), device=dev, generator=g)
    t = run({"partition_perm": lambda: K.partition_order(dest, 8),
             "torch_argsort_bincount": lambda: (torch.argsort(dest, stable=True),
                                                torch.bincount(dest, minlength=8).tolist())}, a.rounds)
    out["partition"] = t
    print(json.dumps({"partition": t}), flush=True)
    if a.json:
        os.makedirs(os.path.dirname(a.json) or ".", exist_ok=True)
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
