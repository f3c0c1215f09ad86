"""Engine-primitive micro-benchmarks (reference: src/serviceBenchmarks — HashMapTest, StringHashMapTest,
ShuffleTest, AllocationTest).

The reference measures its C++ hash maps, the shuffle service and the page allocator on CPU.  Here the
same services are device/collective primitives, measured on whatever device is given:

* hash join     — ``execution.kernels.join_match``: sort the build hashes, binary-search the probes,
                  expand matches (netsDB's JoinMap build + probe)
* group-by      — ``group_ids`` + ``segment_reduce``: unique/inverse + index_add (the aggregation
                  combiner's hash map)
* string keys   — the StringHashMapTest analogue: host strings hashed to int64 keys, then grouped
* shuffle       — ``ClusterContext.all_to_all_rows`` on hash-partitioned rows (needs >1 rank: run under
                  torchrun; with 1 rank the exchange is a local no-op and is skipped)
* allocation    — native ``SlabAllocator`` alloc/free of page-sized extents

    python scripts/bench_services.py [--device cuda:0] [--rows 50000000]
Prints one JSON line per primitive.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from netsdb_amd import _ext  # noqa: E402
from netsdb_amd.execution import kernels as K  # noqa: E402


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def timeit(fn, dev, iters=5):
    fn()
    _sync(dev)
    best = float("inf")
    for _ in range(iters):
        t0 = time.perf_counter()
        fn()
        _sync(dev)
        best = min(best, time.perf_counter() - t0)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", default="cuda:0" if torch.cuda.is_available() else "cpu")
    ap.add_argument("--rows", type=int, default=50_000_000)
    ap.add_argument("--build-rows", type=int, default=5_000_000)
    ap.add_argument("--groups", type=int, default=100_000)
    ap.add_argument("--string-rows", type=int, default=20_000_000)
    a = ap.parse_args()
    dev = torch.device(a.device)
    g = torch.Generator(device=dev).manual_seed(0)

    # ---- hash join: build side unique keys, probe side with ~1 match per probe
    bkeys = torch.randperm(a.build_rows, device=dev, generator=g).to(torch.int64)
    pkeys = torch.randint(0, a.build_rows, (a.rows,), device=dev, generator=g)
    bh, ph = K.hash_keys(bkeys), K.hash_keys(pkeys)
    out = {}

    def join():
        out["m"] = K.join_match(bh, ph)

    t = timeit(join, dev)
    nmatch = int(out["m"][0].numel())
    print(json.dumps({"primitive": "hash_join", "device": str(dev), "build_rows": a.build_rows, "probe_rows": a.rows,
                      "matches": nmatch, "ms": round(t * 1e3, 2), "probe_rows_per_s": round(a.rows / t, 1)}), flush=True)

    # ---- group-by aggregation (sum of a f64 value per key)
    keys = torch.randint(0, a.groups, (a.rows,), device=dev, generator=g)
    vals = torch.rand(a.rows, device=dev, dtype=torch.float64, generator=g)

    def groupby():
        inv, reps, n = K.group_ids(keys)
        out["s"] = K.segment_reduce(vals, inv, n, "sum")

    t = timeit(groupby, dev)
    ref = torch.zeros(a.groups, dtype=torch.float64, device=dev).index_add_(0, keys, vals)
    ok = bool(torch.allclose(out["s"], ref[ref != 0] if out["s"].numel() != a.groups else ref))
    print(json.dumps({"primitive": "group_by_sum", "device": str(dev), "rows": a.rows, "groups": a.groups,
                      "ms": round(t * 1e3, 2), "rows_per_s": round(a.rows / t, 1), "matches_reference": ok}), flush=True)

    # ---- string keys (StringHashMapTest): a device string column (packed UTF-8 in HBM) -> hash kernel ->
    # device group-by; plus a LIKE predicate over the same column
    from netsdb_amd.objects.strings import StringColumn

    strs = [f"key-{i % 5000}-" + "x" * (i % 17) for i in range(a.string_rows)]
    scol = StringColumn.from_list(strs, dev)

    def strgroup():
        inv, reps, n = K.group_ids(scol)
        out["n"] = n

    t = timeit(strgroup, dev, iters=5)
    print(json.dumps({"primitive": "string_key_group_by", "device": str(dev), "rows": a.string_rows,
                      "bytes": scol.payload, "groups": out["n"], "ms": round(t * 1e3, 2),
                      "rows_per_s": round(a.string_rows / t, 1)}), flush=True)

    def strlike():
        out["m"] = scol.like("%-1%xxx%")

    t = timeit(strlike, dev, iters=5)
    print(json.dumps({"primitive": "string_like", "device": str(dev), "rows": a.string_rows,
                      "matches": int(out["m"].sum()), "ms": round(t * 1e3, 3),
                      "GBps": round(scol.payload / t / 1e9, 1)}), flush=True)

    # ---- shuffle over the process group
    from netsdb_amd.parallel.comm import ClusterContext

    ctx = ClusterContext.from_env(device=str(dev)) if int(os.environ.get("WORLD_SIZE", "1")) > 1 else None
    if ctx is not None and ctx.distributed:
        rows = torch.randn(a.rows // 10, 16, device=dev)
        dest = K.partition_of(K.hash_keys(torch.arange(rows.shape[0], device=dev)), ctx.world_size)
        order = torch.argsort(dest)
        counts = torch.bincount(dest, minlength=ctx.world_size).tolist()

        def shuffle():
            out["x"] = ctx.all_to_all_rows(rows[order], counts)

        t = timeit(shuffle, dev)
        nbytes = rows.numel() * rows.element_size()
        t = ctx.all_reduce_scalar(t, "max")
        if ctx.rank == 0:
            print(json.dumps({"primitive": "shuffle_all_to_all", "ranks": ctx.world_size, "bytes_per_rank": nbytes,
                              "ms": round(t * 1e3, 2), "GBps_per_rank": round(nbytes / t / 1e9, 2)}), flush=True)
    else:
        print(json.dumps({"primitive": "shuffle_all_to_all", "skipped": "single rank (run under torchrun)"}), flush=True)

    # ---- allocation (AllocationTest): native slab allocator, 64 MiB pages in a 288 GiB arena
    sa = _ext.native().SlabAllocator(288 << 30, 256)
    n = 4000
    t0 = time.perf_counter()
    offs = [sa.alloc((64 << 20) // (1 + i % 7)) for i in range(n)]     # ~96 GiB of mixed extents
    for o in offs[::2]:
        sa.free(o)
    for o in offs[1::2]:
        sa.free(o)
    t = time.perf_counter() - t0
    print(json.dumps({"primitive": "slab_alloc_free", "ops": 2 * n, "ms": round(t * 1e3, 2),
                      "ops_per_s": round(2 * n / t, 1), "all_fit": min(offs) >= 0, "leak_free": sa.used == 0}),
          flush=True)


if __name__ == "__main__":
    main()
