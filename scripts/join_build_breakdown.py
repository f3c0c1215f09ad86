"""Per-kernel time of the join builds and probes in a rocprofv3 kernel trace of scripts/bench_relops.py.

Builds are grouped by their table size (the region-build grid = regions + 1; the global-atomic insert as 'global'),
each kernel's median over the builds of that size, plus the whole build's span (first to last kernel).

    python scripts/join_build_breakdown.py gpurun_out/<tag>/relopsprof/run_kernel_trace.csv
"""
import collections
import csv
import statistics
import sys

BUILD = ("jpart_", "join_region_build", "join_runs", "join_perm", "join_init", "join_insert", "join_bloom")


def short(name: str) -> str:
    return name.split("(")[0].split("::")[-1].split("<")[0].replace("void ", "")


def main(path: str) -> None:
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    builds, cur, last = [], None, None
    probes = collections.defaultdict(list)
    for r in rows:
        n = short(r["Kernel_Name"])
        t = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if n in ("jpart_hist_kernel", "join_init_kernel"):
            cur = {"_start": int(r["Start_Timestamp"]), "_size": "global"}
            builds.append(cur)
        if cur is not None and n.startswith(BUILD):
            cur[n] = cur.get(n, 0.0) + t
            cur["_end"] = int(r["End_Timestamp"])
            if n == "join_region_build_kernel":
                cur["_size"] = f"{int(r['Grid_Size_X']) // 512 - 1} regions"
            last = cur["_size"]
        if n == "join_probe_kernel":
            probes[last].append(t)
    by = collections.defaultdict(list)
    for b in builds:
        by[b["_size"]].append(b)
    for size, bs in by.items():
        print(f"build, {size}: {len(bs)} builds")
        for k in [k for k in bs[0] if not k.startswith("_")]:
            print(f"    {k:32s} {statistics.median(b.get(k, 0.0) for b in bs):9.1f} us")
        print(f"    {'span':32s} {statistics.median((b['_end'] - b['_start']) / 1e3 for b in bs):9.1f} us")
        if probes.get(size):
            print(f"    {'join_probe_kernel (after)':32s} {statistics.median(probes[size]):9.1f} us")


if __name__ == "__main__":
    main(sys.argv[1])
