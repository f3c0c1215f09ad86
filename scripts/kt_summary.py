"""Summarise a rocprofv3 kernel-trace CSV: per-kernel count / median / mean duration, and the
timeline of the last N dispatches (start offset, duration, name).

    python scripts/kt_summary.py <dir-with-*kernel_trace.csv> [last_n] [name_filter]
"""
import csv
import glob
import os
import statistics
import sys


def load(path):
    files = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def main():
    path = sys.argv[1]
    last = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    rows = load(path)
    if len(sys.argv) > 3:          # keep only kernels whose name contains this substring
        rows = [r for r in rows if sys.argv[3] in r[2]]
    by = {}
    for s, e, n in rows:
        by.setdefault(n, []).append((e - s) / 1e3)
    print(f"{'kernel':80s} {'n':>5s} {'median_us':>10s} {'mean_us':>10s} {'min_us':>9s}")
    for n, d in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        print(f"{n[:80]:80s} {len(d):5d} {statistics.median(d):10.1f} {statistics.mean(d):10.1f} {min(d):9.1f}")
    print(f"\nlast {last} dispatches:")
    t0 = rows[-last][0] if len(rows) >= last else rows[0][0]
    for s, e, n in rows[-last:]:
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} us  {n[:70]}")


if __name__ == "__main__":
    main()
