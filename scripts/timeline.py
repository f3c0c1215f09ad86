"""Print the last N nsdb-kernel dispatches of a rocprofv3 kernel trace as a step timeline.

    python scripts/timeline.py gpurun_out/prof/run_kernel_trace.csv [N]
"""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "nsdb" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
last = rows[-n:]
t0 = int(last[0]["Start_Timestamp"])
for r in last:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1000:9.1f} us  {(e - s) / 1000:8.1f} us  {r['Kernel_Name'][:80]}  grid={r['Grid_Size_X']}")
