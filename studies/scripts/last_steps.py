"""Timeline of the last N bench steps from a rocprofv3 kernel trace (nsdb kernels only): start offset, gap to the
previous kernel, duration.

    python scripts/last_steps.py gpurun_out/prof/run_kernel_trace.csv [N_KERNELS]
"""
import csv
import sys


def main():
    rows = [r for r in csv.DictReader(open(sys.argv[1])) if "nsdb::" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
    last = rows[-n:]
    t0 = int(last[0]["Start_Timestamp"])
    prev = None
    for r in last:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev) / 1000 if prev else 0.0
        name = r["Kernel_Name"].replace("void ", "").replace("nsdb::", "")[:58]
        print(f"{(s - t0) / 1000:9.1f} +{gap:7.1f} {(e - s) / 1000:8.1f}  {name}")
        prev = e


if __name__ == "__main__":
    main()
