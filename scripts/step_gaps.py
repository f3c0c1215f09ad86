"""Per-step GPU busy time vs wall from a rocprofv3 kernel trace of bench.py: the sum of kernel durations
between consecutive FF layer-1 GEMM starts vs the start-to-start interval (idle = host-bound bubbles).

    python scripts/step_gaps.py gpurun_out/prof/run_kernel_trace.csv [last_n_steps]
"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 10
starts = [i for i, r in enumerate(rows) if "gemm_nt_256_8ph" in r["Kernel_Name"] and int(r["Grid_Size_X"]) == 131072]
busy_all, wall_all = 0.0, 0.0
for a, b in list(zip(starts, starts[1:]))[-n:]:
    t0, t1 = int(rows[a]["Start_Timestamp"]), int(rows[b]["Start_Timestamp"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows[a:b]) / 1000
    wall = (t1 - t0) / 1000
    busy_all += busy
    wall_all += wall
    print(f"step wall {wall:8.1f} us  kernels {busy:8.1f} us  idle {wall - busy:7.1f} us")
print(f"mean: wall {wall_all / n:.1f} us, kernels {busy_all / n:.1f} us")
