"""Print the duration series of the FF layer-1 GEMM dispatches (the long 8-phase kernels) from a
rocprofv3 kernel trace: shows the clock ramp / throttling over a bench run.

    python scripts/gemm1_series.py <trace dir> [min_us]
"""
import sys

from kt_summary import load

rows = load(sys.argv[1])
mn = float(sys.argv[2]) if len(sys.argv) > 2 else 300.0
d = [(s, (e - s) / 1e3) for s, e, n in rows if "8ph" in n and (e - s) / 1e3 > mn]
t0 = d[0][0] if d else 0
for i, (s, us) in enumerate(d):
    print(f"{i:4d} t={(s - t0) / 1e6:9.3f} ms  {us:8.1f} us")
