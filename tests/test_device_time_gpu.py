"""Per-stage device time (HIP event pairs, no synchronisation inside a job): a stage's device_seconds against the
sum of its kernels in a rocprofv3 kernel trace of the same run, plus the tracer's device spans.
Reference: src/pdbServer/headers/PDBLogger.h (job / stage timing logs)."""
import csv
import glob
import json
import os
import shutil
import subprocess
import sys
import tempfile

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_stage_device_time_matches_rocprof_kernel_sum():
    rp = shutil.which("rocprofv3")
    if rp is None:
        pytest.skip("rocprofv3 not on PATH")
    out = tempfile.mkdtemp(prefix="nsdb_devtime_prof_")
    runs, gemms = 3, 20
    cmd = [rp, "--kernel-trace", "--output-format", "csv", "-d", out, "-o", "run", "--",
           sys.executable, os.path.join(ROOT, "scripts", "device_time_probe.py"), "--runs", str(runs),
           "--gemms", str(gemms)]
    p = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240,
                       env=dict(os.environ, TMPDIR="/tmp"))
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == runs
    heavy = [max(r["stages"], key=lambda s: s["device_seconds"] or 0) for r in lines]
    dev_s = [h["device_seconds"] for h in heavy]
    assert all(d is not None and d > 0 for d in dev_s), lines
    traces = glob.glob(os.path.join(out, "**", "run_kernel_trace.csv"), recursive=True)
    assert traces, os.listdir(out)
    with open(traces[0]) as f:
        rows = [r for r in csv.DictReader(f) if "gemm_nt" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ns = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows]
    per_run = len(ns) // (runs + 1)                  # the warm-up job ran the same GEMMs first
    assert per_run >= gemms, (len(ns), runs)
    for i in range(runs):
        k = ns[(i + 1) * per_run:(i + 2) * per_run]
        ksum = sum(k) / 1e9
        # the stage's device span holds its GEMMs plus the scan / write work around them: within 10 %
        assert abs(dev_s[i] - ksum) <= 0.10 * ksum, (i, dev_s[i], ksum)


def test_tracer_device_spans_and_history():
    """Tracer(device_time=True) spans carry device_us after resolve(); the self-learning history stores each stage's
    device seconds."""
    from netsdb_amd import ops
    from netsdb_amd.utils.trace import Tracer

    tr = Tracer(device_time=True)
    A = torch.randn(4096, 4096, device="cuda:0").to(torch.bfloat16)
    ops.gemm_nt(A, A)
    torch.cuda.synchronize()
    with tr.span("gemm"):
        for _ in range(10):
            ops.gemm_nt(A, A)
    assert tr.resolve(block=True) == 0
    ev = tr.events[-1]
    assert ev["args"]["device_us"] > 0
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(10):
        ops.gemm_nt(A, A)
    e.record()
    e.synchronize()
    ref_us = s.elapsed_time(e) * 1e3
    assert 0.7 * ref_us < ev["args"]["device_us"] < 1.5 * ref_us, (ev["args"]["device_us"], ref_us)
    path = os.path.join(tempfile.mkdtemp(), "t.json")
    tr.export_chrome(path)
    assert "device_us" in json.load(open(path))["traceEvents"][-1]["args"]

    from netsdb_amd.client import PDBClient
    from netsdb_amd.models import tpch, tpch_gen

    c = PDBClient(root=tempfile.mkdtemp(), device="cuda:0")
    tpch.load(c, "tpch", tpch_gen.generate_fast(0.01, seed=3), device="cuda:0")
    sl = c.enable_self_learning()
    tpch.QUERIES["q06"](c, "tpch")
    tpch.QUERIES["q01"](c, "tpch")
    assert sl.db.flush_device_times(block=True) == 0
    vals = [r[0] for r in sl.db.conn.execute("SELECT device_seconds FROM job_stage")]
    assert vals and all(v is not None and v > 0 for v in vals), vals
