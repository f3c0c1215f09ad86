"""Probe for the engine's per-stage device time (JobStats["stages"][i]["device_seconds"], HIP event pairs): one
job whose only heavy stage is a vectorised native lambda running ``--gemms`` MFMA GEMMs of 8192 x 4096 x 4096 per
batch. Prints one JSON line per timed run with every stage's host and device seconds; tests/test_device_time_gpu.py
runs it under ``rocprofv3 --kernel-trace`` and compares the heavy stage's device time with the sum of its GEMM
kernels in the trace.

    python scripts/device_time_probe.py [--runs 3 --gemms 20]
"""
import argparse
import json
import os
import sys
import tempfile

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--gemms", type=int, default=20)
    ap.add_argument("--rows", type=int, default=8192)
    ap.add_argument("--k", type=int, default=4096)
    ap.add_argument("--device", default="cuda:0")
    a = ap.parse_args()

    from netsdb_amd import ops
    from netsdb_amd.client import PDBClient
    from netsdb_amd.computations import ScanSet, SelectionComp, WriteSet
    from netsdb_amd.lambdas import Literal, make_batch_lambda, make_lambda_from_self
    from netsdb_amd.objects.record import RecordBatch

    dev = torch.device(a.device)
    c = PDBClient(root=tempfile.mkdtemp(prefix="nsdb_devtime_"), device=dev)
    c.create_database("d")
    c.create_set("d", "x", None)
    g = torch.Generator(device=dev).manual_seed(0)
    X = (torch.rand(a.rows, a.k, device=dev, generator=g) - 0.5).to(torch.bfloat16)
    W = (torch.rand(a.k, a.k, device=dev, generator=g) - 0.5).to(torch.bfloat16)
    c.send_data("d", "x", RecordBatch({"x": X}, a.rows))

    def heavy(b):
        y = None
        for _ in range(a.gemms):
            y = ops.gemm_nt(b.columns["x"], W, out_dtype=torch.bfloat16, out=y)
        return y[:, 0].float()

    class Heavy(SelectionComp):
        def get_selection(self, x):
            return Literal(True)

        def get_projection(self, x):
            return make_batch_lambda(make_lambda_from_self(x), heavy)

    def job(i):
        out = f"y{i}"
        c.create_set("d", out, None)
        return c.execute_computations(WriteSet("d", out).set_input(Heavy().set_input(ScanSet("d", "x"))),
                                      job_name="devtime")

    job(-1)                                          # plans / kernels warm
    if dev.type == "cuda":
        torch.cuda.synchronize()
    for i in range(a.runs):
        st = job(i)
        dts = st.device_times(block=True)
        print(json.dumps({"run": i, "stages": [{"id": s["id"], "desc": s["desc"], "seconds": s["seconds"],
                                                "device_seconds": d} for s, d in zip(st["stages"], dts)],
                          "gemms": a.gemms, "shape": [a.rows, a.k, a.k]}), flush=True)


if __name__ == "__main__":
    main()
