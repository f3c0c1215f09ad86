"""dbgen .tbl ingestion throughput (models/tpch_tbl.py): write generated TPC-H tables at scale factor SF in dbgen's
format, then time load_tbl (chunked read + device parse + dispatch into the sets) per table. One JSON line."""
import argparse
import json
import os
import shutil
import sys
import tempfile
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=1.0)
    ap.add_argument("--chunk-mb", type=int, default=256)
    ap.add_argument("--dir", default=None)
    a = ap.parse_args()
    from netsdb_amd.client import PDBClient
    from netsdb_amd.models import tpch_gen, tpch_tbl

    dev = "cuda:0" if torch.cuda.is_available() else "cpu"
    d = a.dir or tempfile.mkdtemp(prefix="tbl_")
    t0 = time.perf_counter()
    tables = tpch_gen.generate_fast(a.sf, seed=1)
    tpch_tbl.write_tbl(tables, d)
    t_write = time.perf_counter() - t0
    del tables
    c = PDBClient(root=tempfile.mkdtemp(), device=dev)
    tpch_tbl.load_tbl(c, "warm", d, device=dev, only=["nation", "region"])    # first-launch costs out of the timing
    t1 = time.perf_counter()
    st = tpch_tbl.load_tbl(c, "tpch", d, device=dev, chunk_bytes=a.chunk_mb << 20)
    total = time.perf_counter() - t1
    nbytes = sum(v["bytes"] for v in st.values())
    rows = sum(v["rows"] for v in st.values())
    print(json.dumps({"sf": a.sf, "device": dev, "bytes": nbytes, "rows": rows, "seconds": round(total, 3),
                      "GB_per_s": round(nbytes / total / 1e9, 3), "Mrows_per_s": round(rows / total / 1e6, 2),
                      "write_seconds": round(t_write, 1),
                      "tables": {k: {"rows": v["rows"], "MB": round(v["bytes"] / 1e6, 1), "s": round(v["seconds"], 3)}
                                 for k, v in st.items()}}), flush=True)
    if a.dir is None:
        shutil.rmtree(d, ignore_errors=True)


if __name__ == "__main__":
    main()
