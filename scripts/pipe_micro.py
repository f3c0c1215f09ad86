"""Micro-benchmark of the fused pipeline kernels (csrc/kernels/pipeline.hip) on synthetic lineitem-shaped columns,
outside the engine: a Q06-shaped filter+aggregate, a Q01-shaped grouped aggregate and a Q14-shaped predicate mask.
Prints one JSON line per kernel (device ms, rows/s, effective GB/s of the columns it must read)."""
import argparse
import json
import os
import struct
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from netsdb_amd import _ext  # noqa: E402
from netsdb_amd.execution import pipeline as PL  # noqa: E402
from netsdb_amd.objects.strings import StringColumn  # noqa: E402


def fb(v: float) -> int:
    return struct.unpack("<q", struct.pack("<d", v))[0]


def col(kind, obj, late=0, L=0):
    if isinstance(obj, StringColumn):
        return (kind, late, L, None, obj.starts.contiguous(), obj.ends.contiguous(), obj.data)
    return (kind, late, L, obj, None, None, None)


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=60_000_000)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--which", default="q06,q01,q14")
    ap.add_argument("--max-wg", type=int, default=0)
    ap.add_argument("--tiles", default="0,-1", help="tile sizes to compare (0: register kernels, -1: auto)")
    args = ap.parse_args()
    h = _ext.hip()
    dev = torch.device("cuda")
    n = args.rows
    g = torch.Generator(device=dev).manual_seed(0)
    ship = torch.randint(8036, 10562, (n,), device=dev, dtype=torch.int32, generator=g)
    disc = torch.randint(0, 11, (n,), device=dev, generator=g).double() / 100
    qty = torch.randint(1, 51, (n,), device=dev, generator=g).double()
    price = torch.rand(n, device=dev, generator=g, dtype=torch.float64) * 1e5
    tax = torch.randint(0, 9, (n,), device=dev, generator=g).double() / 100
    abc = torch.tensor([ord("A"), ord("N"), ord("R")], device=dev)
    fo = torch.tensor([ord("F"), ord("O")], device=dev)
    flags = StringColumn.from_short_codes((abc[torch.randint(0, 3, (n,), device=dev, generator=g)] << 3) | 1, 1)
    status = StringColumn.from_short_codes((fo[torch.randint(0, 2, (n,), device=dev, generator=g)] << 3) | 1, 1)
    lit = torch.zeros(1, dtype=torch.uint8, device=dev)
    out = []
    for tile in [int(x) for x in args.tiles.split(",")]:
        run_all(args, h, n, cols_of=dict(ship=ship, disc=disc, qty=qty, price=price, tax=tax, flags=flags,
                                         status=status), lit=lit, tile=tile, out=out)
    for o in out:
        print(json.dumps(o), flush=True)


def run_all(args, h, n, cols_of, lit, tile, out):
    ship, disc, qty, price, tax = (cols_of[k] for k in ("ship", "disc", "qty", "price", "tax"))
    flags, status = cols_of["flags"], cols_of["status"]
    I = PL.IMM
    if "q06" in args.which:
        # (op, dst, a, b, c, imm): each compare after the first ANDs with the running conjunction (c = 4)
        ins = [(PL.OP_GEI, 4, 0, I, -1, 8766), (PL.OP_LTI, 4, 0, I, 4, 9131), (PL.OP_GEF, 4, 1, I, 4, fb(0.05)),
               (PL.OP_LEF, 4, 1, I, 4, fb(0.07)), (PL.OP_LTF, 4, 2, I, 4, fb(24.0)),
               (PL.OP_MULF, 5, 3, 1, -1, 0)]
        prog = torch.tensor(ins, dtype=torch.int64)
        # the same predicate with range instructions (what the compiler emits): 4 instructions
        rins = [(PL.OP_RNGI, 4, 0, -1, -1, 8766, 0 | (1 << 8)), (PL.OP_RNGF, 4, 1, -1, 4, fb(0.05), 1 | (3 << 8)),
                (PL.OP_LTF, 4, 2, I, 4, fb(24.0), 0), (PL.OP_MULF, 5, 3, 1, -1, 0, 0)]
        rprog, kpool = torch.tensor(rins, dtype=torch.int64), [9131, fb(0.07)]
        cols = [col(PL.C_I32, ship), col(PL.C_F64, disc), col(PL.C_F64, qty), col(PL.C_F64, price)]
        ms = timed(lambda: h.pipe_agg(rprog, 3, cols, lit, n, 4, -1, [5], 0, args.max_wg, tile, kpool), args.reps)
        out.append({"tile": tile, "kernel": "q06_range_agg", "ms": round(ms, 4), "grows_s": round(n / ms / 1e6, 2)})
        for late in (1, 0):
            cols = [col(PL.C_I32, ship), col(PL.C_F64, disc), col(PL.C_F64, qty), col(PL.C_F64, price, late)]
            ms = timed(lambda: h.pipe_agg(prog, 5, cols, lit, n, 4, -1, [5], 0, args.max_wg, tile), args.reps)
            out.append({"tile": tile, "kernel": "q06_agg", "late": late, "ms": round(ms, 4), "grows_s": round(n / ms / 1e6, 2),
                        "gbs": round(n * 28 / ms / 1e6, 1)})
    if "q01" in args.which:
        # key = pack(flag code, status code); values qty, price, price*(1-disc), price*(1-disc)*(1+tax), disc, 1.0
        # string columns first (slots 0, 1), as the compiler orders them
        ins = [(PL.OP_LEI, 7, 2, I, -1, 10471),
               (PL.OP_PACK, 8, 0, 1, -1, 11),
               (PL.OP_SUBF, 9, I, 3, -1, fb(1.0)), (PL.OP_MULF, 9, 5, 9, -1, 0),
               (PL.OP_ADDF, 10, I, 6, -1, fb(1.0)), (PL.OP_MULF, 10, 9, 10, -1, 0),
               (PL.OP_CONST, 11, -1, -1, -1, fb(1.0))]
        prog = torch.tensor(ins, dtype=torch.int64)
        for late in (1, 0):
            cols = [col(PL.C_SCODE, flags, late, 1), col(PL.C_SCODE, status, late, 1), col(PL.C_I32, ship),
                    col(PL.C_F64, disc, late), col(PL.C_F64, qty, late), col(PL.C_F64, price, late),
                    col(PL.C_F64, tax, late)]
            ms = timed(lambda: h.pipe_agg(prog, 1, cols, lit, n, 7, 8, [4, 5, 9, 10, 3, 11], 0, args.max_wg, tile),
                       args.reps)
            out.append({"tile": tile, "kernel": "q01_agg", "late": late, "ms": round(ms, 4), "grows_s": round(n / ms / 1e6, 2),
                        "gbs": round(n * (4 + 32 + 2 * 17) / ms / 1e6, 1)})
        t = h.pipe_agg(prog, 1, cols, lit, n, 7, 8, [4, 5, 9, 10, 3, 11], 0, args.max_wg, tile).cpu()
        out.append({"tile": tile, "kernel": "q01_check", "status": int(t[0]), "kept": int(t[1]),
                    "groups": int((t[2:2050] != -(1 << 63)).sum())})
    if "disp" in args.which:
        # dispatch cost: the Q06 columns with k no-op / AND instructions (k = 1, 6, 12)
        cols = [col(PL.C_I32, ship), col(PL.C_F64, disc), col(PL.C_F64, qty), col(PL.C_F64, price)]
        for name, ins1 in (("nop", (PL.OP_NOP, 4, -1, -1, -1, 0)), ("and", (PL.OP_AND, 4, 1, 2, -1, 0))):
            for k in (1, 6, 12):
                prog = torch.tensor([ins1] * k, dtype=torch.int64)
                ms = timed(lambda: h.pipe_agg(prog, k, cols, lit, n, -1, -1, [3], 0, args.max_wg, tile), args.reps)
                out.append({"tile": tile, "kernel": f"disp_{name}_{k}", "ms": round(ms, 4)})
    if "q01c" in args.which:
        # Q01 with the string keys read through their kept short codes (what the engine passes: plain int64 columns)
        ins = [(PL.OP_LEI, 7, 2, I, -1, 10471),
               (PL.OP_PACK, 8, 0, 1, -1, 11),
               (PL.OP_SUBF, 9, I, 3, -1, fb(1.0)), (PL.OP_MULF, 9, 5, 9, -1, 0),
               (PL.OP_ADDF, 10, I, 6, -1, fb(1.0)), (PL.OP_MULF, 10, 9, 10, -1, 0),
               (PL.OP_CONST, 11, -1, -1, -1, fb(1.0))]
        prog = torch.tensor(ins, dtype=torch.int64)
        cols = [col(PL.C_I64, flags.short_codes(1)), col(PL.C_I64, status.short_codes(1)), col(PL.C_I32, ship),
                col(PL.C_F64, disc), col(PL.C_F64, qty), col(PL.C_F64, price), col(PL.C_F64, tax)]
        ms = timed(lambda: h.pipe_agg(prog, 1, cols, lit, n, 7, 8, [4, 5, 9, 10, 3, 11], 0, args.max_wg, tile),
                   args.reps)
        out.append({"tile": tile, "kernel": "q01_codes_agg", "ms": round(ms, 4), "grows_s": round(n / ms / 1e6, 2),
                    "gbs": round(n * (4 + 32 + 16) / ms / 1e6, 1)})
    if "q14" in args.which:
        ins = [(PL.OP_GEI, 1, 0, I, -1, 9374), (PL.OP_LTI, 1, 0, I, 1, 9404)]
        prog = torch.tensor(ins, dtype=torch.int64)
        cols = [col(PL.C_I32, ship)]
        ms = timed(lambda: h.pipe_mask(prog, cols, lit, n, 1, tile), args.reps)
        out.append({"tile": tile, "kernel": "q14_mask", "ms": round(ms, 4), "grows_s": round(n / ms / 1e6, 2),
                    "gbs": round(n * 5 / ms / 1e6, 1)})
        rprog = torch.tensor([(PL.OP_RNGI, 1, 0, -1, -1, 9374, 1 << 8)], dtype=torch.int64)
        ms = timed(lambda: h.pipe_mask(rprog, cols, lit, n, 1, tile, [9404]), args.reps)
        out.append({"tile": tile, "kernel": "q14_range_mask", "ms": round(ms, 4), "grows_s": round(n / ms / 1e6, 2)})
    if "floor" in args.which:
        # no instructions: the load / loop / store floor of each kernel on the same columns
        empty = torch.zeros(0, 6, dtype=torch.int64)
        cols = [col(PL.C_I32, ship)]
        ms = timed(lambda: h.pipe_mask(empty, cols, lit, n, -1, tile), args.reps)
        out.append({"tile": tile, "kernel": "mask_floor_1xi32", "ms": round(ms, 4), "gbs": round(n * 5 / ms / 1e6, 1)})
        cols = [col(PL.C_I32, ship), col(PL.C_F64, disc), col(PL.C_F64, qty), col(PL.C_F64, price)]
        ms = timed(lambda: h.pipe_agg(empty, 0, cols, lit, n, -1, -1, [3], 0, args.max_wg, tile), args.reps)
        out.append({"tile": tile, "kernel": "agg_floor_q06cols", "ms": round(ms, 4), "gbs": round(n * 28 / ms / 1e6, 1)})
        one = torch.tensor([(PL.OP_GEI, 4, 0, I, -1, 8766)], dtype=torch.int64)
        ms = timed(lambda: h.pipe_agg(one, 1, cols, lit, n, 4, -1, [3], 0, args.max_wg, tile), args.reps)
        out.append({"tile": tile, "kernel": "agg_1ins_q06cols", "ms": round(ms, 4), "gbs": round(n * 28 / ms / 1e6, 1)})


if __name__ == "__main__":
    main()
