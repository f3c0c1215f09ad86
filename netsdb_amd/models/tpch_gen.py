"""Vectorised TPC-H generator for benchmark scale factors (SF 1 / SF 10: 6 M / 60 M lineitems).

Reference: src/tpch/source/tpchDataLoader.cc (loads dbgen .tbl files) and the dbgen domains it reads. The
list-of-Python-strings generator in models/tpch.py is fine for the test scale (SF 0.004) but builds tens of
millions of Python string objects at SF 10; here every column is a numpy array and every text column is a
:class:`GenStrings` — dictionary codes into a small vocabulary (flags, modes, segments, comments as word
tuples) or a fixed-width byte matrix (names, phones, clerks). A GenStrings becomes a device StringColumn with
ONE gather launch (the vocabulary packed once, ``StringColumn.take(codes)`` on the GPU), and a pandas
Categorical / fixed-width string array for the oracle, so the pandas reference runs at SF 10 as well.

Same distributions as models/tpch.generate (dbgen cardinalities: SF x 150 k customers, 1.5 M orders, 1-7
lineitems per order, 200 k parts x 4 suppliers, custkey % 3 == 0 places no orders, 2 % of order comments
carry "special ... requests"), drawn in a different order: not byte-identical to tpch.generate.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import numpy as np
import torch

from ..objects.strings import StringColumn
from . import tpch as T


class GenStrings:
    """A generated text column: ``vocab[codes]`` or the rows of a fixed-width uint8 matrix."""

    def __init__(self, vocab: Optional[List[str]] = None, codes: Optional[np.ndarray] = None,
                 fixed: Optional[np.ndarray] = None):
        self.vocab, self.codes, self.fixed = vocab, codes, fixed

    def __len__(self):
        return len(self.codes) if self.codes is not None else self.fixed.shape[0]

    def __getitem__(self, i):
        if self.codes is not None:
            return self.vocab[int(self.codes[i])]
        return bytes(self.fixed[i]).decode()

    def rows(self, sl) -> "GenStrings":
        """A row subset (slice or index array), e.g. one rank's share of a generated table."""
        if self.codes is not None:
            return GenStrings(self.vocab, self.codes[sl])
        return GenStrings(fixed=self.fixed[sl])

    def tolist(self) -> List[str]:
        if self.codes is not None:
            v = self.vocab
            return [v[c] for c in self.codes.tolist()]
        return self.fixed.view(f"S{self.fixed.shape[1]}").ravel().astype(str).tolist()

    def to_column(self, device=None) -> StringColumn:
        """The column as a StringColumn on ``device`` (vocabulary gather on the device for coded columns)."""
        if self.codes is not None:
            voc = StringColumn.from_list(self.vocab, device)
            codes = torch.from_numpy(self.codes.astype(np.int64))
            return voc.take(codes.to(voc.device))
        n, w = self.fixed.shape
        data = np.zeros(StringColumn._alloc_size(n * w), dtype=np.uint8)
        data[: n * w] = self.fixed.ravel()
        off = np.arange(n + 1, dtype=np.int64) * w
        col = StringColumn(torch.from_numpy(data), torch.from_numpy(off), n * w, maxlen=w)
        return col.to(device) if device is not None else col

    def to_pandas(self):
        import pandas as pd

        if self.codes is not None:
            return pd.Categorical.from_codes(self.codes.astype(np.int64), categories=self.vocab)
        return self.fixed.view(f"S{self.fixed.shape[1]}").ravel().astype(str)


def _digits(x: np.ndarray, width: int) -> np.ndarray:
    """[n, width] ASCII digits of non-negative ints, zero padded."""
    x = x.astype(np.int64)
    out = np.empty((x.size, width), dtype=np.uint8)
    for j in range(width - 1, -1, -1):
        out[:, j] = 48 + (x % 10)
        x = x // 10
    return out


def _fixed(prefix: str, nums: np.ndarray, width: int) -> GenStrings:
    p = np.frombuffer(prefix.encode(), dtype=np.uint8)
    return GenStrings(fixed=np.concatenate([np.broadcast_to(p, (nums.size, p.size)), _digits(nums, width)], 1))


def _phones(nation: np.ndarray, rng) -> GenStrings:
    n = nation.size
    dash = np.full((n, 1), ord("-"), dtype=np.uint8)
    parts = [_digits(nation + 10, 2), dash, _digits(rng.integers(100, 1000, n), 3), dash,
             _digits(rng.integers(100, 1000, n), 3), dash, _digits(rng.integers(1000, 10000, n), 4)]
    return GenStrings(fixed=np.concatenate(parts, 1))


_NW = len(T.WORDS)
_COMMENT_VOCAB: Optional[List[str]] = None


def _comment_vocab() -> List[str]:
    """Every 4-word comment, then the same with " special <word 0> requests" appended (order comments)."""
    global _COMMENT_VOCAB
    if _COMMENT_VOCAB is None:
        w = T.WORDS
        base = [f"{w[a]} {w[b]} {w[c]} {w[d]}" for a in range(_NW) for b in range(_NW) for c in range(_NW)
                for d in range(_NW)]
        _COMMENT_VOCAB = base + [f"{s} special {w[i // _NW ** 3]} requests" for i, s in enumerate(base)]
    return _COMMENT_VOCAB


def _comments(rng, n: int, special_frac: float = 0.0) -> GenStrings:
    t = rng.integers(0, _NW, size=(n, 4))
    code = ((t[:, 0] * _NW + t[:, 1]) * _NW + t[:, 2]) * _NW + t[:, 3]
    if special_frac > 0:
        code = code + (rng.random(n) < special_frac) * _NW ** 4
    return GenStrings(_comment_vocab(), code.astype(np.int32))


def _cat(vocab: List[str], codes: np.ndarray) -> GenStrings:
    return GenStrings(list(vocab), codes.astype(np.int32))


def _ymd(days: np.ndarray) -> np.ndarray:
    """Days since 1970 -> yyyymmdd through a lookup table (datetime64 conversions once per distinct day)."""
    lo, hi = int(days.min()), int(days.max())
    table = T._days_to_ymd(np.arange(lo, hi + 1))
    return table[days - lo]


def generate_fast(sf: float = 1.0, seed: int = 0) -> Dict[str, Dict[str, object]]:
    """Columnar TPC-H tables ``{table: {column: np.ndarray | GenStrings}}`` at scale factor ``sf``."""
    rng = np.random.default_rng(seed)
    n_supp = max(10, int(10000 * sf))
    n_cust = max(30, int(150000 * sf))
    n_part = max(40, int(200000 * sf))
    n_ord = max(150, int(1500000 * sf))
    t: Dict[str, Dict[str, object]] = {}
    t["region"] = {"r_regionkey": np.arange(5), "r_name": _cat(T.REGIONS, np.arange(5)),
                   "r_comment": _comments(rng, 5)}
    t["nation"] = {"n_nationkey": np.arange(25), "n_name": _cat([n for n, _ in T.NATIONS], np.arange(25)),
                   "n_regionkey": np.array([r for _, r in T.NATIONS]), "n_comment": _comments(rng, 25)}
    sk = np.arange(1, n_supp + 1)
    snat = rng.integers(0, 25, n_supp)
    t["supplier"] = {"s_suppkey": sk, "s_name": _fixed("Supplier#", sk, 9), "s_address": _fixed("addr", sk, 9),
                     "s_nationkey": snat, "s_phone": _phones(snat, rng),
                     "s_acctbal": np.round(rng.uniform(-999.99, 9999.99, n_supp), 2), "s_comment": _comments(rng, n_supp)}
    ck = np.arange(1, n_cust + 1)
    cnat = rng.integers(0, 25, n_cust)
    t["customer"] = {"c_custkey": ck, "c_name": _fixed("Customer#", ck, 9), "c_address": _fixed("caddr", ck, 9),
                     "c_nationkey": cnat, "c_phone": _phones(cnat, rng),
                     "c_acctbal": np.round(rng.uniform(-999.99, 9999.99, n_cust), 2),
                     "c_mktsegment": _cat(T.SEGMENTS, rng.integers(0, 5, n_cust)), "c_comment": _comments(rng, n_cust)}
    pk = np.arange(1, n_part + 1)
    retail = np.round((90000 + (pk // 10) % 20001 + 100 * (pk % 1000)) / 100.0, 2)
    m = rng.integers(1, 6, n_part)
    types = [f"{a} {b} {c}" for a in T.TYPE_S1 for b in T.TYPE_S2 for c in T.TYPE_S3]
    conts = [f"{a} {b}" for a in T.CONT_S1 for b in T.CONT_S2]
    pn = rng.integers(0, _NW, size=(n_part, 3))
    t["part"] = {"p_partkey": pk,
                 "p_name": _cat([f"{T.WORDS[a]} {T.WORDS[b]} {T.WORDS[c]}" for a in range(_NW) for b in range(_NW)
                                 for c in range(_NW)], (pn[:, 0] * _NW + pn[:, 1]) * _NW + pn[:, 2]),
                 "p_mfgr": _cat([f"Manufacturer#{x}" for x in range(1, 6)], m - 1),
                 "p_brand": _cat([f"Brand#{x}{y}" for x in range(1, 6) for y in range(1, 6)],
                                 (m - 1) * 5 + rng.integers(0, 5, n_part)),
                 "p_type": _cat(types, rng.integers(0, len(types), n_part)), "p_size": rng.integers(1, 51, n_part),
                 "p_container": _cat(conts, rng.integers(0, len(conts), n_part)),
                 "p_retailprice": retail, "p_comment": _comments(rng, n_part)}
    ps_pk = np.repeat(pk, 4)
    ps_sk = ((ps_pk + np.tile(np.arange(4), n_part) * (n_supp // 4 + (ps_pk - 1) // n_supp)) % n_supp) + 1
    t["partsupp"] = {"ps_partkey": ps_pk, "ps_suppkey": ps_sk, "ps_availqty": rng.integers(1, 10000, 4 * n_part),
                     "ps_supplycost": np.round(rng.uniform(1.0, 1000.0, 4 * n_part), 2),
                     "ps_comment": _comments(rng, 4 * n_part)}
    ok = np.arange(n_ord)
    ok = (ok // 8) * 32 + (ok % 8) + 1
    valid_c = ck[ck % 3 != 0]
    ocust = valid_c[rng.integers(0, len(valid_c), n_ord)]
    start, end = T._ymd_to_days(19920101), T._ymd_to_days(19980802) - 151
    odays = rng.integers(start, end + 1, n_ord)
    nl = rng.integers(1, 8, n_ord)
    li_ord = np.repeat(np.arange(n_ord), nl)
    nli = len(li_ord)
    first = np.cumsum(nl) - nl
    lnum = np.arange(nli) - np.repeat(first, nl) + 1
    lpk = rng.integers(1, n_part + 1, nli)
    lsk = ((lpk + rng.integers(0, 4, nli) * (n_supp // 4 + (lpk - 1) // n_supp)) % n_supp) + 1
    qty = rng.integers(1, 51, nli).astype(np.float64)
    ext = np.round(qty * retail[lpk - 1], 2)
    disc = rng.integers(0, 11, nli) / 100.0
    tax = rng.integers(0, 9, nli) / 100.0
    ship = odays[li_ord] + rng.integers(1, 122, nli)
    commit = odays[li_ord] + rng.integers(30, 91, nli)
    receipt = ship + rng.integers(1, 31, nli)
    ship_y, commit_y, receipt_y = _ymd(ship), _ymd(commit), _ymd(receipt)
    # returnflag: R / A (half each) when received by CURRENT_DATE, else N; linestatus: O after it, else F
    rf = np.where(receipt_y <= T.CURRENT_DATE, (rng.random(nli) < 0.5).astype(np.int32), 2)   # vocab A, R, N
    ls = (ship_y > T.CURRENT_DATE).astype(np.int32)                                             # vocab F, O
    t["lineitem"] = {"l_orderkey": ok[li_ord], "l_partkey": lpk, "l_suppkey": lsk, "l_linenumber": lnum,
                     "l_quantity": qty, "l_extendedprice": ext, "l_discount": disc, "l_tax": tax,
                     "l_returnflag": _cat(["R", "A", "N"], rf), "l_linestatus": _cat(["F", "O"], ls),
                     "l_shipdate": ship_y, "l_commitdate": commit_y, "l_receiptdate": receipt_y,
                     "l_shipinstruct": _cat(T.INSTRUCTS, rng.integers(0, 4, nli)),
                     "l_shipmode": _cat(T.SHIPMODES, rng.integers(0, 7, nli)), "l_comment": _comments(rng, nli)}
    total = np.bincount(li_ord, weights=ext * (1 + tax) * (1 - disc), minlength=n_ord)
    nF = np.bincount(li_ord, weights=(ls == 0).astype(np.float64), minlength=n_ord).astype(np.int64)
    ostatus = np.where(nF == nl, 0, np.where(nF == 0, 1, 2))                                    # vocab F, O, P
    t["orders"] = {"o_orderkey": ok, "o_custkey": ocust, "o_orderstatus": _cat(["F", "O", "P"], ostatus),
                   "o_totalprice": np.round(total, 2), "o_orderdate": _ymd(odays),
                   "o_orderpriority": _cat(T.PRIORITIES, rng.integers(0, 5, n_ord)),
                   "o_clerk": _fixed("Clerk#", rng.integers(1, max(2, int(1000 * sf)) + 1, n_ord), 9),
                   "o_shippriority": np.zeros(n_ord, dtype=np.int64), "o_comment": _comments(rng, n_ord, 0.02)}
    return t


__all__ = ["GenStrings", "generate_fast"]
