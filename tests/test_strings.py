"""Device string columns (objects/strings.py + csrc/kernels/strings.hip).

CPU tests check StringColumn's numpy paths against plain Python string semantics and run TPC-H queries
with ``NSDB_DEVICE_STRINGS=1`` (every str column packed) against the pandas oracle, plus a 2-rank gloo
shuffle of a packed column. GPU tests check the HIP hash / LIKE / gather kernels against the same Python
references and run the TPC-H string queries on cuda:0."""
import math
import re

import pytest
import torch

from netsdb_amd.execution import kernels as K
from netsdb_amd.objects.record import RecordBatch
from netsdb_amd.objects.strings import StringColumn, hash_str
from netsdb_amd.storage.serde import deserialize_batch, serialize_batch

WORDS = ["", "a", "PROMO BRUSHED TIN", "STANDARD POLISHED BRASS", "special x requests", "requests special",
         "héllo wörld", "a_b%c", "MAIL", "SHIP", "x" * 37, "Clerk#000000951", "13-555-1234", "_", "%"]


def _strings(n, seed=0):
    g = torch.Generator().manual_seed(seed)
    idx = torch.randint(0, len(WORDS), (n,), generator=g).tolist()
    extra = torch.randint(0, 1000, (n,), generator=g).tolist()
    return [WORDS[i] + (f" {e}" if e % 3 == 0 else "") for i, e in zip(idx, extra)]


def _like_ref(s, pattern):
    rx = "".join(".*" if ch == "%" else "." if ch == "_" else re.escape(ch) for ch in pattern)
    return re.fullmatch(rx, s, re.S) is not None


PATTERNS = ["PROMO%", "%BRASS", "%special%requests%", "", "%", "a_b%", "_", "%_%", "MAIL", "%ll%w%",
            "%o%o%o%", "x%x", "13-%", "%#0000009__"]


def _check_column(col, strs):
    assert col.tolist() == strs
    assert col.hash64().cpu().tolist() == [hash_str(s) for s in strs]
    for p in PATTERNS:
        assert col.like(p).cpu().tolist() == [_like_ref(s, p) for s in strs], p
        assert col.like(p, negate=True).cpu().tolist() == [not _like_ref(s, p) for s in strs], p
    for lit in ("a_b", "%", "MAIL", "requests"):
        assert col.startswith(lit).cpu().tolist() == [s.startswith(lit) for s in strs]
        assert col.endswith(lit).cpu().tolist() == [s.endswith(lit) for s in strs]
        assert col.contains(lit).cpu().tolist() == [lit in s for s in strs]
        assert col.eq(lit).cpu().tolist() == [s == lit for s in strs]
    assert col.isin(["MAIL", "SHIP", ""]).cpu().tolist() == [s in ("MAIL", "SHIP", "") for s in strs]
    idx = torch.tensor([len(strs) - 1, 0, 3, 3, 1])
    assert col.take(idx).tolist() == [strs[i] for i in idx.tolist()]
    assert col.take(torch.tensor([], dtype=torch.long)).tolist() == []
    sl = col[5:17]
    assert sl.tolist() == strs[5:17] and sl.take(torch.tensor([2, 0])).tolist() == [strs[7], strs[5]]
    assert StringColumn.concat([col[:4], sl, col[:0]]).tolist() == strs[:4] + strs[5:17]
    codes, dic = col.dict_encode()
    assert [dic[c] for c in codes.cpu().tolist()] == strs and len(dic) == len(set(strs))


def test_string_column_cpu():
    strs = _strings(300)
    _check_column(StringColumn.from_list(strs), strs)
    with pytest.raises(IndexError):
        StringColumn.from_list(strs).take(torch.tensor([300]))


def test_string_keys_match_host_keys():
    strs = _strings(200, seed=1)
    col = StringColumn.from_list(strs)
    assert torch.equal(K.column_to_int64(strs), K.column_to_int64(col))
    inv, reps, n = K.group_ids(col)
    assert n == len(set(strs)) and [reps.tolist()[i] for i in inv.tolist()] == strs
    nums = torch.arange(200) % 3
    inv2, reps2, n2 = K.group_ids((col, nums))
    assert n2 == len(set(zip(strs, nums.tolist())))
    r0, r1 = reps2
    assert [(r0.tolist()[g], int(r1[g])) for g in inv2.tolist()] == list(zip(strs, nums.tolist()))


def test_string_column_serde_and_batch_ops():
    strs = _strings(50, seed=2)
    b = RecordBatch({"s": StringColumn.from_list(strs), "x": torch.arange(50)}, 50)
    page = b.slice(10, 30)
    d = deserialize_batch(serialize_batch(page))
    assert isinstance(d["s"], StringColumn) and d["s"].tolist() == strs[10:30]
    assert page.nbytes() < b.nbytes()
    cat = RecordBatch.concat([page, b.take(torch.tensor([0, 1]))])
    assert cat["s"].tolist() == strs[10:30] + strs[:2]


@pytest.fixture()
def device_strings(monkeypatch):
    monkeypatch.setenv("NSDB_DEVICE_STRINGS", "1")


def _tpch_strings(device, tmp_path):
    from netsdb_amd.client import PDBClient
    from netsdb_amd.models import tpch

    t = tpch.generate(0.004, seed=5)
    c = PDBClient(root=str(tmp_path), device=device)
    tpch.load(c, "tpch", t)
    assert tpch.q14(c, "tpch") == pytest.approx(tpch.reference("q14", t), rel=1e-9)
    for q in ("q01", "q12", "q22", "q13", "q04"):
        ref = tpch.reference(q, t)
        if q == "q01":
            ref = sorted(ref, key=lambda x: (x["l_returnflag"], x["l_linestatus"]))
        elif q != "q13":
            ref = sorted(ref, key=lambda x: x[list(x)[0]])
        got = tpch.QUERIES[q](c, "tpch")
        assert len(got) == len(ref), q
        for g, e in zip(got, ref):
            for k, v in e.items():
                ok = math.isclose(g[k], v, rel_tol=1e-9, abs_tol=1e-6) if isinstance(v, float) else g[k] == v
                assert ok, (q, k, g, e)
    return c


def test_tpch_string_queries_packed_cpu(device_strings, tmp_path):
    from netsdb_amd.models import tpch

    seen = []
    orig = StringColumn.like

    def spy(self, *a, **k):                      # Q13's NOT LIKE (a lambda tree) evaluated on the packed column
        seen.append(type(self))
        return orig(self, *a, **k)

    StringColumn.like = spy
    try:
        _tpch_strings("cpu", tmp_path)
    finally:
        StringColumn.like = orig
    assert seen and all(t is StringColumn for t in seen)


def test_string_column_shuffle_two_ranks():
    from tests.test_distributed import _run

    res = _run("_string_shuffle_scenario")
    for rank, got in enumerate(res):
        for src, (s, i, kind) in enumerate(got):
            assert kind == "StringColumn"
            assert i == [k for k in range(40) if k % 2 == rank]
            assert s == [f"r{src}-{k}-" + "z" * (k % 11) for k in i]


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
def test_string_kernels_gpu():
    strs = _strings(5000, seed=3)
    col = StringColumn.from_list(strs, "cuda:0")
    assert col.device.type == "cuda"
    _check_column(col, strs)
    # the payload of a slice starts mid-buffer: unaligned starts for the dword funnel loads
    sl = col[3:4001]
    assert sl.hash64().cpu().tolist() == [hash_str(s) for s in strs[3:4001]]


@pytest.mark.gpu
def test_tpch_string_queries_gpu(tmp_path):
    """Default policy on a GPU: str columns become HBM StringColumns when a set is placed on cuda:0. (The string
    predicates themselves compile into the fused scan kernels on a GPU, so no eager LIKE call is left to spy on:
    the check is on what the queries read.)"""
    c = _tpch_strings("cuda:0", tmp_path)
    for s, col in (("part", "p_type"), ("orders", "o_comment"), ("lineitem", "l_shipmode"),
                   ("customer", "c_phone")):
        data = c.storage.get_set("tpch", s).all().columns[col]
        assert isinstance(data, StringColumn) and data.device.type == "cuda", (s, col, type(data))


def test_substr_cpu():
    """SUBSTRING on bytes: clamped at both ends, empty rows, lengths 0, a start past every row."""
    strs = ["", "a", "ab", "13-555-0199", "27-1", "xyz" * 20, "é-x"]
    col = StringColumn.from_list(strs)
    for start, length in ((0, 2), (1, 3), (5, 0), (40, 10), (0, 100)):
        got = col.substr(start, length)
        raw = [bytes(got.data[got.offsets[i]:got.offsets[i + 1]].numpy()) for i in range(len(strs))]
        assert raw == [x.encode()[start:start + length] for x in strs]
    ascii_col = StringColumn.from_list(strs[:6])
    sub = ascii_col.substr(0, 2)
    assert sub.tolist() == [x[:2] for x in strs[:6]]
    assert sub.hash64().tolist() == [hash_str(x[:2]) for x in strs[:6]]     # group-by keys of the substrings


@pytest.mark.gpu
def test_substr_gpu_matches_cpu_without_host_reads():
    strs = _strings(4000, seed=9)
    cpu = StringColumn.from_list(strs).substr(1, 3)
    col = StringColumn.from_list(strs, "cuda:0")
    calls = []
    orig = {k: getattr(torch.Tensor, k) for k in ("cpu", "tolist", "item")}

    def guard(name):
        def w(self, *a, **kw):
            calls.append(name)
            return orig[name](self, *a, **kw)
        return w

    for k in orig:
        setattr(torch.Tensor, k, guard(k))
    try:
        sub = col.substr(1, 3)
        h = sub.hash64()
    finally:
        for k, f in orig.items():
            setattr(torch.Tensor, k, f)
    assert calls == [], calls
    assert sub.device.type == "cuda"
    assert sub.tolist() == cpu.tolist()
    assert h.cpu().tolist() == cpu.hash64().tolist()


@pytest.mark.gpu
def test_like_contains_random_small_alphabet_gpu():
    """Contains-segments of LIKE (the dword-at-a-time two-byte candidate scan in strings.hip find_seg) against the
    regex reference on random strings over a 3-letter alphabet: overlapping and repeated candidates, matches at
    every alignment and at the very end of a string, '_' inside and at the head of segments."""
    g = torch.Generator().manual_seed(21)
    strs = []
    for _ in range(4000):
        n = int(torch.randint(0, 40, (1,), generator=g))
        strs.append("".join("abc"[int(i)] for i in torch.randint(0, 3, (n,), generator=g)))
    col = StringColumn.from_list(strs, "cuda:0")
    pats = ["%ab%", "%aab%", "%abc%ca%", "%ba%ab%cc%", "%a_c%", "%_b%", "%cc%", "%abcabc%", "a%bc%", "%ab%c",
            "%aa%aa%aa%", "%c_a_b%", "%bb%"]
    for p in pats:
        assert col.like(p).cpu().tolist() == [_like_ref(s, p) for s in strs], p


def test_short_code_decode_host_paths_agree():
    """from_short_codes: the numpy decode of a few host codes (fused aggregation keys) == the torch decode."""
    import random

    rng = random.Random(3)
    for L in (1, 2, 3, 7):
        words = ["".join(rng.choice("AB xyz|") for _ in range(rng.randint(0, L))) for _ in range(200)]
        codes = StringColumn.from_list(words).short_codes(L)
        small = StringColumn.from_short_codes(codes, L)                       # numpy path (n <= 65536)
        big = StringColumn.from_short_codes(codes.repeat(400), L)             # torch path (80 000 rows)
        assert list(small) == words
        assert list(big)[:200] == words and len(big) == 80_000


def test_tpch_result_lists_one_read():
    """models/tpch.py _lists: tensors, string columns and plain lists of a result batch as Python lists."""
    from netsdb_amd.models.tpch import _lists

    sc = StringColumn.from_list(["R", "AF", "", "NO"])
    got = _lists({"k": sc, "v": torch.tensor([1.5, 2.0, 0.0, -1.0]), "n": torch.tensor([1, 2, 3, 4]), "l": [9, 8, 7, 6]})
    assert got == {"k": ["R", "AF", "", "NO"], "v": [1.5, 2.0, 0.0, -1.0], "n": [1, 2, 3, 4], "l": [9, 8, 7, 6]}


@pytest.mark.gpu
def test_like_occurrence_bitmaps_gpu():
    """The buffer-parallel LIKE (strings.hip like_occ_kernel + like_rows_kernel) for floating-segment patterns against
    the per-row search and a Python regex: occurrences straddling row boundaries must not count, '_' inside a segment,
    overlapping candidates ('aab' in 'aaab'), segments up to 16 bytes, a row selection viewing a larger buffer."""
    from netsdb_amd import _ext

    h = _ext.hip()
    g = torch.Generator().manual_seed(11)
    alpha = "abcs pecialrequstx"
    n = 70_000
    lens = torch.randint(0, 40, (n,), generator=g).tolist()
    chars = torch.randint(0, len(alpha), (sum(lens),), generator=g).tolist()
    strs, o = [], 0
    for ln in lens:
        strs.append("".join(alpha[c] for c in chars[o:o + ln]))
        o += ln
    strs[5] = "xx special yy requests zz"
    strs[6], strs[7] = "...spec", "ial requests"                 # a match only across the row boundary
    strs[8] = "aaab" * 3
    col = StringColumn.from_list(strs, "cuda:0")
    pats = ["%special%requests%", "%sp%", "%aab%", "%ec_al%", "%ab%ca%bs%", "%pecialrequstxabcs%",
            "%special requests%"]
    for pat in pats:
        ref = [_like_ref(s, pat) for s in strs]
        h.str_like_occ_min_rows(1 << 62)
        slow = col.like(pat).cpu().tolist()
        h.str_like_occ_min_rows(1)
        fast = col.like(pat).cpu().tolist()
        neg = col.like(pat, negate=True).cpu().tolist()
        h.str_like_occ_min_rows(1 << 16)
        assert slow == ref, pat
        assert fast == ref, pat
        assert neg == [not x for x in ref], pat
    sel = col.take(torch.arange(3, n, 7, device="cuda:0"))
    h.str_like_occ_min_rows(1)
    got = sel.like("%special%requests%").cpu().tolist()
    h.str_like_occ_min_rows(1 << 16)
    assert got == [_like_ref(strs[i], "%special%requests%") for i in range(3, n, 7)]
