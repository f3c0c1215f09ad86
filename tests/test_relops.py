"""Device relational operators (csrc/kernels/relops.hip via execution/kernels.py): hash aggregation, hash join,
partition permutation, and value-exact keys (strings byte-compared after the hash; packed int tuples).

GPU tests compare every kernel against a plain PyTorch / Python reference of the same op; CPU tests cover the
host paths and the collision handling with a deliberately weak string hash."""
import pytest
import torch

from netsdb_amd import _ext
from netsdb_amd.execution import kernels as K
from netsdb_amd.objects.strings import StringColumn

DEV = "cuda:0"


def _ref_groupby(keys, vals, op):
    """dict: key -> (agg row, count) in fp64 / int64 on the host."""
    out = {}
    k = keys.tolist()
    v = vals.tolist() if vals is not None else [[]] * len(k)
    for kk, vv in zip(k, v):
        vv = vv if isinstance(vv, list) else [vv]
        if kk not in out:
            out[kk] = [list(vv), 1]
        else:
            a, c = out[kk]
            for j, x in enumerate(vv):
                a[j] = a[j] + x if op == "sum" else (min(a[j], x) if op == "min" else max(a[j], x))
            out[kk][1] = c + 1
    return out


def _check_agg(keys, vals, op, r, rtol=1e-9):
    reps, aggs, cnt, first, inv, status = r
    ref = _ref_groupby(keys.cpu(), None if vals is None else vals.cpu(), op)
    g = int(status[0])
    assert g == len(ref) == reps.numel()
    assert sorted(reps.tolist()) == sorted(ref.keys())
    kl = keys.cpu().tolist()
    first_of = {}
    for i, kk in enumerate(kl):
        first_of.setdefault(kk, i)
    cl, fl = cnt.cpu().tolist(), first.cpu().tolist()
    al = aggs.cpu().tolist() if vals is not None else None
    for i, kk in enumerate(reps.tolist()):
        a, c = ref[kk]
        assert cl[i] == c
        assert fl[i] == first_of[kk]
        if al is not None:
            for x, y in zip(al[i], a):
                assert abs(x - y) <= rtol * max(1.0, abs(y)), (kk, al[i], a)
    if inv.numel():
        assert torch.equal(reps.index_select(0, inv).cpu(), keys.cpu())


# ------------------------------------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("n,distinct", [(1000, 8), (200_000, 10), (200_000, 5000), (300_000, 250_000),
                                        (50_000, 1), (17, 17)])
@pytest.mark.parametrize("op", ["sum", "min", "max"])
def test_hash_aggregate_f64(n, distinct, op):
    g = torch.Generator(device=DEV).manual_seed(n + distinct)
    keys = torch.randint(0, distinct, (n,), device=DEV, generator=g) * 7919 - 3 * distinct
    vals = torch.rand(n, 3, device=DEV, dtype=torch.float64, generator=g) - 0.5
    r = _ext.hip().hash_aggregate(keys, vals, op, True, 0)
    assert int(r[5][2]) == 1
    _check_agg(keys, vals, op, r)


@pytest.mark.gpu
@pytest.mark.parametrize("F", [1, 3])
def test_hash_aggregate_high_cardinality_subpartitions(F):
    """Mostly-distinct keys: every level-1 bucket is split again on the device (agg_bucket_kernel's sub-partition
    pass), then each sub-bucket is aggregated in LDS and written straight to the dense output."""
    g = torch.Generator(device=DEV).manual_seed(17 + F)
    n = 1_000_000
    keys = torch.randint(0, 800_000, (n,), device=DEV, generator=g) * 1_000_003
    vals = torch.rand(n, F, device=DEV, dtype=torch.float64, generator=g)
    r = _ext.hip().hash_aggregate(keys, vals, "sum", True, 0)
    assert int(r[5][2]) == 1 and int(r[5][1]) == 1                   # PART path
    assert int(r[5][3]) > 200_000                                       # the sample saw a high-cardinality column
    _check_agg(keys, vals, "sum", r)


@pytest.mark.gpu
@pytest.mark.parametrize("op", ["sum", "min", "max"])
def test_hash_aggregate_int64_and_sentinel(op):
    g = torch.Generator(device=DEV).manual_seed(3)
    keys = torch.randint(0, 300, (100_000,), device=DEV, generator=g)
    keys[::97] = torch.iinfo(torch.int64).min            # the empty-slot marker as a real key
    keys[5::101] = torch.iinfo(torch.int64).max
    vals = torch.randint(-10**12, 10**12, (100_000,), device=DEV, generator=g)
    for thr, path in ((100_000, 0), (1, 1)):                # forced LOW, forced PART
        r = _ext.hip().hash_aggregate(keys, vals, op, True, thr)
        assert int(r[5][1]) == path
        _check_agg(keys, vals.unsqueeze(1), op, r, rtol=0)
    r = _ext.hip().hash_aggregate(keys, None, "sum", False, 0)   # counts only, no inverse
    reps, _, cnt, _, inv, _ = r
    assert inv.numel() == 0
    ref = torch.bincount(torch.unique(keys.cpu(), return_inverse=True)[1])
    assert sorted(cnt.cpu().tolist()) == sorted(ref.tolist())


@pytest.mark.gpu
def test_hash_aggregate_paths_agree_on_skew():
    """Skew: four hot keys make four oversized level-1 buckets (each still owned by one workgroup) next to
    buckets of singletons; LOW (thr 100k) and PART must agree."""
    g = torch.Generator(device=DEV).manual_seed(11)
    hot = torch.randint(0, 4, (400_000,), device=DEV, generator=g)
    cold = torch.randint(1000, 10**9, (100_000,), device=DEV, generator=g)
    keys = torch.cat([hot, cold])[torch.randperm(500_000, device=DEV, generator=g)]
    vals = torch.ones(500_000, 1, device=DEV, dtype=torch.float64)
    for thr in (0, 100_000):
        r = _ext.hip().hash_aggregate(keys, vals, "sum", True, thr)
        _check_agg(keys, vals, "sum", r)


@pytest.mark.gpu
def test_group_reduce_matches_segment_reduce():
    g = torch.Generator(device=DEV).manual_seed(5)
    n = 123_457
    a = torch.randint(0, 50, (n,), device=DEV, generator=g)
    b = torch.randint(-3, 3, (n,), device=DEV, generator=g).to(torch.int32)
    v = torch.randn(n, 2, device=DEV, generator=g)
    for op in ("sum", "min", "max", "count", "mean"):
        reps, agg = K.group_reduce((a, b), v, op)
        with K_opts(hash_groupby=False):
            inv, reps2, g2 = K.group_ids((a.cpu(), b.cpu()))
        ref = K.segment_reduce(v.cpu(), inv, g2, op) if op != "count" else torch.bincount(inv)
        assert torch.equal(reps[0].cpu(), reps2[0]) and torch.equal(reps[1].cpu(), reps2[1])
        assert reps[1].dtype == torch.int32
        torch.testing.assert_close(agg.cpu().to(ref.dtype), ref, rtol=1e-5, atol=1e-4)


def K_opts(**kw):
    from netsdb_amd import ops
    return ops.kernel_options(**kw)


@pytest.mark.gpu
def test_group_ids_device_tuple_unpackable_and_floats():
    g = torch.Generator(device=DEV).manual_seed(9)
    n = 50_000
    a = torch.randint(-2**62, 2**62, (30,), device=DEV, generator=g)[torch.randint(0, 30, (n,), device=DEV, generator=g)]
    b = torch.randint(-2**62, 2**62, (7,), device=DEV, generator=g)[torch.randint(0, 7, (n,), device=DEV, generator=g)]
    f = torch.tensor([0.0, -0.0, 1.5, float("inf")], device=DEV)[torch.randint(0, 4, (n,), device=DEV, generator=g)]
    inv, reps, ng = K.group_ids((a, b, f))
    ref = {}
    for t in zip(a.tolist(), b.tolist(), f.tolist()):
        ref.setdefault(t, len(ref))
    assert ng == len(ref)
    got = list(zip(*(r.tolist() for r in reps)))
    assert sorted(got) == sorted(ref.keys())
    rows = list(zip(a.tolist(), b.tolist(), f.tolist()))
    il = inv.tolist()
    for i in range(0, n, 997):
        assert got[il[i]] == rows[i]


@pytest.mark.gpu
def test_join_table_device_vs_host():
    g = torch.Generator(device=DEV).manual_seed(2)
    build = torch.randint(0, 5000, (40_000,), device=DEV, generator=g)
    build[::13] = torch.iinfo(torch.int64).min
    probe = torch.randint(-100, 6000, (70_000,), device=DEV, generator=g)
    probe[::17] = torch.iinfo(torch.int64).min
    jt = K.JoinTable(build)
    bi, pi = jt.probe(probe)
    bi2, pi2 = K.JoinTable(build.cpu()).probe(probe.cpu())
    assert bi.numel() == bi2.numel() > 0
    assert torch.equal(build[bi], probe[pi])
    a = sorted(zip(pi.cpu().tolist(), bi.cpu().tolist()))
    b = sorted(zip(pi2.tolist(), bi2.tolist()))
    assert a == b
    assert bool((pi[1:] >= pi[:-1]).all())                 # probe-major
    e_b, e_p = jt.probe(torch.empty(0, dtype=torch.int64, device=DEV))
    assert e_b.numel() == 0 and e_p.numel() == 0


@pytest.mark.gpu
def test_join_unique_build_keys_and_single_sentinel():
    """Primary-key builds (every key once, one row with the empty-slot marker value): the claiming row is its
    own payload, no CSR run; every probe row finds exactly its build row."""
    g = torch.Generator(device=DEV).manual_seed(4)
    build = torch.randperm(300_000, device=DEV, generator=g) * 3 + 1
    build[123] = torch.iinfo(torch.int64).min
    probe = build[torch.randint(0, 300_000, (1_000_000,), device=DEV, generator=g)]
    bi, pi = K.JoinTable(build).probe(probe)
    assert pi.numel() == probe.numel() and torch.equal(pi, torch.arange(probe.numel(), device=DEV))
    assert torch.equal(build[bi], probe)
    assert _ext.hip().join_build(build)[1].numel() == build.numel()
    # one repeated key (and a second kEmpty-marker row): the CSR path, every pair still found
    b2 = torch.cat([build, build[:1], build[123:124]])
    tab, perm = _ext.hip().join_build(b2)[:2]
    assert perm.numel() == b2.numel()
    bi, pi = K.JoinTable(b2).probe(probe)
    assert bi.numel() == int((torch.isin(probe, b2).long() + (probe == build[0]).long()
                              + (probe == build[123]).long()).sum())
    assert torch.equal(b2[bi], probe[pi])


@pytest.mark.gpu
@pytest.mark.parametrize("P", [1, 2, 8, 255, 1024])
def test_partition_order_stable(P):
    g = torch.Generator(device=DEV).manual_seed(P)
    dest = torch.randint(0, P, (200_003,), device=DEV, generator=g)
    perm, counts = K.partition_order(dest, P)
    assert torch.equal(perm.cpu(), torch.argsort(dest.cpu(), stable=True))
    assert counts == torch.bincount(dest.cpu(), minlength=P).tolist()


@pytest.mark.gpu
def test_string_keys_exact_under_hash_collisions_gpu(monkeypatch):
    strs = [f"longer-key{i % 37}" for i in range(5000)]     # > 7 bytes: the hash + byte re-check path
    col = StringColumn.from_list(strs, DEV)
    orig = StringColumn.hash64
    monkeypatch.setattr(StringColumn, "hash64", lambda self: orig(self) & 3)   # 4 hash values for 37 strings
    inv, reps, ng = K.group_ids(col)
    assert ng == 37 and sorted(reps.tolist()) == sorted(set(strs))
    rl = reps.tolist()
    assert [rl[i] for i in inv.tolist()] == strs
    nums = torch.tensor([i % 2 for i in range(5000)], device=DEV)
    inv2, reps2, ng2 = K.group_ids((col, nums))
    assert ng2 == len(set(zip(strs, nums.tolist())))
    vals = torch.ones(5000, device=DEV)
    # forced collisions: the fused hash aggregation must refuse (its per-row check against the group's
    # representative fails) so the engine takes the exact generic path; that path must then be exact
    assert K.group_reduce(col, vals, "sum") is None
    inv3, reps3, g3 = K.group_ids(col)
    agg3 = K.segment_reduce(vals, inv3, g3, "sum")
    assert sorted(zip(reps3.tolist(), agg3.tolist())) == sorted((s, float(strs.count(s))) for s in set(strs))
    monkeypatch.setattr(StringColumn, "hash64", orig)          # no collisions: the fused path runs and is exact
    r = K.group_reduce(col, vals, "sum")
    assert r is not None
    assert sorted(zip(r[0].tolist(), r[1].tolist())) == sorted((s, float(strs.count(s))) for s in set(strs))
    m = col.isin(["longer-key1", "longer-key5"])
    assert m.tolist() == [s in ("longer-key1", "longer-key5") for s in strs]


@pytest.mark.gpu
def test_str_eq_pairs_kernel():
    a = StringColumn.from_list(["", "a", "abcdefghij", "abcdefghiX", "same", "x" * 100], DEV)
    b = StringColumn.from_list(["", "b", "abcdefghij", "abcdefghij", "same", "x" * 99 + "y"], DEV)
    assert a.eq_rows(None, b, None).tolist() == [True, False, True, False, True, False]
    ia = torch.tensor([4, 2, 0], device=DEV)
    ib = torch.tensor([4, 3, 0], device=DEV)
    assert a.eq_rows(ia, b, ib).tolist() == [True, True, True]


# ------------------------------------------------------------------------------------------------ CPU
def test_string_group_exact_under_collisions_cpu(monkeypatch):
    strs = [f"k{i % 11}" for i in range(400)]
    col = StringColumn.from_list(strs)
    orig = StringColumn.hash64
    monkeypatch.setattr(StringColumn, "hash64", lambda self: orig(self) & 1)
    inv, reps, ng = K.group_ids(col)
    assert ng == 11
    rl = reps.tolist()
    assert [rl[i] for i in inv.tolist()] == strs
    assert col.isin(["k3"]).tolist() == [s == "k3" for s in strs]
    assert col.eq_rows(None, StringColumn.from_list(["k0"] * 400), None).tolist() == [s == "k0" for s in strs]


def test_isin_listed_values_sharing_a_hash(monkeypatch):
    col = StringColumn.from_list(["a", "b", "c", "a"])
    monkeypatch.setattr(StringColumn, "hash64", lambda self: torch.zeros(len(self), dtype=torch.int64))
    assert col.isin(["a", "c"]).tolist() == [True, False, True, True]


def test_join_table_host_path():
    build = torch.tensor([5, 1, 5, 9, 1, 1])
    probe = torch.tensor([1, 2, 5, 9, 9])
    bi, pi = K.JoinTable(build).probe(probe)
    pairs = sorted(zip(pi.tolist(), bi.tolist()))
    assert pairs == [(0, 1), (0, 4), (0, 5), (2, 0), (2, 2), (3, 3), (4, 3)]


def test_partition_order_host_path():
    dest = torch.tensor([2, 0, 2, 1, 0])
    perm, counts = K.partition_order(dest, 3)
    assert perm.tolist() == [1, 4, 3, 0, 2] and counts == [2, 1, 2]


def test_pack_exact_roundtrip():
    a = torch.tensor([3, -5, 3, 100])
    b = torch.tensor([7, 7, 8, 0])
    packed, layout = K._pack_exact([a, b])
    ua, ub = K._unpack(packed, layout)
    assert torch.equal(ua, a) and torch.equal(ub, b)
    # lexicographic order preserved
    order = torch.argsort(packed)
    assert [(int(a[i]), int(b[i])) for i in order] == sorted(zip(a.tolist(), b.tolist()))
    assert K._pack_exact([torch.tensor([-2**62, 2**62]), torch.tensor([0, 1])]) is None


@pytest.mark.gpu
@pytest.mark.parametrize("distinct", [8, 5000, 400_000])
def test_hash_aggregate_without_first_rows(distinct):
    """want_first=False (packed numeric keys): the partition passes carry no row ids; groups, sums and counts
    are unchanged."""
    g = torch.Generator(device=DEV).manual_seed(distinct)
    n = 600_000
    keys = torch.randint(0, distinct, (n,), device=DEV, generator=g) * 7 + 1
    vals = torch.rand(n, 2, device=DEV, dtype=torch.float64, generator=g)
    a = _ext.hip().hash_aggregate(keys, vals, "sum", False, 0, True)
    b = _ext.hip().hash_aggregate(keys, vals, "sum", False, 0, False)
    oa, ob = torch.argsort(a[0]), torch.argsort(b[0])
    assert torch.equal(a[0][oa], b[0][ob]) and torch.equal(a[2][oa], b[2][ob])
    torch.testing.assert_close(a[1][oa], b[1][ob], rtol=1e-12, atol=1e-9)


_SHORT = ["", "a", "ab", "a\x00", "b", "zz", "abcdefg", "\u00e9", "A", "ab"]


def _check_short_codes(col, strs):
    codes = col.short_codes().cpu()
    enc = [x.encode() for x in strs]
    assert len(set(codes.tolist())) == len(set(enc))
    assert all((codes[i] == codes[j]).item() == (enc[i] == enc[j]) for i in range(len(enc)) for j in range(len(enc)))
    order = sorted(range(len(enc)), key=lambda i: enc[i])          # byte-lexicographic
    assert sorted(codes.tolist()) == [codes[i].item() for i in order]
    back = StringColumn.from_short_codes(codes.to(col.device), col.max_len())
    assert back.tolist() == strs


def test_short_string_codes_cpu():
    """Strings of <= 7 bytes as exact, order-preserving int64 codes (no hash, no byte re-check)."""
    col = StringColumn.from_list(_SHORT)
    assert col.max_len() == 7
    _check_short_codes(col, _SHORT)
    _check_short_codes(col.take(torch.tensor([1, 4, 4, 8])), [_SHORT[i] for i in (1, 4, 4, 8)])
    assert StringColumn.from_list(["abcdefgh", "a"]).short_codes() is None       # 8 bytes: hash path
    assert col.isin(["ab", "zz", "much too long"]).tolist() == [x in ("ab", "zz") for x in _SHORT]
    assert col.take(torch.tensor([1, 2])).isin(["abcdefg"]).tolist() == [False, False]


@pytest.mark.gpu
def test_short_string_codes_and_groupby_gpu():
    col = StringColumn.from_list(_SHORT, DEV)
    _check_short_codes(col, _SHORT)
    assert torch.equal(col.short_codes().cpu(), StringColumn.from_list(_SHORT).short_codes())
    # a two-column short string key (the TPC-H Q01 shape): packed into one exact int, groups in byte order
    g = torch.Generator(device=DEV).manual_seed(2)
    n = 300_000
    f1 = StringColumn.from_list(["A", "N", "R"], DEV).take(torch.randint(0, 3, (n,), device=DEV, generator=g))
    f2 = StringColumn.from_list(["F", "O"], DEV).take(torch.randint(0, 2, (n,), device=DEV, generator=g))
    v = torch.rand(n, 2, device=DEV, dtype=torch.float64, generator=g)
    reps, agg = K.group_reduce((f1, f2), v, "sum")
    keys = list(zip(f1.tolist(), f2.tolist()))
    assert list(zip(reps[0].tolist(), reps[1].tolist())) == sorted(set(keys))
    uk = sorted(set(keys))
    gid = torch.tensor([uk.index(k) for k in keys])
    ref = torch.zeros(len(uk), 2, dtype=torch.float64).index_add_(0, gid, v.cpu())
    torch.testing.assert_close(agg.cpu(), ref, rtol=1e-9, atol=1e-9)


@pytest.mark.gpu
@pytest.mark.parametrize("distinct", [6, 3000, 300_000])
def test_hash_aggregate_column_major_values(distinct):
    """A [n, F] value row given column-major (the transpose of a contiguous [F, n] stack) is read in place by both
    paths (LOW / PART) and aggregates exactly like the row-major copy."""
    g = torch.Generator(device=DEV).manual_seed(distinct)
    n = 500_000
    keys = torch.randint(0, distinct, (n,), device=DEV, generator=g) * 3 + 1
    cols = torch.rand(4, n, device=DEV, dtype=torch.float64, generator=g)
    vc = cols.t()
    assert vc.stride() == (1, n)
    a = _ext.hip().hash_aggregate(keys, vc, "sum", True, 0)
    b = _ext.hip().hash_aggregate(keys, vc.contiguous(), "sum", True, 0)
    assert int(a[5][1]) == int(b[5][1]) and int(a[5][2]) == 1
    oa, ob = torch.argsort(a[0]), torch.argsort(b[0])
    assert torch.equal(a[0][oa], b[0][ob]) and torch.equal(a[2][oa], b[2][ob]) and torch.equal(a[3][oa], b[3][ob])
    torch.testing.assert_close(a[1][oa], b[1][ob], rtol=1e-12, atol=1e-9)
    _check_agg(keys[:50_000], vc[:50_000], "max", _ext.hip().hash_aggregate(keys[:50_000], vc[:50_000], "max", True, 0))


@pytest.mark.gpu
def test_low_path_scratch_is_o_groups():
    """LOW-path aggregation: scratch is the LOW table + an output of its capacity, whatever n (no n-sized buffers);
    the PART path's buffers are allocated only when it runs, and are charged to the storage manager meanwhile."""
    from netsdb_amd.execution import kernels as K

    h = _ext.hip()
    sizes = []
    for n in (1 << 20, 1 << 24):
        keys = torch.randint(0, 8, (n,), device=DEV) * 977
        vals = torch.rand(n, device=DEV, dtype=torch.float64)
        r = h.hash_aggregate(keys, vals, "sum", False, 0, False)
        st = r[5].tolist()
        assert st[1] == 0 and st[2] == 1 and st[0] == 8          # LOW path, ok, 8 groups
        sizes.append(st[4])
        ref = torch.zeros(8, dtype=torch.float64, device=DEV).index_add_(0, keys // 977, vals)
        o = torch.argsort(r[0])
        assert torch.allclose(r[1][o, 0], ref, rtol=1e-9)
    # fixed-size tables (the LOW / MID global table holds up to 16 k MID groups: 2.6 MB at F = 1), never n-sized
    assert sizes[0] == sizes[1] and sizes[1] < (4 << 20), sizes
    # PART path: charged while allocated, released after
    calls = []
    n = 1 << 22
    keys = torch.randperm(n, device=DEV)
    r = h.hash_aggregate(keys, None, "sum", False, 0, False, lambda b: calls.append(b))
    st = r[5].tolist()
    assert st[1] == 1 and st[2] == 1 and st[0] == n
    assert len(calls) == 2 and calls[0] > 0 and calls[0] == -calls[1] and st[4] > n * 8
    K.SCRATCH_STATS["charged_bytes"] = 0


_C1, _C2, _M64 = 0xBF58476D1CE4E5B9, 0x94D049BB133111EB, (1 << 64) - 1


def _unxorshift(y, s):
    x, t = y, y
    while t:
        t >>= s
        x ^= t
    return x


def _inv_mix64(h):
    """Inverse of relops.hip mix64 (the splitmix64 finaliser): a key whose hash is h."""
    x = _unxorshift(h, 31)
    x = (x * pow(_C2, -1, 1 << 64)) & _M64
    x = _unxorshift(x, 27)
    x = (x * pow(_C1, -1, 1 << 64)) & _M64
    return _unxorshift(x, 30)


def _mix64(x):
    x ^= x >> 30
    x = (x * _C1) & _M64
    x ^= x >> 27
    x = (x * _C2) & _M64
    return x ^ (x >> 31)


@pytest.mark.gpu
def test_part_overflow_falls_back_exactly():
    """Keys crafted so that every one hashes to the same PART bucket, sub-bucket and LDS start slot: the LDS probe
    windows fill, the overflow table fills, hash_aggregate reports ok = 0, group_reduce returns None, and the
    engine's generic path gives the exact result."""
    from netsdb_amd.execution import kernels as K

    hs = [(0xA5C3F1 << 40) | (m << 16) | 0x1234 for m in range(1, 200_001)]
    ks = [_inv_mix64(h) for h in hs]
    assert all(_mix64(k) == h for k, h in zip(ks[:100], hs[:100]))
    ks = [k - (1 << 64) if k >= (1 << 63) else k for k in ks]
    distinct = torch.tensor(ks, dtype=torch.int64)
    keys = distinct.repeat(5)[torch.randperm(1_000_000)].to(DEV)
    vals = torch.rand(keys.numel(), device=DEV, dtype=torch.float64)
    r = _ext.hip().hash_aggregate(keys, vals, "sum", False, 0, True)
    st = r[5].tolist()
    assert st[1] == 1 and st[2] == 0, st                     # PART path, its overflow table filled
    assert K.group_reduce(keys, vals, "sum") is None         # the fused path refuses ...
    inv, reps, g = K.group_ids(keys.cpu())                    # ... and the generic path is exact
    agg = K.segment_reduce(vals.cpu(), inv, g, "sum")
    u, ui = torch.unique(keys.cpu(), return_inverse=True)
    ref = torch.zeros(u.numel(), dtype=torch.float64).index_add_(0, ui, vals.cpu())
    assert torch.equal(reps, u) and torch.allclose(agg, ref)


@pytest.mark.gpu
def test_chunked_aggregation_matches_unchunked(monkeypatch):
    """Inputs past the per-call row bound are aggregated chunk by chunk and merged (forced with a small bound)."""
    from netsdb_amd.execution import kernels as K

    n = 300_000
    keys = torch.randint(0, 5000, (n,), device=DEV)
    vals = torch.rand(n, 2, device=DEV, dtype=torch.float64)
    full = K.group_reduce(keys, vals, "sum")
    monkeypatch.setattr(K, "AGG_CHUNK_ROWS", 70_000)
    part = K.group_reduce(keys, vals, "sum")
    assert torch.equal(full[0], part[0]) and torch.allclose(full[1], part[1], rtol=1e-9)
    inv, reps, g = K.group_ids(keys)
    u, ui = torch.unique(keys, return_inverse=True)
    assert torch.equal(reps, u) and torch.equal(inv, ui)


@pytest.mark.gpu
def test_large_join_build_with_clusters_matches_host():
    """A build of >= 1 M rows with repeated keys, kEmpty-marker rows and a crafted cluster of 3000 keys sharing one
    home slot (a 3000-slot probe chain that crosses an eighth of the table): every (build, probe) pair equals the
    host join's."""
    g = torch.Generator(device=DEV).manual_seed(7)
    n = 1_200_000
    build = torch.randint(0, 500_000, (n,), device=DEV, generator=g) * 7 + 3
    build[::50_000] = torch.iinfo(torch.int64).min
    cap = 1 << 22                                   # pow2_at_least(2 n): the table the binding sizes
    home = cap // 8 - 5
    crafted = [_inv_mix64((j << 22) | home) for j in range(1, 3001)]
    crafted = torch.tensor([c - (1 << 64) if c >= 1 << 63 else c for c in crafted], dtype=torch.int64, device=DEV)
    assert all((_mix64(int(c) & _M64) & (cap - 1)) == home for c in crafted[:5].tolist())
    build = torch.cat([build, crafted, crafted[:100]])          # the first 100 crafted keys twice
    assert build.numel() >= 1 << 20 and 2 * build.numel() <= cap
    probe = torch.cat([build[torch.randint(0, build.numel(), (200_000,), device=DEV, generator=g)],
                       torch.randint(0, 4_000_000, (50_000,), device=DEV, generator=g), crafted[:500]])
    bi, pi = K.JoinTable(build).probe(probe)
    assert torch.equal(build[bi], probe[pi])
    bi2, pi2 = K.JoinTable(build.cpu()).probe(probe.cpu())
    assert bi.numel() == bi2.numel()
    assert sorted(zip(pi.cpu().tolist(), bi.cpu().tolist())) == sorted(zip(pi2.tolist(), bi2.tolist()))


@pytest.mark.gpu
def test_mix64_kernel_matches_torch_expression():
    """relops.hip mix64_kernel == the torch splitmix64 expression (wrapping int64), with and without the xor input,
    odd lengths and a view at an odd offset (realigned by the binding)."""
    from netsdb_amd import _ext
    from netsdb_amd.execution import kernels as K

    def ref(x, y=None):
        if y is not None:
            x = x ^ y
        x = x + K._GOLD
        x = (x ^ K._lsr(x, 30)) * K._M1
        x = (x ^ K._lsr(x, 27)) * K._M2
        return x ^ K._lsr(x, 31)

    g = torch.Generator().manual_seed(5)
    for n in (1, 2, 3, 1001, 1 << 20):
        x = torch.randint(-(1 << 62), 1 << 62, (n,), generator=g, dtype=torch.int64)
        y = torch.randint(-(1 << 62), 1 << 62, (n,), generator=g, dtype=torch.int64)
        xd, yd = x.cuda(), y.cuda()
        assert torch.equal(_ext.hip().mix64(xd).cpu(), ref(x))
        assert torch.equal(_ext.hip().mix64(xd, yd).cpu(), ref(x, y))
        if n > 2:
            assert torch.equal(_ext.hip().mix64(xd[1:], yd[1:]).cpu(), ref(x[1:], y[1:]))
    big = torch.randint(-(1 << 62), 1 << 62, (1 << 16,), generator=g, dtype=torch.int64)
    assert torch.equal(K.mix64(big.cuda()).cpu(), ref(big))            # the engine entry takes the kernel


@pytest.mark.gpu
def test_group_reduce_many_groups_unsorted_is_exact():
    """Past SORTED_GROUPS_MAX groups group_reduce returns the groups in the table's order (no key sort): the same
    set of (key, aggregate) pairs as torch.unique + index_add."""
    g = torch.Generator(device=DEV).manual_seed(8)
    n = 3_000_000
    keys = torch.randint(0, 1 << 40, (n,), device=DEV, generator=g)
    keys[: n // 3] = keys[n // 3: 2 * (n // 3)]                       # repeats: ~2 M groups of 1-2 rows
    vals = torch.rand(n, device=DEV, dtype=torch.float64, generator=g)
    reps, agg = K.group_reduce(keys, vals, "sum")
    assert reps.numel() > K.SORTED_GROUPS_MAX
    o = torch.argsort(reps)
    u, ui = torch.unique(keys, return_inverse=True)
    ref = torch.zeros(u.numel(), dtype=torch.float64, device=DEV).index_add_(0, ui, vals)
    assert torch.equal(reps[o], u)
    torch.testing.assert_close(agg[o], ref, rtol=1e-12, atol=1e-12)


@pytest.mark.gpu
def test_compact_matches_nonzero():
    """relops.hip stable compaction == torch.nonzero: bool and uint8 (bytes > 1 count as set) masks, dense / sparse /
    empty / full, ragged tails, an unaligned view."""
    g = torch.Generator(device=DEV).manual_seed(9)
    for n in (1, 15, 16, 17, 8191, 8192, 8193, 100_003, 3_000_001):
        for p in (0.0, 0.01, 0.5, 1.0):
            m = torch.rand(n, device=DEV, generator=g) < p
            assert torch.equal(_ext.hip().compact(m), torch.nonzero(m).flatten()), (n, p)
        u = torch.randint(0, 4, (n,), device=DEV, generator=g).to(torch.uint8)
        assert torch.equal(_ext.hip().compact(u), torch.nonzero(u).flatten()), n
        if n > 3:
            assert torch.equal(_ext.hip().compact(u[3:]), torch.nonzero(u[3:]).flatten()), n
    big = torch.rand(1 << 20, device=DEV, generator=g) < 0.3
    assert torch.equal(K.selected_rows(big), torch.nonzero(big).flatten())      # the engine entry


@pytest.mark.gpu
@pytest.mark.parametrize("distinct", [600, 1500, 3000, 5000])
@pytest.mark.parametrize("op", ["sum", "min", "max"])
def test_hash_aggregate_mid_path(distinct, op):
    """The MID path (hash-partitioned LDS tables, one pass over the rows; relops.hip agg_low_kernel MODE 2) for
    group counts between the LOW tables and the PART path: exact groups, aggregates, counts, first rows and inverse,
    double and int64 values, and the same groups as with the MID path switched off (the PART path)."""
    h = _ext.hip()
    g = torch.Generator(device=DEV).manual_seed(distinct)
    n = 400_003
    keys = torch.randint(0, distinct, (n,), device=DEV, generator=g) * 7919 - 123456
    keys[:5] = -(1 << 63)                                           # the kEmpty marker as a real key
    vals = torch.rand(n, 2, device=DEV, dtype=torch.float64, generator=g)
    r = h.hash_aggregate(keys, vals, op, True)
    assert int(r[5][1]) == 0, "LOW / MID path expected"              # status path: 0 = the LDS-table paths
    _check_agg(keys, vals, op, r)
    ivals = torch.randint(-1000, 1000, (n, 1), device=DEV, generator=g)
    ri = h.hash_aggregate(keys, ivals, op, False)
    _check_agg(keys, ivals, op, ri)
    h.agg_set_mid(False)
    try:
        rp = h.hash_aggregate(keys, vals, op, True)
    finally:
        h.agg_set_mid(True)
    assert int(rp[5][1]) == 1                                        # the PART path ran
    o1, o2 = torch.argsort(r[0]), torch.argsort(rp[0])
    assert torch.equal(r[0][o1], rp[0][o2]) and torch.equal(r[2][o1], rp[2][o2])
    torch.testing.assert_close(r[1][o1], rp[1][o2], rtol=1e-12, atol=1e-12)


@pytest.mark.gpu
def test_join_probe_filter_gpu():
    """Probe filters (relops.hip join_bloom_kernel, a blocked Bloom filter per large table): probing with the filter
    finds exactly the pairs probing without it finds, for unique and repeated build keys, the empty-marker key and
    mostly-absent probe keys; the fused TPC-H join stages give the same answers with a filter on every table."""
    h = _ext.hip()
    g = torch.Generator(device=DEV).manual_seed(9)
    build = torch.randperm(2_000_000, device=DEV, generator=g)[:600_000] * 5 + 3
    build = torch.cat([build, build[:1000], torch.tensor([torch.iinfo(torch.int64).min], device=DEV)])
    probe = torch.randint(0, 10_000_000, (3_000_000,), device=DEV, generator=g)
    probe[:5000] = build[:5000]
    probe[5000] = torch.iinfo(torch.int64).min
    try:
        h.join_set_bloom(True, 0)
        t_on = K.JoinTable(build)
        assert t_on._dev[2].numel() > 0
        h.join_set_bloom(False)
        t_off = K.JoinTable(build)
        assert t_off._dev[2].numel() == 0
    finally:
        h.join_set_bloom(True)
    b1, p1 = t_on.probe(probe)
    b0, p0 = t_off.probe(probe)
    assert torch.equal(p1, p0) and torch.equal(b1, b0)
    assert torch.equal(build[b1], probe[p1]) and p1.numel() >= 5001


@pytest.mark.gpu
def test_tpch_join_queries_with_probe_filters_gpu(tmp_path):
    from netsdb_amd.client import PDBClient
    from netsdb_amd.models import tpch

    h = _ext.hip()
    t = tpch.generate(0.01, seed=3)
    c = PDBClient(root=str(tmp_path), device=DEV)
    tpch.load(c, "tpch", t)
    try:
        h.join_set_bloom(True, 0)                 # a filter on every join table, however small
        for q in ("q03", "q12", "q14", "q17", "q04"):
            got = tpch.QUERIES[q](c, "tpch")
            ref = tpch.reference(q, t)
            if isinstance(ref, float):
                assert got == pytest.approx(ref, rel=1e-9), q
                continue
            assert len(got) == len(ref), q
            key = lambda r: tuple(str(v) for v in r.values())  # noqa: E731
            for a, b in zip(sorted(got, key=key), sorted(ref, key=key)):
                for k, v in b.items():
                    assert (a[k] == pytest.approx(v, rel=1e-9, abs=1e-6)) if isinstance(v, float) else a[k] == v, (q, k)
    finally:
        h.join_set_bloom(True)


@pytest.mark.gpu
def test_take_many_matches_index_select():
    """relops take_many (one launch for many columns) equals index_select per column: every row width (1/2/4/8 B,
    16-B multiples, odd multiples of the element), views at unaligned offsets, 2-D rows, and the bad-id word."""
    from netsdb_amd.objects.record import take_many, take_many_check

    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(5)
    n = 10_000
    cols = [torch.randint(0, 255, (n,), device=dev, dtype=torch.uint8),
            torch.randn(n, device=dev).to(torch.bfloat16),
            torch.randn(n, device=dev),
            torch.randint(-2**62, 2**62, (n,), device=dev, generator=g),
            torch.randn(n, 4, device=dev),                       # 16-B rows
            torch.randn(n, 3, device=dev, dtype=torch.float64),  # 24-B rows: 8-B elements
            torch.randn(n, 3, device=dev),                       # 12-B rows
            torch.randn(n + 1, device=dev, dtype=torch.float64)[1:],   # an 8-B-aligned view
            torch.randn(n * 4 + 1, device=dev)[1:].view(n, 4)]         # 16-B rows at a 4-B offset
    idx = torch.randint(0, n, (3000,), device=dev, generator=g)
    got = take_many(cols, idx)
    for c, o in zip(cols, got):
        assert o.shape == (3000,) + tuple(c.shape[1:]) and torch.equal(o, c.index_select(0, idx))
    assert take_many_check()
    bad = idx.clone()
    bad[7] = n + 5
    take_many(cols[:2], bad)
    assert not take_many_check() and take_many_check()
    take_many(cols[:2], bad)
    from netsdb_amd.objects.strings import to_host

    with pytest.raises(IndexError):                      # surfaces at the next batched host read
        to_host(idx)
    assert take_many_check()
    assert [o.numel() for o in take_many(cols[:3], idx[:0])] == [0, 0, 0]


@pytest.mark.gpu
def test_lazy_selection_group_gather(monkeypatch):
    """A small lazy selection's first read gathers all of its pending columns (strings too) in one take_many launch;
    the values are those of per-column takes, a large one still gathers column by column."""
    from netsdb_amd.objects import record as R

    dev = "cuda"
    n = 5000
    s = StringColumn.from_list([f"s{i % 97}" * (1 + i % 3) for i in range(n)], dev)
    src = {"a": torch.arange(n, device=dev), "b": torch.randn(n, device=dev), "s": s,
           "t": torch.randn(n, 2, device=dev)}
    idx = torch.randint(0, n, (777,), device=dev)
    calls = []
    real = R.take_many
    monkeypatch.setattr(R, "take_many", lambda c, i: calls.append(len(c)) or real(c, i))
    lz = R.LazyTakeColumns(src, idx)
    assert torch.equal(lz["b"], src["b"][idx])
    assert calls == [5]                                   # a, b, t, s.starts, s.ends
    assert torch.equal(lz["a"], idx) and torch.equal(lz["t"], src["t"][idx])
    assert lz["s"].tolist() == s.take(idx).tolist() and calls == [5]
    monkeypatch.setattr(R, "GROUP_TAKE_MAX_ROWS", 100)
    lz2 = R.LazyTakeColumns(src, idx)
    assert torch.equal(lz2["b"], src["b"][idx]) and calls == [5]


def _unmix64(y: int) -> int:
    """Inverse of relops.hip mix64 (splitmix64's finaliser): keys whose table home slots the test chooses."""
    m = (1 << 64) - 1
    y ^= (y >> 31) ^ (y >> 62)
    y = (y * pow(0x94D049BB133111EB, -1, 1 << 64)) & m
    y ^= (y >> 27) ^ (y >> 54)
    y = (y * pow(0xBF58476D1CE4E5B9, -1, 1 << 64)) & m
    y ^= (y >> 30) ^ (y >> 60)
    return y


def test_unmix64_inverts_mix64():
    from netsdb_amd.objects.strings import _mix_py

    for x in (0, 1, 12345, (1 << 64) - 1, 0x8000000000000001):
        assert _unmix64(_mix_py(x)) == x


@pytest.mark.gpu
@pytest.mark.parametrize("n,distinct", [(50_000, 50_000), (600_000, 150_000), (3_000_000, 3_000_000),
                                        (6_000_000, 2_000_000)])   # the last: a two-level partition (4096 regions)
def test_join_partitioned_build_matches_global_insert(n, distinct):
    """The LDS region build (tables of more than one 4096-slot region) and the global-atomic insert give the same
    pairs, with repeated keys (CSR runs), kEmpty-marker rows and the probe filter; the table's slot contents agree
    as a set (claims may differ in which row of a repeated key is rank 0)."""
    g = torch.Generator(device=DEV).manual_seed(11)
    build = torch.randint(0, distinct, (n,), device=DEV, generator=g) * 7 + 3
    build[::1001] = torch.iinfo(torch.int64).min
    probe = torch.randint(0, distinct + distinct // 3, (200_000,), device=DEV, generator=g) * 7 + 3
    probe[::37] = torch.iinfo(torch.int64).min
    h = _ext.hip()
    outs = []
    for part in (True, False):
        h.join_set_part(part)
        h.join_set_bloom(True, 4 << 20, 1 << 40)              # filters on every table past 4 MiB, however large
        try:
            tab, perm, bloom, stat = h.join_build(build)
            if tab.shape[0] - 1 > (1 << 22):              # region tables carry the build's host read
                m = int(torch.unique(build, return_counts=True)[1].max())   # the kEmpty slot counts +1: a bound
                assert stat.numel() == 2 and int(stat[0]) == 0 and m <= int(stat[1]) + 1 <= m + 1
            else:
                assert stat.numel() == 0                   # whole-table tables: no host read in the build
            bi, pi = h.join_probe(tab, perm, probe, bloom)
        finally:
            h.join_set_part(True)
            h.join_set_bloom(True)
        assert torch.equal(build[bi], probe[pi]) and bool((pi[1:] >= pi[:-1]).all())
        keys = tab[:, 0].sort().values
        outs.append((sorted(zip(pi.tolist(), bi.tolist())), keys, bloom))
    assert outs[0][0] == outs[1][0]
    assert torch.equal(outs[0][1], outs[1][1])
    assert torch.equal(outs[0][2], outs[1][2])          # probe filters built in the region pass = the filter kernel's


@pytest.mark.gpu
def test_join_region_overflow_rebuilds_larger():
    """A region table (past 2^22 slots): 6,000 distinct keys whose home slots all fall in ONE 4096-slot region of the
    first 2^23-slot table, next to 1.1 M random keys. The build sees a region without an empty slot, doubles the table
    (the crafted keys then split over two regions) and every key is found."""
    rng = torch.Generator().manual_seed(3)
    hi = torch.randint(0, 1 << 38, (6000,), generator=rng).tolist()
    lo = torch.randint(0, 1 << 12, (6000,), generator=rng).tolist()
    vals = {(int(a) << 24) | (int(a) & 1) << 23 | (int(b) & 0xFFF) for a, b in zip(hi, lo)}   # bits 12..22 zero
    crafted = [(_unmix64(v) ^ (1 << 63)) - (1 << 63) for v in vals]    # as signed int64
    crafted = torch.tensor([k for k in crafted if k != -(1 << 63)], dtype=torch.int64)
    rnd = torch.randint(-(1 << 62), 1 << 62, (1_100_000,), generator=rng)
    build = torch.unique(torch.cat([crafted, rnd]))
    build = build[torch.randperm(build.numel(), generator=rng)].to(DEV)
    tab, perm, bloom, stat = _ext.hip().join_build(build)
    assert tab.shape[0] - 1 == 1 << 24 and int(stat[0]) == 0             # rebuilt once, larger
    bi, pi = _ext.hip().join_probe(tab, perm, build, bloom)
    assert torch.equal(pi, torch.arange(build.numel(), device=DEV)) and torch.equal(bi, pi)


def test_join_region_constants_agree():
    """relops.hip and pipeline_core.h (the fused probes) must walk the same probe order."""
    import re
    from pathlib import Path

    kd = Path(__file__).resolve().parents[1] / "netsdb_amd" / "csrc" / "kernels"
    r = (kd / "relops.hip").read_text()
    c = (kd / "pipeline_core.h").read_text()
    assert re.search(r"constexpr int kJRegionBits = 12;", r) and "constexpr u64 kJWholeWrap = 1ull << 22;" in r
    assert "constexpr unsigned long long JREGION = 4096, JWHOLE = 1ull << 22;" in c
