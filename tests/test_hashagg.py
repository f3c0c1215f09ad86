"""Device hash-table group-by (csrc/kernels/relops.hip hash_aggregate, ops path execution/kernels.py group_ids) vs
torch.unique(sorted=True, return_inverse=True) — the reference groups through C++ hash maps
(src/queryExecution aggregation processors); the result must be the exact sorted distinct keys and inverse."""
import pytest
import torch

from netsdb_amd import _ext
from netsdb_amd.execution import kernels as K

I64_MIN = -(1 << 63)


def _check(keys):
    inv, uniq = _ext.hip().hash_group_ids(keys)
    ru, ri = torch.unique(keys, sorted=True, return_inverse=True)
    assert torch.equal(uniq, ru)
    assert torch.equal(inv, ri)


@pytest.mark.gpu
def test_hash_group_ids_matches_unique_gpu():
    dev = "cuda:0"
    g = torch.Generator(device=dev).manual_seed(0)
    # wide keys (mostly distinct), low cardinality (heavy contention on a few slots), mid cardinality with
    # negatives and the empty-slot sentinel value itself, tiny and single-row columns
    _check(torch.randint(-(1 << 62), 1 << 62, (1 << 20,), device=dev, generator=g))
    _check(torch.randint(0, 7, (1 << 22,), device=dev, generator=g))
    k = torch.randint(-5000, 5000, (300_001,), device=dev, generator=g)
    k[::97] = I64_MIN
    _check(k)
    _check(torch.tensor([I64_MIN], device=dev))
    _check(torch.tensor([42, 42, 42], device=dev))
    inv, uniq = _ext.hip().hash_group_ids(torch.empty(0, dtype=torch.int64, device=dev))
    assert inv.numel() == 0 and uniq.numel() == 0


@pytest.mark.gpu
def test_group_ids_uses_hash_table_gpu():
    dev = "cuda:0"
    from netsdb_amd import ops
    keys32 = torch.randint(-100, 100, (100_000,), device=dev, dtype=torch.int32)
    with ops.kernel_options(hash_groupby=True):
        inv, reps, n = K.group_ids(keys32)
    ru, ri = torch.unique(keys32, return_inverse=True)
    assert n == ru.numel() and reps.dtype == torch.int32 and torch.equal(reps, ru) and torch.equal(inv, ri)
    # string keys group by their device hash through the same table
    from netsdb_amd.objects.strings import StringColumn
    words = ["ab", "c", "ab", "", "xyz", "c", "ab"] * 1000
    col = StringColumn.from_list(words, dev)
    with ops.kernel_options(hash_groupby=True):
        inv, reps, n = K.group_ids(col)
    assert n == 4 and sorted(reps.tolist()) == sorted(set(words))
    back = [reps.tolist()[i] for i in inv.tolist()]
    assert back == words
    with ops.kernel_options(hash_groupby=False):          # torch.unique path, same result
        inv2, reps2, n2 = K.group_ids(keys32)
    assert n2 == ru.numel() and torch.equal(reps2, ru) and torch.equal(inv2, ri)


def test_hash_group_ids_rejects_bad_input_cpu():
    if not _ext.hip_available():
        pytest.skip("HIP extension not built")
    with pytest.raises(RuntimeError):
        _ext.hip().hash_group_ids(torch.zeros(4, dtype=torch.int64))   # host tensor


@pytest.mark.gpu
def test_run_aggregate_clustered_keys_gpu():
    """Clustered-key group-by (relops.hip run_*_kernel) against the hash path and a torch fp64 reference: ordered keys
    in runs (the lineitem-by-orderkey shape, with negative keys and a run crossing every tile boundary), sums / min /
    max over f64 and int64 values in both layouts, count only; unordered keys must be refused (empty result)."""
    h = _ext.hip()
    dev = "cuda:0"
    g = torch.Generator().manual_seed(7)
    n = 300_000
    run = torch.randint(1, 9, (n,), generator=g)
    keys = (torch.repeat_interleave(torch.arange(n), run)[:n] * 3 - 1000).to(dev)
    keys[8192 * 3 - 2: 8192 * 3 + 5] = keys[8192 * 3 - 2]        # one run across a tile boundary
    keys = torch.cummax(keys, 0).values
    vals_f = torch.randn(n, 3, generator=g, dtype=torch.float64).to(dev)
    vals_i = torch.randint(-50, 50, (n, 2), generator=g).to(dev)
    uk, inv, cnt = torch.unique_consecutive(keys, return_inverse=True, return_counts=True)
    first = torch.cat([torch.zeros(1, dtype=torch.int64, device=dev), torch.cumsum(cnt, 0)[:-1]])
    for vals in (vals_f, vals_f.t().contiguous().t(), vals_i):
        for op in ("sum", "min", "max"):
            r = h.run_aggregate(keys, vals, op)
            assert r, "ordered keys must take the run path"
            rk, ra, rc, rf = r
            assert torch.equal(rk, uk) and torch.equal(rc, cnt) and torch.equal(rf, first)
            ref = torch.zeros(uk.numel(), vals.shape[1], dtype=vals.dtype, device=dev)
            if op == "sum":
                ref.index_add_(0, inv, vals)
            else:
                ref = ref.index_reduce_(0, inv, vals, "amin" if op == "min" else "amax", include_self=False)
            tol = 1e-9 if vals.dtype == torch.float64 else 0
            assert torch.allclose(ra, ref, rtol=tol, atol=tol), op
    r = h.run_aggregate(keys, None, "sum")
    assert r and torch.equal(r[2], cnt) and r[1].shape == (uk.numel(), 0)
    shuffled = keys[torch.randperm(n, generator=g).to(dev)]
    assert not h.run_aggregate(shuffled, vals_f, "sum")
    # group_reduce takes the run path for ordered packed keys and agrees with the hash path on unordered ones
    K.LAST_RUN_AGG.update(tried=0, used=0)
    rk, ra = K.group_reduce(keys, vals_f[:, 0], "sum")
    assert K.LAST_RUN_AGG["used"] == 1
    pk, pa = K.group_reduce(shuffled, vals_f[:, 0][torch.randperm(n, generator=g).to(dev)], "count")
    assert K.LAST_RUN_AGG["used"] == 1 and int(pa.sum()) == n
    o1, o2 = torch.argsort(rk), torch.argsort(pk)
    assert torch.equal(rk[o1], pk[o2]) and torch.equal(pa[o2].long(), cnt)
    assert torch.allclose(ra[o1], ref_sum(vals_f[:, 0], inv, uk.numel()), rtol=1e-12, atol=1e-9)


def ref_sum(v, inv, g):
    return torch.zeros(g, dtype=v.dtype, device=v.device).index_add_(0, inv, v)
