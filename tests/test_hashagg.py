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
