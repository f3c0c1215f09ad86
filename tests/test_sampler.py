"""Sampler utilities vs the reference formulas (src/utilities/headers/Sampler.h)."""
import math

import torch

from netsdb_amd.utils.sampler import fraction_for_sample_size, num_std, randomize_in_place


def test_fraction_formulas():
    assert num_std(3) == 12.0 and num_std(10) == 9.0 and num_std(100) == 6.0
    # with replacement: (k + numStd(k) sqrt(k)) / total
    assert math.isclose(fraction_for_sample_size(100, 10**6, True), (100 + 6.0 * 10) / 10**6)
    f = fraction_for_sample_size(4, 1000, False)
    g = -math.log(1e-4) / 1000
    assert math.isclose(f, 0.004 + g + math.sqrt(g * g + 2 * g * 0.004))
    assert fraction_for_sample_size(10, 5, False) == 1.0


def test_bernoulli_sample_reaches_lower_bound():
    # the bound holds with probability >= 1 - 1e-4: every seed here must draw >= k records
    total, k = 20000, 8
    f = fraction_for_sample_size(k, total)
    for seed in range(50):
        g = torch.Generator().manual_seed(seed)
        assert int((torch.rand(total, generator=g) < f).sum()) >= k


def test_randomize_in_place_is_permutation():
    x = torch.arange(100).reshape(50, 2)
    y = randomize_in_place(x.clone(), torch.Generator().manual_seed(1))
    assert not torch.equal(x, y)
    assert torch.equal(y[y[:, 0].argsort()], x)
