"""Sampling utilities (reference: src/utilities/headers/Sampler.h — used by the k-means driver to size
the Bernoulli sample that seeds the centroids).

``fraction_for_sample_size`` keeps the reference's bound: with replacement, mean + numStd·sqrt(mean)
Poisson slack; without replacement, the Bernoulli bound with failure probability 1e-4, so a sample of
at least ``lower_bound`` records is drawn with high probability.  ``randomize_in_place`` is the
reference's Fisher-Yates shuffle, done as one device permutation gather instead of a host loop.
"""
from __future__ import annotations

import math
from typing import Optional

import torch


def num_std(lower_bound: int) -> float:
    """Sampler::numStd — tighter slack for larger samples."""
    if lower_bound < 6:
        return 12.0
    if lower_bound < 16:
        return 9.0
    return 6.0


def fraction_for_sample_size(lower_bound: int, total: int, with_replacement: bool = False) -> float:
    """Sampler::computeFractionForSampleSize."""
    total = max(1, int(total))
    if with_replacement:
        return max(lower_bound + num_std(lower_bound) * math.sqrt(lower_bound), 1e-15) / total
    fraction = lower_bound / total
    gamma = -math.log(1e-4) / total
    return min(1.0, max(1e-10, fraction + gamma + math.sqrt(gamma * gamma + 2 * gamma * fraction)))


def randomize_in_place(x: torch.Tensor, generator: Optional[torch.Generator] = None) -> torch.Tensor:
    """Sampler::randomizeInPlace — uniform shuffle of the rows of ``x`` (in place; returns ``x``)."""
    n = x.shape[0]
    if n <= 1:
        return x
    perm = torch.randperm(n, generator=generator).to(x.device)
    x.copy_(x.index_select(0, perm))
    return x
