"""Data dispatcher: how client-sent records are partitioned over the worker ranks.

Reference: src/dispatcher (PartitionPolicy, RoundRobinPolicy, RandomPolicy, FairPolicy,
LambdaPolicy, IRPolicy, PartitionPolicyFactory, DispatcherServer) and the self-learning
partitioner (src/selfLearning SimplePartitioner / DispatchComp).
"""
from __future__ import annotations

import random
from typing import List, Optional

import torch

from ..objects.record import RecordBatch
from ..execution import kernels as K


class PartitionPolicy:
    name = "base"

    def assign(self, batch: RecordBatch, nparts: int, loads: Optional[List[int]] = None) -> torch.Tensor:
        raise NotImplementedError


class RoundRobinPolicy(PartitionPolicy):
    """Pages/records dealt round-robin (netsDB default)."""

    name = "roundrobin"

    def __init__(self):
        self.next = 0

    def assign(self, batch, nparts, loads=None):
        d = (torch.arange(batch.n) + self.next) % nparts
        self.next = (self.next + batch.n) % nparts
        return d


class RandomPolicy(PartitionPolicy):
    name = "random"

    def __init__(self, seed: int = 0):
        self.rng = random.Random(seed)

    def assign(self, batch, nparts, loads=None):
        g = torch.Generator().manual_seed(self.rng.randrange(1 << 30))
        return torch.randint(0, nparts, (batch.n,), generator=g)


class FairPolicy(PartitionPolicy):
    """Send to the least-loaded ranks (by bytes), balancing the running totals."""

    name = "fair"

    def assign(self, batch, nparts, loads=None):
        loads = list(loads or [0] * nparts)
        per = max(1, batch.nbytes() // max(1, batch.n))
        out = []
        for _ in range(batch.n):
            r = min(range(nparts), key=lambda i: loads[i])
            loads[r] += per
            out.append(r)
        return torch.tensor(out, dtype=torch.int64)


class LambdaPolicy(PartitionPolicy):
    """Hash-partition by a key function of the record batch (``key_fn(batch) -> column``); the
    policy netsDB's self-learning optimizer (Lachesis) installs for co-partitioned joins."""

    name = "lambda"

    def __init__(self, key_fn, description: str = ""):
        self.key_fn = key_fn
        self.description = description

    def assign(self, batch, nparts, loads=None):
        return K.partition_of(K.hash_keys(self.key_fn(batch)), nparts).cpu()


class RangePolicy(PartitionPolicy):
    """Contiguous ranges of an integer key (block-row partitioning of matrix sets)."""

    name = "range"

    def __init__(self, key_fn, num_keys: int):
        self.key_fn = key_fn
        self.num_keys = num_keys

    def assign(self, batch, nparts, loads=None):
        k = self.key_fn(batch).long().cpu()
        per = (self.num_keys + nparts - 1) // nparts
        return torch.clamp(k // max(1, per), max=nparts - 1)


class IRPolicy(PartitionPolicy):
    """Inverse-ratio: probability inversely proportional to current load."""

    name = "ir"

    def __init__(self, seed: int = 0):
        self.gen = torch.Generator().manual_seed(seed)

    def assign(self, batch, nparts, loads=None):
        loads = torch.tensor(loads or [0] * nparts, dtype=torch.float64)
        w = 1.0 / (loads + 1.0)
        return torch.multinomial(w / w.sum(), batch.n, replacement=True, generator=self.gen)


_POLICIES = {"roundrobin": RoundRobinPolicy, "random": RandomPolicy, "fair": FairPolicy, "ir": IRPolicy}


def make_policy(spec) -> PartitionPolicy:
    """PartitionPolicyFactory."""
    if isinstance(spec, PartitionPolicy):
        return spec
    if spec is None:
        return RoundRobinPolicy()
    if callable(spec):
        return LambdaPolicy(spec)
    return _POLICIES[spec]()


__all__ = ["PartitionPolicy", "RoundRobinPolicy", "RandomPolicy", "FairPolicy", "LambdaPolicy", "RangePolicy",
           "IRPolicy", "make_policy"]
