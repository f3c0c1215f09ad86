"""Packing deduplicated tensor blocks into storage pages.

Reference: model-inference/deduplication/page-packing (algorithms/PagePacking.py: Baseline
``bin_pack_base``, Greedy-2 ``bin_pack_greedy``, Greedy-1 ``*_greedy1`` and Two-Stage ``*_twostage``;
driven by runBaseline/runGreedy-1/runGreedy-2/runTwo-Stage.py on word2vec and text-classification
block sets).  Goal: place the distinct blocks of several models (tensors = sets of distinct block
ids) into pages of ``l`` blocks so that (1) few pages are used in total and (2) each model needs to
read few pages — a model whose blocks are spread over many half-foreign pages pays extra I/O
(netsDB's shared-page sets load whole pages).

Re-implemented on sets and dicts (the reference's 0/1 page matrix with ``list.index`` lookups is
quadratic); the equivalence-class algorithms are generalised from the reference's fixed six-tensor
word2vec case to any number of tensors: an equivalence class is the set of blocks owned by exactly the
same set of tensors.

All functions return a :class:`Packing`.
"""
from __future__ import annotations

import math
from collections import Counter
from dataclasses import dataclass, field
from typing import Dict, Hashable, List, Sequence, Set

Block = Hashable


@dataclass
class Packing:
    pages: List[List[Block]] = field(default_factory=list)

    @property
    def num_pages(self) -> int:
        return len(self.pages)

    def page_of(self) -> Dict[Block, int]:
        return {b: i for i, p in enumerate(self.pages) for b in p}

    def tensor_pages(self, tensors: Sequence[Set[Block]]) -> List[Set[int]]:
        """Pages each tensor must read (its I/O cost in pages)."""
        po = self.page_of()
        return [{po[b] for b in t} for t in tensors]

    def validate(self, tensors: Sequence[Set[Block]], l: int):
        seen: Set[Block] = set()
        for p in self.pages:
            if not 0 < len(p) <= l:
                raise AssertionError(f"page with {len(p)} blocks (limit {l})")
            for b in p:
                if b in seen:
                    raise AssertionError(f"block {b!r} packed twice")
                seen.add(b)
        need = set().union(*tensors) if tensors else set()
        if seen != need:
            raise AssertionError(f"{len(need - seen)} blocks unpacked, {len(seen - need)} foreign")
        return True


def lower_bound(tensors: Sequence[Set[Block]], l: int) -> int:
    return math.ceil(len(set().union(*tensors)) / l) if tensors else 0


def _freq(tensors: Sequence[Set[Block]]) -> Counter:
    c: Counter = Counter()
    for t in tensors:
        c.update(t)
    return c


def _append_pages(pk: Packing, items: Sequence[Block], l: int, fill_tail: bool = False):
    items = list(items)
    if fill_tail and pk.pages and len(pk.pages[-1]) < l and items:
        room = l - len(pk.pages[-1])
        pk.pages[-1].extend(items[:room])
        items = items[room:]
    for s in range(0, len(items), l):
        pk.pages.append(list(items[s: s + l]))


def _full_pages_of(pk: Packing, t: Set[Block], page_sets: List[frozenset]) -> Set[Block]:
    """Blocks of ``t`` already sitting in pages that ``t`` uses completely (the reference's
    findMinBinsMaxCover keeps only fully covered pages; partially covered ones are not reused)."""
    covered: Set[Block] = set()
    for ps in page_sets:
        if ps <= t:
            covered |= ps
    return covered


def _incremental(tensors: Sequence[Set[Block]], l: int, order_first_by_freq: bool, fill_tail: bool = False) -> Packing:
    freq = _freq(tensors)
    pk = Packing()
    first = tensors[0]
    items = sorted(first, key=lambda b: (-freq[b], repr(b))) if order_first_by_freq else sorted(first, key=repr)
    _append_pages(pk, items, l)
    placed = set(items)
    for t in tensors[1:]:
        page_sets = [frozenset(p) for p in pk.pages]
        covered = _full_pages_of(pk, t, page_sets)
        rest = [b for b in t if b not in covered and b not in placed]
        # blocks of t already placed in partially shared pages stay where they are
        rest.sort(key=lambda b: (-freq[b], repr(b)))
        _append_pages(pk, rest, l, fill_tail)
        placed.update(rest)
    return pk


def baseline(tensors: Sequence[Set[Block]], l: int) -> Packing:
    """Baseline (bin_pack_base): tensors in the given order; each new tensor reuses the pages it fully
    covers and packs its remaining blocks (by frequency) into new pages."""
    return _incremental(list(tensors), l, order_first_by_freq=False)


def greedy2(tensors: Sequence[Set[Block]], l: int, fill_tail: bool = False) -> Packing:
    """Greedy-2 (bin_pack_greedy): as Baseline, but tensors largest-first and every tensor's new blocks
    ordered by how many tensors share them (shared blocks cluster into the same pages).  ``fill_tail``
    tops up the last partial page before opening new ones (fewer pages, a few foreign-block reads)."""
    ts = sorted(tensors, key=len, reverse=True)
    return _incremental(ts, l, order_first_by_freq=True, fill_tail=fill_tail)


def equivalence_classes(tensors: Sequence[Set[Block]]) -> Dict[frozenset, List[Block]]:
    owners: Dict[Block, Set[int]] = {}
    for i, t in enumerate(tensors):
        for b in t:
            owners.setdefault(b, set()).add(i)
    classes: Dict[frozenset, List[Block]] = {}
    for b, o in owners.items():
        classes.setdefault(frozenset(o), []).append(b)
    for v in classes.values():
        v.sort(key=repr)
    return classes


def _class_order(classes: Dict[frozenset, List[Block]]):
    return sorted(classes, key=lambda k: (-len(k), sorted(k)))


def greedy1(tensors: Sequence[Set[Block]], l: int) -> Packing:
    """Greedy-1: every equivalence class gets its own pages — a tensor never reads a block it does not
    own, at the price of partially filled pages (one per class)."""
    classes = equivalence_classes(tensors)
    pk = Packing()
    for k in _class_order(classes):
        _append_pages(pk, classes[k], l)
    return pk


def two_stage(tensors: Sequence[Set[Block]], l: int) -> Packing:
    """Two-Stage: stage 1 packs only FULL pages of each equivalence class; stage 2 packs the leftovers
    of all classes together with Greedy-2, topping up partial pages (at most one page per class of
    leftovers, so the foreign reads stay bounded while the page count approaches the lower bound)."""
    classes = equivalence_classes(tensors)
    pk = Packing()
    left: Set[Block] = set()
    for k in _class_order(classes):
        items = classes[k]
        full = len(items) // l * l
        _append_pages(pk, items[:full], l)
        left.update(items[full:])
    if left:
        sub = [t & left for t in tensors]
        sub = [t for t in sub if t]
        pk.pages.extend(greedy2(sub, l, fill_tail=True).pages)
    return pk


ALGORITHMS = {"baseline": baseline, "greedy1": greedy1, "greedy2": greedy2, "two_stage": two_stage}


def pack(tensors: Sequence[Set[Block]], l: int, algorithm: str = "two_stage") -> Packing:
    pk = ALGORITHMS[algorithm]([set(t) for t in tensors], l)
    return pk


def report(tensors: Sequence[Set[Block]], l: int) -> Dict[str, dict]:
    """num_pages and total per-tensor page reads of every algorithm, plus the lower bound."""
    out = {"lower_bound": {"num_pages": lower_bound(tensors, l),
                           "page_reads": sum(math.ceil(len(t) / l) for t in tensors)}}
    for name, fn in ALGORITHMS.items():
        pk = fn([set(t) for t in tensors], l)
        pk.validate(tensors, l)
        out[name] = {"num_pages": pk.num_pages, "page_reads": sum(len(s) for s in pk.tensor_pages(tensors))}
    return out


def synthetic_shared_models(n_tensors: int = 6, blocks_per_tensor: int = 500, unshared_per_tensor: int = 50,
                            seed: int = 0) -> List[Set[int]]:
    """Replica of detector_output_same_size_unshared_located_random: every tensor has the same
    ``blocks_per_tensor - unshared`` shared blocks plus ``unshared`` private ones at random positions."""
    import random

    rnd = random.Random(seed)
    shared = list(range(blocks_per_tensor - unshared_per_tensor))
    nxt = len(shared)
    out = []
    for _ in range(n_tensors):
        own = list(range(nxt, nxt + unshared_per_tensor))
        nxt += unshared_per_tensor
        t = shared + own
        rnd.shuffle(t)
        out.append(set(t))
    return out


__all__ = ["Packing", "baseline", "greedy1", "greedy2", "two_stage", "pack", "report", "lower_bound",
           "equivalence_classes", "synthetic_shared_models", "ALGORITHMS"]
