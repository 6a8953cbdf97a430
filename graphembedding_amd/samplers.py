"""Pair samplers (model/Siamese/samplers.py:5-68) as explicit state machines.

Both reference samplers draw only from fresh `random.Random(seed)` generators with
fixed seeds, so their streams are functions of small tables computed once:

* RandomSampler: state (idx, list order).  A call emits (list[idx], list[idx + 1]);
  reaching the end of the list re-orders it IN PLACE by sigma, the permutation that
  `random.Random(123).shuffle` applies to a list of that length (samplers.py:28), and
  restarts at 0.  The list is ModelGraphList.gs, so after training
  `get_orig_train_graph(j)` returns a permuted graph (quirk A6).
* DistributionSampler: state (cur, item).  Graphs are ranked by (density, index) and
  cut into bins of `bin_size`; the bin walk is a `Random(123)`-shuffled bin list, and the
  item taken inside a bin at cursor c is `Random(123 + c).randint(0, bin_size - 1)`
  (samplers.py:44-68).  The stream is periodic in cur.

csrc/sg_sampler.hip runs the same two machines on the device from the same tables
(device_sampler.py); tests/test_golden.py pins both streams against the reference's
own samplers (fixture F2) and the list order after whole training loops (F7).
"""
from __future__ import annotations

import random
from typing import Dict, List

import networkx as nx

_SIGMA: Dict[tuple, List[int]] = {}


def shuffle_permutation(n: int, seed: int = 123) -> List[int]:
    """sigma with random.Random(seed).shuffle(x) == [x[sigma[i]] for i in range(n)]:
    shuffle's swaps depend only on n and the generator, not on the contents."""
    key = (int(n), int(seed))
    if key not in _SIGMA:
        sigma = list(range(n))
        random.Random(seed).shuffle(sigma)
        _SIGMA[key] = sigma
    return _SIGMA[key]


def bin_item(cur: int, bin_size: int) -> int:
    """The in-bin item index DistributionSampler uses at cursor `cur`."""
    return random.Random(123 + cur).randint(0, bin_size - 1)


class Sampler(object):
    """The graph list (shared with its ModelGraphList, re-ordered in place) and the
    reference's sampler options."""

    def __init__(self, gs, sample_num, sampler_duplicate_removal):
        if len(gs) < 2:
            raise AssertionError('a sampler needs at least 2 graphs, got {}'.format(len(gs)))
        self.gs = gs
        self.sample_num = sample_num
        self.sampler_duplicate_removal = sampler_duplicate_removal

    def get_pair(self):
        raise NotImplementedError()

    def get_triple_for_hinge_loss(self):
        raise NotImplementedError()


class RandomSampler(Sampler):
    def __init__(self, gs, sample_num, sampler_duplicate_removal):
        super().__init__(gs, sample_num, sampler_duplicate_removal)
        self.idx = 0

    def _wrap(self):
        sigma = shuffle_permutation(len(self.gs))
        self.gs[:] = [self.gs[k] for k in sigma]
        self.idx = 0

    def get_pair(self):
        first = self.gs[self.idx]
        self.idx += 1
        if self.idx >= len(self.gs):
            self._wrap()
        return first, self.gs[self.idx]


class DistributionSampler(Sampler):
    def __init__(self, gs, sample_num, sampler_duplicate_removal, bin_size=5):
        super().__init__(gs, sample_num, sampler_duplicate_removal)
        # rank by (density, index): the order the bins are cut from
        self.dens_list = sorted((nx.density(g.nxgraph), k) for k, g in enumerate(self.gs))
        self.bin_size = bin_size
        self.bin_number = len(self.gs) // self.bin_size
        self.bin_idx = self.shuffle_idx()
        self.cur = 0
        self.item_idx = bin_item(0, self.bin_size)

    def shuffle_idx(self):
        walk = list(shuffle_permutation(self.bin_number))   # Random(123).shuffle(range)
        if self.sample_num > 0:
            walk = walk[:2 * self.sample_num]
        return walk

    def _graph(self, slot):
        rank = self.bin_idx[slot] * self.bin_size + self.item_idx
        return self.gs[self.dens_list[rank][1]]

    def get_pair(self):
        pair = (self._graph(self.cur), self._graph(self.cur + 1))
        nxt = self.cur + 2
        self.cur = nxt if nxt < len(self.bin_idx) - 1 else 0
        self.item_idx = bin_item(self.cur, self.bin_size)
        return pair
