"""Datasets (src/data.py:9-132) plus the synthetic AIDS-shaped stand-ins of
BASELINE.md §3 (the real AIDS gexf archives are not available offline).

`Data(name_str)` keeps the reference's pickle-cache contract (data.py:10-21):
the object's __dict__ is cached under save/<ClassName>_<name>.pickle.
"""
from __future__ import annotations

import random
from glob import glob
from random import randint

import networkx as nx
import numpy as np

from .utils import (get_data_path, get_save_path, get_train_str, load, save, sorted_nicely)

# The 29 AIDS atom types (SimGNN AIDS700nef); Zipf-weighted so 'C' dominates.
AIDS_TYPES = ['C', 'O', 'N', 'Cl', 'F', 'S', 'Se', 'P', 'Na', 'I', 'Co', 'Br', 'Li', 'Si', 'Mg',
              'Cu', 'As', 'B', 'Pt', 'Ru', 'K', 'Pd', 'Au', 'Te', 'W', 'Rh', 'Zn', 'Bi', 'Sn']


class Data(object):
    def __init__(self, name_str, use_cache=True):
        name = self.__class__.__name__ + '_' + name_str + self.name_suffix()
        self.name = name
        sfn = self.save_filename()
        temp = load(sfn) if use_cache else None
        if temp:
            self.__dict__ = temp
        else:
            self.init()
            if use_cache:
                save(sfn, self.__dict__)

    def init(self):
        raise NotImplementedError()

    def name_suffix(self):
        return ''

    def save_filename(self):
        return '{}/{}'.format(get_save_path(), self.name)

    def get_gids(self):
        return [g.graph['gid'] for g in self.graphs]


class SynData(Data):
    """data.py:36-59 — unseeded gnm graphs (kept for interface parity)."""
    train_num_graphs = 20
    test_num_graphs = 10

    def __init__(self, train):
        self.num_graphs = SynData.train_num_graphs if train else SynData.test_num_graphs
        super().__init__(get_train_str(train))

    def init(self):
        self.graphs = []
        for i in range(self.num_graphs):
            n = randint(5, 20)
            m = randint(n - 1, n * (n - 1) // 2)
            g = nx.gnm_random_graph(n, m)
            g.graph['gid'] = i
            for v in g.nodes():
                g.nodes[v]['type'] = 'C'
            self.graphs.append(g)

    def name_suffix(self):
        return '_{}_{}'.format(SynData.train_num_graphs, SynData.test_num_graphs)


class AIDSData(Data):
    def __init__(self, train):
        self.train = train
        super().__init__(get_train_str(train))

    def init(self):
        self.graphs = []
        datadir = '{}/{}/{}'.format(get_data_path(), self.get_folder_name(),
                                    'train' if self.train else 'test')
        files = self.sort()(glob(datadir + '/*.gexf'))
        if not files:
            raise RuntimeError('No gexf files under {} (the AIDS archives are not shipped; '
                               'use a syn_* dataset offline)'.format(datadir))
        for file in files:
            gid = int(file.split('/')[-1].split('.')[0])
            g = nx.read_gexf(file)
            g.graph['gid'] = gid
            self.graphs.append(g)
            if not nx.is_connected(g):
                raise RuntimeError('{} not connected'.format(gid))
        if 'nef' in self.get_folder_name():
            for g in self.graphs:
                self._remove_valence(g)

    def get_folder_name(self):
        raise NotImplementedError()

    def sort(self):
        raise NotImplementedError()

    def _remove_valence(self, g):
        for n1, n2, d in g.edges(data=True):
            d.pop('valence', None)


class AIDS10kData(AIDSData):
    def get_folder_name(self):
        return 'AIDS10k'

    def sort(self):
        return sorted_nicely


class AIDS10kNEFData(AIDS10kData):
    def init(self):
        self.graphs = AIDS10kData(self.train).graphs
        for g in self.graphs:
            self._remove_valence(g)


class AIDS700nefData(AIDSData):
    def get_folder_name(self):
        return 'AIDS700nef'

    def sort(self):
        return sorted_nicely


class AIDS80nefData(AIDS700nefData):
    def init(self):
        self.graphs = AIDS700nefData(self.train).graphs
        random.Random(123).shuffle(self.graphs)       # data.py:127
        self.graphs = self.graphs[0:70] if self.train else self.graphs[0:10]


# ---------------------------------------------------------------------------
# Synthetic AIDS-shaped datasets
# ---------------------------------------------------------------------------
SYNTHETIC = {
    # name: (n_train, n_test, n_lo, n_hi, n_types)
    'syn_aids80nef': (70, 10, 5, 10, 29),
    'syn_aids700nef': (560, 140, 5, 10, 29),
    'syn_aids10knef': (10000, 18, 5, 30, 29),
    'syn_web': (1000, 100, 64, 512, 29),
}
# mean extra-edge degree of the sparse synthetic sets (p_extra = deg / (n - 1));
# the others use p_extra = 0.15 (AIDS-like density)
SYNTHETIC_EXTRA_DEGREE = {'syn_web': 4.0}


def synthetic_graph(rng: np.random.Generator, n: int, gid: int, n_types: int = 29,
                    p_extra: float = 0.15, zipf_s: float = 1.5) -> nx.Graph:
    """Connected graph: random recursive spanning tree + each non-edge with
    probability p_extra; node types Zipf(zipf_s) over n_types AIDS atom types;
    node ids are strings like gexf's."""
    g = nx.Graph(gid=gid)
    w = 1.0 / np.arange(1, n_types + 1) ** zipf_s
    w /= w.sum()
    types = rng.choice(n_types, size=n, p=w)
    for v in range(n):
        g.add_node(str(v), type=AIDS_TYPES[types[v] % len(AIDS_TYPES)]
                   if n_types <= len(AIDS_TYPES) else 'T{}'.format(types[v]))
    for v in range(1, n):
        g.add_edge(str(v), str(int(rng.integers(0, v))))
    if p_extra > 0:
        iu, ju = np.triu_indices(n, 1)
        extra = rng.random(iu.shape[0]) < p_extra
        for a, b in zip(iu[extra], ju[extra]):
            g.add_edge(str(a), str(b))
    return g


def synthetic_graphs(name: str, seed: int = 123):
    n_train, n_test, lo, hi, nt = SYNTHETIC[name]
    rng = np.random.default_rng(seed)
    deg = SYNTHETIC_EXTRA_DEGREE.get(name)
    gs = []
    for gid in range(n_train + n_test):
        n = int(rng.integers(lo, hi + 1))
        pe = 0.15 if deg is None else min(0.15, deg / max(n - 1, 1))
        gs.append(synthetic_graph(rng, n, gid, nt, p_extra=pe))
    return gs[:n_train], gs[n_train:]


class SyntheticAIDSData(Data):
    def __init__(self, name, train):
        self.syn_name = name
        self.train = train
        super().__init__(name + '_' + get_train_str(train), use_cache=False)

    def init(self):
        tr, te = synthetic_graphs(self.syn_name)
        self.graphs = tr if self.train else te


def synthetic_ged_matrix(graphs, seed: int = 7) -> np.ndarray:
    """Stand-in GED labels for all pairs: d(i,j) ~ U{0..max(n_i,n_j)},
    symmetric, d(i,i) = 0."""
    n = len(graphs)
    sizes = np.array([g.number_of_nodes() for g in graphs])
    rng = np.random.default_rng(seed)
    hi = np.maximum(sizes[:, None], sizes[None, :])
    d = np.floor(rng.random((n, n)) * (hi + 1)).astype(np.int64)
    d = np.triu(d, 1)
    return d + d.T
