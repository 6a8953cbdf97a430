"""Ground-truth distance lookup (model/Siamese/dist_calculator.py:6-44).

The cache is the reference's `OrderedDict{(gid1, gid2): int}` pickle under
save/<ds>_<metric>_<algo>[_revtakemin]_gidpair_dist_map (read with a
restricted unpickler).  A miss falls back to `distance.ged`, which raises in
this build (the Java GED solver is out of scope).  `from_matrix` builds the
same map from an in-memory matrix (synthetic labels).
"""
from __future__ import annotations

from collections import OrderedDict

import numpy as np

from .distance import ged, normalized_dist
from .utils import get_save_path, safe_load, save


class DistCalculator(object):
    def __init__(self, dataset, dist_metric, algo, gidpair_dist_map=None, persist=False):
        self.sfn = '{}/{}_{}_{}{}_gidpair_dist_map'.format(
            get_save_path(), dataset, dist_metric, algo, '' if algo == 'astar' else '_revtakemin')
        self.algo = algo
        self.persist = persist
        if gidpair_dist_map is not None:
            self.gidpair_dist_map = gidpair_dist_map
        else:
            self.gidpair_dist_map = safe_load(self.sfn) or OrderedDict()
        if dist_metric == 'ged':
            self.dist_func = ged
        else:
            raise RuntimeError('Unknwon distance metric {}'.format(dist_metric))

    @classmethod
    def from_matrix(cls, dataset, graphs, dmat, dist_metric='ged', algo='astar'):
        m = OrderedDict()
        gids = [g.graph['gid'] for g in graphs]
        for i, a in enumerate(gids):
            for j, b in enumerate(gids):
                m[(a, b)] = int(dmat[i][j])
        obj = cls(dataset, dist_metric, algo, gidpair_dist_map=m)
        # the dense matrix too: device_sampler.label_matrix gathers from it directly
        obj.matrix = ({g: i for i, g in enumerate(gids)}, np.asarray(dmat))
        return obj

    def calculate_dist(self, g1, g2):
        gid1 = g1.graph['gid']
        gid2 = g2.graph['gid']
        pair = (gid1, gid2)
        d = self.gidpair_dist_map.get(pair)
        if d is None:
            rev_d = self.gidpair_dist_map.get((gid2, gid1))
            if rev_d:                      # sic: a cached reverse 0 is a miss (quirk A15)
                d = rev_d
            else:
                d = self.dist_func(g1, g2, self.algo)
            self.gidpair_dist_map[pair] = d
            if self.persist:
                save(self.sfn, self.gidpair_dist_map)
        return d, normalized_dist(d, g1, g2)
