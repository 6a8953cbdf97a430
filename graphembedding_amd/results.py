"""Result objects (src/results.py:11-399): the sink of the path's m×n scores.

Same interface: m_n, dist_sim_mat, dist_sim, sim_mat, top_k_ids (tie-inclusive
option), ranking, time/time_mat, mat, sort_id_mat; load_result dispatches on the
model name exactly like results.py:384-395.  Distance results are built from
result/<ds>/<metric>/<metric>_<metric>_mat_<ds>_<model>_*.npy (results.py:182-192)
or directly from in-memory matrices (DistanceMatrixResult).
"""
from __future__ import annotations

from glob import glob

import numpy as np

from .distance import normalized_dist
from .similarity import create_sim_kernel
from .utils import get_result_path, load_data


class Result(object):
    """m = number of queries, n = number of database graphs."""

    def model(self):
        return self.model_

    def m_n(self):
        return self.dist_sim_mat(norm=False).shape

    def dist_sim_mat(self, norm):
        raise NotImplementedError()

    def dist_sim(self, qid, gid, norm):
        raise NotImplementedError()

    def sim_mat(self, sim_kernel, yeta, norm):
        raise NotImplementedError()

    def top_k_ids(self, qid, k, norm, inclusive):
        """Ids of the top-k database graphs for query qid; with inclusive=True
        graphs tied with the k-th are included (len >= k)."""
        order = self.sort_id_mat(norm)
        n = order.shape[1]
        if k < 0 or k >= n:
            raise RuntimeError('Invalid k {}'.format(k))
        row = order[qid]
        if not inclusive:
            return row[:k]
        vals = self.dist_sim_mat(norm)[qid]
        while k < n and vals[row[k - 1]] == vals[row[k]]:
            k += 1
        return row[:k]

    def ranking(self, qid, gid, norm, one_based=True):
        """Rank of database graph gid for query qid, ties resolved to the best rank."""
        row = self.sort_id_mat(norm)[qid]
        hits = np.where(row == gid)[0]
        assert len(hits) == 1
        pos = int(hits[0])
        vals = self.dist_sim_mat(norm)[qid]
        while pos > 0 and vals[row[pos - 1]] == vals[row[pos]]:
            pos -= 1
        return pos + 1 if one_based else pos

    def time(self, qid, gid):
        raise NotImplementedError()

    def time_mat(self):
        raise NotImplementedError()

    def mat(self, metric, norm):
        raise NotImplementedError()

    def sort_id_mat(self, norm):
        raise NotImplementedError()


class DistanceModelResult(Result):
    """Ground-truth style result holding a distance matrix (results.py:129-198)."""

    def __init__(self, dataset, model, dist_mat=None, dist_norm_mat=None, time_mat=None):
        self.dataset = dataset
        self.model_ = model
        if dist_mat is None:
            dist_mat = self._load_result_mat(dataset, self.dist_metric())
            time_mat = self._load_result_mat(dataset, 'time')
        self.dist_mat_ = np.asarray(dist_mat)
        if dist_norm_mat is None:
            dist_norm_mat = self._normalize(dataset, self.dist_mat_)
        self.dist_norm_mat_ = np.asarray(dist_norm_mat)
        self.time_mat_ = None if time_mat is None else np.asarray(time_mat)
        self.sort_id_mat_ = np.argsort(self.dist_mat_, kind='mergesort')
        self.dist_norm_sort_id_mat_ = np.argsort(self.dist_norm_mat_, kind='mergesort')

    def dist_metric(self):
        raise NotImplementedError()

    @staticmethod
    def _normalize(dataset, dm):
        train = load_data(dataset, True).graphs
        test = load_data(dataset, False).graphs
        out = np.array(dm, dtype=np.float64, copy=True)
        for i in range(dm.shape[0]):
            for j in range(dm.shape[1]):
                out[i][j] = normalized_dist(dm[i][j], test[i], train[j])
        return out

    def dist_mat(self, norm):
        return self.dist_norm_mat_ if norm else self.dist_mat_

    def dist_sim_mat(self, norm):
        return self.dist_mat(norm)

    def dist_sim(self, qid, gid, norm):
        return self.dist_metric(), self.dist_mat(norm)[qid][gid]

    def sim_mat(self, sim_kernel, yeta, norm):
        return create_sim_kernel(sim_kernel, yeta).dist_to_sim_np(self.dist_mat(norm))

    def time(self, qid, gid):
        return self.time_mat_[qid][gid]

    def time_mat(self):
        return self.time_mat_

    def mat(self, metric, norm):
        if metric == self.dist_metric():
            return self.dist_mat(norm)
        if metric == 'time':
            return self.time_mat_
        raise RuntimeError('Unknown metric {} for model {}'.format(metric, self.model_))

    def sort_id_mat(self, norm):
        return self.dist_norm_sort_id_mat_ if norm else self.sort_id_mat_

    def _load_result_mat(self, dataset, metric):
        pattern = get_result_path() + '/{}/{}/{}_{}_mat_{}_{}_*.npy'.format(
            dataset, metric, self.dist_metric(), metric, dataset, self.model_)
        files = glob(pattern)
        if not files:
            raise RuntimeError('No results found {}'.format(pattern))
        return np.load(files[0], allow_pickle=False)


class PairwiseGEDModelResult(DistanceModelResult):
    def dist_metric(self):
        return 'ged'


class PairwiseMCSModelResult(DistanceModelResult):
    def dist_metric(self):
        return 'mcs'


class DistanceMatrixResult(PairwiseGEDModelResult):
    """In-memory GED result (e.g. synthetic ground truth)."""

    def __init__(self, dataset, model, dist_mat, dist_norm_mat, time_mat=None):
        super().__init__(dataset, model, dist_mat=dist_mat, dist_norm_mat=dist_norm_mat,
                         time_mat=time_mat)


class SimilarityBasedModelResult(Result):
    def sim_mat(self, sim_kernel=None, yeta=None, norm=None):
        return self.sim_mat_

    def dist_sim_mat(self, norm=False):
        return self.sim_mat()

    def dist_sim(self, qid, gid, norm=False):
        return 'sim', self.sim_mat_[qid][gid]

    def sort_id_mat(self, norm=False):
        # most similar first: reversed stable ascending sort (results.py:221-224)
        return np.argsort(self.sim_mat_, kind='mergesort')[:, ::-1]


class SiameseModelResult(SimilarityBasedModelResult):
    def __init__(self, dataset, model, sim_mat=None, time_mat=None, model_info=None):
        self.model_ = model
        self.dataset = dataset
        if sim_mat is None or time_mat is None:
            raise NotImplementedError('SiameseModelResult needs in-memory sim_mat and time_mat '
                                      '(the reference never implemented loading them)')
        self.sim_mat_ = np.asarray(sim_mat)
        self.time_mat_ = np.asarray(time_mat)
        self.sort_id_mat_ = self.sort_id_mat()

    def time(self, qid, gid):
        return self.time_mat_[qid][gid]

    def time_mat(self):
        return self.time_mat_

    def mat(self, metric, *unused):
        if metric == 'sim':
            return self.sim_mat_
        if metric == 'time':
            return self.time_mat_
        raise RuntimeError('Unknown metric {} for model {}'.format(metric, self.model_))


class TransductiveResult(SimilarityBasedModelResult):
    def __init__(self, dataset, model, sim_mat=None, model_info=None):
        self.model_ = model
        self.dataset = dataset
        if sim_mat is None:
            raise NotImplementedError('TransductiveResult needs an in-memory sim_mat')
        self.sim_mat_ = np.asarray(sim_mat)
        self.sort_id_mat_ = self.sort_id_mat()

    def mat(self, metric, *unused):
        if metric == 'sim':
            return self.sim_mat_
        raise RuntimeError('Unknown metric {} for model {}'.format(metric, self.model_))


def load_results_as_dict(dataset, models, sim='dot', sim_mat=None, time_mat=None,
                         model_info=None):
    return {m: load_result(dataset, m, sim, sim_mat, time_mat, model_info) for m in models}


def load_result(dataset, model, sim=None, sim_mat=None, time_mat=None, model_info=None):
    if 'beam' in model or model in ['astar', 'hungarian', 'vj']:
        return PairwiseGEDModelResult(dataset, model)
    elif model == 'graph2vec':
        raise RuntimeError('graph2vec results are an out-of-scope baseline (results.py:227-310)')
    elif 'siamese' in model:
        return SiameseModelResult(dataset, model, sim_mat, time_mat, model_info)
    elif 'transductive' in model:
        return TransductiveResult(dataset, model, sim_mat, model_info)
    else:
        raise RuntimeError('Unknown model {}'.format(model))
