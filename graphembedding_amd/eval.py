"""Test-matrix evaluation (model/Siamese/eval.py:5-42) without the plotting:
ap@k, MRR, "mse" and time via metrics.py against the ground-truth result."""
from __future__ import annotations

import numpy as np

from . import metrics
from .results import DistanceMatrixResult, load_result, load_results_as_dict


class Eval(object):
    def __init__(self, dataset, true_model, sim_kernel_name, yeta, plot_results=False,
                 true_result=None):
        if plot_results:
            raise RuntimeError('plotting (exp.plot_apk / plot_mrr_mse_time) is out of scope')
        self.dataset = dataset
        self.models = [true_model]
        self.rs = {true_model: true_result} if true_result is not None else \
            load_results_as_dict(dataset, self.models)
        self.true_result = self.rs[true_model]
        self.sim_kernel_name = sim_kernel_name
        self.yeta = yeta
        self.results = {}

    @classmethod
    def from_calculator(cls, data, dist_calculator, flags):
        """Ground truth of the m×n test matrix from a gid-pair distance map."""
        from .distance import normalized_dist
        m, n = data.m_n()
        d = np.zeros((m, n))
        dn = np.zeros((m, n))
        for i in range(m):
            g1 = data.test_data.get_graph(i).nxgraph
            for j, g2 in enumerate(data.orig_train_graphs):
                d[i][j], dn[i][j] = dist_calculator.calculate_dist(g1, g2)
        true = DistanceMatrixResult(flags.dataset, flags.dist_algo, d, dn)
        return cls(flags.dataset, flags.dist_algo, flags.sim_kernel, flags.yeta,
                   true_result=true)

    def get_true_sim(self, query_id, train_id, norm):
        return self.true_result.sim_mat(self.sim_kernel_name, self.yeta, norm)[query_id][train_id]

    def eval_test(self, cur_model, sim_mat, time_mat):
        pred = load_result(self.dataset, cur_model, sim_mat=sim_mat, time_mat=time_mat)
        self.rs[cur_model] = pred
        _, n = self.true_result.m_n()
        ks = [k for k in (1, 2, 5, 10, 20, 50, 100) if k < n]
        out = {}
        for norm in (True, False):
            sfx = '_norm' if norm else '_nonorm'
            out['apk' + sfx] = {cur_model: {'ks': ks, 'aps': metrics.precision_at_ks(
                self.true_result, pred, norm, ks)}}
            out['mrr' + sfx] = {cur_model: metrics.mean_reciprocal_rank(self.true_result, pred,
                                                                        norm)}
            out['mse' + sfx] = {cur_model: metrics.mean_squared_error(
                self.true_result, pred, self.sim_kernel_name, self.yeta, norm)}
        if time_mat is not None:
            out['time'] = {cur_model: metrics.average_time(pred)}
        self.results.update(out)
        return self.results
