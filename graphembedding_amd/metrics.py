"""Ranking / regression metrics over Result objects (src/metrics.py:14-91)."""
from __future__ import annotations

import numpy as np
from scipy.stats import hmean


class Metric(object):
    def __init__(self, name, ylabel):
        self.name = name
        self.ylabel = ylabel

    def __str__(self):
        return self.name


def precision_at_ks(true_r, pred_r, norm, ks, print_ids=()):
    """Mean over queries of |true top-k (tie-inclusive) ∩ predicted top-k| / k."""
    m, n = true_r.m_n()
    assert true_r.m_n() == pred_r.m_n()
    ps = np.zeros((m, len(ks)))
    for q in range(m):
        for c, k in enumerate(ks):
            assert type(k) is int and 0 < k < n
            truth = set(true_r.top_k_ids(q, k, norm, inclusive=True))
            guess = set(pred_r.top_k_ids(q, k, norm, inclusive=False))
            ps[q][c] = len(truth & guess) / k
        if q in print_ids:
            print('query {}\nks:    {}\nprecs: {}'.format(q, ks, ps[q]))
    return np.mean(ps, axis=0)


def mean_reciprocal_rank(true_r, pred_r, norm, print_ids=()):
    """1 / harmonic mean of the best predicted rank among the true top-1 (ties)."""
    m, n = true_r.m_n()
    assert true_r.m_n() == pred_r.m_n()
    best = np.zeros(m)
    for q in range(m):
        tops = true_r.top_k_ids(q, 1, norm, inclusive=True)
        assert len(tops) >= 1
        best[q] = min(pred_r.ranking(q, t, norm, one_based=True) for t in tops)
        if q in print_ids:
            print('query {}\nrank: {}'.format(q, best[q]))
    return 1.0 / hmean(best)


def mean_squared_error(true_r, pred_r, sim_kernel, yeta, norm):
    """Frobenius norm of the similarity-matrix difference divided by m·n (sic)."""
    m, n = true_r.m_n()
    assert true_r.m_n() == pred_r.m_n()
    diff = true_r.sim_mat(sim_kernel, yeta, norm) - pred_r.sim_mat(sim_kernel, yeta, norm)
    return np.linalg.norm(diff) / (m * n)


def average_time(r):
    return np.mean(r.time_mat())
