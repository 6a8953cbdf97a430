"""Driver mirror of model/Siamese/train.py:8-111 and main.py:14-27.

`run` replaces `run_tf` (train.py:77-102): the timed region is the device work
of one batch (the reference timed `sess.run` only).  `test` scores the whole
m×n test matrix in ONE fused-kernel launch instead of the reference's m·n
batch-1 `sess.run`s; `test_matrix='compat_diag'` reproduces the
reference's `test_sim_mat[i][i] = sim` write (quirk A5).
"""
from __future__ import annotations

import time as _time

import numpy as np

from .config import FLAGS, check_flags
from .eval import Eval


def _sync():
    import torch
    if torch.cuda.is_available():
        torch.cuda.synchronize()


def print_msec(sec):
    return '{:.2f}msec'.format(sec * 1000)


def run(data, dist_calculator, model, tvt, test_id=None, train_id=None, iter=None):
    batch = model.get_feed_dict(data, dist_calculator, tvt, test_id, train_id)
    _sync()
    t = _time.time()
    if tvt == 'train':
        out = model.train_step(batch)
    elif tvt == 'val':
        out = model.val_loss(batch)
    elif tvt == 'test':
        s = model.test_scores(batch)
        assert len(s) == 1
        out = model.apply_final_act_np(s[0])
    else:
        raise RuntimeError('Unknown train_val_test {}'.format(tvt))
    _sync()
    return out, _time.time() - t


def train_val(data, dist_calculator, model, flags=None, verbose=True):
    f = flags or FLAGS
    train_costs, train_times, val_costs, val_times = [], [], [], []
    for it in range(f.iters):
        c, t = run(data, dist_calculator, model, 'train', iter=it)
        train_costs.append(c)
        train_times.append(t)
        vc, vt = run(data, dist_calculator, model, 'val', iter=it)
        val_costs.append(vc)
        val_times.append(vt)
        if verbose:
            print('Iter:', '%04d' % (it + 1), 'train_loss=', '{:.5f}'.format(c),
                  'time=', print_msec(t), 'val_loss=', '{:.5f}'.format(vc),
                  'time=', print_msec(vt))
        if f.early_stopping:
            if it > f.early_stopping and \
                    val_costs[-1] > np.mean(val_costs[-(f.early_stopping + 1):-1]):
                if verbose:
                    print('Early stopping...')
                break
    return train_costs, train_times, val_costs, val_times


def test(data, dist_calculator, model, flags=None, evaluator=None, verbose=True):
    """All m×n (test i, original train j) pairs in one launch (train.py:47-74)."""
    f = flags or FLAGS
    m, n = data.m_n()
    g1s, g2s = [], []
    for i in range(m):
        for j in range(n):
            g1s.append(data.test_data.get_graph(i))
            g2s.append(data.get_orig_train_graph(j))   # permuted after training (A6)
    batch = model.make_batch(g1s, g2s)
    _sync()
    t0 = _time.time()
    s = model.test_scores(batch)
    _sync()
    elapsed = _time.time() - t0
    sims = np.asarray(model.apply_final_act_np(s), dtype=np.float64).reshape(m, n)
    time_mode = getattr(f, 'test_time', 'batched')
    if time_mode == 'per_pair':
        # train.py:57-69: every (i, j) timed around its own single-pair run (msec); the
        # same dropout keys as the batched launch (pair index i * n + j), so the scores
        # equal the batched ones
        time_mat = np.zeros((m, n))
        for i in range(m):
            for j in range(n):
                one = model.make_batch([g1s[i * n + j]], [g2s[i * n + j]], pair_offset=i * n + j,
                                       batch_total=m * n)
                _sync()
                t = _time.time()
                s1 = model.test_scores(one)
                _sync()
                time_mat[i][j] = (_time.time() - t) * 1000.0
                # same keys, same kernel: bit-identical (bit patterns, so NaN == NaN)
                if np.float64(s1[0]).view(np.uint64) != np.float64(s[i * n + j]).view(np.uint64):
                    raise RuntimeError('per_pair score ({}, {}) = {!r} differs from the batched '
                                       'score {!r}'.format(i, j, float(s1[0]),
                                                           float(s[i * n + j])))
    elif time_mode == 'batched':
        time_mat = np.full((m, n), elapsed * 1000.0 / max(1, m * n))   # msec per pair
    else:
        raise RuntimeError('Unknown test_time {}'.format(time_mode))
    if f.test_matrix == 'compat_diag':
        sim_mat = np.zeros((m, n))
        for i in range(m):
            sim_mat[i][i] = sims[i][n - 1]             # train.py:68 writes [i][i]
    else:
        sim_mat = sims
    results = None
    if evaluator is not None:
        results = evaluator.eval_test(f.model, sim_mat, time_mat)
        # the deviation is stated on the result: 'batched' entries are a launch average
        results['time_mat_mode'] = {f.model: time_mode}
        evaluator.rs[f.model].time_mat_mode = time_mode
    if verbose:
        print('scored {}x{} pairs in {}'.format(m, n, print_msec(elapsed)))
    return sim_mat, time_mat, results


def main(flags=None, device='cuda', return_objects=False):
    """main.py:14-27 (returns costs/times and the test results; with return_objects also
    the (data, dist_calculator, model) the run trained and scored with)."""
    from .data import synthetic_ged_matrix
    from .data_siamese import SiameseModelData
    from .dist_calculator import DistCalculator
    from .model_mse import create_model
    f = flags or FLAGS
    check_flags(f)
    data = SiameseModelData(f)
    if f.dataset.startswith('syn_'):
        gs = list(data.orig_train_graphs) + list(data.test_data.gs[i].nxgraph
                                                 for i in range(data.m))
        dc = DistCalculator.from_matrix(f.dataset, gs, synthetic_ged_matrix(gs),
                                        f.dist_metric, f.dist_algo)
    else:
        dc = DistCalculator(f.dataset, f.dist_metric, f.dist_algo)
    model = create_model(f.model, data.input_dim(), f, device=device,
                         n_max=f.n_max or max(g.num_nodes() for g in
                                              data.train_data.gs + data.valid_data.gs +
                                              data.test_data.gs))
    tr = train_val(data, dc, model, f)
    evaluator = Eval.from_calculator(data, dc, f) if f.dataset.startswith('syn_') else None
    res = test(data, dc, model, f, evaluator)
    if return_objects:
        return tr, res, (data, dc, model)
    return tr, res


if __name__ == '__main__':
    from .config import parse_args
    main(parse_args())
