"""End-to-end on the GPU: the reference's main() flow (train_val + test + eval)
on the synthetic AIDS80nef stand-in, and all-pairs training that decreases the
loss.  Numerics are covered by test_gpu_parity.py; this checks the wiring."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_main_flow_syn_aids80nef(gpu, capsys):
    from graphembedding_amd.config import Flags
    from graphembedding_amd.train import main
    f = Flags(dataset='syn_aids80nef', iters=4, n_max=10, node_feat_order='sorted')
    (tc, tt, vc, vt), (sim_mat, time_mat, results) = main(f, device=gpu)
    assert len(tc) == 4 and all(np.isfinite(tc)) and all(np.isfinite(vc))
    assert sim_mat.shape == (10, 70) and np.all((sim_mat > 0) & (sim_mat <= 1))
    assert 'mrr_norm' in results and 'apk_nonorm' in results and 'time' in results
    out = capsys.readouterr().out
    assert 'Iter: 0001 train_loss=' in out


def test_compat_diag_test_matrix(gpu):
    from graphembedding_amd.config import Flags
    from graphembedding_amd.train import main
    f = Flags(dataset='syn_aids80nef', iters=1, n_max=10, node_feat_order='sorted',
              test_matrix='compat_diag')
    _, (sim_mat, _, _) = main(f, device=gpu)
    assert np.count_nonzero(sim_mat) <= 10          # only [i][i] written (train.py:68, A5)
    assert np.all(np.diag(sim_mat[:, :10]) > 0)


def test_allpairs_training_reduces_loss(gpu):
    import torch
    from graphembedding_amd.allpairs import AllPairsShard, load_graph_set
    from graphembedding_amd.config import Flags
    from graphembedding_amd.model_mse import SiameseGCNTNMSE
    f = Flags(dropout=0.0, learning_rate=0.003)
    gs = load_graph_set('syn_aids80nef', n_max=10)
    labels = gs.label_matrix(f.yeta)
    model = SiameseGCNTNMSE(gs.d_in, f, device=gpu, n_max=10)
    shard = AllPairsShard(gs, labels, device=gpu)
    batch = shard.batch(model)
    losses = [model.train_step(batch) for _ in range(40)]
    torch.cuda.synchronize()
    assert losses[-1] < losses[0], losses[::8]


def test_per_pair_test_times(gpu):
    """test_time='per_pair': every test-matrix entry timed around its own single-pair run,
    as train.py:57-69 times each sess.run; 'batched' states its launch average on the
    result (time_mat_mode)."""
    from graphembedding_amd.config import Flags
    from graphembedding_amd.train import main
    f = Flags(dataset='syn_aids80nef', iters=1, n_max=10, node_feat_order='sorted',
              test_time='per_pair')
    _, (sim_mat, time_mat, results) = main(f, device=gpu)
    assert time_mat.shape == (10, 70) and np.all(time_mat > 0)
    assert len(np.unique(time_mat)) > 1
    assert results['time_mat_mode'] == {f.model: 'per_pair'}
    f2 = Flags(dataset='syn_aids80nef', iters=1, n_max=10, node_feat_order='sorted')
    _, (sim2, time2, res2) = main(f2, device=gpu)
    assert res2['time_mat_mode'] == {f2.model: 'batched'}
    assert len(np.unique(time2)) == 1


def _expected_columns(f):
    """get_orig_train_graph(j) after the default loop, from the REFERENCE sampler's list
    order (F7, tests/golden/make_golden.py): fresh (unshuffled) train / val lists indexed
    by the reference's permutation after 30 * iters get_pair calls each."""
    import json
    import os
    from graphembedding_amd.data_siamese import SiameseModelData
    with open(os.path.join(os.path.dirname(__file__), 'golden', 'f7_loop_lists.json')) as fh:
        f7 = json.load(fh)
    fresh = SiameseModelData(f)
    tr, va = fresh.train_data.gs, fresh.valid_data.gs
    calls = 30 * f.iters
    pt = f7['random_{}_after_{}_calls'.format(len(tr), calls)]['gs']
    pv = f7['random_{}_after_{}_calls'.format(len(va), calls)]['gs']
    return fresh, [tr[k] for k in pt] + [va[k] for k in pv]


def test_main_test_matrix_matches_oracle(gpu):
    """f1 end to end: main() (train_val 20 iterations, then test + Eval) on AIDS80nef-shaped
    data; every sim_mat[i][j] equals the oracle's exp(-η s²) for (test i, the PERMUTED train
    graph j) — the reference scores get_orig_train_graph(j) after the in-place shuffles
    (train.py:57-69, samplers.py:28, A6) — within 1e-4, with dropout on (A4) and the eval
    seed; the compat_diag matrix (train.py:68, A5) holds exactly sims[i][n-1] at [i][i];
    Eval.eval_test's metrics equal metrics.py (pinned by F4) on the same matrix."""
    from oracle import siamese_oracle as O
    from graphembedding_amd import metrics
    from graphembedding_amd.config import Flags
    from graphembedding_amd.eval import Eval
    from graphembedding_amd.packer import record_words, unpack_host
    from graphembedding_amd.results import SiameseModelResult
    from graphembedding_amd.train import test, main
    f = Flags(dataset='syn_aids80nef', n_max=10, node_feat_order='sorted')
    assert f.iters == 20 and f.dropout == 0.1
    tr, (sim_mat, time_mat, results), (data, dc, model) = main(f, device=gpu,
                                                               return_objects=True)
    m, n = data.m_n()
    assert sim_mat.shape == (m, n) == (10, 70)
    fresh, cols = _expected_columns(f)
    assert [data.get_orig_train_graph(j).nxgraph.graph['gid'] for j in range(n)] == \
        [g.nxgraph.graph['gid'] for g in cols]
    # orig_train_graphs (networkx graphs) keep the load order: train list, then val list
    assert [g.graph['gid'] for g in data.orig_train_graphs] == \
        [g.nxgraph.graph['gid'] for g in fresh.train_data.gs + fresh.valid_data.gs]
    seed = model._seed(None)                   # the eval launch's seed (no step since)
    g1s = [fresh.test_data.get_graph(i) for i in range(m) for _ in range(n)]
    g2s = [cols[j] for _ in range(m) for j in range(n)]
    words = model.make_batch(g1s, g2s).records.cpu().numpy().view(np.uint32).reshape(
        m * n, record_words(model.n_max, model.record_dtype))
    r = unpack_host(words, model.n_max)
    og = ([], [])
    for k in range(m * n):
        for side in (0, 1):
            c = int(r['n'][k, side])
            og[side].append(O.Graph(adj=r['adj'][k, side, :c, :c].astype(np.float64),
                                    types=r['types'][k, side, :c].astype(np.int64)))
    spec = O.OracleSpec(layers=model.layers, d_in=model.input_dim, keep_prob=1.0 - f.dropout,
                        final_act=f.final_act, sim_kernel=f.sim_kernel, yeta=f.yeta,
                        loss_mode=f.loss_mode, ntn_mode=f.ntn_mode,
                        weight_decay=f.weight_decay, dist_norm=f.dist_norm)
    s_ref = O.forward(spec, model.params.cpu().numpy().astype(np.float64), og[0], og[1], seed)
    want = O.final_act(spec, s_ref).reshape(m, n)
    err = float(np.abs(sim_mat - want).max())
    print('test matrix {}x{}: max |sim - oracle| {:.3g}'.format(m, n, err))
    assert err <= 1e-4, err
    # A5: the reference's [i][i] write, from a second test() of the same model and lists
    fc = f.copy(test_matrix='compat_diag')
    diag, _, _ = test(data, dc, model, fc, None, verbose=False)
    expect = np.zeros((m, n))
    for i in range(m):
        expect[i][i] = sim_mat[i][n - 1]
    assert np.array_equal(diag, expect)
    # Eval.eval_test == metrics.py on the same matrices
    true_r = Eval.from_calculator(data, dc, f).true_result
    pred_r = SiameseModelResult(f.dataset, f.model, sim_mat=sim_mat, time_mat=time_mat)
    ks = results['apk_norm'][f.model]['ks']
    for norm, sfx in ((True, '_norm'), (False, '_nonorm')):
        assert np.array_equal(results['apk' + sfx][f.model]['aps'],
                              metrics.precision_at_ks(true_r, pred_r, norm, ks))
        assert results['mrr' + sfx][f.model] == metrics.mean_reciprocal_rank(true_r, pred_r,
                                                                             norm)
        assert results['mse' + sfx][f.model] == metrics.mean_squared_error(
            true_r, pred_r, f.sim_kernel, f.yeta, norm)
