"""End-to-end on the GPU: the reference's main() flow (train_val + test + eval)
on the synthetic AIDS80nef stand-in, and all-pairs training that decreases the
loss.  Numerics are covered by test_gpu_parity.py; this checks the wiring."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_main_flow_syn_aids80nef(gpu, capsys):
    from graphembedding_amd.config import Flags
    from graphembedding_amd.train import main
    f = Flags(dataset='syn_aids80nef', iters=4, n_max=10)
    (tc, tt, vc, vt), (sim_mat, time_mat, results) = main(f, device=gpu)
    assert len(tc) == 4 and all(np.isfinite(tc)) and all(np.isfinite(vc))
    assert sim_mat.shape == (10, 70) and np.all((sim_mat > 0) & (sim_mat <= 1))
    assert 'mrr_norm' in results and 'apk_nonorm' in results and 'time' in results
    out = capsys.readouterr().out
    assert 'Iter: 0001 train_loss=' in out


def test_compat_diag_test_matrix(gpu):
    from graphembedding_amd.config import Flags
    from graphembedding_amd.train import main
    f = Flags(dataset='syn_aids80nef', iters=1, n_max=10, test_matrix='compat_diag')
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
    f = Flags(dataset='syn_aids80nef', iters=1, n_max=10, test_time='per_pair')
    _, (sim_mat, time_mat, results) = main(f, device=gpu)
    assert time_mat.shape == (10, 70) and np.all(time_mat > 0)
    assert len(np.unique(time_mat)) > 1
    assert results['time_mat_mode'] == {f.model: 'per_pair'}
    f2 = Flags(dataset='syn_aids80nef', iters=1, n_max=10)
    _, (sim2, time2, res2) = main(f2, device=gpu)
    assert res2['time_mat_mode'] == {f2.model: 'batched'}
    assert len(np.unique(time2)) == 1
