"""GPU parity: libsiamese_hip.so (through the C-ABI) against the numpy oracle on
identical seeded inputs, dropout on (shared counter RNG) and off.
Tolerance: 1e-4 (north_star: per-pair scores within 1e-4 fp32)."""
import numpy as np
import pytest

from _fixtures import AVERAGE_STACK, check_grad_per_var, run_oracle_step, small_problem
from oracle import siamese_oracle as O

pytestmark = pytest.mark.gpu

TOL = 1e-4

STACKS = {
    'default': {},
    'default_nodrop': dict(dropout=0.0),
    'average': AVERAGE_STACK,
    'attention': dict(AVERAGE_STACK, layer_2='Attention:input_dim=16'),
    'attention_nodrop': dict(AVERAGE_STACK, layer_2='Attention:input_dim=16', dropout=0.0),
    'attention_intended_aligned': dict(AVERAGE_STACK, layer_2='Attention:input_dim=16',
                                       ntn_mode='intended', loss_mode='aligned'),
    'attention_bf16_records': dict(AVERAGE_STACK, layer_2='Attention:input_dim=16',
                                   record_dtype='bf16'),
    'dot': dict(num_layers=5, layer_4='Dot'),
    'dense_after_pad': dict(num_layers=6,
                            layer_3='Padding:max_in_dims=10,padding_value=0',
                            layer_4='Dense:input_dim=1,output_dim=1,dropout=True,act=tanh,bias=True',
                            layer_5='NTN:input_dim=10,feature_map_dim=10,inneract=sigmoid,'
                                    'dropout=True,bias=False'),
    'intended_aligned': dict(ntn_mode='intended', loss_mode='aligned'),
    'sigmoid_final': dict(final_act='sigmoid'),
    # config C3: Â stored as bf16 in the records (fused path and generic path)
    'default_bf16_records': dict(record_dtype='bf16'),
    'average_bf16_records': dict(AVERAGE_STACK, record_dtype='bf16'),
}


def _check_grad(g_gpu, g_ref, prob, tol=TOL):
    """Per variable, each against its own largest reference component (_fixtures)."""
    check_grad_per_var(g_gpu, g_ref, prob.layers, prob.d_in, tol)


@pytest.mark.parametrize('name', list(STACKS))
def test_forward_and_step_match_oracle(gpu, name):
    prob = small_problem(n_graphs=16, n_pairs=40, seed=21, flags_overrides=STACKS[name])
    model, batch = prob.make_gpu_model(device=gpu)
    seed = 1234
    s = model.pred_sim_without_act(batch, seed=seed).cpu().numpy()
    ref = run_oracle_step(prob, seed)
    np.testing.assert_allclose(s, ref.s, rtol=TOL, atol=TOL)
    model.fwd_bwd(batch, seed=seed)
    _check_grad(model.grad.cpu().numpy(), ref.grad_mse, prob)
    loss_mse = float(model.loss_buf[0].item())
    assert abs(loss_mse - ref.loss_mse) <= TOL * max(1.0, abs(ref.loss_mse))
    model.apply_adam()
    reg = float(model.reg_buf[0].item())
    assert abs(loss_mse + reg - ref.loss) <= TOL * max(1.0, abs(ref.loss))
    np.testing.assert_allclose(model.params.cpu().numpy(), ref.new_params, rtol=0, atol=2e-5)


def test_large_batch_properties(gpu):
    """Size-independent properties at a few thousand pairs: sharded forward ==
    unsharded, gradient of a batch == sum of its halves, deterministic replay."""
    import torch
    prob = small_problem(n_graphs=64, n_pairs=4096, seed=8)
    model, batch = prob.make_gpu_model(device=gpu)
    seed = 42
    s_full = model.pred_sim_without_act(batch, seed=seed).cpu().numpy()
    half = batch.n_pairs // 2
    W = batch.records.numel() // batch.n_pairs
    b0 = model.batch_from_records(batch.records[:half * W], half, batch.labels[:half], 0,
                                  batch.n_pairs, y_stats=batch.y_stats)
    b1 = model.batch_from_records(batch.records[half * W:], batch.n_pairs - half,
                                  batch.labels[half:], half, batch.n_pairs, y_stats=batch.y_stats)
    s0 = model.pred_sim_without_act(b0, seed=seed).cpu().numpy()
    s1 = model.pred_sim_without_act(b1, seed=seed).cpu().numpy()
    assert np.array_equal(np.concatenate([s0, s1]), s_full)
    model.fwd_bwd(batch, seed=seed)
    g_full = model.grad.clone()
    model.fwd_bwd(batch, seed=seed)
    assert torch.equal(g_full, model.grad), 'fwd_bwd is not bitwise reproducible'
    model.fwd_bwd(b0, seed=seed, add_label_term=True)
    g0 = model.grad.clone()
    model.fwd_bwd(b1, seed=seed, add_label_term=False)
    g_sum = (g0 + model.grad).cpu().numpy()
    _check_grad(g_sum, g_full.cpu().numpy(), prob, tol=1e-5)


@pytest.mark.parametrize('dtype', ['f32', 'bf16'])
def test_pack_pairs_device_matches_host(gpu, dtype):
    import torch
    from graphembedding_amd.packer import pack_device
    prob = small_problem(n_graphs=10, n_pairs=50, seed=2)
    store = prob.store()
    words_h = store.pack_host(prob.pairs, prob.labels, dtype=dtype)
    recs, status = pack_device(store, prob.pairs, prob.labels, device=gpu, dtype=dtype)
    torch.cuda.synchronize()
    assert int(status.item()) == 0
    assert np.array_equal(recs.cpu().numpy().view(np.uint32).reshape(words_h.shape), words_h)
    bad = prob.pairs.copy()
    bad[3, 1] = 10_000
    _, status = pack_device(store, bad, prob.labels, device=gpu, dtype=dtype)
    assert int(status.item()) != 0


@pytest.mark.parametrize('dtype', ['f32', 'bf16'])
def test_label_stats(gpu, dtype):
    import torch
    from graphembedding_amd import _lib
    prob = small_problem(n_graphs=10, n_pairs=3000, seed=4,
                         flags_overrides=dict(record_dtype=dtype))
    model, batch = prob.make_gpu_model(device=gpu)
    stats = torch.zeros(2, dtype=torch.float32, device=gpu)
    _lib.label_stats(batch.records, batch.n_pairs, prob.n_max, stats, model.workspace(3000),
                     dtype=dtype)
    y = prob.labels.astype(np.float64)
    st = stats.cpu().numpy()
    assert abs(st[0] - y.mean()) < 1e-6
    assert abs(st[1] - 0.5 * ((y - y.mean()) ** 2).sum()) < 1e-4 * max(1, st[1])


def test_edge_cases(gpu):
    """Single-node graphs, graphs at the padding capacity, empty batch."""
    import torch
    prob = small_problem(n_graphs=12, n_pairs=30, seed=9, n_lo=1, n_hi=10)
    model, batch = prob.make_gpu_model(device=gpu)
    s = model.pred_sim_without_act(batch, seed=3).cpu().numpy()
    ref = run_oracle_step(prob, 3)
    np.testing.assert_allclose(s, ref.s, rtol=TOL, atol=TOL)
    empty = model.batch_from_records(batch.records[:0], 0, batch.labels[:0],
                                     y_stats=batch.y_stats)
    model.fwd_bwd(empty, seed=1)
    assert float(model.grad.abs().max().item()) == 0.0


def test_nmax30_aids10k_shape(gpu):
    """AIDS10k-shaped graphs (N <= 30, Padding/NTN input_dim 30)."""
    prob = small_problem(n_graphs=10, n_pairs=12, seed=13, n_lo=5, n_hi=30, n_max=30)
    model, batch = prob.make_gpu_model(device=gpu)
    s = model.pred_sim_without_act(batch, seed=5).cpu().numpy()
    ref = run_oracle_step(prob, 5)
    np.testing.assert_allclose(s, ref.s, rtol=TOL, atol=TOL)
    model.fwd_bwd(batch, seed=5)
    _check_grad(model.grad.cpu().numpy(), ref.grad_mse, prob)


@pytest.mark.parametrize('stack', ['default', 'average', 'attention'])
def test_fast_path_matches_generic_path(gpu, monkeypatch, stack):
    """The fused MFMA kernel and the generic LDS kernel agree on the default, the
    tuning.py Average and the Attention-pooling stacks (dropout on) — the generic path
    is the on-GPU cross-check."""
    prob = small_problem(n_graphs=40, n_pairs=2000, seed=17,
                         flags_overrides=None if stack == 'default' else STACKS[stack])
    model, batch = prob.make_gpu_model(device=gpu)
    assert model.kernel_path == 1, 'the stack must take the fused path'
    seed = 99
    s_fast = model.pred_sim_without_act(batch, seed=seed).cpu().numpy()
    model.fwd_bwd(batch, seed=seed)
    g_fast = model.grad.cpu().numpy()
    l_fast = float(model.loss_buf[0].item())
    monkeypatch.setenv('SG_DISABLE_FAST', '1')
    s_gen = model.pred_sim_without_act(batch, seed=seed).cpu().numpy()
    model.fwd_bwd(batch, seed=seed)
    g_gen = model.grad.cpu().numpy()
    np.testing.assert_allclose(s_fast, s_gen, rtol=1e-5, atol=1e-5)
    _check_grad(g_fast, g_gen, prob, tol=2e-5)
    assert abs(l_fast - float(model.loss_buf[0].item())) <= 1e-5 * max(1.0, abs(l_fast))


@pytest.mark.parametrize('case', ['one_type', 'types_32', 'nmax12', 'heavy_dropout',
                                  'self_and_repeated_pairs', 'attention_nmax12',
                                  'attention_single_nodes', 'attention_heavy_dropout'])
def test_fused_path_edge_shapes(gpu, case):
    """Fused-kernel boundaries against the oracle: a single node type (d_in = 1), the
    largest one-hot width the fused kernel takes (d_in = 32), Padding / NTN width 12 with
    12-node graphs (the third Â k-step full), dropout 0.9 (most elements dropped), and
    self-pairs (g, g) plus repeated pairs (distinct pair keys, so distinct masks); the
    Attention-pooling kernel at capacity 12, on 1- to 4-node graphs and at dropout 0.9."""
    kw = dict(n_graphs=14, n_pairs=48, seed=17)
    if case == 'one_type':
        kw.update(n_types=1)
    elif case == 'types_32':
        kw.update(n_types=32, n_lo=8, n_hi=10, n_graphs=40)
    elif case == 'nmax12':
        kw.update(n_max=12, n_lo=9, n_hi=12)
    elif case == 'heavy_dropout':
        kw.update(flags_overrides=dict(dropout=0.9))
    elif case == 'attention_nmax12':
        kw.update(n_max=12, n_lo=9, n_hi=12, flags_overrides=STACKS['attention'])
    elif case == 'attention_single_nodes':
        kw.update(n_lo=1, n_hi=4, flags_overrides=STACKS['attention'])
    elif case == 'attention_heavy_dropout':
        kw.update(flags_overrides=dict(STACKS['attention'], dropout=0.9))
    prob = small_problem(**kw)
    if case == 'self_and_repeated_pairs':
        prob.pairs[:16, 1] = prob.pairs[:16, 0]
        prob.pairs[16:24] = prob.pairs[0]
    if case == 'types_32':
        assert prob.d_in > 16, prob.d_in   # the second 16-type tile of the gW0 product
    model, batch = prob.make_gpu_model(device=gpu)
    assert model.kernel_path == 1, (case, model.kernel_path)
    seed = 4321
    s = model.pred_sim_without_act(batch, seed=seed).cpu().numpy()
    ref = run_oracle_step(prob, seed)
    np.testing.assert_allclose(s, ref.s, rtol=TOL, atol=TOL)
    model.fwd_bwd(batch, seed=seed)
    _check_grad(model.grad.cpu().numpy(), ref.grad_mse, prob)
    loss_mse = float(model.loss_buf[0].item())
    assert abs(loss_mse - ref.loss_mse) <= TOL * max(1.0, abs(ref.loss_mse))
