"""Processing order (sg_pair_order, sg_forward_ex / sg_fwd_bwd_ex; include/siamese_hip.h)
and the class-exclusive schedule (sg_pair_order_cls, sg_forward_cls / sg_fwd_bwd_cls).

sg_pair_order must be the stable sort of the records by cost class, and walking
it must change nothing but the gradient's summation order: scores bit-identical,
gradient and loss within fp32 reassociation error, still bitwise reproducible
(fused path), and still equal to the oracle."""
import numpy as np
import pytest

from _fixtures import AVERAGE_STACK, run_oracle_step, small_problem

pytestmark = pytest.mark.gpu

TOL = 1e-4


def _node_counts(prob):
    n = np.array([g.number_of_nodes() for g in prob.graphs])
    return np.minimum(n[prob.pairs[:, 0]], prob.n_max), np.minimum(n[prob.pairs[:, 1]], prob.n_max)


def _expected_order(prob, fused):
    n0, n1 = _node_counts(prob)
    key = (n0 > 8).astype(int) + 2 * (n1 > 8).astype(int) if fused else n0 + n1
    return np.argsort(key, kind='stable').astype(np.int32)


@pytest.mark.parametrize('name,fused', [('default', True), ('average', True),
                                        ('attention', True), ('dot', False),
                                        ('default_bf16', True)])
def test_pair_order_is_stable_class_sort(gpu, name, fused):
    ov = {'default': {}, 'average': AVERAGE_STACK, 'default_bf16': dict(record_dtype='bf16'),
          'attention': dict(AVERAGE_STACK, layer_2='Attention:input_dim=16'),
          'dot': dict(num_layers=5, layer_4='Dot')}[name]
    # > 2 sort chunks (8192 records), ragged last chunk, 1..10-node graphs
    prob = small_problem(n_graphs=50, n_pairs=20011, seed=31, n_lo=1, n_hi=10,
                         flags_overrides=ov)
    model, batch = prob.make_gpu_model(device=gpu)
    assert (model.kernel_path == 1) == fused
    model.balance(batch)
    got = batch.order.cpu().numpy()
    assert np.array_equal(got, _expected_order(prob, fused))


@pytest.mark.parametrize('name', ['default', 'average', 'attention', 'default_bf16'])
def test_ordered_step_equals_batch_order(gpu, name):
    import torch
    ov = {'default': {}, 'average': AVERAGE_STACK, 'default_bf16': dict(record_dtype='bf16'),
          'attention': dict(AVERAGE_STACK, layer_2='Attention:input_dim=16')}[name]
    prob = small_problem(n_graphs=48, n_pairs=5000, seed=12, n_lo=2, n_hi=10,
                         flags_overrides=ov)
    model, batch = prob.make_gpu_model(device=gpu)
    seed = 77
    s_plain = model.pred_sim_without_act(batch, seed=seed).cpu().numpy()
    s_out = torch.empty(batch.n_pairs, dtype=torch.float32, device=gpu)
    model.fwd_bwd(batch, seed=seed, s_out=s_out)
    g_plain = model.grad.cpu().numpy()
    l_plain = float(model.loss_buf[0].item())
    s_bwd_plain = s_out.cpu().numpy()

    model.balance(batch)
    assert batch.order is not None
    s_ord = model.pred_sim_without_act(batch, seed=seed).cpu().numpy()
    assert np.array_equal(s_ord, s_plain), 'scores must not depend on the processing order'
    s_out.zero_()
    model.fwd_bwd(batch, seed=seed, s_out=s_out)
    assert np.array_equal(s_out.cpu().numpy(), s_bwd_plain)
    g_ord = model.grad.clone()
    scale = max(1.0, float(np.abs(g_plain).max()))
    assert float(np.abs(g_ord.cpu().numpy() - g_plain).max()) <= 1e-5 * scale
    assert abs(float(model.loss_buf[0].item()) - l_plain) <= 1e-5 * max(1.0, abs(l_plain))
    model.fwd_bwd(batch, seed=seed)
    if model.kernel_path == 1:
        # the fused kernel sums in a fixed order; the generic one accumulates a
        # workgroup's waves with LDS float atomics (reproducible to fp32 rounding)
        assert torch.equal(g_ord, model.grad), 'ordered fwd_bwd is not bitwise reproducible'
    else:
        assert float((g_ord - model.grad).abs().max().item()) <= 1e-5 * scale


def test_ordered_step_matches_oracle(gpu):
    prob = small_problem(n_graphs=16, n_pairs=40, seed=21, n_lo=2, n_hi=10)
    model, batch = prob.make_gpu_model(device=gpu)
    model.balance(batch)
    seed = 1234
    ref = run_oracle_step(prob, seed)
    np.testing.assert_allclose(model.pred_sim_without_act(batch, seed=seed).cpu().numpy(), ref.s,
                               rtol=TOL, atol=TOL)
    model.fwd_bwd(batch, seed=seed)
    g = model.grad.cpu().numpy()
    assert float(np.abs(g - ref.grad_mse).max()) <= TOL * max(1.0, float(np.abs(ref.grad_mse).max()))


def test_order_edge_cases(gpu):
    """One pair, and an order with out-of-range entries (clamped, no fault)."""
    import torch
    prob = small_problem(n_graphs=4, n_pairs=1, seed=3)
    model, batch = prob.make_gpu_model(device=gpu)
    s1 = model.pred_sim_without_act(batch, seed=5).cpu().numpy()
    model.balance(batch)
    assert batch.order.cpu().tolist() == [0]
    assert np.array_equal(model.pred_sim_without_act(batch, seed=5).cpu().numpy(), s1)

    prob = small_problem(n_graphs=8, n_pairs=300, seed=4)
    model, batch = prob.make_gpu_model(device=gpu)
    batch.order = torch.full((300,), 1 << 30, dtype=torch.int32, device=gpu)
    batch.order[::7] = -5
    model.fwd_bwd(batch, seed=1)
    torch.cuda.synchronize()
    assert bool(torch.isfinite(model.grad).all())


@pytest.mark.parametrize('n_pairs', [3, 37, 5000, 20011])
def test_class_schedule_equals_mixed_schedule(gpu, n_pairs):
    """sg_pair_order_cls's class table is the stable sort's class boundaries; the
    class-exclusive schedule (each wave runs one class's pair body) gives the mixed
    schedule's scores bit for bit, its gradient up to summation order, is bitwise
    reproducible, and matches the oracle."""
    import torch
    prob = small_problem(n_graphs=40, n_pairs=n_pairs, seed=n_pairs, n_lo=3, n_hi=10)
    model, batch = prob.make_gpu_model(device=gpu)
    assert model.kernel_path == 1
    seed = 4242
    model.balance(batch, classes=False)
    assert batch.cls is None
    s_mix = model.pred_sim_without_act(batch, seed=seed).cpu().numpy()
    model.fwd_bwd(batch, seed=seed)
    g_mix = model.grad.cpu().numpy()
    l_mix = float(model.loss_buf[0].item())
    model.balance(batch, classes=True)
    assert batch.cls is not None
    n0, n1 = _node_counts(prob)
    key = (n0 > 8).astype(int) + 2 * (n1 > 8).astype(int)
    expect = np.concatenate([[0], np.cumsum(np.bincount(key, minlength=4))])
    assert batch.cls.cpu().tolist() == expect.tolist()
    assert np.array_equal(batch.order.cpu().numpy(), _expected_order(prob, True))
    s_cls = model.pred_sim_without_act(batch, seed=seed).cpu().numpy()
    assert np.array_equal(s_cls, s_mix)
    s_out = torch.full((batch.n_pairs,), float('nan'), dtype=torch.float32, device=gpu)
    model.fwd_bwd(batch, seed=seed, s_out=s_out)
    assert np.array_equal(s_out.cpu().numpy(), s_mix)
    g_cls = model.grad.clone()
    scale = max(1.0, float(np.abs(g_mix).max()))
    assert float(np.abs(g_cls.cpu().numpy() - g_mix).max()) <= 1e-5 * scale
    assert abs(float(model.loss_buf[0].item()) - l_mix) <= 1e-5 * max(1.0, abs(l_mix))
    model.fwd_bwd(batch, seed=seed)
    assert torch.equal(g_cls, model.grad), 'class-schedule fwd_bwd is not bitwise reproducible'
    if n_pairs <= 40:
        ref = run_oracle_step(prob, seed)
        np.testing.assert_allclose(s_cls, ref.s, rtol=TOL, atol=TOL)
        from _fixtures import check_grad_per_var
        check_grad_per_var(g_cls.cpu().numpy(), ref.grad_mse, prob.layers, prob.d_in, TOL)


def test_class_table_needs_the_fused_path(gpu):
    """sg_pair_order_cls is the fused path's (path 1); other paths keep the plain order."""
    prob = small_problem(n_graphs=12, n_pairs=200, seed=5,
                         flags_overrides=dict(num_layers=5, layer_4='Dot'))
    model, batch = prob.make_gpu_model(device=gpu)
    assert model.kernel_path == 0
    model.balance(batch)
    assert batch.order is not None and batch.cls is None
