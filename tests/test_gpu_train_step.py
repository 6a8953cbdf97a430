"""sg_train_step (include/siamese_hip.h, library 1.9): fwd_bwd + ApplyAdam in one call;
on the fused path the gradient reduction applies the update in the same launch
(sg_reduce_adam, with the step scalars α, β powers and wd·½Σθ² from the fused kernel's
block 0).

It must leave θ, m, v, the β powers, the gradient and the loss bitwise as sg_fwd_bwd_cls +
sg_adam_tf do (models.py:28-36's train op), and wd·½Σθ² within double-summation order,
step after step (the β powers advance once per call)."""
import numpy as np
import pytest

from _fixtures import AVERAGE_STACK, small_problem

pytestmark = pytest.mark.gpu


def _state(model):
    return [t.clone() for t in (model.params, model.adam_m, model.adam_v, model.beta_powers,
                                model.grad, model.loss_buf)]


@pytest.mark.parametrize('name,classes', [('default', True), ('default', False),
                                          ('average', True), ('attention', True),
                                          ('cap32', False)])
def test_train_step_equals_two_calls(gpu, name, classes):
    import torch
    ov = {'default': {}, 'average': AVERAGE_STACK, 'cap32': {},
          'attention': dict(AVERAGE_STACK, layer_2='Attention:input_dim=16')}[name]
    d = 30 if name == 'cap32' else 10   # cap32: the capacity-32 kernel, two calls inside
    prob = small_problem(n_graphs=40, n_pairs=3001, seed=5, n_lo=2, n_hi=d, n_max=d,
                         flags_overrides=ov)
    ma, ba = prob.make_gpu_model(device=gpu)
    mb, bb = prob.make_gpu_model(device=gpu)
    assert ma.kernel_path == (2 if name == 'cap32' else 1)
    if classes:
        ma.balance(ba)
        mb.balance(bb)
    for step in range(4):
        seed = 1000 + step
        ma.fwd_bwd(ba, seed=seed)
        ma.apply_adam()
        mb.fwd_bwd_adam(bb, seed=seed)
        torch.cuda.synchronize()
        for k, (x, y) in enumerate(zip(_state(ma), _state(mb))):
            assert torch.equal(x, y), (name, step, k)
        ra, rb = float(ma.reg_buf[0].item()), float(mb.reg_buf[0].item())
        assert abs(ra - rb) <= 1e-6 * max(1.0, abs(ra)), (step, ra, rb)
    assert not torch.equal(ma.params, torch.zeros_like(ma.params))


def test_train_step_matches_train_loop_step(gpu):
    """model.train_step takes sg_train_step when no gradient hook is set; with a hook it
    keeps the separate calls (the hook sits between them)."""
    import torch
    prob = small_problem(n_graphs=30, n_pairs=500, seed=9, n_lo=2, n_hi=10)
    ma, ba = prob.make_gpu_model(device=gpu)
    mb, bb = prob.make_gpu_model(device=gpu)
    calls = []
    mb.grad_hook = lambda m: calls.append(1)
    la = [ma.train_step(ba) for _ in range(3)]
    lb = [mb.train_step(bb) for _ in range(3)]
    assert len(calls) == 3
    assert torch.equal(ma.params, mb.params)
    assert np.allclose(la, lb, rtol=1e-6, atol=0)
