"""The numpy oracle's hand-written backward against an independent torch
autograd restatement of the same TF graph (layers.py / model_mse.py), with
dropout ON (shared counter RNG masks), for every layer stack the engine
supports.  CPU only."""
import numpy as np
import pytest
import torch

from _fixtures import AVERAGE_STACK, small_problem
from oracle import siamese_oracle as O



@pytest.fixture(autouse=True, scope='module')
def _float64_default():
    """float64 for this module's torch restatement only: a module-level
    set_default_dtype would leak into every test collected after it (the GPU tests'
    float32 buffers included)."""
    old = torch.get_default_dtype()
    torch.set_default_dtype(torch.float64)
    yield
    torch.set_default_dtype(old)


def _act(name, x):
    return {'relu': torch.relu, 'identity': lambda v: v, 'sigmoid': torch.sigmoid,
            'tanh': torch.tanh}[name](x)


def torch_forward(spec, P, g, side, pair, seed):
    x = None
    for li, L in enumerate(spec.layers):
        k = L['kind']
        keep = spec.layer_keep(L)
        if k == 'GraphConvolution':
            W = P[(li, 'weights_0')]
            if L['sparse_inputs']:
                m = torch.as_tensor(O.dropout_mask(seed, pair, side, li, g.n, keep))
                X = torch.zeros(g.n, W.shape[0])
                X[torch.arange(g.n), torch.as_tensor(g.types, dtype=torch.long)] = 1.0
                X = X * m[:, None] / keep
                sup = X @ W
            else:
                m = torch.as_tensor(O.dropout_mask(seed, pair, side, li, x.numel(), keep)).reshape(x.shape)
                sup = (x / keep * m) @ W
            out = torch.as_tensor(g.adj) @ sup
            if (li, 'bias') in P:
                out = out + P[(li, 'bias')]
            x = _act(L['act'], out)
        elif k == 'Dense':
            m = torch.as_tensor(O.dropout_mask(seed, pair, side, li, x.numel(), keep)).reshape(x.shape)
            out = (x / keep * m) @ P[(li, 'weights')]
            if (li, 'bias') in P:
                out = out + P[(li, 'bias')]
            x = _act(L['act'], out)
        elif k == 'Padding':
            x = torch.nn.functional.pad(x, (0, 0, 0, L['max_in_dims'] - x.shape[0]),
                                        value=float(L['padding_value']))
        elif k == 'Average':
            x = x.mean(0)
        elif k == 'Attention':
            W = P[(li, 'weights')]
            temp = x.mean(0).reshape(1, -1)
            h = torch.tanh((temp @ W).reshape(-1, 1))
            att = torch.sigmoid(x @ h)
            x = (att.reshape(1, -1) @ x).squeeze()
        else:
            break
    return x


def torch_loss(spec, flat, g1s, g2s, labels, seed):
    P, off = {}, 0
    leaves = []
    for li, name, shape in O.param_shapes(spec):
        n = int(np.prod(shape))
        t = torch.tensor(flat[off:off + n].reshape(shape), requires_grad=True)
        P[(li, name)] = t
        leaves.append(t)
        off += n
    hi = O._head_index(spec)
    H = spec.layers[hi]
    ss = []
    for i, (a, b) in enumerate(zip(g1s, g2s)):
        e1 = torch_forward(spec, P, a, 0, i, seed)
        e2 = torch_forward(spec, P, b, 1, i, seed)
        if H['kind'] == 'Dot':
            ss.append((e1 * e2).sum())
            continue
        keep = spec.layer_keep(H)
        D = H['input_dim']
        m1 = torch.as_tensor(O.dropout_mask(seed, i, 0, hi, D, keep))
        m2 = torch.as_tensor(O.dropout_mask(seed, i, 1, hi, D, keep))
        x1 = (e1.reshape(-1) / keep * m1).reshape(1, -1)
        x2 = (e2.reshape(-1) / keep * m2).reshape(1, -1)
        fm = []
        for k in range(H['feature_map_dim']):
            v = P[(hi, 'weights_V')][k].reshape(1, -1) @ torch.cat([x1.T, x2.T], 0)
            h = ((x1 @ P[(hi, 'weights_W')][:, :, k]) * x2).sum()
            mid = v + h
            if (hi, 'bias') in P:
                mid = mid + P[(hi, 'bias')][k]
            fm.append(mid)
        r = _act(H['inneract'], torch.stack(fm))                 # (K,1,1)
        if spec.ntn_mode == 'reference':
            ss.append((P[(hi, 'weights_U')] * r).sum())          # broadcast quirk A1
        else:
            ss.append((P[(hi, 'weights_U')].reshape(-1) * r.reshape(-1)).sum())
    s = torch.stack(ss)
    if spec.final_act == 'sim_kernel':
        yhat = torch.exp(-spec.yeta * s ** 2)
    else:
        yhat = _act(spec.final_act, s)
    y = torch.as_tensor(labels)
    if spec.loss_mode == 'broadcast':
        mse = 0.5 * ((y.reshape(-1, 1) - yhat.reshape(1, -1)) ** 2).sum() / len(ss)
    else:
        mse = 0.5 * ((y - yhat) ** 2).sum() / len(ss)
    wd = sum(spec.weight_decay * 0.5 * (t ** 2).sum() for t in leaves)
    loss = mse + wd
    loss.backward()
    grad = torch.cat([t.grad.reshape(-1) for t in leaves]).numpy()
    return s.detach().numpy(), float(loss), grad


STACKS = {
    'default': {},
    'average': AVERAGE_STACK,
    'attention': dict(AVERAGE_STACK, layer_2='Attention:input_dim=16'),
    'dot': dict(num_layers=5, layer_4='Dot'),
    'dense_after_pad': dict(num_layers=6,
                            layer_3='Padding:max_in_dims=10,padding_value=0',
                            layer_4='Dense:input_dim=1,output_dim=1,dropout=True,act=tanh,bias=True',
                            layer_5='NTN:input_dim=10,feature_map_dim=10,inneract=sigmoid,'
                                    'dropout=True,bias=False'),
    'intended_aligned': dict(ntn_mode='intended', loss_mode='aligned'),
    'sigmoid_final': dict(final_act='sigmoid', dropout=0.0),
}


@pytest.mark.parametrize('name', list(STACKS))
def test_oracle_matches_torch_autograd(name):
    prob = small_problem(n_graphs=8, n_pairs=6, seed=11, flags_overrides=STACKS[name])
    spec = prob.oracle_spec()
    g1, g2 = prob.oracle_graphs()
    flat = prob.params.astype(np.float64)
    res = O.fwd_bwd(spec, flat, g1, g2, prob.labels.astype(np.float64), seed=99)
    s_t, loss_t, grad_t = torch_loss(spec, flat, g1, g2, prob.labels.astype(np.float64), 99)
    np.testing.assert_allclose(res.s, s_t, rtol=1e-12, atol=1e-12)
    assert abs(res.loss - loss_t) < 1e-10 * max(1, abs(loss_t))
    np.testing.assert_allclose(res.grad, grad_t, rtol=1e-9, atol=1e-11)


def test_oracle_finite_difference():
    prob = small_problem(n_graphs=6, n_pairs=4, seed=3, flags_overrides=dict(dropout=0.0))
    spec = prob.oracle_spec()
    g1, g2 = prob.oracle_graphs()
    flat = prob.params.astype(np.float64)
    y = prob.labels.astype(np.float64)
    res = O.fwd_bwd(spec, flat, g1, g2, y, seed=1)
    rng = np.random.default_rng(0)
    for idx in rng.choice(flat.size, 25, replace=False):
        e = np.zeros_like(flat)
        e[idx] = 1e-6
        lp = O.fwd_bwd(spec, flat + e, g1, g2, y, seed=1).loss
        lm = O.fwd_bwd(spec, flat - e, g1, g2, y, seed=1).loss
        fd = (lp - lm) / 2e-6
        assert abs(fd - res.grad[idx]) < 1e-6 + 1e-4 * abs(fd), (idx, fd, res.grad[idx])


def test_broadcast_loss_closed_form():
    # l2_loss((B,1) - (B,)) / B  ==  ½Σ(ŷ-ȳ)² + ½Σ(y-ȳ)²   (model_mse.py:148-151, quirk A2)
    rng = np.random.default_rng(1)
    y, yhat = rng.random(7), rng.random(7)
    direct = 0.5 * np.sum((y[:, None] - yhat[None, :]) ** 2) / 7
    closed = 0.5 * np.sum((yhat - y.mean()) ** 2) + 0.5 * np.sum((y - y.mean()) ** 2)
    assert abs(direct - closed) < 1e-13


def test_ntn_broadcast_quirk():
    # layers.py:305-308: reduce_sum(U(K,1) * stack(K,1,1)) == ΣU · Σr
    rng = np.random.default_rng(2)
    U, r = rng.random((10, 1)), rng.random((10, 1, 1))
    assert abs(np.sum(U * r) - U.sum() * r.sum()) < 1e-12
    assert abs(np.sum(U * r) - float(U[:, 0] @ r[:, 0, 0])) > 1e-3


def test_dropout_mask_statistics_and_determinism():
    m = O.dropout_mask(123, 7, 1, 2, 200000, 0.9)
    assert abs(m.mean() - 0.9) < 0.003
    assert np.array_equal(m, O.dropout_mask(123, 7, 1, 2, 200000, 0.9))
    assert not np.array_equal(m[:1000], O.dropout_mask(123, 8, 1, 2, 1000, 0.9))
    assert O.dropout_mask(5, 1, 0, 0, 50, 1.0).all()
    assert O.keep_threshold(0.9) == 58982


def test_adam_tf_form():
    st = O.adam_init(3)
    p = np.array([1.0, -2.0, 0.5])
    g = np.array([0.1, -0.2, 0.0])
    p1 = O.adam_tf_step(p, g, st, lr=0.01)
    # first step: alpha = lr*sqrt(1-b2)/(1-b1); m = 0.1 g; v = 0.001 g²
    alpha = 0.01 * np.sqrt(1 - 0.999) / (1 - 0.9)
    exp = p - alpha * (0.1 * g) / (np.sqrt(0.001 * g * g) + 1e-8)
    np.testing.assert_allclose(p1, exp, rtol=1e-12)
    assert abs(st.beta1_power - float(np.float32(0.9) * np.float32(0.9))) < 1e-9
