"""TEST INFRASTRUCTURE ONLY — float64 numpy restatement of the reference's
Siamese GCN → pooling → NTN → Gaussian similarity → MSE path.

Every function cites the reference file:line it restates (paths relative to
/root/reference).  Parity status: graph preprocessing / sampler / kernels are
pinned by tests/golden (generated from the reference's own importable modules);
the TF layer arithmetic is "parity unpinned" by TF itself (TF absent here) and is
cross-checked against torch autograd and finite differences in tests/.

The dropout masks are NOT TF's (TF 1.x used an unseeded RNG, `layers.py:332-338`,
`tf.nn.dropout`), they come from the counter-based hash below, which the HIP
kernels implement bit-exactly, so that dropout-on runs are comparable too.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np

# ----------------------------------------------------------------------------
# Counter-based dropout RNG (shared bit-exactly with graphembedding_amd/csrc)
# ----------------------------------------------------------------------------
_M32 = 0xFFFFFFFF


def sg_mix(x):
    """24-bit-multiply variant of Wellons' lowbias32 mixer (uint64 arrays holding
    u32): both multiplies take the low 24 bits of x, i.e. the gfx950
    full-rate v_mul_u32_u24 instruction."""
    x = np.asarray(x, dtype=np.uint64) & _M32
    x ^= x >> np.uint64(16)
    x = ((x & np.uint64(0xFFFFFF)) * np.uint64(0x7FEB35)) & _M32
    x ^= x >> np.uint64(15)
    x = ((x & np.uint64(0xFFFFFF)) * np.uint64(0x846CA7)) & _M32
    x ^= x >> np.uint64(16)
    return x


def seed_key(seed: int) -> int:
    lo = seed & _M32
    hi = (seed >> 32) & _M32
    return ((lo * 0x85EBCA6B) & _M32) ^ hi


def keep_threshold(keep: float) -> int:
    """16-bit keep threshold; 65536 means "always keep"."""
    if keep >= 1.0:
        return 65536
    return int(min(65536, max(0, round(keep * 65536.0))))


def dropout_mask(seed: int, pair: int, side: int, layer: int, count: int,
                 keep: float) -> np.ndarray:
    """Keep-mask (bool[count]) of one dropout site.

    Replaces TF's `floor(keep_prob + random_uniform(shape))` (layers.py:334-336,
    tf.nn.dropout) with draw(seed, pair, side, layer, e) < round(keep*65536), where
    e is the row-major element index of the logical (unpadded) tensor of one side.
    One hash sg_mix(pk ^ (layer << 26 | e)) serves the element e of both sides:
    its low 16 bits are side 0's draw, its high 16 bits side 1's.
    """
    if keep >= 1.0:
        return np.ones(count, dtype=bool)
    assert count <= (1 << 26)
    thr = keep_threshold(keep)
    pk = sg_mix(np.uint64((pair & _M32) ^ seed_key(seed)))
    e = np.arange(count, dtype=np.uint64)
    ctr = (np.uint64(layer) << np.uint64(26)) | e
    h = sg_mix(ctr ^ pk)
    draw = (h >> np.uint64(16 * int(side))) & np.uint64(0xFFFF)
    return draw < np.uint64(thr)


# ----------------------------------------------------------------------------
# Activations (layers_factory.py:101-127)
# ----------------------------------------------------------------------------
def _act(name: str, x):
    if name == 'relu':
        return np.maximum(x, 0.0)
    if name == 'identity':
        return x
    if name == 'sigmoid':
        return 1.0 / (1.0 + np.exp(-x))
    if name == 'tanh':
        return np.tanh(x)
    raise RuntimeError('Unknown activation function {}'.format(name))


def _act_grad(name: str, pre, out, g):
    """TF gradients: ReluGrad uses (features > 0) (relu'(0) = 0)."""
    if name == 'relu':
        return g * (pre > 0)
    if name == 'identity':
        return g
    if name == 'sigmoid':
        return g * out * (1.0 - out)
    if name == 'tanh':
        return g * (1.0 - out * out)
    raise RuntimeError('Unknown activation function {}'.format(name))


# ----------------------------------------------------------------------------
# Model spec
# ----------------------------------------------------------------------------
@dataclass
class OracleSpec:
    """Plain-data model description (the layer list of config.py:44-66)."""
    layers: List[dict]
    d_in: int
    keep_prob: float = 0.9            # 1 - FLAGS.dropout (config.py:104)
    final_act: str = 'sim_kernel'     # config.py:83
    sim_kernel: str = 'gaussian'      # config.py:77
    yeta: float = 0.6                 # config.py:81
    loss_mode: str = 'broadcast'      # 'broadcast' = reference quirk A2; 'aligned'
    ntn_mode: str = 'reference'       # 'reference' = broadcast quirk A1; 'intended'
    weight_decay: float = 5e-4        # config.py:105
    dist_norm: bool = True            # config.py:73

    def layer_keep(self, layer: dict) -> float:
        # layers.py:45-49: dropout=True -> FLAGS.dropout, else 0.
        return self.keep_prob if layer.get('dropout', False) else 1.0


def param_shapes(spec: OracleSpec) -> List[Tuple[int, str, Tuple[int, ...]]]:
    """(layer index, var name, shape) in model variable order (layers.py:68-73,
    151-152, 174-178, 268-277)."""
    out = []
    for li, L in enumerate(spec.layers):
        k = L['kind']
        if k == 'GraphConvolution':
            din = L['input_dim'] if L.get('input_dim') else spec.d_in
            out.append((li, 'weights_0', (din, L['output_dim'])))
            if L['bias']:
                out.append((li, 'bias', (L['output_dim'],)))
        elif k == 'Dense':
            out.append((li, 'weights', (L['input_dim'], L['output_dim'])))
            if L['bias']:
                out.append((li, 'bias', (L['output_dim'],)))
        elif k == 'Attention':
            out.append((li, 'weights', (L['input_dim'], L['input_dim'])))
        elif k == 'NTN':
            D, K = L['input_dim'], L['feature_map_dim']
            out.append((li, 'weights_W', (D, D, K)))
            out.append((li, 'weights_V', (K, 2 * D)))
            out.append((li, 'weights_U', (K, 1)))
            if L['bias']:
                out.append((li, 'bias', (K,)))
    return out


def n_params(spec: OracleSpec) -> int:
    return int(sum(int(np.prod(s)) for _, _, s in param_shapes(spec)))


def unflatten(spec: OracleSpec, flat: np.ndarray) -> Dict[Tuple[int, str], np.ndarray]:
    p, off = {}, 0
    for li, name, shape in param_shapes(spec):
        sz = int(np.prod(shape))
        p[(li, name)] = np.asarray(flat[off:off + sz], dtype=np.float64).reshape(shape)
        off += sz
    assert off == len(flat)
    return p


def flatten(spec: OracleSpec, p: Dict[Tuple[int, str], np.ndarray]) -> np.ndarray:
    return np.concatenate([np.asarray(p[(li, name)], dtype=np.float64).ravel()
                           for li, name, _ in param_shapes(spec)])


def glorot_init(spec: OracleSpec, seed: int = 0) -> np.ndarray:
    """inits.py:11-21 (glorot uses shape[0], shape[1] only; zeros for biases)."""
    rng = np.random.default_rng(seed)
    parts = []
    for li, name, shape in param_shapes(spec):
        if name == 'bias':
            parts.append(np.zeros(shape))
        else:
            r = math.sqrt(6.0 / (shape[0] + shape[1]))
            parts.append(rng.uniform(-r, r, size=shape))
    return np.concatenate([x.ravel() for x in parts]).astype(np.float32).astype(np.float64)


# ----------------------------------------------------------------------------
# Per-graph / per-pair forward + backward
# ----------------------------------------------------------------------------
@dataclass
class Graph:
    """One preprocessed graph: Â (graphs.py:64-76) and one-hot type columns
    (graphs.py:55-62, 98-111)."""
    adj: np.ndarray    # [n, n] float (D^-1/2 (A+I) D^-1/2)
    types: np.ndarray  # [n] int  (column of the one-hot row; row value 1.0)

    @property
    def n(self) -> int:
        return int(self.types.shape[0])


def _node_forward(spec: OracleSpec, P, g: Graph, side: int, pair: int, seed: int):
    """Node-level stack + pooling for one graph instance (layers.py:91-227)."""
    x = None          # current tensor (rows x D); None = sparse one-hot X
    rows = g.n
    caches = []
    for li, L in enumerate(spec.layers):
        k = L['kind']
        keep = spec.layer_keep(L)
        if k == 'GraphConvolution':
            W = P[(li, 'weights_0')]
            b = P.get((li, 'bias'))
            if L['sparse_inputs']:
                # sparse_dropout over the nnz of X (layers.py:97-98, 332-338);
                # num_features_nonzero = (N,) (graphs.py:49-50), one nnz per row.
                if x is not None:
                    raise RuntimeError('sparse_inputs GCN must be the first layer')
                m = dropout_mask(seed, pair, side, li, rows, keep)
                scale = np.where(m, 1.0 / keep, 0.0)
                pre_sup = W[g.types] * scale[:, None]           # X·W (row gather)
                cache = dict(kind=k, li=li, scale=scale)
            else:
                m = dropout_mask(seed, pair, side, li, x.size, keep).reshape(x.shape)
                xd = np.where(m, x / keep, 0.0)                  # layers.py:100
                pre_sup = xd @ W
                cache = dict(kind=k, li=li, xd=xd, m=m, keep=keep)
            pre = g.adj @ pre_sup                                # layers.py:110
            if b is not None:
                pre = pre + b
            out = _act(L['act'], pre)
            cache.update(pre=pre, out=out, act=L['act'])
            caches.append(cache)
            x = out
        elif k == 'Dense':
            W = P[(li, 'weights')]
            b = P.get((li, 'bias'))
            m = dropout_mask(seed, pair, side, li, x.size, keep).reshape(x.shape)
            xd = np.where(m, x / keep, 0.0)                      # layers.py:196
            pre = xd @ W
            if b is not None:
                pre = pre + b
            out = _act(L['act'], pre)
            caches.append(dict(kind=k, li=li, xd=xd, m=m, keep=keep, pre=pre, out=out, act=L['act']))
            x = out
        elif k == 'Padding':
            P_ = L['max_in_dims']
            if x.shape[0] > P_:
                # tf.pad with a negative padding raises (layers.py:226, quirk A9)
                raise RuntimeError('Padding: {} rows > max_in_dims {}'.format(x.shape[0], P_))
            out = np.full((P_, x.shape[1]), float(L.get('padding_value', 0)))
            out[:x.shape[0]] = x
            caches.append(dict(kind=k, li=li, rows=x.shape[0]))
            x = out
        elif k == 'Average':
            caches.append(dict(kind=k, li=li, rows=x.shape[0]))
            x = x.mean(axis=0)                                   # layers.py:136-140
        elif k == 'Attention':
            W = P[(li, 'weights')]
            temp = x.mean(axis=0).reshape(1, -1)                 # layers.py:154-160
            h = np.tanh((temp @ W).reshape(-1, 1))
            att = 1.0 / (1.0 + np.exp(-(x @ h)))                 # (rows, 1)
            out = (att.reshape(1, -1) @ x).reshape(-1)
            caches.append(dict(kind=k, li=li, x=x, temp=temp, h=h, att=att))
            x = out
        elif k in ('NTN', 'Dot'):
            break
        else:
            raise RuntimeError('Unknown layer {}'.format(k))
    return x, caches


def _node_backward(spec: OracleSpec, P, G, g: Graph, caches, gx):
    """Reverse of _node_forward; accumulates into G (dict like P)."""
    for c in reversed(caches):
        k, li = c['kind'], c['li']
        if k == 'GraphConvolution':
            gpre = _act_grad(c['act'], c['pre'], c['out'], gx)
            if (li, 'bias') in P:
                G[(li, 'bias')] += gpre.sum(axis=0)
            gsup = g.adj.T @ gpre                                # adjoint of sparse matmul
            if 'scale' in c:                                     # sparse one-hot input
                contrib = gsup * c['scale'][:, None]
                np.add.at(G[(li, 'weights_0')], g.types, contrib)
                gx = None
            else:
                W = P[(li, 'weights_0')]
                G[(li, 'weights_0')] += c['xd'].T @ gsup
                gxd = gsup @ W.T
                gx = np.where(c['m'], gxd / c['keep'], 0.0)
        elif k == 'Dense':
            gpre = _act_grad(c['act'], c['pre'], c['out'], gx)
            if (li, 'bias') in P:
                G[(li, 'bias')] += gpre.sum(axis=0)
            W = P[(li, 'weights')]
            G[(li, 'weights')] += c['xd'].T @ gpre
            gxd = gpre @ W.T
            gx = np.where(c['m'], gxd / c['keep'], 0.0)
        elif k == 'Padding':
            gx = gx[:c['rows']]
        elif k == 'Average':
            gx = np.tile(gx / c['rows'], (c['rows'], 1))
        elif k == 'Attention':
            W = P[(li, 'weights')]
            x, temp, h, att = c['x'], c['temp'], c['h'], c['att']
            gout = gx.reshape(1, -1)                             # out = attᵀ x
            gatt = (gout @ x.T).reshape(-1, 1)                   # (rows, 1)
            gx_direct = att.reshape(-1, 1) @ gout                # (rows, D)
            gz = gatt * att * (1.0 - att)                        # sigmoid'
            gh = x.T @ gz                                        # (D, 1)
            gx_att = gz @ h.T                                    # (rows, D)
            gu = (gh.reshape(1, -1)) * (1.0 - h.reshape(1, -1) ** 2)  # tanh'
            G[(li, 'weights')] += temp.T @ gu
            gtemp = gu @ W.T                                     # (1, D)
            gx = gx_direct + gx_att + np.tile(gtemp / x.shape[0], (x.shape[0], 1))
    return gx


def _head_index(spec: OracleSpec) -> int:
    for li, L in enumerate(spec.layers):
        if L['kind'] in ('NTN', 'Dot'):
            return li
    raise RuntimeError('model has no pair head (NTN or Dot)')


def pair_forward(spec: OracleSpec, P, g1: Graph, g2: Graph, pair: int, seed: int):
    """One input pair through the Siamese model (models.py:39-65,
    model_mse.py:117-126 pairs ins[i] with ins[i+B]). Returns (s, cache)."""
    e1, c1 = _node_forward(spec, P, g1, 0, pair, seed)
    e2, c2 = _node_forward(spec, P, g2, 1, pair, seed)
    hi = _head_index(spec)
    L = spec.layers[hi]
    if L['kind'] == 'Dot':
        if e1.shape != e2.shape:
            raise RuntimeError('Dot: shape mismatch {} vs {}'.format(e1.shape, e2.shape))
        s = float(np.sum(e1 * e2))                               # layers.py:249-252
        return s, dict(kind='Dot', e1=e1, e2=e2, c1=c1, c2=c2)
    # NTN (layers.py:282-310)
    keep = spec.layer_keep(L)
    D, K = L['input_dim'], L['feature_map_dim']
    f1, f2 = e1.reshape(-1), e2.reshape(-1)
    if f1.size != D or f2.size != D:
        raise RuntimeError('NTN input_dim {} != {}'.format(D, f1.size))
    m1 = dropout_mask(seed, pair, 0, hi, D, keep)
    m2 = dropout_mask(seed, pair, 1, hi, D, keep)
    x1 = np.where(m1, f1 / keep, 0.0)
    x2 = np.where(m2, f2 / keep, 0.0)
    W = P[(hi, 'weights_W')]
    V = P[(hi, 'weights_V')]
    U = P[(hi, 'weights_U')][:, 0]
    b = P.get((hi, 'bias'))
    x12 = np.concatenate([x1, x2])
    u = np.einsum('abk,b->ak', W, x2)                            # W[:,:,k] x2
    m = V @ x12 + np.einsum('a,ak->k', x1, u)
    if b is not None:
        m = m + b
    r = _act(L['inneract'], m)
    if spec.ntn_mode == 'reference':
        s = float(U.sum() * r.sum())                             # quirk A1 (layers.py:305-308)
    else:
        s = float(U @ r)
    return s, dict(kind='NTN', hi=hi, e1=e1, e2=e2, c1=c1, c2=c2, m1=m1, m2=m2,
                   keep=keep, x1=x1, x2=x2, u=u, m=m, r=r)


def pair_backward(spec: OracleSpec, P, G, g1: Graph, g2: Graph, cache, gs: float):
    if cache['kind'] == 'Dot':
        ge1 = gs * cache['e2']
        ge2 = gs * cache['e1']
    else:
        hi = cache['hi']
        L = spec.layers[hi]
        W = P[(hi, 'weights_W')]
        V = P[(hi, 'weights_V')]
        U = P[(hi, 'weights_U')][:, 0]
        x1, x2, u, m, r = cache['x1'], cache['x2'], cache['u'], cache['m'], cache['r']
        D = x1.size
        if spec.ntn_mode == 'reference':
            G[(hi, 'weights_U')][:, 0] += gs * r.sum()
            gr = gs * U.sum() * np.ones_like(r)
        else:
            G[(hi, 'weights_U')][:, 0] += gs * r
            gr = gs * U
        gm = _act_grad(L['inneract'], m, r, gr)
        if (hi, 'bias') in P:
            G[(hi, 'bias')] += gm
        x12 = np.concatenate([x1, x2])
        G[(hi, 'weights_V')] += np.outer(gm, x12)
        G[(hi, 'weights_W')] += np.einsum('a,b,k->abk', x1, x2, gm)
        gx12 = V.T @ gm
        gx1 = gx12[:D] + u @ gm
        gx2 = gx12[D:] + np.einsum('a,abk,k->b', x1, W, gm)
        keep = cache['keep']
        ge1 = np.where(cache['m1'], gx1 / keep, 0.0).reshape(cache['e1'].shape)
        ge2 = np.where(cache['m2'], gx2 / keep, 0.0).reshape(cache['e2'].shape)
    _node_backward(spec, P, G, g1, cache['c1'], ge1)
    _node_backward(spec, P, G, g2, cache['c2'], ge2)


# ----------------------------------------------------------------------------
# Final activation, labels, loss (similarity.py:44-60, model_mse.py:145-151)
# ----------------------------------------------------------------------------
def sim_kernel_np(spec: OracleSpec, d):
    if spec.sim_kernel == 'gaussian':
        return np.exp(-spec.yeta * np.square(d))                 # similarity.py:55-56
    if spec.sim_kernel == 'identity':
        return d
    raise RuntimeError('Unknown sim kernel {}'.format(spec.sim_kernel))


def final_act(spec: OracleSpec, s):
    if spec.final_act == 'sim_kernel':
        return sim_kernel_np(spec, s)
    return _act(spec.final_act, s)


def final_act_grad(spec: OracleSpec, s, yhat):
    fa = spec.final_act
    if fa == 'sim_kernel':
        if spec.sim_kernel == 'gaussian':
            return -2.0 * spec.yeta * s * yhat
        return np.ones_like(s)
    if fa == 'identity':
        return np.ones_like(s)
    if fa == 'relu':
        return (s > 0).astype(np.float64)
    if fa == 'sigmoid':
        return yhat * (1.0 - yhat)
    if fa == 'tanh':
        return 1.0 - yhat * yhat
    raise RuntimeError('Unknown activation function {}'.format(fa))


def labels_from_dists(spec: OracleSpec, dists, norm_dists):
    """model_mse.py:146 + similarity.py:58-60: y = kernel(norm_d or d)."""
    d = norm_dists if spec.dist_norm else dists
    return sim_kernel_np(spec, np.asarray(d, dtype=np.float64))


def weight_decay_loss(spec: OracleSpec, flat: np.ndarray) -> float:
    """models.py:69-73: wd * l2_loss(var) summed over every var (quirk A10)."""
    return float(spec.weight_decay * 0.5 * np.sum(np.asarray(flat, np.float64) ** 2))


@dataclass
class StepResult:
    s: np.ndarray          # [B] pre-activation scores (pred_sim_without_act)
    yhat: np.ndarray       # [B] final_act(s)
    loss: float            # full loss incl. weight decay (models.py:67-88)
    loss_mse: float
    grad_mse: np.ndarray   # d loss_mse / d params (flat)
    grad: np.ndarray       # grad_mse + wd * params (what Adam consumes)


def forward(spec: OracleSpec, flat: np.ndarray, g1s: Sequence[Graph], g2s: Sequence[Graph],
            seed: int, pair_offset: int = 0) -> np.ndarray:
    P = unflatten(spec, flat)
    return np.array([pair_forward(spec, P, a, b, pair_offset + i, seed)[0]
                     for i, (a, b) in enumerate(zip(g1s, g2s))])


def fwd_bwd(spec: OracleSpec, flat: np.ndarray, g1s: Sequence[Graph], g2s: Sequence[Graph],
            labels: np.ndarray, seed: int, pair_offset: int = 0,
            y_mean: Optional[float] = None) -> StepResult:
    """One training batch (train.py:88-93 'train' objs, without the update)."""
    P = unflatten(spec, flat)
    G = {k: np.zeros_like(v) for k, v in P.items()}
    B = len(g1s)
    y = np.asarray(labels, dtype=np.float64)
    caches, s = [], np.zeros(B)
    for i, (a, b) in enumerate(zip(g1s, g2s)):
        s[i], c = pair_forward(spec, P, a, b, pair_offset + i, seed)
        caches.append(c)
    yhat = final_act(spec, s)
    if spec.loss_mode == 'broadcast':
        # l2_loss((B,1) - (B,)) / B == 1/2 sum_j (yhat_j - ybar)^2 + 1/2 sum_i (y_i - ybar)^2
        ybar = float(y.mean()) if y_mean is None else float(y_mean)
        loss_mse = 0.5 * np.sum((yhat - ybar) ** 2) + 0.5 * np.sum((y - ybar) ** 2)
        gyhat = yhat - ybar
    elif spec.loss_mode == 'aligned':
        loss_mse = 0.5 * np.sum((y - yhat) ** 2) / B
        gyhat = (yhat - y) / B
    else:
        raise RuntimeError('Unknown loss mode {}'.format(spec.loss_mode))
    gs = gyhat * final_act_grad(spec, s, yhat)
    for i, (a, b) in enumerate(zip(g1s, g2s)):
        pair_backward(spec, P, G, a, b, caches[i], float(gs[i]))
    grad_mse = flatten(spec, G)
    grad = grad_mse + spec.weight_decay * np.asarray(flat, np.float64)
    loss = float(loss_mse) + weight_decay_loss(spec, flat)
    return StepResult(s=s, yhat=yhat, loss=loss, loss_mse=float(loss_mse),
                      grad_mse=grad_mse, grad=grad)


# ----------------------------------------------------------------------------
# Adam, TF ApplyAdam form (models.py:28-29,36; quirk A13)
# ----------------------------------------------------------------------------
@dataclass
class AdamState:
    m: np.ndarray
    v: np.ndarray
    beta1_power: float
    beta2_power: float


def adam_init(n: int, beta1=0.9, beta2=0.999) -> AdamState:
    return AdamState(np.zeros(n), np.zeros(n), beta1, beta2)


def adam_tf_step(params, grad, st: AdamState, lr=0.01, beta1=0.9, beta2=0.999, eps=1e-8):
    """alpha = lr*sqrt(1-b2^t)/(1-b1^t); m += (g-m)(1-b1); v += (g^2-v)(1-b2);
    var -= alpha*m/(sqrt(v)+eps); then beta powers *= beta (float32 variables)."""
    alpha = lr * math.sqrt(1.0 - st.beta2_power) / (1.0 - st.beta1_power)
    st.m = st.m + (grad - st.m) * (1.0 - beta1)
    st.v = st.v + (grad * grad - st.v) * (1.0 - beta2)
    new = params - alpha * st.m / (np.sqrt(st.v) + eps)
    st.beta1_power = float(np.float32(st.beta1_power) * np.float32(beta1))
    st.beta2_power = float(np.float32(st.beta2_power) * np.float32(beta2))
    return new


def adam_tf_step_f32(params, grad_mse, st: AdamState, lr=0.01, beta1=0.9, beta2=0.999,
                     eps=1e-8, weight_decay=0.0):
    """The same update in float32 arithmetic, as the reference trains (TF fp32 variables,
    models.py:28-36).  Restates TF 1.x's CPU ApplyAdam functor (training_ops.cc, the
    non-Nesterov branch; TF is absent here, version per SURVEY §8(c)):
      alpha = lr*sqrt(1-b2p)/(1-b1p); m += (g-m)*(1-b1); v += (g*g-v)*(1-b2);
      var -= (m*alpha)/(sqrt(v)+eps)
    with g = dL_mse/dvar + wd*var, the AddN of the MSE gradient and l2_loss's gradient
    (models.py:69-74).  st.m / st.v are kept float32."""
    f = np.float32
    th = np.asarray(params, f)
    g = np.asarray(grad_mse, f) + f(weight_decay) * th
    b1p, b2p = f(st.beta1_power), f(st.beta2_power)
    alpha = f(lr) * np.sqrt(f(1) - b2p) / (f(1) - b1p)
    m = np.asarray(st.m, f)
    v = np.asarray(st.v, f)
    m = m + (g - m) * (f(1) - f(beta1))
    v = v + (g * g - v) * (f(1) - f(beta2))
    st.m, st.v = m, v
    st.beta1_power = float(b1p * f(beta1))
    st.beta2_power = float(b2p * f(beta2))
    return th - (m * alpha) / (np.sqrt(v) + f(eps))


# ----------------------------------------------------------------------------
# Default layer stacks (config.py:44-66; tuning.py:74-93)
# ----------------------------------------------------------------------------
def default_layers(n_max: int = 10, ntn_k: int = 10) -> List[dict]:
    return [
        dict(kind='GraphConvolution', input_dim=None, output_dim=32, act='relu',
             dropout=True, bias=True, sparse_inputs=True),
        dict(kind='GraphConvolution', input_dim=32, output_dim=16, act='identity',
             dropout=True, bias=True, sparse_inputs=False),
        dict(kind='Dense', input_dim=16, output_dim=1, act='relu', dropout=True, bias=True),
        dict(kind='Padding', max_in_dims=n_max, padding_value=0),
        dict(kind='NTN', input_dim=n_max, feature_map_dim=ntn_k, inneract='relu',
             dropout=True, bias=True),
    ]


def average_layers(ntn_k: int = 10) -> List[dict]:
    return [
        dict(kind='GraphConvolution', input_dim=None, output_dim=32, act='relu',
             dropout=True, bias=True, sparse_inputs=True),
        dict(kind='GraphConvolution', input_dim=32, output_dim=16, act='identity',
             dropout=True, bias=True, sparse_inputs=False),
        dict(kind='Average'),
        dict(kind='NTN', input_dim=16, feature_map_dim=ntn_k, inneract='relu',
             dropout=True, bias=True),
    ]
