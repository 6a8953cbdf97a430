"""Shared test fixtures: small synthetic AIDS-shaped problems, the oracle twin
of the GPU model, and helpers to run both on identical inputs."""
from __future__ import annotations

import os
import sys
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from graphembedding_amd.config import Flags  # noqa: E402
from graphembedding_amd.data import synthetic_graph  # noqa: E402
from graphembedding_amd.graphs import ModelGraph, NodeFeatureOneHotEncoder  # noqa: E402
from graphembedding_amd.layers_factory import create_layers  # noqa: E402
from graphembedding_amd.model_mse import glorot_flat  # noqa: E402
from graphembedding_amd.packer import GraphStore  # noqa: E402
from oracle import siamese_oracle as O  # noqa: E402

AVERAGE_STACK = dict(
    num_layers=4,
    layer_0='GraphConvolution:output_dim=32,act=relu,dropout=True,bias=True,sparse_inputs=True',
    layer_1='GraphConvolution:input_dim=32,output_dim=16,act=identity,dropout=True,bias=True,'
            'sparse_inputs=False',
    layer_2='Average',
    layer_3='NTN:input_dim=16,feature_map_dim=10,inneract=relu,dropout=True,bias=True')


@dataclass
class Problem:
    flags: Flags
    graphs: list                    # networkx graphs
    mgs: List[ModelGraph]
    d_in: int
    n_max: int
    pairs: np.ndarray               # [P, 2] graph indices
    labels: np.ndarray              # [P] float32 similarities
    params: np.ndarray              # float32 flat
    layers: list = field(default_factory=list)

    def oracle_spec(self) -> O.OracleSpec:
        f = self.flags
        return O.OracleSpec(layers=self.layers, d_in=self.d_in, keep_prob=1.0 - f.dropout,
                            final_act=f.final_act, sim_kernel=f.sim_kernel, yeta=f.yeta,
                            loss_mode=f.loss_mode, ntn_mode=f.ntn_mode,
                            weight_decay=f.weight_decay, dist_norm=f.dist_norm)

    def oracle_graphs(self):
        from graphembedding_amd.packer import bf16_round
        rd = getattr(self.flags, 'record_dtype', 'f32')
        # bf16 records store Â rounded to bf16 (RNE); the kernels compute with that Â
        cast = (lambda a: bf16_round(a.astype(np.float32))) if rd == 'bf16' else \
            (lambda a: a.astype(np.float32))
        gs = [O.Graph(adj=cast(m.adj).astype(np.float64), types=m.types) for m in self.mgs]
        return [gs[i] for i in self.pairs[:, 0]], [gs[j] for j in self.pairs[:, 1]]

    def store(self) -> GraphStore:
        return GraphStore(self.mgs, self.n_max, self.d_in)

    def make_gpu_model(self, device='cuda'):
        from graphembedding_amd.model_mse import SiameseGCNTNMSE
        import torch
        model = SiameseGCNTNMSE(self.d_in, self.flags, device=device, n_max=self.n_max,
                                params=self.params)
        # records at the model's node capacity (the fused kernels pick their own)
        words = GraphStore(self.mgs, model.n_max, self.d_in).pack_host(
            self.pairs, self.labels, dtype=model.record_dtype)
        recs = torch.from_numpy(words.view(np.int32).reshape(-1)).to(device)
        batch = model.batch_from_records(recs, len(self.pairs), self.labels)
        return model, batch

    def make_gpu_web_model(self, device='cuda', chunk=None):
        """Graph-store path (kernel path 3): CSR store + pair ids instead of records."""
        from graphembedding_amd.model_mse import SiameseGCNTNMSE
        model = SiameseGCNTNMSE(self.d_in, self.flags, device=device, n_max=self.n_max,
                                params=self.params)
        assert model.is_web, model.kernel_path
        batch = model.make_web_batch([self.mgs[i] for i in self.pairs[:, 0]],
                                     [self.mgs[j] for j in self.pairs[:, 1]], self.labels,
                                     chunk=chunk)
        return model, batch


def small_problem(n_graphs=12, n_pairs=24, seed=5, n_lo=3, n_hi=10, n_max=10, n_types=29,
                  flags_overrides=None, all_types=True, p_extra=0.15) -> Problem:
    rng = np.random.default_rng(seed)
    graphs = []
    for gid in range(n_graphs):
        n = int(rng.integers(n_lo, n_hi + 1))
        graphs.append(synthetic_graph(rng, n, gid, n_types, p_extra=p_extra))
    enc = NodeFeatureOneHotEncoder(graphs, 'type').pin_sorted()
    mgs = [ModelGraph(g, enc) for g in graphs]
    ov = dict(flags_overrides or {})
    if n_max != 10 and 'layer_3' not in ov and ov.get('num_layers', 5) == 5:
        ov['layer_3'] = 'Padding:max_in_dims={},padding_value=0'.format(n_max)
        ov['layer_4'] = 'NTN:input_dim={},feature_map_dim=10,inneract=relu,dropout=True,' \
                        'bias=True'.format(n_max)
    flags = Flags(**ov)
    d_in = enc.input_dim()
    layers = create_layers(flags, d_in)
    pairs = rng.integers(0, n_graphs, size=(n_pairs, 2)).astype(np.int32)
    d = rng.integers(0, 8, size=n_pairs)
    nn = np.array([graphs[i].number_of_nodes() + graphs[j].number_of_nodes() for i, j in pairs])
    labels = np.exp(-flags.yeta * (2.0 * d / nn) ** 2).astype(np.float32)
    params = glorot_flat(layers, d_in, seed + 1)
    # non-zero biases so bias paths are exercised
    params = params + np.float32(0.05) * rng.standard_normal(params.shape).astype(np.float32)
    return Problem(flags=flags, graphs=graphs, mgs=mgs, d_in=d_in, n_max=n_max, pairs=pairs,
                   labels=labels, params=params.astype(np.float32), layers=layers)


def run_oracle_step(prob: Problem, seed: int, adam: bool = True):
    spec = prob.oracle_spec()
    g1, g2 = prob.oracle_graphs()
    flat = prob.params.astype(np.float64)
    res = O.fwd_bwd(spec, flat, g1, g2, prob.labels.astype(np.float64), seed)
    if adam:
        st = O.adam_init(flat.size)
        res.new_params = O.adam_tf_step(flat, res.grad, st, lr=prob.flags.learning_rate)
    return res


def check_grad_per_var(g_gpu, g_ref, layers, d_in, tol=1e-4, what=''):
    """Per-variable gradient check: every variable of the flat gradient (the
    reference's variable order, model_mse.param_shapes) must match within `tol` x the
    largest |component| of that variable's own reference gradient — a few-percent error
    in a small-magnitude tensor (NTN bias, U, b1) cannot hide behind the largest one.
    The floor (1e-7 x the global max) only keeps an all-zero variable from dividing by
    zero.  Returns {variable: relative error} for reporting."""
    from graphembedding_amd.model_mse import param_shapes
    g_gpu = np.asarray(g_gpu, np.float64).reshape(-1)
    g_ref = np.asarray(g_ref, np.float64).reshape(-1)
    assert g_gpu.shape == g_ref.shape, (g_gpu.shape, g_ref.shape)
    floor = 1e-7 * max(float(np.abs(g_ref).max()), 1e-30)
    off, rel, bad = 0, {}, []
    for li, name, shape in param_shapes(layers, d_in):
        n = int(np.prod(shape))
        a, b = g_gpu[off:off + n], g_ref[off:off + n]
        scale = max(float(np.abs(b).max()), floor)
        r = float(np.abs(a - b).max()) / scale
        key = '{}.{}'.format(li, name)
        rel[key] = r
        if not r <= tol:
            bad.append((key, r, scale))
        off += n
    assert off == g_ref.size
    assert not bad, '{} per-variable gradient errors above {}: {}'.format(what, tol, bad)
    return rel
