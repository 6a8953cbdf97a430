"""The host mirror against golden fixtures produced by the reference's own
modules (tests/golden/make_golden.py).  CPU only, bit-exact where the
reference computes on the host."""
import json
import os

import networkx as nx
import numpy as np
import pytest

from graphembedding_amd import metrics, similarity
from graphembedding_amd.data import synthetic_graph
from graphembedding_amd.graphs import ModelGraph, NodeFeatureOneHotEncoder
from graphembedding_amd.results import DistanceMatrixResult, SiameseModelResult
from graphembedding_amd.samplers import DistributionSampler, RandomSampler
from graphembedding_amd.utils import sorted_nicely

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def _load(name):
    with open(os.path.join(G, name)) as f:
        return json.load(f)


def _graph(spec):
    g = nx.Graph(gid=spec['gid'])
    for n, t in spec['nodes']:
        g.add_node(n, type=t)
    for u, v, w in spec['edges']:
        if w != 1.0:
            g.add_edge(u, v, weight=w)
        else:
            g.add_edge(u, v)
    return g


def test_f1_preprocessing_bit_exact():
    f1 = _load('f1_preprocess.json')
    arr = np.load(os.path.join(G, 'f1_preprocess.npz'))
    gs = [_graph(s) for s in f1['graphs']]
    enc = NodeFeatureOneHotEncoder(gs, 'type')
    assert enc.input_dim() == f1['input_dim']
    assert set(enc.feat_idx_dic) == set(f1['feat_idx_dic'])
    enc.feat_idx_dic = dict(f1['feat_idx_dic'])   # set order is hash-seed dependent (A7)
    for k, g in enumerate(gs):
        mg = ModelGraph(g, enc)
        ref_adj = arr['adj_%d' % k]
        assert mg.adj.shape == ref_adj.shape
        assert np.array_equal(mg.adj, ref_adj), 'graph %d: Â differs' % k
        assert np.array_equal(mg.adj.astype(np.float32), ref_adj.astype(np.float32))
        assert np.array_equal(enc.encode(g), arr['x_%d' % k])
        assert tuple(mg.get_node_inputs_num_nonzero()) == tuple(arr['nnz_%d' % k])
        # the COO views the reference fed TF
        (c, v, shp) = mg.get_laplacians()[0]
        dense = np.zeros(shp)
        dense[c[:, 0], c[:, 1]] = v
        assert np.array_equal(dense, ref_adj)


def test_f2_random_sampler_streams():
    f2 = _load('f2_samplers.json')
    for n in (52, 420, 7500):
        items = list(range(n))
        s = RandomSampler(items, -1, False)
        got = [list(s.get_pair()) for _ in range(2 * n + 37)]
        assert got == f2['random_%d' % n]
        assert list(s.gs) == f2['random_%d_final_list' % n]   # in-place shuffle (A6)


def test_f2_distribution_sampler_streams():
    f2 = _load('f2_samplers.json')
    rng = np.random.default_rng(7)

    class _G:
        def __init__(self, g, i):
            self.nxgraph = g
            self.i = i
    gs = []
    for gid in range(48):
        gs.append(synthetic_graph(rng, int(rng.integers(3, 13)), gid, 29))
    g = gs[0].copy()
    u, v = next(iter(g.edges()))
    g[u][v]['weight'] = 2.5
    gs.append(g)
    g2 = gs[1].copy()
    g2.add_edge('0', '0')
    gs.append(g2)
    dgs = [_G(x, i) for i, x in enumerate(gs)]
    for num in (-1, 3):
        ds = DistributionSampler(dgs, num, False)
        got = [[a.i, b.i] for a, b in (ds.get_pair() for _ in range(40))]
        assert got == f2['density_%d' % num]


def test_f3_similarity_kernels():
    f3 = _load('f3_similarity.json')
    d = np.array(f3['d'])
    assert np.array_equal(similarity.create_sim_kernel('gaussian', 0.6).dist_to_sim_np(d),
                          np.array(f3['gaussian_0.6']))
    assert np.array_equal(similarity.create_sim_kernel('gaussian', 1.0).dist_to_sim_np(d),
                          np.array(f3['gaussian_1.0']))
    assert list(similarity.create_sim_kernel('identity').dist_to_sim_np(d)) == f3['identity']
    assert similarity.GaussianKernel(0.6).name() == f3['name_0.6']
    assert similarity.GaussianKernel(0.6).shortname() == f3['shortname_0.6']
    assert similarity.GaussianKernel(0.001).name() == f3['name_0.001']
    with pytest.raises(RuntimeError):
        similarity.create_sim_kernel('linear')


def test_f4_metrics_and_result_ranking():
    f4 = _load('f4_metrics.json')
    true_d = np.array(f4['true_dist'])
    pred_s = np.array(f4['pred_sim'])
    true_r = DistanceMatrixResult('syn', 'astar', true_d, true_d * 0.5)
    pred_r = SiameseModelResult('syn', 'siamese_gcntn_mse', sim_mat=pred_s,
                                time_mat=np.zeros_like(pred_s))
    for norm in (False, True):
        np.testing.assert_allclose(metrics.precision_at_ks(true_r, pred_r, norm, f4['ks']),
                                   f4['apk_%s' % norm], rtol=0, atol=0)
        assert metrics.mean_reciprocal_rank(true_r, pred_r, norm) == f4['mrr_%s' % norm]
        assert metrics.mean_squared_error(true_r, pred_r, 'gaussian', 0.6, norm) == \
            f4['mse_%s' % norm]


def test_f5_sorted_nicely():
    f5 = _load('f5_utils.json')
    assert sorted_nicely(f5['in']) == f5['sorted_nicely']
