"""Generate golden fixtures by importing the REFERENCE's own (non-TF) modules
from /root/reference in this container.  Run once; the outputs (.npz/.json) are
committed and travel to the GPU box — the reference itself never does.

  python tests/golden/make_golden.py

Pinned here (reference modules imported read-only, PYTHONDONTWRITEBYTECODE):
  model/Siamese/graphs.py     ModelGraph (Â, X COO tuples), NodeFeatureOneHotEncoder
  model/Siamese/samplers.py   RandomSampler / DistributionSampler pair streams
  src/similarity.py           GaussianKernel / IdentityKernel, create_sim_kernel
  src/metrics.py              precision_at_ks, mean_reciprocal_rank, mean_squared_error
  src/utils.py                sorted_nicely, save (F6: the label-store pickle)
  src/data.py                 AIDS700nefData / AIDS80nefData gexf loaders (F6)
  model/Siamese/samplers.py   list order after the default 20-iteration loop (F7)
Not importable here: TF (absent), src/distance.py and src/results.py (need bs4
via nx_to_gxl.py) — their logic is restated and tested against these fixtures
where it feeds them.
"""
import json
import os
import sys

import numpy as np

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = '/root/reference'
sys.path.insert(0, REF + '/model/Siamese')
sys.path.insert(0, REF + '/src')
sys.path.insert(1, ROOT)

import networkx as nx  # noqa: E402

import graphs as ref_graphs  # noqa: E402  (reference)
import samplers as ref_samplers  # noqa: E402  (reference)
import similarity as ref_similarity  # noqa: E402  (reference)
import metrics as ref_metrics  # noqa: E402  (reference)
import utils as ref_utils  # noqa: E402  (reference)

from graphembedding_amd.data import synthetic_graph  # noqa: E402


def graph_set(seed, count, lo, hi):
    rng = np.random.default_rng(seed)
    gs = []
    for gid in range(count):
        gs.append(synthetic_graph(rng, int(rng.integers(lo, hi + 1)), gid, 29))
    # one weighted graph and one with a self loop to pin nx.adjacency_matrix semantics
    g = gs[0].copy()
    u, v = next(iter(g.edges()))
    g[u][v]['weight'] = 2.5
    g.graph['gid'] = count
    gs.append(g)
    g2 = gs[1].copy()
    g2.add_edge('0', '0')
    g2.graph['gid'] = count + 1
    gs.append(g2)
    return gs


def gexf_like(g):
    return {'gid': g.graph['gid'], 'nodes': [[n, g.nodes[n]['type']] for n in g.nodes()],
            'edges': [[u, v, g[u][v].get('weight', 1.0)] for u, v in g.edges()]}


def main():
    out = {}
    # ---- F1: preprocessing (graphs.py:34-117) ----
    gs = graph_set(seed=2024, count=12, lo=1, hi=12)
    enc = ref_graphs.NodeFeatureOneHotEncoder(gs, 'type')
    f1 = {'graphs': [gexf_like(g) for g in gs], 'feat_idx_dic': enc.feat_idx_dic,
          'input_dim': int(enc.input_dim())}
    arrays = {}
    for k, g in enumerate(gs):
        mg = ref_graphs.ModelGraph(g, enc)
        (xc, xv, xs) = mg.get_node_inputs()
        (ac, av, ash) = mg.get_laplacians()[0]
        dense = np.zeros(ash)
        dense[ac[:, 0], ac[:, 1]] = av
        arrays['adj_%d' % k] = dense
        xd = np.zeros(xs)
        xd[xc[:, 0], xc[:, 1]] = xv
        arrays['x_%d' % k] = xd
        arrays['nnz_%d' % k] = np.array(mg.get_node_inputs_num_nonzero())
    np.savez_compressed(os.path.join(HERE, 'f1_preprocess.npz'), **arrays)
    with open(os.path.join(HERE, 'f1_preprocess.json'), 'w') as f:
        json.dump(f1, f, indent=1, sort_keys=True)

    # ---- F2: pair streams (samplers.py:19-68), B + B*B draws per step (A3) ----
    f2 = {}
    for n in (52, 420, 7500):
        items = list(range(n))
        s = ref_samplers.RandomSampler(items, -1, False)
        f2['random_%d' % n] = [list(s.get_pair()) for _ in range(2 * n + 37)]
        f2['random_%d_final_list' % n] = list(s.gs)

    class _G:  # the density sampler reads g.nxgraph
        def __init__(self, g, i):
            self.nxgraph = g
            self.i = i
    dgs = [_G(g, i) for i, g in enumerate(graph_set(seed=7, count=48, lo=3, hi=12))]
    for num in (-1, 3):
        ds = ref_samplers.DistributionSampler(dgs, num, False)
        f2['density_%d' % num] = [[a.i, b.i] for a, b in (ds.get_pair() for _ in range(40))]
    with open(os.path.join(HERE, 'f2_samplers.json'), 'w') as f:
        json.dump(f2, f)

    # ---- F3: similarity kernels (similarity.py:44-76) ----
    d = np.linspace(0.0, 3.0, 31)
    f3 = {'d': d.tolist(),
          'gaussian_0.6': ref_similarity.create_sim_kernel('gaussian', 0.6).dist_to_sim_np(d).tolist(),
          'gaussian_1.0': ref_similarity.create_sim_kernel('gaussian', 1.0).dist_to_sim_np(d).tolist(),
          'identity': list(ref_similarity.create_sim_kernel('identity').dist_to_sim_np(d)),
          'name_0.6': ref_similarity.GaussianKernel(0.6).name(),
          'shortname_0.6': ref_similarity.GaussianKernel(0.6).shortname(),
          'name_0.001': ref_similarity.GaussianKernel(0.001).name()}
    with open(os.path.join(HERE, 'f3_similarity.json'), 'w') as f:
        json.dump(f3, f)

    # ---- F4: metrics on synthetic result matrices, via duck-typed result objects ----
    from graphembedding_amd.results import DistanceMatrixResult, SiameseModelResult
    rng = np.random.default_rng(11)
    m, n = 6, 25
    true_d = rng.integers(0, 8, size=(m, n)).astype(float)       # GED-like with ties
    pred_s = rng.random((m, n))
    pred_s[:, 3] = pred_s[:, 4]                                    # ties in predictions too
    true_r = DistanceMatrixResult('syn', 'astar', true_d, true_d * 0.5)
    pred_r = SiameseModelResult('syn', 'siamese_gcntn_mse', sim_mat=pred_s,
                                time_mat=rng.random((m, n)))
    ks = [1, 2, 5, 10, 20]
    f4 = {'true_dist': true_d.tolist(), 'pred_sim': pred_s.tolist(), 'ks': ks}
    for norm in (False, True):
        f4['apk_%s' % norm] = ref_metrics.precision_at_ks(true_r, pred_r, norm, ks).tolist()
        f4['mrr_%s' % norm] = float(ref_metrics.mean_reciprocal_rank(true_r, pred_r, norm))
        f4['mse_%s' % norm] = float(ref_metrics.mean_squared_error(true_r, pred_r, 'gaussian', 0.6,
                                                                   norm))
    f4['time'] = float(ref_metrics.average_time(pred_r))
    with open(os.path.join(HERE, 'f4_metrics.json'), 'w') as f:
        json.dump(f4, f)

    # ---- F5: natural sort (utils.py:148-160) ----
    names = ['g10.gexf', 'g2.gexf', 'g1.gexf', 'a100', 'a20', 'a3', '7', '11', 'b']
    with open(os.path.join(HERE, 'f5_utils.json'), 'w') as f:
        json.dump({'in': names, 'sorted_nicely': ref_utils.sorted_nicely(names)}, f)
    print('golden fixtures written to', HERE)


def f6_gexf_tree(root):
    """A small AIDS700nef-shaped gexf tree (data/AIDS700nef/{train,test}/<gid>.gexf):
    84 train + 14 test connected graphs of 3-8 nodes, gids deliberately not in
    lexicographic order (sorted_nicely matters), node ids in a shuffled file order (the
    node order of read_gexf is the file order, quirk A8), and a 'valence' edge attribute
    on some edges (the nef loaders drop it, data.py:80-83,91-93)."""
    rng = np.random.default_rng(606)
    gid = 0
    for split, count in (('train', 84), ('test', 14)):
        d = os.path.join(root, 'AIDS700nef', split)
        os.makedirs(d, exist_ok=True)
        for k in range(count):
            gid += int(rng.integers(1, 40))
            n = int(rng.integers(3, 9))
            g0 = synthetic_graph(rng, n, gid, 29, p_extra=0.2)
            order = [str(v) for v in rng.permutation(n)]
            g = nx.Graph()
            for v in order:
                g.add_node(v, type=g0.nodes[v]['type'], label=v)
            for u, v in g0.edges():
                if rng.random() < 0.5:
                    g.add_edge(u, v, valence=int(rng.integers(1, 3)))
                else:
                    g.add_edge(u, v)
            nx.write_gexf(g, os.path.join(d, '{}.gexf'.format(gid)))


def f6_loaders():
    """F6 (rows f2/f3): the reference's own on-disk loaders and label store.

    f2: gexf files read by the reference's AIDS700nefData / AIDS80nefData
        (src/data.py:62-132, nx.read_gexf + sorted_nicely + connectivity check + valence
        removal; AIDS80nef = Random(123).shuffle then the first 70 / 10), with
        get_data_path / get_save_path pointed at a temporary tree.
    f3: a gid-pair distance map (OrderedDict{(gid1, gid2): int},
        model/Siamese/dist_calculator.py:8-20) written by the reference's utils.save
        (src/utils.py:203-234), and GED / time result matrices saved under the names
        src/exp.py:263-266 writes (result/<ds>/ged/ged_ged_mat_<ds>_<model>_<ts>_...npy),
        which src/results.py:182-192 globs."""
    import shutil
    import tempfile
    from collections import OrderedDict
    import data as ref_data  # noqa: E402  (reference)
    fx = os.path.join(HERE, 'f6')
    if os.path.isdir(fx):
        shutil.rmtree(fx)
    data_root = os.path.join(fx, 'data')
    f6_gexf_tree(data_root)
    out = {}
    with tempfile.TemporaryDirectory() as save_dir:
        # the reference module bound these names at import (from utils import ...)
        ref_data.get_data_path = lambda: data_root
        ref_data.get_save_path = lambda: save_dir
        for cls in ('AIDS700nefData', 'AIDS80nefData'):
            for train in (True, False):
                d = getattr(ref_data, cls)(train)
                key = '{}_{}'.format(cls, 'train' if train else 'test')
                out[key] = [{'gid': g.graph['gid'],
                             'nodes': [[v, g.nodes[v].get('type')] for v in g.nodes()],
                             'edges': sorted([sorted([u, v]) + [sorted(a.keys())]
                                              for u, v, a in g.edges(data=True)])}
                            for g in d.graphs]
    # f3: the label store
    tr = [g['gid'] for g in out['AIDS80nefData_train']]
    te = [g['gid'] for g in out['AIDS80nefData_test']]
    sizes = {g['gid']: len(g['nodes']) for k in ('AIDS80nefData_train', 'AIDS80nefData_test')
             for g in out[k]}
    rng = np.random.default_rng(808)
    dmap = OrderedDict()
    entries = []
    for a in te:
        for b in tr[:20]:
            d = int(rng.integers(0, 9))
            rev = bool(rng.random() < 0.5)
            if not rev:
                dmap[(a, b)] = d
            else:                       # stored reversed: found through the reverse key
                dmap[(b, a)] = d
            entries.append([a, b, d, rev])
    # a cached reverse distance of 0 is treated as a miss (dist_calculator.py:33-37, A15)
    zero_pair = [te[0], tr[25]]
    dmap[(tr[25], te[0])] = 0
    save_dir = os.path.join(fx, 'save')
    os.makedirs(save_dir, exist_ok=True)
    ref_utils.save(os.path.join(save_dir, 'aids80nef_ged_astar_gidpair_dist_map'), dmap)
    m, n = len(te), len(tr)
    ged_mat = np.zeros((m, n))                       # exp.py:219-220
    time_mat = np.zeros((m, n))
    for i in range(m):
        for j in range(n):
            ged_mat[i][j] = int(rng.integers(0, 9))
            time_mat[i][j] = float(np.round(rng.random() * 3, 2))
    rdir = os.path.join(fx, 'result', 'aids80nef')
    os.makedirs(os.path.join(rdir, 'ged'), exist_ok=True)
    os.makedirs(os.path.join(rdir, 'time'), exist_ok=True)
    stamp = '2018-06-01T10:00:00_host_8cpus'
    np.save(os.path.join(rdir, 'ged', 'ged_ged_mat_aids80nef_astar_{}'.format(stamp)), ged_mat)
    np.save(os.path.join(rdir, 'time', 'ged_time_mat_aids80nef_astar_{}'.format(stamp)),
            time_mat)
    # normalized_dist (distance.py:59-60) of every (test i, train j) result entry
    norm = np.array([[2.0 * ged_mat[i][j] / (sizes[te[i]] + sizes[tr[j]]) for j in range(n)]
                     for i in range(m)])
    out['dist_map_entries'] = entries
    out['dist_map_reverse_zero_pair'] = zero_pair
    out['dist_map_len'] = len(dmap)
    out['ged_mat'] = ged_mat.tolist()
    out['time_mat'] = time_mat.tolist()
    out['ged_norm_mat'] = norm.tolist()
    with open(os.path.join(HERE, 'f6_loaders.json'), 'w') as f:
        json.dump(out, f)
    print('F6 fixtures written to', fx)


def f7_train_loop_lists():
    """F7 (row f1, quirks A3 + A6): the reference RandomSampler's list order after a whole
    default training loop.  train_val (train.py:8-44) makes, per iteration, one train and
    one val get_feed_dict; each draws B + B² = 30 pairs (A3), so after `iters` iterations
    both the 52-graph train list and the 18-graph val list of AIDS80nef
    (data_siamese.py:85-87) have seen 30 * iters get_pair calls, each wrap shuffling the
    list in place (samplers.py:28).  test() then scores column j against that permuted
    list (data_siamese.py:58-66)."""
    out = {}
    for n in (52, 18):
        for iters in (1, 4, 20):
            s = ref_samplers.RandomSampler(list(range(n)), -1, False)
            for _ in range(30 * iters):
                s.get_pair()
            out['random_{}_after_{}_calls'.format(n, 30 * iters)] = {'gs': list(s.gs),
                                                                     'idx': int(s.idx)}
    with open(os.path.join(HERE, 'f7_loop_lists.json'), 'w') as f:
        json.dump(out, f)
    print('F7 fixtures written to', HERE)


if __name__ == '__main__':
    if '--only-f6' in sys.argv:
        f6_loaders()
    elif '--only-f7' in sys.argv:
        f7_train_loop_lists()
    else:
        main()
        f6_loaders()
        f7_train_loop_lists()
