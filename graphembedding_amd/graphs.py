"""Per-graph preprocessing (model/Siamese/graphs.py:8-117).

ModelGraph keeps Â = D^-½ (A+I) D^-½ as a dense float64 matrix computed with
the reference's exact operation order ((A·D)ᵀ·D, graphs.py:64-76), so its
float32 cast is bit-identical to what the reference fed TF (quirk A11), and the
one-hot column of every node (row-normalised one-hot rows have value 1.0,
graphs.py:55-62).  The COO tuples of the reference are still available from
get_node_inputs / get_laplacians.
"""
from __future__ import annotations

import networkx as nx
import numpy as np

from .samplers import DistributionSampler, RandomSampler


class ModelGraphList(object):
    def __init__(self, sampler, sample_num, sampler_duplicate_removal, gs, node_feat_encoder):
        self.gs = [ModelGraph(g, node_feat_encoder) for g in gs]
        if sampler == 'random':
            self.sampler = RandomSampler(self.gs, sample_num, sampler_duplicate_removal)
        elif sampler == 'density':
            self.sampler = DistributionSampler(self.gs, sample_num, sampler_duplicate_removal)
        else:
            raise RuntimeError('Unknown sampler {}'.format(sampler))

    def num_graphs(self):
        return len(self.gs)

    def get_graph_pair(self):
        return self.sampler.get_pair()

    def get_triple_for_hinge_loss(self):
        return self.sampler.get_triple_for_hinge_loss()

    def get_graph(self, id):
        return self.gs[id]


def normalized_adjacency(nxgraph) -> np.ndarray:
    """graphs.py:64-76 in dense float64, same operation order as scipy's."""
    n = nxgraph.number_of_nodes()
    A = nx.to_numpy_array(nxgraph, nodelist=list(nxgraph.nodes()), dtype=np.float64)
    A = A + np.eye(n)
    rowsum = A.sum(axis=1)
    with np.errstate(divide='ignore'):
        d = np.power(rowsum, -0.5)
    d[np.isinf(d)] = 0.
    T = A * d[None, :]            # (A·D)[i][j] = A[i][j]·d[j]
    return T.T * d[None, :]       # ((A·D)ᵀ·D)[j][i] = (A[i][j]·d[j])·d[i]


class ModelGraph(object):
    def __init__(self, nxgraph, node_feat_encoder):
        self.nxgraph = nxgraph
        self.types = np.asarray(node_feat_encoder.encode_columns(nxgraph), dtype=np.int32)
        self.d_in = node_feat_encoder.input_dim()
        self.adj = normalized_adjacency(nxgraph)

    def get_nxgraph(self):
        return self.nxgraph

    def num_nodes(self):
        return int(self.types.shape[0])

    def get_node_inputs(self):
        n = self.num_nodes()
        coords = np.stack([np.arange(n, dtype=np.int32), self.types], axis=1)
        return coords, np.ones(n), (n, self.d_in)

    def get_node_inputs_num_nonzero(self):
        return self.get_node_inputs()[1].shape

    def get_laplacians(self):
        r, c = np.nonzero(self.adj)
        coords = np.stack([r, c], axis=1).astype(np.int32)
        return [(coords, self.adj[r, c], self.adj.shape)]


class NodeFeatureOneHotEncoder(object):
    """graphs.py:98-117: the type→column map comes from Python set iteration
    order (quirk A7); it is an explicit, recorded input of the packer."""

    def __init__(self, gs, node_feat_name, feat_idx_dic=None):
        self.node_feat_name = node_feat_name
        if feat_idx_dic is not None:
            self.feat_idx_dic = dict(feat_idx_dic)
            return
        inputs_set = set()
        for g in gs:
            inputs_set = inputs_set | set(self._node_feat_dic(g).values())
        self.feat_idx_dic = {feat: idx for idx, feat in enumerate(inputs_set)}

    def pin_sorted(self):
        """Replace the hash-seed-dependent set order with sorted order, so that
        every process (rank) encodes identically.  Returns self."""
        self.feat_idx_dic = {f: i for i, f in enumerate(sorted(self.feat_idx_dic, key=str))}
        return self

    def encode_columns(self, g):
        node_feat_dic = self._node_feat_dic(g)
        return [self.feat_idx_dic[node_feat_dic[n]] for n in g.nodes()]

    def encode(self, g):
        cols = self.encode_columns(g)
        out = np.zeros((len(cols), self.input_dim()))
        out[np.arange(len(cols)), cols] = 1.0
        return out

    def input_dim(self):
        return len(self.feat_idx_dic)

    def _node_feat_dic(self, g):
        return nx.get_node_attributes(g, self.node_feat_name)
