"""Graph store and pair-record packer (replaces get_feed_dict's per-pair
sparse-tuple feeds, model_mse.py:65-81).

A GraphStore holds every graph of a dataset as fixed-capacity slots
(adj [G][n_max][n_max] f32 — Â cast from float64 like the reference's float32
placeholders, quirk A11 —, one-hot columns [G][n_max] i32, node counts [G]).
Pair records (layout in include/siamese_hip.h) are gathered from it either on
the device (sg_pack_pairs, the product path) or on the host (pack_host, used
for small batches and by tests).
"""
from __future__ import annotations

from typing import Optional, Sequence

import numpy as np


def record_words(n_max: int) -> int:
    return 2 * n_max * n_max + 2 * n_max + 4


def record_bytes(n_max: int) -> int:
    return 4 * record_words(n_max)


class GraphStore(object):
    def __init__(self, model_graphs: Sequence, n_max: int, d_in: Optional[int] = None):
        G = len(model_graphs)
        self.n_max = int(n_max)
        self.adj = np.zeros((G, n_max, n_max), dtype=np.float32)
        self.types = np.zeros((G, n_max), dtype=np.int32)
        self.n = np.zeros(G, dtype=np.int32)
        self.gids = []
        for k, mg in enumerate(model_graphs):
            n = mg.num_nodes()
            if n > n_max:
                # tf.pad fails for N > max_in_dims (layers.py:226, quirk A9)
                raise RuntimeError('graph {} has {} nodes > n_max {}'.format(
                    mg.nxgraph.graph.get('gid'), n, n_max))
            if d_in is not None and n and int(mg.types.max()) >= d_in:
                raise RuntimeError('node type column out of range')
            if not np.array_equal(mg.adj, mg.adj.T):
                raise RuntimeError('Â must be symmetric (undirected graphs)')
            self.adj[k, :n, :n] = mg.adj.astype(np.float32)
            self.types[k, :n] = mg.types
            self.n[k] = n
            self.gids.append(mg.nxgraph.graph.get('gid'))
        self._dev = None

    def __len__(self):
        return int(self.n.shape[0])

    def to_device(self, device):
        import torch
        if self._dev is None or self._dev[0].device != torch.device(device):
            self._dev = (torch.from_numpy(self.adj).to(device),
                         torch.from_numpy(self.types).to(device),
                         torch.from_numpy(self.n).to(device))
        return self._dev

    def pack_host(self, pair_idx: np.ndarray, labels: Optional[np.ndarray] = None) -> np.ndarray:
        """Host twin of sg_pack_pairs: uint32 words [n_pairs][record_words]."""
        pair_idx = np.asarray(pair_idx, dtype=np.int64).reshape(-1, 2)
        P = pair_idx.shape[0]
        nm = self.n_max
        W = record_words(nm)
        out = np.zeros((P, W), dtype=np.uint32)
        a, b = pair_idx[:, 0], pair_idx[:, 1]
        nn = nm * nm
        out[:, 0:nn] = self.adj[a].reshape(P, nn).view(np.uint32)
        out[:, nn:2 * nn] = self.adj[b].reshape(P, nn).view(np.uint32)
        out[:, 2 * nn:2 * nn + nm] = self.types[a].view(np.uint32)
        out[:, 2 * nn + nm:2 * nn + 2 * nm] = self.types[b].view(np.uint32)
        out[:, 2 * nn + 2 * nm] = self.n[a].view(np.uint32)
        out[:, 2 * nn + 2 * nm + 1] = self.n[b].view(np.uint32)
        lab = np.zeros(P, np.float32) if labels is None else np.asarray(labels, np.float32)
        out[:, 2 * nn + 2 * nm + 2] = lab.view(np.uint32)
        out[:, 2 * nn + 2 * nm + 3] = (np.arange(P) & 0x7FFFFFFF).astype(np.uint32)
        return out


def pack_device(store: GraphStore, pair_idx, labels=None, device='cuda', stream=None):
    """Device packing via sg_pack_pairs. pair_idx: int32 [n,2] (numpy or torch)."""
    import torch
    from . import _lib
    adj, types, n = store.to_device(device)
    pi = torch.as_tensor(pair_idx, dtype=torch.int32, device=device).reshape(-1, 2).contiguous()
    P = int(pi.shape[0])
    lab = None
    if labels is not None:
        lab = torch.as_tensor(labels, dtype=torch.float32, device=device).reshape(-1).contiguous()
    recs = torch.empty(P * record_words(store.n_max), dtype=torch.int32, device=device)
    status = torch.zeros(1, dtype=torch.int32, device=device)
    if P:
        _lib.pack_pairs(adj, types, n, store.n_max, pi, lab, recs, status, stream=stream)
    return recs, status


def unpack_host(words: np.ndarray, n_max: int):
    """Split host record words into fields (for tests / debugging)."""
    words = np.asarray(words, dtype=np.uint32).reshape(-1, record_words(n_max))
    nn = n_max * n_max
    adj = words[:, :2 * nn].view(np.float32).reshape(-1, 2, n_max, n_max)
    types = words[:, 2 * nn:2 * nn + 2 * n_max].view(np.int32).reshape(-1, 2, n_max)
    n = words[:, 2 * nn + 2 * n_max:2 * nn + 2 * n_max + 2].view(np.int32)
    label = words[:, 2 * nn + 2 * n_max + 2].view(np.float32)
    tag = words[:, 2 * nn + 2 * n_max + 3].view(np.int32)
    return dict(adj=adj, types=types, n=n, label=label, tag=tag)
