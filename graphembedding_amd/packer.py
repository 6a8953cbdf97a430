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


def adj_words(n_max: int, dtype: str = 'f32') -> int:
    """Words of the Â block: f32 entries, or bf16 entries packed two per word."""
    return n_max * n_max if dtype == 'bf16' else 2 * n_max * n_max


def record_words(n_max: int, dtype: str = 'f32') -> int:
    """Record words, padded to 16 B (include/siamese_hip.h)."""
    if dtype not in ('f32', 'bf16'):
        raise RuntimeError('Unknown record dtype {}'.format(dtype))
    return (adj_words(n_max, dtype) + 2 * n_max + 4 + 3) & ~3


def record_bytes(n_max: int, dtype: str = 'f32') -> int:
    return 4 * record_words(n_max, dtype)


def f32_to_bf16_bits(x: np.ndarray) -> np.ndarray:
    """RNE float32 → bf16 bit patterns (uint16), the SG_DTYPE_BF16 encoding."""
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    return ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)


def bf16_round(x: np.ndarray) -> np.ndarray:
    """Values of f32 → bf16 → f32 (what a bf16 record's kernels compute with)."""
    return (f32_to_bf16_bits(x).astype(np.uint32) << 16).view(np.float32)


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

    def pack_host(self, pair_idx: np.ndarray, labels: Optional[np.ndarray] = None,
                  dtype: str = 'f32') -> np.ndarray:
        """Host twin of sg_pack_pairs_ex: uint32 words [n_pairs][record_words]."""
        pair_idx = np.asarray(pair_idx, dtype=np.int64).reshape(-1, 2)
        P = pair_idx.shape[0]
        nm = self.n_max
        W = record_words(nm, dtype)
        out = np.zeros((P, W), dtype=np.uint32)
        a, b = pair_idx[:, 0], pair_idx[:, 1]
        nn = nm * nm
        adj = np.concatenate([self.adj[a].reshape(P, nn), self.adj[b].reshape(P, nn)], axis=1)
        if dtype == 'bf16':
            bits = f32_to_bf16_bits(adj).astype(np.uint32)             # [P, 2 nn]
            out[:, 0:nn] = bits[:, 0::2] | (bits[:, 1::2] << 16)
        else:
            out[:, 0:2 * nn] = adj.view(np.uint32)
        o = adj_words(nm, dtype)
        out[:, o:o + nm] = self.types[a].view(np.uint32)
        out[:, o + nm:o + 2 * nm] = self.types[b].view(np.uint32)
        out[:, o + 2 * nm] = self.n[a].view(np.uint32)
        out[:, o + 2 * nm + 1] = self.n[b].view(np.uint32)
        lab = np.zeros(P, np.float32) if labels is None else np.asarray(labels, np.float32)
        out[:, o + 2 * nm + 2] = lab.view(np.uint32)
        out[:, o + 2 * nm + 3] = (np.arange(P) & 0x7FFFFFFF).astype(np.uint32)
        return out


def pack_device(store: GraphStore, pair_idx, labels=None, device='cuda', stream=None,
                dtype: str = 'f32'):
    """Device packing via sg_pack_pairs_ex. pair_idx: int32 [n,2] (numpy or torch)."""
    import torch
    from . import _lib
    adj, types, n = store.to_device(device)
    pi = torch.as_tensor(pair_idx, dtype=torch.int32, device=device).reshape(-1, 2).contiguous()
    P = int(pi.shape[0])
    lab = None
    if labels is not None:
        lab = torch.as_tensor(labels, dtype=torch.float32, device=device).reshape(-1).contiguous()
    recs = torch.empty(P * record_words(store.n_max, dtype), dtype=torch.int32, device=device)
    status = torch.zeros(1, dtype=torch.int32, device=device)
    if P:
        _lib.pack_pairs(adj, types, n, store.n_max, pi, lab, recs, status, stream=stream,
                        dtype=dtype)
    return recs, status


def pack_device_into(store: GraphStore, pair_idx, labels, records, status, stream=None,
                     dtype: str = 'f32'):
    """sg_pack_pairs_ex into caller-owned device buffers (no allocation): pair_idx
    int32 [n,2] and labels float32 [n] (or None) as device tensors, records with
    room for n records."""
    from . import _lib
    adj, types, n = store.to_device(records.device)
    P = int(pair_idx.shape[0])
    assert records.numel() >= P * record_words(store.n_max, dtype)
    if P:
        _lib.pack_pairs(adj, types, n, store.n_max, pair_idx, labels, records, status,
                        stream=stream, dtype=dtype)


def unpack_host(words: np.ndarray, n_max: int, dtype: str = 'f32'):
    """Split host record words into fields (for tests / debugging); a bf16 Â is
    returned widened to f32."""
    words = np.asarray(words, dtype=np.uint32).reshape(-1, record_words(n_max, dtype))
    nn = n_max * n_max
    if dtype == 'bf16':
        a = words[:, :nn]
        bits = np.stack([a << 16, a & 0xFFFF0000], axis=2).reshape(-1, 2 * nn)
        adj = bits.astype(np.uint32).view(np.float32).reshape(-1, 2, n_max, n_max)
    else:
        adj = words[:, :2 * nn].view(np.float32).reshape(-1, 2, n_max, n_max)
    o = adj_words(n_max, dtype)
    types = words[:, o:o + 2 * n_max].view(np.int32).reshape(-1, 2, n_max)
    n = words[:, o + 2 * n_max:o + 2 * n_max + 2].view(np.int32)
    label = words[:, o + 2 * n_max + 2].view(np.float32)
    tag = words[:, o + 2 * n_max + 3].view(np.int32)
    return dict(adj=adj, types=types, n=n, label=label, tag=tag)
