"""Graph-store path for Web-sized graphs (BASELINE config C5; kernel path 3).

The reference feeds every graph as sparse tuples (model_mse.py:65-81; Â from
graphs.py:64-76).  For graphs of hundreds of nodes a dense pair record (Â as
n_max² per side) is the wrong layout, so this path keeps ONE device copy of the
dataset in CSR form and hands the kernels pair ids:

  CsrStore        node_off / types / row_ptr / col / val of every graph
                  (include/siamese_hip.h, sg_csr_store_t), built from ModelGraphs.
  size_order      a stable ordering of a pair list by node-count bucket, so the
                  NTN GEMM tiles of sg_web_* see pairs of similar size (the
                  kernels skip feature tiles beyond every pair's node count).
  WebAllPairs     one rank's shard of the all-pairs stream on the graph store
                  (the C5 bench workload), stepped through sg_web_fwd_bwd.

Dropout masks are keyed by the pair's position in the (ordered) list plus
pair_offset, exactly like the record path's keys.
"""
from __future__ import annotations

from typing import Optional, Sequence

import numpy as np

from .shard import shard_range


class CsrStore(object):
    """CSR form of a list of ModelGraphs (Â symmetric, float32 cast, quirk A11)."""

    def __init__(self, model_graphs: Sequence, d_in: Optional[int] = None,
                 n_cap: Optional[int] = None):
        G = len(model_graphs)
        ns = np.array([mg.num_nodes() for mg in model_graphs], dtype=np.int64)
        if G and ns.min() < 1:
            raise RuntimeError('graph with no nodes')
        if n_cap is not None and G and ns.max() > n_cap:
            # tf.pad fails for N > max_in_dims (layers.py:226, quirk A9)
            raise RuntimeError('graph with {} nodes > max_in_dims {}'.format(int(ns.max()), n_cap))
        self.n = ns.astype(np.int32)
        self.node_off = np.zeros(G + 1, dtype=np.int32)
        self.node_off[1:] = np.cumsum(ns)
        total = int(self.node_off[-1])
        self.types = np.zeros(total, dtype=np.int32)
        row_ptr = [np.zeros(1, dtype=np.int64)]
        cols, vals = [], []
        base = 0
        for k, mg in enumerate(model_graphs):
            a = np.asarray(mg.adj)
            if not np.array_equal(a, a.T):
                raise RuntimeError('Â must be symmetric (undirected graphs)')
            if d_in is not None and int(mg.types.max()) >= d_in:
                raise RuntimeError('node type column out of range')
            o = int(self.node_off[k])
            self.types[o:o + mg.num_nodes()] = mg.types
            r, c = np.nonzero(a)                       # row-major, columns ascending
            cnt = np.bincount(r, minlength=mg.num_nodes())
            row_ptr.append(base + np.cumsum(cnt))
            cols.append(c.astype(np.int32))
            vals.append(a[r, c].astype(np.float32))
            base += r.size
        self.row_ptr = np.concatenate(row_ptr).astype(np.int64)
        if self.row_ptr[-1] >= 2 ** 31:
            raise RuntimeError('store has more than 2^31 Â entries')
        self.row_ptr = self.row_ptr.astype(np.int32)
        self.col = np.concatenate(cols) if cols else np.zeros(0, np.int32)
        self.val = np.concatenate(vals) if vals else np.zeros(0, np.float32)
        self.n_max = int(ns.max()) if G else 1
        self.max_nnz = int(np.diff(self.row_ptr[self.node_off]).max()) if G else 0
        self.gids = [mg.nxgraph.graph.get('gid') for mg in model_graphs]
        self._dev = None
        self._struct = None

    def __len__(self):
        return int(self.n.shape[0])

    @property
    def nnz(self) -> int:
        return int(self.val.shape[0])

    def to_device(self, device):
        """Device arrays and the sg_csr_store_t pointing at them (cached)."""
        import torch
        from . import _lib
        if self._dev is None or self._dev[0].device != torch.device(device):
            t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)  # noqa: E731
            self._dev = (t(self.node_off), t(self.types), t(self.row_ptr),
                         t(self.col if self.col.size else np.zeros(1, np.int32)),
                         t(self.val if self.val.size else np.zeros(1, np.float32)))
            self._struct = _lib.csr_struct(len(self), self.n_max, *self._dev,
                                           max_nnz=self.max_nnz)
        return self._struct


def size_order(pairs: np.ndarray, n_nodes: np.ndarray, bucket: int = 32) -> np.ndarray:
    """Stable permutation of a pair list sorted by (n1 bucket, n2 bucket)."""
    pairs = np.asarray(pairs)
    if pairs.shape[0] == 0:
        return np.zeros(0, dtype=np.int64)
    b1 = n_nodes[pairs[:, 0]] // bucket
    b2 = n_nodes[pairs[:, 1]] // bucket
    return np.lexsort((b2, b1)).astype(np.int64)


def dealt_size_order(pairs: np.ndarray, n_nodes: np.ndarray, block: int = 128,
                     virtual: int = 8, seed: int = 0) -> np.ndarray:
    """size_order, cut into `block`-pair blocks (size-homogeneous for the GEMM
    tiles), then dealt stratified into `virtual` contiguous groups: each run of
    `virtual` consecutive (similar-cost) blocks gives one block, in a fixed
    pseudo-random assignment, to every group.  Any contiguous rank shard for a world
    size dividing `virtual` then holds the same size mix.  Independent of the world
    size, so the list position (the dropout key) of a pair is too."""
    order = size_order(pairs, n_nodes)
    nb = (order.size + block - 1) // block
    if nb == 0:
        return order
    rng = np.random.default_rng(seed)
    groups = [[] for _ in range(virtual)]
    for s0 in range(0, nb, virtual):
        run = np.arange(s0, min(s0 + virtual, nb))
        dest = rng.permutation(virtual)[:run.size]
        for b, v in zip(run, dest):
            groups[v].append(b)
    return np.concatenate([order[b * block:(b + 1) * block] for g in groups for b in g])


def allpairs_ids(G: int, start: int, end: int) -> np.ndarray:
    p = np.arange(start, end, dtype=np.int64)
    return np.stack([p // G, p % G], axis=1).astype(np.int32)


class WebAllPairs(object):
    """This rank's shard of the all-pairs stream on the graph store.

    The ordered pair space of G graphs is ordered once on the host by
    dealt_size_order (the same permutation on every rank and for every world
    size), then split into contiguous rank shards with equal size mixes; list
    position = dropout key, so a sharded step computes the unsharded one.  Labels
    stay on the device with the pair ids.
    """

    def __init__(self, gs, labels: np.ndarray, rank: int = 0, world: int = 1, device='cuda',
                 chunk: int = 32768, n_pairs: Optional[int] = None, d_in: Optional[int] = None,
                 n_cap: Optional[int] = None):
        import torch
        G = len(gs.graphs)
        self.total = int(n_pairs if n_pairs is not None else G * G)
        self.store = CsrStore(gs.mgs, d_in if d_in is not None else gs.d_in, n_cap)
        ids = allpairs_ids(G, 0, self.total)
        order = dealt_size_order(ids, self.store.n)
        ids = ids[order]
        flat = labels.reshape(-1)[:self.total][order]
        self.start, self.end = shard_range(self.total, rank, world)
        self.n = self.end - self.start
        self.pairs = torch.from_numpy(np.ascontiguousarray(ids[self.start:self.end])).to(device)
        self.labels = torch.from_numpy(np.ascontiguousarray(flat[self.start:self.end])).to(device)
        y = flat.astype(np.float64)
        ybar = y.mean() if y.size else 0.0
        self.y_stats = torch.tensor([ybar, 0.5 * ((y - ybar) ** 2).sum()], dtype=torch.float32,
                                    device=device)
        self.chunk = int(max(1, min(chunk, max(self.n, 1))))
        self.device = device
        self.n_nodes = self.store.n[ids[self.start:self.end]] if self.n else np.zeros((0, 2))

    def batch(self, model):
        return model.web_batch(self.store, self.pairs, self.labels, pair_offset=self.start,
                               batch_total=self.total, y_stats=self.y_stats, chunk=self.chunk)
