"""All-pairs Siamese training over a graph set (the BASELINE workload:
AIDS700nef all-pairs, 700² = 490,000 ordered pairs per step).

The pair stream is the ordered pair space p ↦ (p // G, p % G); each rank packs
its contiguous shard once into HBM-resident pair records (sg_pack_pairs) and
every step runs the fused fwd+bwd kernel over them, all-reduces the gradient
(N > 1) and applies Adam.  Labels are y = exp(-η (2d/(n_i+n_j))²) from a GED
matrix (synthetic offline).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional

import weakref

import numpy as np

from .data import synthetic_ged_matrix, synthetic_graphs
from .graphs import ModelGraph, NodeFeatureOneHotEncoder
from .packer import GraphStore, pack_device, pack_device_into, record_words
from .shard import shard_range


@dataclass
class GraphSet:
    graphs: list
    mgs: List[ModelGraph]
    d_in: int
    n_max: int
    store: GraphStore
    ged: np.ndarray

    def label_matrix(self, yeta: float, dist_norm: bool = True) -> np.ndarray:
        sizes = np.array([g.number_of_nodes() for g in self.graphs], dtype=np.float64)
        d = self.ged.astype(np.float64)
        if dist_norm:
            d = 2.0 * d / (sizes[:, None] + sizes[None, :])   # normalized_dist, distance.py:59-60
        d = d.astype(np.float32).astype(np.float64)           # float32 placeholder feed
        return np.exp(-yeta * d * d).astype(np.float32)

    def flops_per_pair_web(self, h1=32, h2=16, K=10) -> float:
        """Config C5: SURVEY §8(d) per-graph GCN/Dense terms, and the NTN terms on the
        pair's nonzero structure (x is zero beyond each graph's nodes, so the
        bilinear term is n1·n2 per k instead of D²): fwd K(2 n1 n2 + 2(n1+n2)),
        bwd twice that.  Averaged over the all-pairs stream."""
        n = np.array([g.number_of_nodes() for g in self.graphs], dtype=np.float64)
        e = np.array([g.number_of_edges() for g in self.graphs], dtype=np.float64)
        nnz = n + 2 * e
        fwd = 2 * h1 * n + 2 * h1 * nnz + 2 * n * h1 * h2 + 2 * h2 * nnz + 2 * n * h2
        bwd = (2 * h1 * nnz + 2 * h1 * n) + (2 * h2 * nnz + 4 * n * h1 * h2) + 4 * n * h2
        nm = n.mean()
        ntn_f = K * (2 * (n[:, None] * n[None, :]).mean() + 2 * 2 * nm)
        return float(2 * (fwd + bwd).mean() + 3 * ntn_f)

    def csr_bytes_per_pair(self) -> float:
        """Algorithmic input bytes of a pair on the graph-store path: both graphs'
        CSR rows (row_ptr + col + val) and types, plus the pair ids and label."""
        n = np.array([g.number_of_nodes() for g in self.graphs], dtype=np.float64)
        e = np.array([g.number_of_edges() for g in self.graphs], dtype=np.float64)
        per_graph = 4 * (n + 1) + 4 * n + 8 * (n + 2 * e)
        return float(2 * per_graph.mean() + 12)

    def flops_per_pair(self, h1=32, h2=16, D=10, K=10, pool='padding') -> float:
        """Algorithmic FLOPs per pair, fwd+bwd (SURVEY §8(d) formula), averaged
        over the all-pairs stream (every graph is g1 G times and g2 G times).
        pool='average': the tuning.py stack (no Dense; mean over nodes, NTN D = h2);
        pool='attention': the same with Attention pooling (layers.py:143-160)."""
        n = np.array([g.number_of_nodes() for g in self.graphs], dtype=np.float64)
        e = np.array([g.number_of_edges() for g in self.graphs], dtype=np.float64)
        nnz = n + 2 * e
        if pool == 'padding':
            head_f, head_b = 2 * n * h2, 4 * n * h2
        elif pool == 'attention':
            # layers.py:154-160: mean n h2, h = tanh(temp Wa) 2 h2², att = σ(H2 h) 2 n h2,
            # attᵀ H2 2 n h2; backward gatt and gh 2 n h2 each, gWa and gtemp 2 h2² each,
            # ∂H2 = att gout + gz h + gtemp / n 4 n h2
            head_f, head_b = 5 * n * h2 + 2 * h2 * h2, 8 * n * h2 + 4 * h2 * h2
        else:
            head_f, head_b = n * h2, n * h2
        if pool != 'padding':
            D = h2
        fwd = 2 * h1 * n + 2 * h1 * nnz + 2 * n * h1 * h2 + 2 * h2 * nnz + head_f
        bwd = (2 * h1 * nnz + 2 * h1 * n) + (2 * h2 * nnz + 4 * n * h1 * h2) + head_b
        ntn_f = K * (4 * D + 2 * D * D + 2 * D)
        return float(2 * (fwd + bwd).mean() + 3 * ntn_f)


def load_graph_set(name: str = 'syn_aids700nef', n_max: int = 10, seed: int = 123,
                   with_store: bool = True) -> GraphSet:
    tr, te = synthetic_graphs(name, seed)
    graphs = tr + te
    # sorted (not set-order) columns: identical encoding on every rank (quirk A7)
    enc = NodeFeatureOneHotEncoder(graphs, 'type').pin_sorted()
    mgs = [ModelGraph(g, enc) for g in graphs]
    # dense-slot store for the record paths; the graph-store path (web.py) builds CSR
    store = GraphStore(mgs, n_max, enc.input_dim()) if with_store else None
    return GraphSet(graphs=graphs, mgs=mgs, d_in=enc.input_dim(), n_max=n_max, store=store,
                    ged=synthetic_ged_matrix(graphs))


class AllPairsShard(object):
    """This rank's slice of the all-pairs stream, packed once into HBM."""

    def __init__(self, gs: GraphSet, labels: np.ndarray, rank: int = 0, world: int = 1,
                 device='cuda', n_pairs: Optional[int] = None, dtype: str = 'f32'):
        import torch
        G = len(gs.graphs)
        self.total = int(n_pairs if n_pairs is not None else G * G)
        self.start, self.end = shard_range(self.total, rank, world)
        p = np.arange(self.start, self.end, dtype=np.int64)
        pairs = np.stack([p // G, p % G], axis=1).astype(np.int32)
        flat_labels = labels.reshape(-1)[:self.total]
        lab = flat_labels[self.start:self.end]
        self.dtype = dtype
        self.records, status = pack_device(gs.store, pairs, lab, device=device, dtype=dtype)
        torch.cuda.synchronize()
        if int(status.item()) != 0:
            raise RuntimeError('sg_pack_pairs reported invalid graph ids')
        self.labels = torch.from_numpy(lab.copy()).to(device)
        y = flat_labels.astype(np.float64)
        ybar = y.mean()
        self.y_stats = torch.tensor([ybar, 0.5 * ((y - ybar) ** 2).sum()], dtype=torch.float32,
                                    device=device)
        self.n = self.end - self.start
        self.record_bytes = 4 * record_words(gs.n_max, dtype)
        self.store_n = gs.store.n

    def batch(self, model, rank: int = 0, balance: bool = True):
        model.check_node_counts(self.store_n, 'AllPairsShard')
        b = model.batch_from_records(self.records, self.n, self.labels,
                                     pair_offset=self.start, batch_total=self.total,
                                     y_stats=self.y_stats)
        return model.balance(b) if balance else b


class AllPairsStream(object):
    """This rank's slice of the all-pairs stream, packed and stepped chunk by chunk.

    For shards whose records do not fit HBM at once: AIDS10knef all-pairs (config
    C4) is 10,018² = 100.4 M pairs, 850 GB of capacity-32 f32 records.  One device
    buffer holds `chunk` records; for every chunk the pair ids (p // G, p % G) are
    generated on the device, packed (sg_pack_pairs_ex) and run through fwd_bwd with
    pair_offset = the chunk's global start, so dropout masks and the broadcast loss
    are those of the unchunked step.  The chunk gradients and losses are summed in
    chunk order (deterministic), leaving model.grad / model.loss_buf as one fwd_bwd
    over the whole shard would (up to fp32 summation order).

    source='auto' skips the records when the model runs a fused kernel with f32 Â
    (config C4's capacity-32 one in particular): the kernel then gathers every pair's
    graphs from the store
    (sg_fwd_bwd_src, library 1.6) and the pack pass with its 8.5 KB-per-pair write and
    read-back disappears.  source='records' always packs.
    """

    def __init__(self, gs: GraphSet, labels: np.ndarray, rank: int = 0, world: int = 1,
                 device='cuda', chunk: int = 4_000_000, dtype: str = 'f32',
                 n_pairs: Optional[int] = None, balance: bool = True, source: str = 'auto',
                 keep_orders: bool = True):
        import torch
        self.torch = torch
        G = len(gs.graphs)
        self.G = G
        self.total = int(n_pairs if n_pairs is not None else G * G)
        self.start, self.end = shard_range(self.total, rank, world)
        self.n = self.end - self.start
        self.chunk = int(max(1, min(chunk, max(self.n, 1))))
        self.dtype = dtype
        self.store = gs.store
        self.balance = balance
        self.device = device
        flat = labels.reshape(-1)[:self.total]
        # the shard's labels stay on the device (4 B per pair)
        self.labels = torch.from_numpy(np.ascontiguousarray(flat[self.start:self.end])).to(device)
        y = flat.astype(np.float64)
        ybar = y.mean()
        self.y_stats = torch.tensor([ybar, 0.5 * ((y - ybar) ** 2).sum()], dtype=torch.float32,
                                    device=device)
        self.record_bytes = 4 * record_words(gs.n_max, dtype)
        if source not in ('auto', 'records'):
            raise RuntimeError('Unknown pair source {}'.format(source))
        self.source = source
        self.records = None   # allocated on the first packed chunk
        self.status = torch.zeros(1, dtype=torch.int32, device=device)
        # store-sourced chunks need no records, so their batches (with the class order, 4 B
        # per pair) are built once and reused by every step, as AllPairsShard reuses its
        # packed, ordered batch; keep_orders=False rebuilds them per step
        self.keep_orders = keep_orders
        self._batches = {}
        self._batches_owner = None

    def chunks(self):
        for c0 in range(self.start, self.end, self.chunk):
            yield c0, min(self.chunk, self.end - c0)

    def uses_store(self, model) -> bool:
        return (self.source == 'auto' and model.kernel_path in (1, 2) and self.dtype == 'f32' and
                model.record_dtype == 'f32' and self.store.n_max == model.n_max)

    def _pack(self, model, c0: int, n: int):
        torch = self.torch
        model.check_node_counts(self.store.n, 'AllPairsStream')
        lab = self.labels[c0 - self.start:c0 - self.start + n]
        if self.uses_store(model):
            # the kept batches belong to one model (a weak reference: a later model that
            # reuses a dead one's id() must not get its batches)
            owner = self._batches_owner() if self._batches_owner is not None else None
            if owner is not model:
                self._batches = {}
                self._batches_owner = weakref.ref(model)
            key = (c0, n)
            if self.keep_orders and key in self._batches:
                return self._batches[key]
            b = model.batch_from_store(self.store, n, lab, grid_base=c0, pair_offset=c0,
                                       batch_total=self.total, y_stats=self.y_stats,
                                       status=self.status)
            b = model.balance(b) if self.balance else b
            if self.keep_orders:
                self._batches[key] = b
            return b
        if self.records is None:
            self.records = torch.empty(self.chunk * record_words(self.store.n_max, self.dtype),
                                       dtype=torch.int32, device=self.device)
        p = torch.arange(c0, c0 + n, dtype=torch.int64, device=self.device)
        pi = torch.stack([p // self.G, p % self.G], dim=1).to(torch.int32).contiguous()
        pack_device_into(self.store, pi, lab, self.records, self.status, dtype=self.dtype)
        b = model.batch_from_records(self.records, n, lab, pair_offset=c0,
                                     batch_total=self.total, y_stats=self.y_stats)
        return model.balance(b) if self.balance else b

    def prepare(self, model):
        """Build (and keep) every store-sourced chunk's batch and class order before the
        timed steps; returns the number of chunks prepared."""
        if not (self.keep_orders and self.uses_store(model)):
            return 0
        for c0, n in self.chunks():
            self._pack(model, c0, n)
        return len(self._batches)

    def fwd_bwd(self, model, add_label_term: bool = True):
        """One fwd+bwd over the shard; leaves the summed gradient / loss_mse in
        model.grad / model.loss_buf (like model.fwd_bwd on one batch)."""
        torch = self.torch
        acc = None
        model.workspace(self.chunk)
        for i, (c0, n) in enumerate(self.chunks()):
            batch = self._pack(model, c0, n)
            model.fwd_bwd(batch, add_label_term=(add_label_term and i == 0))
            if acc is None:
                acc = model.grad_loss.clone()
            else:
                acc += model.grad_loss
        if acc is None:
            model.grad_loss.zero_()
        else:
            model.grad_loss.copy_(acc)

    def check_status(self):
        if int(self.status.item()) != 0:
            raise RuntimeError('sg_pack_pairs reported invalid graph ids')
