"""SiameseGCNTNMSE — host mirror of model/Siamese/model_mse.py:9-168 +
models.py:6-131 on top of the HIP C-ABI.

What was `sess.run` in the reference is now a sequence of stream-ordered
C-ABI calls on torch's current stream:
  train  (train.py:85)  sg_fwd_bwd → [all-reduce] → sg_adam_tf
  val    (train.py:86)  sg_fwd_bwd (loss only)
  test   (train.py:87)  sg_forward → pre-activation s (pred_sim_without_act)
Parameters are one flat fp32 device vector in the reference's variable order.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _lib
from .config import FLAGS
from .layers_factory import create_activation, create_layers, padding_dims
from .packer import GraphStore, record_words
from .similarity import create_sim_kernel


def param_shapes(layers: List[dict], d_in: int) -> List[Tuple[int, str, Tuple[int, ...]]]:
    """(layer index, variable name, shape) in variable creation order
    (layers.py:68-73, 151-152, 174-178, 268-277)."""
    out = []
    for li, L in enumerate(layers):
        k = L['kind']
        if k == 'GraphConvolution':
            din = L.get('input_dim') or d_in
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
            out += [(li, 'weights_W', (D, D, K)), (li, 'weights_V', (K, 2 * D)),
                    (li, 'weights_U', (K, 1))]
            if L['bias']:
                out.append((li, 'bias', (K,)))
    return out


def glorot_flat(layers: List[dict], d_in: int, seed: int = 0) -> np.ndarray:
    """inits.py:11-21 (uniform ±√(6/(s0+s1)); zeros for biases), numpy-seeded."""
    rng = np.random.default_rng(seed)
    parts = []
    for li, name, shape in param_shapes(layers, d_in):
        if name == 'bias':
            parts.append(np.zeros(shape))
        else:
            r = math.sqrt(6.0 / (shape[0] + shape[1]))
            parts.append(rng.uniform(-r, r, size=shape))
    return np.concatenate([p.ravel() for p in parts]).astype(np.float32)


def splitmix64(x: int) -> int:
    """Steele et al.'s splitmix64 finaliser (a bijection of 64-bit integers)."""
    m = 0xFFFFFFFFFFFFFFFF
    x = (int(x) + 0x9E3779B97F4A7C15) & m
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & m
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & m
    return x ^ (x >> 31)


@dataclass
class Batch:
    """A packed batch resident on the device (what get_feed_dict returns)."""
    records: object                 # torch.int32 [n * record_words]
    n_pairs: int
    labels: object                  # torch.float32 [n] (per input pair, for aligned loss)
    y_stats: object                 # torch.float32 [2] {ȳ, ½Σ(y-ȳ)²} of the label set
    pair_offset: int = 0            # global index of record 0 (dropout RNG / sharding)
    batch_total: int = 0            # global batch size B
    gid_pairs: Optional[np.ndarray] = None
    order: object = None            # torch.int32 [n] processing order (balance()) or None
    cls: object = None              # torch.int32 [5] class table of the order (fused path)
    # graph-store path (kernel path 3, config C5): pair ids into a CSR store instead of records
    csr: object = None              # web.CsrStore
    pairs: object = None            # torch.int32 [n, 2] store graph ids
    chunk: int = 0                  # pairs per internal chunk (workspace size)
    # store-sourced pairs (library 1.6, kernel path 2): the fused kernel gathers each pair
    # from a dense GraphStore instead of a packed record (records is None)
    src: object = None              # _lib.SgPairSource
    src_keep: tuple = ()            # the device tensors src points into (kept alive)


class SiameseGCNTNMSE(object):
    def __init__(self, input_dim, flags=None, device='cuda', n_max=None, params=None):
        f = flags or FLAGS
        assert f.loss_func == 'mse'
        self.flags = f
        self.input_dim = int(input_dim)
        self.device = device
        self.layers = create_layers(f, self.input_dim)
        pd = padding_dims(self.layers)
        self.n_max = int(n_max or f.n_max or pd or 10)
        # the reference's tf.pad fails for N > max_in_dims (layers.py:226, quirk A9); the
        # kernels would drop the extra nodes instead, so every store is checked on entry
        # (check_node_counts) even when the record capacity n_max exceeds the Padding dim
        self.max_nodes = pd
        self.sim_kernel = create_sim_kernel(f.sim_kernel, f.yeta)
        self.final_act_np = create_activation(f.final_act, self.sim_kernel)
        self.record_dtype = getattr(f, 'record_dtype', 'f32') or 'f32'
        def make(cap):
            return _lib.make_model(self.layers, self.input_dim, cap, 1.0 - f.dropout,
                                   f.final_act, f.sim_kernel, f.yeta, f.loss_mode, f.ntn_mode,
                                   self.record_dtype)
        self.sg = make(self.n_max)
        self.n_params, self.kernel_path = _lib.validate(self.sg)
        # Record node capacity: any capacity >= the largest graph is valid, and the
        # fused kernels want a specific one (the Padding dim <= 12, or 32 for
        # Padding dims in (12, 31]: config C4), so take it when the stack qualifies.
        if self.kernel_path == 0 and pd is not None and self.n_max <= pd:
            for cap in (pd, 32):
                if cap <= self.n_max:
                    continue
                sg2 = make(cap)
                n2, path2 = _lib.validate(sg2)
                if path2:
                    self.sg, self.n_max, self.n_params, self.kernel_path = sg2, cap, n2, path2
                    break
        import torch
        self.torch = torch
        init = glorot_flat(self.layers, self.input_dim, f.param_seed) if params is None else \
            np.asarray(params, np.float32)
        assert init.shape[0] == self.n_params, (init.shape, self.n_params)
        self.params = torch.from_numpy(init.copy()).to(device)
        self.adam_m = torch.zeros_like(self.params)
        self.adam_v = torch.zeros_like(self.params)
        self.beta1, self.beta2, self.eps = 0.9, 0.999, 1e-8
        self.beta_powers = torch.tensor([self.beta1, self.beta2], dtype=torch.float32, device=device)
        # grad and loss_mse share one flat buffer: the data-parallel all-reduce
        # (shard.make_allreduce_hook) is then a single in-place collective
        n = self.params.numel()
        self.grad_loss = torch.zeros(n + 2, dtype=torch.float32, device=device)
        self.grad = self.grad_loss[:n]
        self.loss_buf = self.grad_loss[n:]
        self.reg_buf = torch.zeros(1, dtype=torch.float32, device=device)
        self._ws = None
        self._ws_pairs = -1
        self.seed = int(f.seed)
        self.step_count = 0
        self.grad_hook = None   # e.g. the data-parallel all-reduce (shard.py)
        self._adam_ws = None
        if self.n_params > 65536:   # multi-block Adam (config C5: D²K NTN weights)
            self._adam_ws = torch.empty(_lib.adam_workspace_bytes(self.n_params) // 8 + 1,
                                        dtype=torch.float64, device=device)

    @property
    def is_web(self) -> bool:
        """Graph-store path (sg_web_*, config C5): Padding/NTN width in [32, 512]."""
        return self.kernel_path == _lib.PATH_WEB

    def check_node_counts(self, n_nodes, what='graph store'):
        """Raise like the reference's tf.pad (layers.py:226, quirk A9) when a graph has
        more nodes than the Padding layer's max_in_dims."""
        n = np.asarray(n_nodes).reshape(-1)
        if self.max_nodes is not None and n.size and int(n.max()) > self.max_nodes:
            k = int(np.argmax(n))
            raise _lib.SiameseHipError(
                '{}: graph {} has {} nodes > Padding max_in_dims {} (layers.py:226)'.format(
                    what, k, int(n[k]), self.max_nodes))

    # ---- reference API ------------------------------------------------------
    def apply_final_act_np(self, score):
        return self.final_act_np(score)

    def pred_sim_without_act(self, batch: Batch, seed: Optional[int] = None):
        """Pre-activation scores of the batch (train.py:87 'test')."""
        torch = self.torch
        s = torch.empty(batch.n_pairs, dtype=torch.float32, device=self.device)
        if batch.csr is not None:
            _lib.web_forward(self.sg, batch.csr.to_device(self.device), batch.pairs, batch.n_pairs,
                             batch.pair_offset, self.params, self._seed(seed), s,
                             self.web_workspace(batch.chunk, batch.n_pairs), batch.chunk)
            return s
        if batch.src is not None:
            _lib.forward_src(self.sg, batch.src, batch.n_pairs, batch.pair_offset, self.params,
                             self._seed(seed), s, order=batch.order)
            return s
        _lib.forward(self.sg, batch.records, batch.n_pairs, batch.pair_offset, self.params,
                     self._seed(seed), s, order=batch.order, class_start=batch.cls)
        return s

    def get_feed_dict(self, data, dist_calculator, tvt, test_id=None, train_id=None):
        """model_mse.py:52-94, same sampler-call pattern (quirk A3 in 'compat')."""
        B = self.flags.batch_size
        if tvt in ('train', 'val'):
            assert test_id is None and train_id is None
            pairs = [data.get_graph_pair(tvt) for _ in range(B)]
        else:
            assert tvt == 'test'
            pairs = [(data.test_data.get_graph(test_id), data.get_orig_train_graph(train_id))]
        dists = norm_dists = None
        if tvt in ('train', 'val'):
            if self.flags.label_stream == 'compat':
                # the label block sits inside the per-pair loop: B redraws of B pairs
                for _ in range(len(pairs)):
                    dists, norm_dists = np.zeros(B), np.zeros(B)
                    for i in range(B):
                        g1, g2 = data.get_graph_pair(tvt)
                        d, nd = data.get_dist(g1.get_nxgraph(), g2.get_nxgraph(), dist_calculator)
                        dists[i], norm_dists[i] = d, nd
            else:
                dists, norm_dists = np.zeros(B), np.zeros(B)
                for i, (g1, g2) in enumerate(pairs):
                    d, nd = data.get_dist(g1.get_nxgraph(), g2.get_nxgraph(), dist_calculator)
                    dists[i], norm_dists[i] = d, nd
        labels = None
        if dists is not None:
            d = norm_dists if self.flags.dist_norm else dists
            labels = self.sim_kernel.dist_to_sim_np(np.asarray(d, np.float32).astype(np.float64))
        return self.make_batch([p[0] for p in pairs], [p[1] for p in pairs], labels)

    def make_batch(self, g1s: Sequence, g2s: Sequence, labels=None, pair_offset=0,
                   batch_total=None) -> Batch:
        """Pack ModelGraph pairs on the host and move them to the device."""
        torch = self.torch
        if self.is_web:
            return self.make_web_batch(g1s, g2s, labels, pair_offset, batch_total)
        uniq, index = [], {}
        idx = np.zeros((len(g1s), 2), np.int32)
        for k, (a, b) in enumerate(zip(g1s, g2s)):
            for c, g in enumerate((a, b)):
                if id(g) not in index:
                    index[id(g)] = len(uniq)
                    uniq.append(g)
                idx[k, c] = index[id(g)]
        store = GraphStore(uniq, self.n_max, self.input_dim)
        self.check_node_counts(store.n, 'make_batch')
        lab = np.zeros(len(g1s), np.float32) if labels is None else np.asarray(labels, np.float32)
        words = store.pack_host(idx, lab, dtype=self.record_dtype)
        recs = torch.from_numpy(words.view(np.int32).reshape(-1)).to(self.device)
        gids = np.array([[a.nxgraph.graph.get('gid', -1), b.nxgraph.graph.get('gid', -1)]
                         for a, b in zip(g1s, g2s)])
        return self.batch_from_records(recs, len(g1s), lab, pair_offset, batch_total, gids)

    def make_web_batch(self, g1s: Sequence, g2s: Sequence, labels=None, pair_offset=0,
                       batch_total=None, chunk=None) -> Batch:
        """ModelGraph pairs → a CSR store of the distinct graphs + pair ids (path 3)."""
        from .web import CsrStore
        torch = self.torch
        uniq, index = [], {}
        idx = np.zeros((len(g1s), 2), np.int32)
        for k, (a, b) in enumerate(zip(g1s, g2s)):
            for c, g in enumerate((a, b)):
                if id(g) not in index:
                    index[id(g)] = len(uniq)
                    uniq.append(g)
                idx[k, c] = index[id(g)]
        store = CsrStore(uniq, self.input_dim, self.n_max)
        lab = np.zeros(len(g1s), np.float32) if labels is None else np.asarray(labels, np.float32)
        gids = np.array([[a.nxgraph.graph.get('gid', -1), b.nxgraph.graph.get('gid', -1)]
                         for a, b in zip(g1s, g2s)])
        b = self.web_batch(store, torch.from_numpy(idx).to(self.device), lab, pair_offset,
                           batch_total, chunk=chunk)
        b.gid_pairs = gids
        return b

    def web_batch(self, store, pairs, labels, pair_offset=0, batch_total=None, y_stats=None,
                  chunk=None) -> Batch:
        n = int(pairs.shape[0])
        self.check_node_counts(store.n, 'web_batch')
        b = self.batch_from_records(None, n, labels, pair_offset, batch_total, y_stats=y_stats)
        b.csr, b.pairs = store, pairs
        b.chunk = int(chunk or min(max(n, 1), 32768))
        return b

    def web_workspace(self, chunk, n_pairs=-1):
        """Graph-store workspace for calls of up to n_pairs pairs in chunks of `chunk`
        (n_pairs <= chunk: one pipeline slot, about half the bytes; -1: any n_pairs).  A
        cached workspace is reused when it is at least as large as the call needs."""
        torch = self.torch
        one = 0 <= int(n_pairs) <= int(chunk)
        key = ('web', int(chunk), one)
        have = getattr(self, '_web_ws_key', None)
        if have is not None and have[:2] == key[:2] and (not have[2] or one):
            return self._web_ws
        nbytes = _lib.web_workspace_bytes(self.sg, int(chunk), 0 if one else -1)
        self._web_ws = None
        self._web_ws = torch.empty(nbytes // 4 + 64, dtype=torch.float32, device=self.device)
        self._web_ws_key = key
        return self._web_ws

    def batch_from_records(self, recs, n_pairs, labels, pair_offset=0, batch_total=None,
                           gid_pairs=None, y_stats=None) -> Batch:
        torch = self.torch
        if recs is not None:   # the kernels read n_pairs whole records
            need = int(n_pairs) * record_words(self.n_max, self.record_dtype)
            if recs.numel() * recs.element_size() < 4 * need:
                raise _lib.SiameseHipError('records hold fewer than n_pairs = {} records of '
                                           '{} B'.format(int(n_pairs), 4 * need // max(1, int(n_pairs))))
        lab = torch.as_tensor(np.asarray(labels, np.float32) if not torch.is_tensor(labels)
                              else labels, dtype=torch.float32, device=self.device)
        if y_stats is None:
            y64 = lab.double()
            ybar = y64.mean() if n_pairs else torch.zeros((), dtype=torch.float64,
                                                          device=self.device)
            half = 0.5 * ((y64 - ybar) ** 2).sum()
            y_stats = torch.stack([ybar, half]).float()
        return Batch(records=recs, n_pairs=int(n_pairs), labels=lab, y_stats=y_stats,
                     pair_offset=int(pair_offset),
                     batch_total=int(batch_total if batch_total is not None else n_pairs),
                     gid_pairs=gid_pairs)

    def batch_from_store(self, store, n_pairs, labels, pair_idx=None, grid_base=0,
                         pair_offset=0, batch_total=None, y_stats=None, status=None) -> Batch:
        """A batch whose pairs the fused kernel gathers from the dense store itself
        (sg_*_src, library 1.6; kernel paths 1 and 2 with f32 Â): store = packer.GraphStore,
        pair_idx int32 [n, 2] device tensor or None for the all-pairs grid (pair i =
        divmod(grid_base + i, G)), labels float32 [n] device tensor.  Same results as
        packing the pairs into records (sg_pack_pairs) and stepping those."""
        if self.kernel_path not in (1, 2) or self.record_dtype != 'f32':
            raise _lib.SiameseHipError('store-sourced batches need a fused kernel path with '
                                       'f32 records (kernel path {})'.format(self.kernel_path))
        if store.n_max != self.n_max:
            raise _lib.SiameseHipError('store n_max {} != model n_max {}'.format(store.n_max,
                                                                                 self.n_max))
        torch = self.torch
        n_pairs = int(n_pairs)
        self.check_node_counts(store.n, 'batch_from_store')
        # the kernel reads pair_idx[0 .. 2n) and labels[0 .. n): check before it does
        if pair_idx is not None:
            if (not torch.is_tensor(pair_idx) or pair_idx.dtype != torch.int32 or
                    not pair_idx.is_contiguous() or pair_idx.numel() < 2 * n_pairs):
                raise _lib.SiameseHipError('pair_idx must be a contiguous int32 [n, 2] tensor')
        elif int(grid_base) < 0:
            raise _lib.SiameseHipError('grid_base must be >= 0')
        if torch.is_tensor(labels) and labels.numel() < n_pairs:
            raise _lib.SiameseHipError('labels has fewer than n_pairs entries')
        dev = store.to_device(self.device)
        b = self.batch_from_records(None, n_pairs, labels, pair_offset=pair_offset,
                                    batch_total=batch_total, y_stats=y_stats)
        b.src = _lib.pair_source(dev, store.n_max, pair_idx=pair_idx, grid_base=grid_base,
                                 labels=b.labels, status=status)
        b.src_keep = (dev, pair_idx, b.labels, status)
        return b

    # ---- steps ----------------------------------------------------------------
    def _seed(self, seed):
        return (self.seed * 1000003 + self.step_count) if seed is None else int(seed)

    def workspace(self, n_pairs):
        torch = self.torch
        if self._ws is None or n_pairs > self._ws_pairs:
            nbytes = _lib.workspace_bytes(self.sg, max(int(n_pairs), 1))
            self._ws = torch.empty(nbytes // 4 + 64, dtype=torch.float32, device=self.device)
            self._ws_pairs = int(n_pairs)
        return self._ws

    def fwd_bwd(self, batch: Batch, seed=None, s_out=None, add_label_term=True):
        """Forward + loss + backward; leaves Σ∂loss_mse/∂θ in self.grad and the
        shard's loss_mse in self.loss_buf[0]."""
        if batch.csr is not None:
            _lib.web_fwd_bwd(self.sg, batch.csr.to_device(self.device), batch.pairs, batch.labels,
                             batch.n_pairs, batch.pair_offset, batch.batch_total, self.params,
                             self._seed(seed), batch.y_stats, 1 if add_label_term else 0, s_out,
                             self.grad, self.loss_buf,
                             self.web_workspace(batch.chunk, batch.n_pairs), batch.chunk)
            return
        if batch.src is not None:
            _lib.fwd_bwd_src(self.sg, batch.src, batch.n_pairs, batch.pair_offset,
                             batch.batch_total, self.params, self._seed(seed), batch.y_stats,
                             1 if add_label_term else 0, s_out, self.grad, self.loss_buf,
                             self.workspace(batch.n_pairs), order=batch.order)
            return
        _lib.fwd_bwd(self.sg, batch.records, batch.n_pairs, batch.pair_offset,
                     batch.batch_total, self.params, self._seed(seed), batch.y_stats,
                     1 if add_label_term else 0, s_out, self.grad, self.loss_buf,
                     self.workspace(batch.n_pairs), order=batch.order, class_start=batch.cls)

    # SG_CLASS_SCHEDULE=0 keeps the mixed (snake) schedule on the fused path
    CLASS_SCHEDULE = True

    def balance(self, batch: Batch, classes: Optional[bool] = None) -> Batch:
        """Attach the class-sorted processing order of the batch's records
        (sg_pair_order): every wavefront then gets the same mix of cheap and
        expensive pairs.  On the fused path (kernel path 1) the order comes with its
        class table (sg_pair_order_cls) and every wavefront runs the pairs of one class
        (class-exclusive schedule).  Scores are unchanged; the gradient differs only by
        summation order.  Worth it for batches that are stepped repeatedly (all-pairs
        epochs), not for the reference's B = 5 feeds."""
        import os
        torch = self.torch
        if batch.n_pairs == 0 or batch.csr is not None:
            return batch
        if classes is None:
            classes = self.CLASS_SCHEDULE and os.environ.get('SG_CLASS_SCHEDULE', '1') != '0'
        ws = torch.empty(_lib.pair_order_workspace_bytes(self.sg, batch.n_pairs) // 4 + 1,
                         dtype=torch.int32, device=self.device)
        order = torch.empty(batch.n_pairs, dtype=torch.int32, device=self.device)
        batch.cls = None
        if batch.src is not None:
            _lib.pair_order_src(self.sg, batch.src, batch.n_pairs, order, ws)
        elif classes and self.kernel_path == 1:
            cls = torch.empty(_lib.FAST_CLASSES_P1, dtype=torch.int32, device=self.device)
            _lib.pair_order_cls(self.sg, batch.records, batch.n_pairs, order, cls, ws)
            batch.cls = cls
        else:
            _lib.pair_order(self.sg, batch.records, batch.n_pairs, order, ws)
        batch.order = order
        return batch

    def apply_adam(self):
        f = self.flags
        if self._adam_ws is not None:
            _lib.adam_tf_ex(self.params, self.adam_m, self.adam_v, self.grad, f.learning_rate,
                            self.beta1, self.beta2, self.eps, f.weight_decay, self.beta_powers,
                            self.reg_buf, self._adam_ws)
            return
        _lib.adam_tf(self.params, self.adam_m, self.adam_v, self.grad, f.learning_rate,
                     self.beta1, self.beta2, self.eps, f.weight_decay, self.beta_powers,
                     self.reg_buf)

    def fwd_bwd_adam(self, batch: Batch, seed=None, s_out=None, add_label_term=True):
        """fwd_bwd + apply_adam as one library call (sg_train_step: on the fused path the
        gradient reduction applies Adam in the same launch).  Same results as the two calls
        (θ, m, v, grad, loss bitwise; reg_buf summed in another order).  Record batches
        only; other batches take the two calls."""
        if batch.csr is not None or batch.src is not None or self._adam_ws is not None:
            self.fwd_bwd(batch, seed, s_out, add_label_term)
            self.apply_adam()
            return
        f = self.flags
        _lib.train_step(self.sg, batch.records, batch.n_pairs, batch.pair_offset,
                        batch.batch_total, self.params, self._seed(seed), batch.y_stats,
                        1 if add_label_term else 0, s_out, self.grad, self.loss_buf,
                        self.workspace(batch.n_pairs), self.adam_m, self.adam_v,
                        f.learning_rate, self.beta1, self.beta2, self.eps, f.weight_decay,
                        self.beta_powers, self.reg_buf, order=batch.order,
                        class_start=batch.cls)

    def train_step(self, batch: Batch, seed=None, sync=True):
        """sess.run([opt_op, loss]) (train.py:85,92): returns the loss evaluated
        at the pre-update parameters (incl. weight decay, models.py:67-88)."""
        if self.grad_hook is None:
            self.fwd_bwd_adam(batch, seed)
        else:
            self.fwd_bwd(batch, seed)
            self.grad_hook(self)
            self.apply_adam()
        self.step_count += 1
        if not sync:
            return None
        return float(self.loss_buf[0].item() + self.reg_buf[0].item())

    def capture_train_steps(self, feed, n_steps: int = 1):
        """A hipGraph of n_steps reference train steps (train.py:8-44: get_feed_dict
        then sess.run([opt_op, loss]) with B = 5 pairs): DeviceFeed.next_batch →
        sg_fwd_bwd_dseed → ApplyAdam → seed + 1, all stream-ordered with no host sync.
        The dropout seed lives on the device, so every replay draws the masks an eager
        step with the same step_count would.  Returns a GraphSteps whose replay() runs
        the captured steps; fused path (default / Average stack) only."""
        return GraphSteps(self, feed, n_steps)

    # validation draws its dropout masks from a stream of its own: the reference's val
    # sess.run (train.py:19-21) samples independently of the train steps
    VAL_SEED_STREAM = 0x5641_4C5F_5354_524D   # 'VAL_STRM'

    def val_seed(self, seed=None):
        """An explicit seed is used as given; the default is the step's seed tagged with
        the validation stream and put through splitmix64, so both 32-bit halves (and the
        kernels' 32-bit key lo*C ^ hi) change in every bit position, not by one fixed
        XOR of the train key (which would make a val pair's masks another pair's train
        masks)."""
        if seed is not None:
            return int(seed)
        return splitmix64(self._seed(None) ^ self.VAL_SEED_STREAM)

    def val_loss(self, batch: Batch, seed=None):
        """sess.run([merged, loss]) on valid_data (train.py:19-21): the loss at the current
        parameters, with independent dropout masks (val_seed); self.grad / loss_buf keep
        the last training step's values."""
        saved = self.grad_loss.clone()
        self.fwd_bwd(batch, self.val_seed(seed))
        loss = float(self.loss_buf[0].item())
        self.grad_loss.copy_(saved)
        reg = self.flags.weight_decay * 0.5 * float((self.params.double() ** 2).sum().item())
        return loss + reg

    def test_scores(self, batch: Batch, seed=None):
        return self.pred_sim_without_act(batch, seed).cpu().numpy().astype(np.float64)

    def flat_params(self) -> np.ndarray:
        return self.params.detach().cpu().numpy()

    def set_params(self, flat):
        self.params.copy_(self.torch.as_tensor(np.asarray(flat, np.float32)))

    # ---- checkpoint / resume (models.py:118-131 counterpart) -------------------
    def state_dict(self):
        return dict(params=self.params.cpu(), adam_m=self.adam_m.cpu(), adam_v=self.adam_v.cpu(),
                    beta_powers=self.beta_powers.cpu(),
                    step_count=self.torch.tensor(self.step_count))

    def load_state_dict(self, sd):
        self.params.copy_(sd['params'])
        self.adam_m.copy_(sd['adam_m'])
        self.adam_v.copy_(sd['adam_v'])
        self.beta_powers.copy_(sd['beta_powers'])
        self.step_count = int(sd['step_count'])

    def save(self, path):
        self.torch.save(self.state_dict(), path)

    def load(self, path):
        self.load_state_dict(self.torch.load(path, weights_only=True))


class GraphSteps(object):
    """Captured train steps of SiameseGCNTNMSE (see capture_train_steps)."""

    def __init__(self, model, feed, n_steps: int = 1):
        import torch
        if model.kernel_path != 1:
            raise RuntimeError('graph-captured steps need the fused path (kernel path 1)')
        if model.grad_hook is not None:
            # a data-parallel hook is host-driven (torch.distributed / gloo): it cannot be
            # recorded into a hipGraph, and a replay would silently skip the exchange
            raise RuntimeError('graph-captured steps do not support a grad_hook (the '
                               'all-reduce of a sharded step); run eager train_step instead')
        self.model, self.feed, self.n_steps = model, feed, int(n_steps)
        m = model
        self.seed_dev = torch.tensor([m._seed(None)], dtype=torch.int64, device=m.device)
        ws = m.workspace(feed.B)
        state = self._snapshot()
        # warm-up on a side stream (allocator pools, lazy handles), then restore
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            self._body(ws)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self._restore(state)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            for _ in range(self.n_steps):
                self._body(ws)
        torch.cuda.synchronize()
        self._restore(state)   # capture records the work; the state must not move

    def _body(self, ws):
        m = self.model
        b = self.feed.next_batch()
        if m._adam_ws is None:   # reduction + Adam in one launch
            f = m.flags
            _lib.train_step_dseed(m.sg, b.records, b.n_pairs, b.pair_offset, b.batch_total,
                                  m.params, self.seed_dev, b.y_stats, 1, None, m.grad,
                                  m.loss_buf, ws, m.adam_m, m.adam_v, f.learning_rate, m.beta1,
                                  m.beta2, m.eps, f.weight_decay, m.beta_powers, m.reg_buf)
        else:
            _lib.fwd_bwd_dseed(m.sg, b.records, b.n_pairs, b.pair_offset, b.batch_total,
                               m.params, self.seed_dev, b.y_stats, 1, None, m.grad, m.loss_buf,
                               ws)
            m.apply_adam()
        _lib.seed_advance(self.seed_dev, 1)

    def _snapshot(self):
        m, f = self.model, self.feed
        return [t.clone() for t in (m.params, m.adam_m, m.adam_v, m.beta_powers,
                                    f.sampler.state, self.seed_dev)]

    def _restore(self, st):
        m, f = self.model, self.feed
        for dst, src in zip((m.params, m.adam_m, m.adam_v, m.beta_powers, f.sampler.state,
                             self.seed_dev), st):
            dst.copy_(src)

    def replay(self, times: int = 1):
        """Run the captured steps `times` times; leaves the last step's loss_mse in
        model.loss_buf and advances model.step_count like eager steps."""
        for _ in range(int(times)):
            self.graph.replay()
        self.model.step_count += self.n_steps * int(times)


def create_model(model, input_dim, flags=None, **kw):
    """models_factory.py:5-11."""
    if model == 'siamese_gcntn_mse':
        return SiameseGCNTNMSE(input_dim, flags, **kw)
    elif model == 'siamese_gcntn_hinge':
        raise RuntimeError('siamese_gcntn_hinge is an unimplemented stub in the reference '
                           '(model_hinge.py:5-45)')
    raise RuntimeError('Unknown model {}'.format(model))
