"""Device-side pair samplers and training feed.

The reference's samplers (model/Siamese/samplers.py:19-68) draw only from fresh
random.Random(seed) generators with known seeds.  RandomSampler re-shuffles its
list with random.Random(123) on every wrap (samplers.py:28), i.e. applies one
fixed permutation σ each time.  DistributionSampler walks bins shuffled by
random.Random(123) and takes its item index from random.Random(123 + cur)
(samplers.py:51-68).  So the tables come from CPython's own `random`, computed
once here exactly as the reference computes them, and csrc/sg_sampler.hip
advances the state and emits the pair stream on the device.

DeviceFeed replaces get_feed_dict (model_mse.py:52-94) for train/val steps:
- sample the step's B + B² pairs on the device (quirk A3: inputs are the first B
  calls, labels those of the last B) or B in 'aligned' mode;
- gather the labels from a device label matrix;
- pack the input pairs from a device graph store.
Nothing crosses PCIe per step.
"""
from __future__ import annotations

from typing import Optional

import numpy as np

from . import _lib
from . import samplers
from .packer import GraphStore, pack_device_into, record_words
from .samplers import DistributionSampler, RandomSampler


def shuffle_permutation(n: int, seed: int = 123) -> np.ndarray:
    """σ with random.Random(seed).shuffle(x) == [x[σ[i]] for i in range(n)]."""
    return np.asarray(samplers.shuffle_permutation(n, seed), dtype=np.int32)


class DeviceRandomSampler(object):
    """RandomSampler (samplers.py:19-31) on the device.  Starts from the host
    sampler's current state: the list as it is now (store ids 0..n-1 of `gs`
    snapshot) and its idx."""

    def __init__(self, host: RandomSampler, device='cuda'):
        import torch
        self.torch = torch
        self.n = len(host.gs)
        self.gs = list(host.gs)   # store order = the list as it is now
        self.host = host
        st = np.zeros(1 + 2 * self.n, dtype=np.int32)
        st[0] = host.idx
        st[1:1 + self.n] = np.arange(self.n, dtype=np.int32)
        self.state = torch.from_numpy(st).to(device)
        self.sigma = torch.from_numpy(shuffle_permutation(self.n)).to(device)
        self.device = device

    def sample(self, count: int, out=None):
        """count get_pair() calls -> int32 [count, 2] store ids (device)."""
        torch = self.torch
        out = out if out is not None else torch.empty((count, 2), dtype=torch.int32,
                                                       device=self.device)
        _lib.sampler_random(self.state, self.sigma, self.n, count, out)
        return out

    def sync_host(self):
        """Leave the host sampler (and its graph list, which the reference shuffles
        in place: quirk A6) in the state the device stream reached."""
        st = self.state.cpu().numpy()
        order = st[1:1 + self.n]
        self.host.gs[:] = [self.gs[i] for i in order]
        self.host.idx = int(st[0])


class DeviceDistributionSampler(object):
    """DistributionSampler (samplers.py:37-68) on the device."""

    def __init__(self, host: DistributionSampler, device='cuda'):
        import torch
        self.torch = torch
        self.host = host
        self.gs = list(host.gs)
        n_bins = len(host.bin_idx)
        if n_bins < 2:
            raise RuntimeError('DistributionSampler needs at least 2 bins')
        self.dens_order = torch.tensor([i for _, i in host.dens_list], dtype=torch.int32,
                                       device=device)
        self.bins = torch.tensor(host.bin_idx, dtype=torch.int32, device=device)
        items = [samplers.bin_item(c, host.bin_size) for c in range(0, n_bins, 2)]
        self.item_table = torch.tensor(items, dtype=torch.int32, device=device)
        self.state = torch.tensor([host.cur, host.item_idx], dtype=torch.int32, device=device)
        self.bin_size = host.bin_size
        self.device = device

    def sample(self, count: int, out=None):
        torch = self.torch
        out = out if out is not None else torch.empty((count, 2), dtype=torch.int32,
                                                       device=self.device)
        _lib.sampler_density(self.state, self.dens_order, self.bins, self.bin_size,
                             self.item_table, count, out)
        return out

    def sync_host(self):
        st = self.state.cpu().numpy()
        self.host.cur, self.host.item_idx = int(st[0]), int(st[1])


def device_sampler(host, device='cuda'):
    if isinstance(host, RandomSampler):
        return DeviceRandomSampler(host, device)
    if isinstance(host, DistributionSampler):
        return DeviceDistributionSampler(host, device)
    raise RuntimeError('Unknown sampler {}'.format(type(host).__name__))


def label_matrix(model, graph_list, dist_calculator, data) -> np.ndarray:
    """float32 [n, n]: the label get_feed_dict would compute for (gs[i], gs[j])
    (data.get_dist -> normalized_dist when dist_norm -> sim kernel)."""
    gs = [g.get_nxgraph() for g in graph_list]
    n = len(gs)
    mat = getattr(dist_calculator, 'matrix', None)
    if mat is not None:   # DistCalculator.from_matrix: gather (same doubles as normalized_dist)
        index, dm = mat
        ix = np.array([index[g.graph['gid']] for g in gs])
        d = dm[np.ix_(ix, ix)].astype(np.int64).astype(np.float64)
        sizes = np.array([g.number_of_nodes() for g in gs], dtype=np.float64)
        nd = 2 * d / (sizes[:, None] + sizes[None, :])
    else:
        d = np.zeros((n, n), np.float64)
        nd = np.zeros((n, n), np.float64)
        for i in range(n):
            for j in range(n):
                d[i, j], nd[i, j] = data.get_dist(gs[i], gs[j], dist_calculator)
    dd = nd if model.flags.dist_norm else d
    return model.sim_kernel.dist_to_sim_np(dd.astype(np.float32).astype(np.float64)).astype(
        np.float32)


class DeviceFeed(object):
    """get_feed_dict(data, dc, tvt) for tvt in {'train', 'val'}, on the device."""

    def __init__(self, model, data, dist_calculator, tvt: str = 'train',
                 labels: Optional[np.ndarray] = None):
        import torch
        assert tvt in ('train', 'val')
        self.torch = torch
        self.model = model
        coll = data.train_data if tvt == 'train' else data.valid_data
        self.sampler = device_sampler(coll.sampler, model.device)
        gl = self.sampler.gs
        self.store = GraphStore(gl, model.n_max, model.input_dim)
        model.check_node_counts(self.store.n, 'DeviceFeed')
        Y = labels if labels is not None else label_matrix(model, gl, dist_calculator, data)
        self.Y = torch.from_numpy(np.ascontiguousarray(Y, dtype=np.float32)).to(model.device)
        B = model.flags.batch_size
        self.B = B
        self.compat = model.flags.label_stream == 'compat'
        self.count = B + B * B if self.compat else B
        dev = model.device
        self.pairs = torch.empty((self.count, 2), dtype=torch.int32, device=dev)
        self.records = torch.empty(B * record_words(model.n_max, model.record_dtype),
                                   dtype=torch.int32, device=dev)
        self.status = torch.zeros(1, dtype=torch.int32, device=dev)
        self.labels = torch.empty(B, dtype=torch.float32, device=dev)
        self.y_stats = torch.empty(2, dtype=torch.float32, device=dev)
        # sg_feed_t: sampler calls + label gather + label stats + packing in one launch
        sadj, stypes, sn = self.store.to_device(dev)
        smp = self.sampler
        f = _lib.SgFeed()
        if isinstance(smp, DeviceRandomSampler):
            f.kind, f.state, f.sigma, f.n = 0, smp.state.data_ptr(), smp.sigma.data_ptr(), smp.n
        else:
            f.kind, f.state = 1, smp.state.data_ptr()
            f.dens_order, f.bins = smp.dens_order.data_ptr(), smp.bins.data_ptr()
            f.item_table, f.n_bins = smp.item_table.data_ptr(), int(smp.bins.numel())
            f.bin_size = smp.bin_size
        f.batch, f.compat = B, 1 if self.compat else 0
        f.label_matrix, f.label_n = self.Y.data_ptr(), int(self.Y.shape[0])
        f.store_adj, f.store_types, f.store_n = sadj.data_ptr(), stypes.data_ptr(), sn.data_ptr()
        f.n_graphs, f.n_max = len(self.store), model.n_max
        f.adj_dtype = _lib.dtype_code(model.record_dtype)
        self._feed = f

    def next_batch(self):
        """One step's batch (device only, one launch): the first B calls are the
        inputs, the labels belong to the last B calls in 'compat' mode (quirk A3)."""
        _lib.feed_step(self._feed, self.pairs, self.records, self.labels, self.y_stats,
                       self.status)
        return self.model.batch_from_records(self.records, self.B, self.labels,
                                             y_stats=self.y_stats)

    def store_ids_to_graphs(self, ids):
        """Host bookkeeping: store ids -> ModelGraph objects."""
        return [self.sampler.gs[int(i)] for i in np.asarray(ids).reshape(-1)]
