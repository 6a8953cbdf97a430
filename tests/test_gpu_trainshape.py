"""Gradient parity at the C4 and C5 TRAINING launch shapes the bench runs (VERDICT r3,
item 1): every score, the per-variable gradient and the loss of one training launch,
against the C restatement (oracle/siamese_cpu.c, float32 per-pair arithmetic like
TF-CPU, gradient summed in double) on the same pairs, dropout 0.1 (shared counter RNG).

- C4 (AIDS10knef, N <= 30, Padding/NTN 30): one store-sourced sg_fwd_bwd_src launch of
  4,194,304 consecutive pairs of the 10,018^2 all-pairs grid at a nonzero, unaligned
  grid_base, in class order — the batch AllPairsStream builds for the bench's
  25 M-pair launches (same kernel, same order kernel, same split-K NTN weight-gradient
  reduction over every workgroup), only shorter.  fp32 register accumulation over
  ~2e3 pairs per wave is checked against the checker's double sums.
- C5 (Web, N <= 512, Padding/NTN 512): 4,096 pairs drawn uniformly from the bench's
  dealt all-pairs list, put in dealt size order, stepped in 5 chunks of <= 1,000 pairs with
  the bench's machinery on: the two-stream chunk pipeline, the 16-way weight-gradient
  split, the forward's D2 rows and dropout keep bits.

The checker runs at record capacity D (30 / 512): the C port's NTN width is its record
capacity, and dropout keys do not depend on the capacity.
Tolerances: scores 1e-4 (north_star); gradient 1e-4 of each variable's own largest
component; loss 1e-4 relative.  Reference math: layers.py:91-310, model_mse.py:145-151,
models.py:67-73."""
import os

import numpy as np
import pytest

from _fixtures import check_grad_per_var
from oracle import cpu_ref

pytestmark = pytest.mark.gpu

TOL = 1e-4
C4_FLAGS = dict(layer_3='Padding:max_in_dims=30,padding_value=0',
                layer_4='NTN:input_dim=30,feature_map_dim=10,inneract=relu,dropout=True,'
                        'bias=True')
WEB_FLAGS = dict(layer_3='Padding:max_in_dims=512,padding_value=0',
                 layer_4='NTN:input_dim=512,feature_map_dim=10,inneract=relu,dropout=True,'
                         'bias=True')


def _check_pairs(store, pairs, labels, D, d_in, params, seed, keep, yeta, ybar, offset,
                 block):
    """The C restatement over `pairs` (global keys offset + i), in blocks of host records
    (capacity-D records of 4M pairs would not fit host memory at once)."""
    from concurrent.futures import ThreadPoolExecutor
    P = pairs.shape[0]
    s = np.empty(P, np.float32)
    g = None
    loss = 0.0
    th = cpu_ref.default_threads()
    starts = list(range(0, P, block))

    def pack(b0):
        b1 = min(P, b0 + block)
        return store.pack_host(pairs[b0:b1], labels[b0:b1], dtype='f32')

    # pack block i + 1 on a helper thread while the C port (GIL released) runs block i
    with ThreadPoolExecutor(1) as ex:
        nxt = ex.submit(pack, starts[0]) if starts else None
        for i, b0 in enumerate(starts):
            words = nxt.result()
            nxt = ex.submit(pack, starts[i + 1]) if i + 1 < len(starts) else None
            sb, gb, lb = cpu_ref.fwd_bwd_records(words, D, d_in, params, seed, keep, yeta,
                                                 ybar, pair_offset=offset + b0, threads=th,
                                                 f64_acc=True)
            s[b0:b0 + sb.shape[0]] = sb
            g = gb.astype(np.float64) if g is None else g + gb
            loss += lb
            del words
    return s, g, loss


@pytest.mark.timeout(900)
def test_c4_store_sourced_training_launch(gpu):
    import torch
    from graphembedding_amd.allpairs import AllPairsStream, load_graph_set
    from graphembedding_amd.config import Flags
    from graphembedding_amd.model_mse import SiameseGCNTNMSE
    from graphembedding_amd.packer import GraphStore
    f = Flags(dropout=0.1, **C4_FLAGS)
    gs = load_graph_set('syn_aids10knef', n_max=32)
    G = len(gs.graphs)
    assert G == 10018
    labels = gs.label_matrix(f.yeta)
    model = SiameseGCNTNMSE(gs.d_in, f, device=gpu, n_max=gs.n_max)
    assert model.kernel_path == 2
    n = 4_194_304
    c0 = 37_000_003                     # nonzero, not a multiple of G or of any tile
    stream = AllPairsStream(gs, labels, 0, 1, device=gpu, chunk=n, balance=True)
    assert stream.uses_store(model)
    batch = stream._pack(model, c0, n)  # what AllPairsStream.fwd_bwd launches per chunk
    assert batch.src is not None and batch.order is not None and batch.n_pairs == n
    seed = 424242
    model.workspace(n)
    s_out = torch.full((n,), float('nan'), dtype=torch.float32, device=gpu)
    model.fwd_bwd(batch, seed=seed, s_out=s_out, add_label_term=False)
    stream.check_status()
    g_gpu = model.grad.cpu().numpy().astype(np.float64)
    loss_gpu = float(model.loss_buf[0].item())
    s_gpu = s_out.cpu().numpy()
    assert not np.isnan(s_gpu).any()
    # the checker: capacity-30 records of the same pairs, keys c0 + i
    p = np.arange(c0, c0 + n, dtype=np.int64)
    pairs = np.stack([p // G, p % G], axis=1)
    lab = labels.reshape(-1)[c0:c0 + n]
    ybar = float(stream.y_stats[0].item())
    store30 = GraphStore(gs.mgs, 30, gs.d_in)
    s_ref, g_ref, loss_ref = _check_pairs(store30, pairs, lab, 30, gs.d_in,
                                          model.params.cpu().numpy(), seed,
                                          1.0 - f.dropout, f.yeta, ybar, c0, 262_144)
    np.testing.assert_allclose(s_gpu, s_ref, rtol=TOL, atol=TOL)
    rel = check_grad_per_var(g_gpu, g_ref, model.layers, model.input_dim, TOL, what='C4')
    assert abs(loss_gpu - loss_ref) <= TOL * max(1.0, abs(loss_ref)), (loss_gpu, loss_ref)
    print('C4 {} pairs at grid_base {}: worst |ds| {:.3g}; per-variable relative gradient '
          'error {}; loss {} vs {}'.format(n, c0, float(np.abs(s_gpu - s_ref).max()), rel,
                                           loss_gpu, loss_ref))


@pytest.mark.timeout(900)
def test_c5_web_training_chunks(gpu):
    import torch
    from graphembedding_amd import _lib
    from graphembedding_amd.allpairs import load_graph_set
    from graphembedding_amd.config import Flags
    from graphembedding_amd.model_mse import SiameseGCNTNMSE
    from graphembedding_amd.packer import GraphStore
    from graphembedding_amd.web import WebAllPairs, dealt_size_order
    for k in ('SG_WEB_PIPE', 'SG_WEB_MASKS', 'SG_WEB_D2', 'SG_WEB_WSPLIT'):
        assert os.environ.get(k, '1') != '0', '{} must be on (the bench runs with it)'.format(k)
    f = Flags(dropout=0.1, **WEB_FLAGS)
    gs = load_graph_set('syn_web', n_max=512, with_store=False)
    labels = gs.label_matrix(f.yeta)
    model = SiameseGCNTNMSE(gs.d_in, f, device=gpu, n_max=gs.n_max)
    assert model.kernel_path == _lib.PATH_WEB
    full = WebAllPairs(gs, labels, 0, 1, device=gpu)
    # 4,096 pairs drawn uniformly from the bench's dealt list, then dealt-size-ordered
    # among themselves (homogeneous GEMM tiles, as in the bench)
    pos = np.sort(np.random.default_rng(2026).choice(full.n, 4096, replace=False))
    ids = full.pairs.cpu().numpy()[pos]
    labs = full.labels.cpu().numpy()[pos]
    o = dealt_size_order(ids, full.store.n)
    ids, labs = np.ascontiguousarray(ids[o]), np.ascontiguousarray(labs[o])
    chunk = 1000                        # 5 chunks, the last one partial
    offset = 777
    batch = model.web_batch(full.store, torch.from_numpy(ids).to(gpu),
                            torch.from_numpy(labs).to(gpu), pair_offset=offset,
                            batch_total=full.total, y_stats=full.y_stats, chunk=chunk)
    assert (batch.n_pairs + chunk - 1) // chunk == 5
    seed = 31337
    s_out = torch.full((batch.n_pairs,), float('nan'), dtype=torch.float32, device=gpu)
    model.fwd_bwd(batch, seed=seed, s_out=s_out, add_label_term=False)
    g_gpu = model.grad.cpu().numpy().astype(np.float64)
    loss_gpu = float(model.loss_buf[0].item())
    s_gpu = s_out.cpu().numpy()
    assert not np.isnan(s_gpu).any()
    s_fwd = model.pred_sim_without_act(batch, seed=seed).cpu().numpy()
    assert np.array_equal(s_fwd, s_gpu), 'eval-path scores differ from the training scores'
    store = GraphStore(gs.mgs, 512, gs.d_in)
    ybar = float(full.y_stats[0].item())
    s_ref, g_ref, loss_ref = _check_pairs(store, ids, labs, 512, gs.d_in,
                                          model.params.cpu().numpy(), seed, 1.0 - f.dropout,
                                          f.yeta, ybar, offset, 64)
    np.testing.assert_allclose(s_gpu, s_ref, rtol=TOL, atol=TOL)
    rel = check_grad_per_var(g_gpu, g_ref, model.layers, model.input_dim, TOL, what='C5')
    assert abs(loss_gpu - loss_ref) <= TOL * max(1.0, abs(loss_ref)), (loss_gpu, loss_ref)
    nn = full.store.n[ids]
    print('C5 {} pairs (N {}..{}, mean {:.0f}) in {} chunks: worst |ds| {:.3g}; per-variable '
          'relative gradient error {}; loss {} vs {}'.format(
              batch.n_pairs, int(nn.min()), int(nn.max()), float(nn.mean()),
              (batch.n_pairs + chunk - 1) // chunk, float(np.abs(s_gpu - s_ref).max()), rel,
              loss_gpu, loss_ref))
