"""Parity at the BASELINE configs' full sizes (the bench workloads), where the numpy
oracle cannot run the whole batch: a seeded sample of pairs of the full step is
checked against the oracle, and size-independent properties cover the rest
(ordered == batch-order scores bitwise, bitwise replay, gradient of the step == sum
of its 8 rank shards).  Tolerance 1e-4 (north_star)."""
import numpy as np
import pytest

from oracle import siamese_oracle as O

pytestmark = pytest.mark.gpu

TOL = 1e-4
C4_FLAGS = dict(layer_3='Padding:max_in_dims=30,padding_value=0',
                layer_4='NTN:input_dim=30,feature_map_dim=10,inneract=relu,dropout=True,'
                        'bias=True')
WEB_FLAGS = dict(layer_3='Padding:max_in_dims=512,padding_value=0',
                 layer_4='NTN:input_dim=512,feature_map_dim=10,inneract=relu,dropout=True,'
                         'bias=True')


def _spec(model, f):
    return O.OracleSpec(layers=model.layers, d_in=model.input_dim, keep_prob=1.0 - f.dropout,
                        final_act=f.final_act, sim_kernel=f.sim_kernel, yeta=f.yeta,
                        loss_mode=f.loss_mode, ntn_mode=f.ntn_mode,
                        weight_decay=f.weight_decay, dist_norm=f.dist_norm)


def _graphs(gs, bf16=False):
    from graphembedding_amd.packer import bf16_round
    # bf16 records hold Â rounded to bf16 (RNE); the kernels compute with that Â
    cast = (lambda a: bf16_round(a.astype(np.float32))) if bf16 else \
        (lambda a: a.astype(np.float32))
    return [O.Graph(adj=cast(m.adj).astype(np.float64), types=m.types) for m in gs.mgs]


def _oracle_scores(model, f, gs, pairs, keys, seed, bf16=False):
    spec = _spec(model, f)
    P = O.unflatten(spec, model.params.cpu().numpy().astype(np.float64))
    og = _graphs(gs, bf16)
    return np.array([O.pair_forward(spec, P, og[i], og[j], int(k), seed)[0]
                     for (i, j), k in zip(pairs, keys)])


def test_c2_full_allpairs_step(gpu):
    """C2: AIDS700nef all-pairs, 490,000 pairs, the headline bench's resident batch."""
    import torch
    from graphembedding_amd.allpairs import AllPairsShard, load_graph_set
    from graphembedding_amd.config import Flags
    from graphembedding_amd.model_mse import SiameseGCNTNMSE
    f = Flags(dropout=0.1)
    gs = load_graph_set('syn_aids700nef', n_max=10)
    labels = gs.label_matrix(f.yeta)
    model = SiameseGCNTNMSE(gs.d_in, f, device=gpu, n_max=gs.n_max)
    assert model.kernel_path == 1
    shard = AllPairsShard(gs, labels, 0, 1, device=gpu)
    batch = shard.batch(model, balance=False)
    assert batch.n_pairs == 490000
    seed = 2024
    s = model.pred_sim_without_act(batch, seed=seed)
    G = len(gs.graphs)
    idx = np.random.default_rng(7).choice(batch.n_pairs, 48, replace=False)
    ref = _oracle_scores(model, f, gs, [(i // G, i % G) for i in idx], idx, seed)
    np.testing.assert_allclose(s.cpu().numpy()[idx], ref, rtol=TOL, atol=TOL)
    model.fwd_bwd(batch, seed=seed)
    g_batch = model.grad_loss.clone()
    model.balance(batch)
    assert torch.equal(model.pred_sim_without_act(batch, seed=seed), s)
    model.fwd_bwd(batch, seed=seed)
    g_full = model.grad_loss.clone()
    model.fwd_bwd(batch, seed=seed)
    assert torch.equal(g_full, model.grad_loss), 'fwd_bwd is not bitwise reproducible'
    scale = max(1.0, float(g_full.abs().max().item()))
    assert float((g_batch - g_full).abs().max().item()) <= 1e-5 * scale
    acc = torch.zeros_like(g_full)
    for r in range(8):
        sh = AllPairsShard(gs, labels, r, 8, device=gpu)
        model.fwd_bwd(sh.batch(model), seed=seed, add_label_term=(r == 0))
        acc += model.grad_loss
    assert float((acc - g_full).abs().max().item()) <= 1e-5 * scale


def test_c3_full_allpairs_bf16_sampled_pairs(gpu):
    """C3: the C2 step with bf16 Â records (496 B/pair): sampled pairs vs the oracle on
    the bf16-rounded Â."""
    from graphembedding_amd.allpairs import AllPairsShard, load_graph_set
    from graphembedding_amd.config import Flags
    from graphembedding_amd.model_mse import SiameseGCNTNMSE
    f = Flags(dropout=0.1, record_dtype='bf16')
    gs = load_graph_set('syn_aids700nef', n_max=10)
    labels = gs.label_matrix(f.yeta)
    model = SiameseGCNTNMSE(gs.d_in, f, device=gpu, n_max=gs.n_max)
    assert model.kernel_path == 1 and model.record_dtype == 'bf16'
    batch = AllPairsShard(gs, labels, 0, 1, device=gpu, dtype='bf16').batch(model)
    seed = 77
    s = model.pred_sim_without_act(batch, seed=seed).cpu().numpy()
    G = len(gs.graphs)
    idx = np.random.default_rng(13).choice(batch.n_pairs, 48, replace=False)
    ref = _oracle_scores(model, f, gs, [(i // G, i % G) for i in idx], idx, seed, bf16=True)
    np.testing.assert_allclose(s[idx], ref, rtol=TOL, atol=TOL)


def test_c4_full_grid_sampled_pairs(gpu):
    """C4: AIDS10knef all-pairs grid (10,018² = 100.4 M pairs): sampled pairs through
    the store-sourced kernel (each at its global pair index) against the oracle."""
    import torch
    from graphembedding_amd.allpairs import load_graph_set
    from graphembedding_amd.config import Flags
    from graphembedding_amd.model_mse import SiameseGCNTNMSE
    f = Flags(dropout=0.1, **C4_FLAGS)
    gs = load_graph_set('syn_aids10knef', n_max=32)
    G = len(gs.graphs)
    assert G == 10018
    model = SiameseGCNTNMSE(gs.d_in, f, device=gpu, n_max=gs.n_max)
    assert model.kernel_path == 2
    seed = 99
    idx = np.random.default_rng(11).choice(G * G, 32, replace=False)
    lab = torch.zeros(1, dtype=torch.float32, device=gpu)
    got = []
    for q in idx:
        b = model.batch_from_store(gs.store, 1, lab, grid_base=int(q), pair_offset=int(q))
        got.append(float(model.pred_sim_without_act(b, seed=seed).item()))
    ref = _oracle_scores(model, f, gs, [(q // G, q % G) for q in idx], idx, seed)
    np.testing.assert_allclose(np.array(got), ref, rtol=TOL, atol=TOL)


def test_c5_web_sampled_pairs(gpu):
    """C5: Web-sized all-pairs (1,100 graphs, N up to 512, 1.21 M pairs) in the bench's
    dealt size order: sampled positions of the full list against the oracle."""
    import torch
    from graphembedding_amd import _lib
    from graphembedding_amd.allpairs import load_graph_set
    from graphembedding_amd.config import Flags
    from graphembedding_amd.model_mse import SiameseGCNTNMSE
    from graphembedding_amd.web import WebAllPairs
    f = Flags(dropout=0.1, **WEB_FLAGS)
    gs = load_graph_set('syn_web', n_max=512, with_store=False)
    labels = gs.label_matrix(f.yeta)
    model = SiameseGCNTNMSE(gs.d_in, f, device=gpu, n_max=gs.n_max)
    assert model.kernel_path == _lib.PATH_WEB
    shard = WebAllPairs(gs, labels, 0, 1, device=gpu)
    batch = shard.batch(model)
    assert batch.n_pairs == len(gs.graphs) ** 2
    seed = 5
    s = model.pred_sim_without_act(batch, seed=seed).cpu().numpy()
    idx = np.random.default_rng(3).choice(batch.n_pairs, 6, replace=False)
    pairs = batch.pairs.cpu().numpy()[idx]
    ref = _oracle_scores(model, f, gs, pairs, idx, seed)
    np.testing.assert_allclose(s[idx], ref, rtol=TOL, atol=TOL)


def test_c2_fused_scores_cover_every_pair(gpu):
    """Every pair of a launch is scored exactly where it belongs: fused fwd_bwd's s_out
    (NaN-filled before the launch) equals the forward-only scores bit for bit, class
    order on and off, at an emulated 8-rank shard (61,250 pairs) and the full step."""
    import torch
    from graphembedding_amd.allpairs import AllPairsShard, load_graph_set
    from graphembedding_amd.config import Flags
    from graphembedding_amd.model_mse import SiameseGCNTNMSE
    f = Flags(dropout=0.1)
    gs = load_graph_set('syn_aids700nef', n_max=10)
    labels = gs.label_matrix(f.yeta)
    model = SiameseGCNTNMSE(gs.d_in, f, device=gpu, n_max=gs.n_max)
    seed = 99
    for world in (8, 1):
        shard = AllPairsShard(gs, labels, 0, world, device=gpu)
        for balance in (False, True):
            batch = shard.batch(model, balance=balance)
            if balance:
                o = np.sort(batch.order.cpu().numpy())
                assert np.array_equal(o, np.arange(batch.n_pairs)), 'order is not a permutation'
            so = torch.full((batch.n_pairs,), float('nan'), dtype=torch.float32, device=gpu)
            model.fwd_bwd(batch, seed=seed, s_out=so)
            assert int(torch.isnan(so).sum()) == 0, (world, balance)
            assert torch.equal(so, model.pred_sim_without_act(batch, seed=seed)), (world, balance)
