"""Chunked all-pairs stepping (allpairs.AllPairsStream, config C4's path when a
shard's records do not fit HBM) equals one fwd_bwd over the resident shard."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('world,rank', [(1, 0), (3, 1)])
def test_stream_equals_resident_shard(gpu, world, rank):
    from graphembedding_amd.allpairs import AllPairsShard, AllPairsStream, load_graph_set
    from graphembedding_amd.config import Flags
    from graphembedding_amd.model_mse import SiameseGCNTNMSE
    flags = Flags(dropout=0.1)
    gs = load_graph_set('syn_aids80nef', n_max=10)
    labels = gs.label_matrix(flags.yeta)
    model = SiameseGCNTNMSE(gs.d_in, flags, device=gpu, n_max=gs.n_max)
    seed = 11
    res = AllPairsShard(gs, labels, rank, world, device=gpu)
    batch = res.batch(model, balance=False)
    model.fwd_bwd(batch, seed=seed, add_label_term=(rank == 0))
    g_ref = model.grad_loss.cpu().numpy().copy()
    stream = AllPairsStream(gs, labels, rank, world, device=gpu, chunk=777, balance=True)
    assert stream.n == res.n and len(list(stream.chunks())) > 1
    # model.fwd_bwd's default seed depends on step_count: pin it for both runs
    orig = model.fwd_bwd
    model.fwd_bwd = lambda b, add_label_term=True: orig(b, seed=seed, add_label_term=add_label_term)
    stream.fwd_bwd(model, add_label_term=(rank == 0))
    stream.check_status()
    g = model.grad_loss.cpu().numpy()
    scale = max(1.0, float(np.abs(g_ref).max()))
    assert float(np.abs(g - g_ref).max()) <= 1e-5 * scale


C4_FLAGS = dict(layer_3='Padding:max_in_dims=30,padding_value=0',
                layer_4='NTN:input_dim=30,feature_map_dim=10,inneract=relu,dropout=True,'
                        'bias=True')


@pytest.mark.parametrize('world,rank', [(1, 0), (3, 2)])
def test_stream_from_store_equals_resident_records(gpu, world, rank):
    """The C4 kernel's streamed step gathers pairs from the graph store (no records,
    sg_fwd_bwd_src) and equals one fwd_bwd over the shard's packed records."""
    from graphembedding_amd.allpairs import AllPairsShard, AllPairsStream, load_graph_set
    from graphembedding_amd.config import Flags
    from graphembedding_amd.model_mse import SiameseGCNTNMSE
    flags = Flags(dropout=0.1, **C4_FLAGS)
    gs = load_graph_set('syn_aids80nef', n_max=32)
    labels = gs.label_matrix(flags.yeta)
    model = SiameseGCNTNMSE(gs.d_in, flags, device=gpu, n_max=gs.n_max)
    assert model.kernel_path == 2
    seed = 5
    res = AllPairsShard(gs, labels, rank, world, device=gpu)
    batch = res.batch(model, balance=False)
    model.fwd_bwd(batch, seed=seed, add_label_term=(rank == 0))
    g_ref = model.grad_loss.cpu().numpy().copy()
    stream = AllPairsStream(gs, labels, rank, world, device=gpu, chunk=501, balance=True)
    assert stream.uses_store(model) and len(list(stream.chunks())) > 1
    orig = model.fwd_bwd
    model.fwd_bwd = lambda b, add_label_term=True: orig(b, seed=seed, add_label_term=add_label_term)
    stream.fwd_bwd(model, add_label_term=(rank == 0))
    stream.check_status()
    assert stream.records is None   # nothing was packed
    g = model.grad_loss.cpu().numpy()
    scale = max(1.0, float(np.abs(g_ref).max()))
    assert float(np.abs(g - g_ref).max()) <= 1e-5 * scale


def test_stream_kept_batches_are_per_model(gpu):
    """Store-sourced chunk batches are built once (prepare) and reused by later steps of the
    same model; a second model gets batches of its own, and a step over the kept batches
    equals one that rebuilds them (keep_orders=False)."""
    from graphembedding_amd.allpairs import AllPairsStream, load_graph_set
    from graphembedding_amd.config import Flags
    from graphembedding_amd.model_mse import SiameseGCNTNMSE
    flags = Flags(dropout=0.1, **C4_FLAGS)
    gs = load_graph_set('syn_aids80nef', n_max=32)
    labels = gs.label_matrix(flags.yeta)
    m1 = SiameseGCNTNMSE(gs.d_in, flags, device=gpu, n_max=gs.n_max)
    m2 = SiameseGCNTNMSE(gs.d_in, flags, device=gpu, n_max=gs.n_max)
    kept = AllPairsStream(gs, labels, 0, 1, device=gpu, chunk=1111, balance=True)
    fresh = AllPairsStream(gs, labels, 0, 1, device=gpu, chunk=1111, balance=True,
                           keep_orders=False)
    n_chunks = len(list(kept.chunks()))
    assert kept.prepare(m1) == n_chunks > 1
    b1 = kept._pack(m1, kept.start, min(kept.chunk, kept.end - kept.start))
    assert kept._pack(m1, kept.start, min(kept.chunk, kept.end - kept.start)) is b1
    b2 = kept._pack(m2, kept.start, min(kept.chunk, kept.end - kept.start))
    assert b2 is not b1
    seed = 7
    grads = []
    for st in (kept, fresh):
        orig = m2.fwd_bwd
        m2.fwd_bwd = lambda b, add_label_term=True: orig(b, seed=seed,
                                                          add_label_term=add_label_term)
        st.fwd_bwd(m2)
        m2.fwd_bwd = orig
        grads.append(m2.grad_loss.cpu().numpy().copy())
    assert np.array_equal(grads[0], grads[1])
