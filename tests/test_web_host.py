"""CPU tests of the graph-store path's host side (config C5): model validation
routes Web-sized stacks to path 3, the CSR store reproduces Â and the one-hot
columns exactly, the size ordering and rank shards partition the all-pairs list,
and the workspace / LDS sizing calls are host-only."""
import numpy as np
import pytest

from _fixtures import small_problem
from graphembedding_amd import _lib
from graphembedding_amd.web import (CsrStore, WebAllPairs, allpairs_ids, dealt_size_order,
                                    size_order)


def _model(prob, n_max, **kw):
    return _lib.make_model(prob.layers, prob.d_in, n_max, 0.9, 'sim_kernel', 'gaussian', 0.6,
                           **kw)


@pytest.mark.parametrize('D', [32, 64, 200, 512])
def test_web_stacks_take_path_3(D):
    prob = small_problem(n_graphs=4, n_pairs=4, seed=2, n_lo=5, n_hi=min(D, 40), n_max=D)
    n, path = _lib.validate(_model(prob, D))
    assert path == _lib.PATH_WEB
    assert n == prob.d_in * 32 + 32 + 32 * 16 + 16 + 16 + 1 + D * D * 10 + 10 * 2 * D + 10 + 10
    assert _lib.web_workspace_bytes(_model(prob, D), 1000) > 0


def test_web_path_limits():
    prob = small_problem(n_graphs=4, n_pairs=4, seed=2, n_lo=5, n_hi=30, n_max=30)
    assert _lib.validate(_model(prob, 32))[1] == 2            # C4 capacity-32 kernel
    big = small_problem(n_graphs=2, n_pairs=2, seed=2, n_lo=5, n_hi=30, n_max=520)
    with pytest.raises(_lib.SiameseHipError):                  # D > 512: no kernel
        _lib.validate(_model(big, 520))
    mid = small_problem(n_graphs=2, n_pairs=2, seed=2, n_lo=5, n_hi=30, n_max=64)
    with pytest.raises(_lib.SiameseHipError):                  # N > max_in_dims (A9)
        _lib.validate(_model(mid, 65))


def test_csr_store_reproduces_adjacency():
    prob = small_problem(n_graphs=9, n_pairs=4, seed=6, n_lo=1, n_hi=70, n_max=128,
                         p_extra=0.05)
    st = CsrStore(prob.mgs, prob.d_in, 128)
    assert st.node_off[-1] == sum(m.num_nodes() for m in prob.mgs)
    for g, mg in enumerate(prob.mgs):
        o, n = int(st.node_off[g]), int(st.n[g])
        A = np.zeros((n, n), np.float32)
        for r in range(n):
            e0, e1 = st.row_ptr[o + r], st.row_ptr[o + r + 1]
            A[r, st.col[e0:e1]] = st.val[e0:e1]
        assert np.array_equal(A, mg.adj.astype(np.float32))
        assert np.array_equal(st.types[o:o + n], mg.types)
    assert st.max_nnz == max(int(np.count_nonzero(m.adj)) for m in prob.mgs)
    with pytest.raises(RuntimeError):
        CsrStore(prob.mgs, prob.d_in, 10)                      # tf.pad: N > max_in_dims


def test_size_order_and_shards():
    n_nodes = np.array([300, 64, 500, 64, 120], np.int32)
    ids = allpairs_ids(5, 0, 25)
    order = size_order(ids, n_nodes)
    assert sorted(order.tolist()) == list(range(25))
    key = (n_nodes[ids[order, 0]] // 32) * 64 + n_nodes[ids[order, 1]] // 32
    assert np.all(np.diff(key) >= 0)


def test_dealt_order_balances_shards():
    rng = np.random.default_rng(0)
    G = 600
    n_nodes = rng.integers(64, 513, size=G).astype(np.int32)
    P = G * G
    ids = allpairs_ids(G, 0, P)
    order = dealt_size_order(ids, n_nodes)
    assert np.array_equal(np.sort(order), np.arange(P))
    cost = (n_nodes[ids[order, 0]].astype(np.float64) * n_nodes[ids[order, 1]])
    for W in (2, 4, 8):
        per = [cost[r * P // W:(r + 1) * P // W].sum() for r in range(W)]
        assert max(per) / min(per) < 1.03, (W, per)
    b1 = (n_nodes[ids[order[:128 * 64], 0]] // 32).reshape(-1, 128)
    assert np.mean(b1.max(1) - b1.min(1) <= 1) > 0.9   # blocks stay size-homogeneous


def test_web_allpairs_shards_partition_the_list():
    from types import SimpleNamespace
    prob = small_problem(n_graphs=7, n_pairs=2, seed=4, n_lo=3, n_hi=60, n_max=64)
    gs = SimpleNamespace(graphs=prob.graphs, mgs=prob.mgs, d_in=prob.d_in)
    labels = np.arange(49, dtype=np.float32).reshape(7, 7) / 49
    full = WebAllPairs(gs, labels, 0, 1, device='cpu')
    parts = [WebAllPairs(gs, labels, r, 3, device='cpu') for r in range(3)]
    assert sum(p.n for p in parts) == 49
    cat = np.concatenate([p.pairs.numpy() for p in parts])
    assert np.array_equal(cat, full.pairs.numpy())
    lab = np.concatenate([p.labels.numpy() for p in parts])
    assert np.array_equal(lab, labels[cat[:, 0], cat[:, 1]])
    assert all(np.allclose(p.y_stats.numpy(), full.y_stats.numpy()) for p in parts)
    assert [p.start for p in parts] == [0, parts[0].end, parts[1].end]


def test_workspace_one_slot_for_single_chunk_calls():
    """sg_web_workspace_bytes_ex: a call of at most one chunk never pipelines, so it needs
    one of the two per-chunk slots; several chunks need both, as
    sg_web_workspace_bytes reports."""
    prob = small_problem(n_graphs=6, n_pairs=6, n_lo=20, n_hi=60, n_max=64)
    m = _model(prob, 64)
    two = _lib.web_workspace_bytes(m, 4096)
    assert _lib.web_workspace_bytes(m, 4096, 4097) == two
    one = _lib.web_workspace_bytes(m, 4096, 4096)
    assert one == _lib.web_workspace_bytes(m, 4096, 0) and one < two
    # the slots dominate: the second one is most of the difference from the per-call part
    assert two - one > 0.4 * two
    # chunk 0 = one chunk of the whole call (sg_web_run): sized for n_pairs, not for 1 pair
    assert _lib.web_workspace_bytes(m, 0, 4096) == one
    assert _lib.web_workspace_bytes(m, 0, 1) == _lib.web_workspace_bytes(m, 1, 1)
    with pytest.raises(_lib.SiameseHipError):
        _lib.web_workspace_bytes(m, 0)           # any n_pairs in chunk 0: not sizable


def test_model_web_workspace_slots():
    """model.web_workspace: a batch that fits one chunk gets the one-slot size, a longer one
    both slots; a two-slot workspace already allocated serves one-chunk calls too."""
    from graphembedding_amd.model_mse import SiameseGCNTNMSE
    prob = small_problem(n_graphs=6, n_pairs=6, n_lo=20, n_hi=60, n_max=64)
    m = SiameseGCNTNMSE(prob.d_in, prob.flags, device='cpu', n_max=64)
    assert m.is_web
    one = _lib.web_workspace_bytes(m.sg, 512, 512)
    two = _lib.web_workspace_bytes(m.sg, 512)
    w1 = m.web_workspace(512, 100)
    assert w1.numel() * 4 >= one and w1.numel() * 4 < two
    w2 = m.web_workspace(512, 5000)               # several chunks: grows to both slots
    assert w2.numel() * 4 >= two
    assert m.web_workspace(512, 10).data_ptr() == w2.data_ptr()   # reused
    w3 = m.web_workspace(256, 10)                 # another chunk size: reallocated
    assert w3.numel() * 4 >= _lib.web_workspace_bytes(m.sg, 256, 10)
