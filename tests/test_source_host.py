"""Host-side logic of store-sourced pairs (library 1.6): when AllPairsStream skips the
pack pass, and the sg_pair_source_t the host builds (CPU only, no kernel calls)."""
from types import SimpleNamespace

import numpy as np
import pytest
import torch

from graphembedding_amd import _lib
from graphembedding_amd.allpairs import AllPairsStream, load_graph_set


@pytest.fixture(scope='module')
def gs():
    return load_graph_set('syn_aids80nef', n_max=32)


def test_stream_source_selection(gs):
    labels = gs.label_matrix(0.6)
    st = AllPairsStream(gs, labels, 0, 1, device='cpu', chunk=1000)
    fused32 = SimpleNamespace(kernel_path=2, record_dtype='f32', n_max=32)
    assert st.uses_store(fused32)
    assert st.records is None                      # no record buffer up front
    assert not st.uses_store(SimpleNamespace(kernel_path=0, record_dtype='f32', n_max=32))
    assert not st.uses_store(SimpleNamespace(kernel_path=2, record_dtype='bf16', n_max=32))
    assert not st.uses_store(SimpleNamespace(kernel_path=1, record_dtype='f32', n_max=10))
    rec = AllPairsStream(gs, labels, 0, 1, device='cpu', chunk=1000, source='records')
    assert not rec.uses_store(fused32)
    with pytest.raises(RuntimeError):
        AllPairsStream(gs, labels, 0, 1, device='cpu', source='bogus')


def test_stream_chunks_cover_the_shard(gs):
    labels = gs.label_matrix(0.6)
    G = len(gs.graphs)
    for world in (1, 3):
        seen = []
        for r in range(world):
            st = AllPairsStream(gs, labels, r, world, device='cpu', chunk=777)
            seen += [(c0, n) for c0, n in st.chunks()]
        flat = np.concatenate([np.arange(c0, c0 + n) for c0, n in seen])
        assert np.array_equal(np.sort(flat), np.arange(G * G))   # grid_base = c0 per chunk


def test_pair_source_struct(gs):
    adj, types, n = gs.store.to_device('cpu')
    pi = torch.zeros((4, 2), dtype=torch.int32)
    lab = torch.zeros(4, dtype=torch.float32)
    src = _lib.pair_source((adj, types, n), 32, pair_idx=pi, grid_base=5, labels=lab)
    assert src.n_graphs == len(gs.graphs) and src.n_max == 32 and src.grid_base == 5
    assert src.adj == adj.data_ptr() and src.pair_idx == pi.data_ptr()
    assert src.labels == lab.data_ptr() and not src.status
    grid = _lib.pair_source((adj, types, n), 32)
    assert not grid.pair_idx and grid.grid_base == 0


def test_batch_from_store_checks(gs):
    """Bad pair lists are refused on the host (the kernel would read past them)."""
    from graphembedding_amd.config import Flags
    from graphembedding_amd.model_mse import SiameseGCNTNMSE
    f = Flags(dropout=0.1, layer_3='Padding:max_in_dims=30,padding_value=0',
              layer_4='NTN:input_dim=30,feature_map_dim=10,inneract=relu,dropout=True,'
                      'bias=True')
    model = SiameseGCNTNMSE(gs.d_in, f, device='cpu', n_max=32)
    assert model.kernel_path == 2
    lab = torch.zeros(8)
    with pytest.raises(_lib.SiameseHipError):
        model.batch_from_store(gs.store, 8, lab, pair_idx=torch.zeros((4, 2), dtype=torch.int32))
    with pytest.raises(_lib.SiameseHipError):
        model.batch_from_store(gs.store, 8, lab, pair_idx=torch.zeros((8, 2)))
    with pytest.raises(_lib.SiameseHipError):
        model.batch_from_store(gs.store, 8, torch.zeros(3), grid_base=0)
    with pytest.raises(_lib.SiameseHipError):
        model.batch_from_store(gs.store, 8, lab, grid_base=-1)
    b = model.batch_from_store(gs.store, 8, lab, grid_base=3, pair_offset=3)
    assert b.records is None and b.src.grid_base == 3 and b.n_pairs == 8
