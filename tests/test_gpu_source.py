"""Store-sourced pairs (sg_*_src, library 1.6) on the AIDS700nef fused kernel (path 1,
default and tuning.py Average stacks): the kernel gathers each pair's graphs from the
dense store and must equal the same pairs packed into records, bit for bit.  (The
capacity-32 kernel's case is tests/test_gpu_fast32.py.)"""
import numpy as np
import pytest

from _fixtures import AVERAGE_STACK, small_problem

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('stack', ['default', 'average', 'attention'])
def test_fused_store_source_matches_records(gpu, stack):
    import torch
    from graphembedding_amd import _lib
    from graphembedding_amd.packer import GraphStore
    ov = {'default': {}, 'average': dict(AVERAGE_STACK),
          'attention': dict(AVERAGE_STACK, layer_2='Attention:input_dim=16')}[stack]
    prob = small_problem(n_graphs=40, n_pairs=8, seed=31, n_lo=1, n_hi=10, n_max=10,
                         flags_overrides=ov)
    model, _ = prob.make_gpu_model(device=gpu)
    assert model.kernel_path == 1
    G, base, n = 40, 37, 1500   # inside the 40 x 40 grid
    q = np.arange(base, base + n)
    pairs = np.stack([q // G, q % G], axis=1).astype(np.int32)
    labels = np.random.default_rng(4).random(n).astype(np.float32)
    store = GraphStore(prob.mgs, model.n_max, prob.d_in)
    words = store.pack_host(pairs, labels, dtype='f32')
    recs = torch.from_numpy(words.view(np.int32).reshape(-1)).to(gpu)
    b_rec = model.batch_from_records(recs, n, labels, pair_offset=base)
    pi = torch.from_numpy(pairs).to(gpu)
    lab = torch.from_numpy(labels).to(gpu)
    status = torch.zeros(1, dtype=torch.int32, device=gpu)
    b_list = model.batch_from_store(store, n, lab, pair_idx=pi, pair_offset=base, status=status)
    b_grid = model.batch_from_store(store, n, lab, grid_base=base, pair_offset=base,
                                    status=status)
    seed = 13

    def run(b):
        s = model.pred_sim_without_act(b, seed=seed).clone()
        so = torch.empty(n, dtype=torch.float32, device=gpu)
        model.fwd_bwd(b, seed=seed, s_out=so)
        return s, so, model.grad.clone(), model.loss_buf.clone()

    ref = run(b_rec)
    for b in (b_list, b_grid):
        for x, y in zip(ref, run(b)):
            assert torch.equal(x, y)
    # the store-sourced path walks the order with the mixed schedule (no class table),
    # so the record batch does too for a bitwise comparison
    model.balance(b_rec, classes=False)
    model.balance(b_grid)
    assert torch.equal(b_rec.order, b_grid.order)
    for x, y in zip(run(b_rec), run(b_grid)):
        assert torch.equal(x, y)
    assert int(status.item()) == 0
    bad = pi.clone()
    bad[7, 0] = -1
    b_bad = model.batch_from_store(store, n, lab, pair_idx=bad, pair_offset=base, status=status)
    model.fwd_bwd(b_bad, seed=seed)
    torch.cuda.synchronize()
    assert int(status.item()) == _lib.SG_ERR_ARG
