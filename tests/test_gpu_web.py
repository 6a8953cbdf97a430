"""GPU parity of the graph-store path (kernel path 3, BASELINE config C5: Web-sized
graphs, Padding / NTN width D in [32, 512]) against the numpy oracle, through the
C-ABI (sg_web_forward / sg_web_fwd_bwd).  Tolerance 1e-4 as for the record path;
the oracle's layer math is the same restatement (oracle/siamese_oracle.py) — the
reference has no Web loader (preprocess_web.py is empty), so the graphs
are synthetic and the parity anchor is the oracle, not reference fixtures."""
import numpy as np
import pytest

from _fixtures import check_grad_per_var, run_oracle_step, small_problem

pytestmark = pytest.mark.gpu

TOL = 1e-4

# name: (n_graphs, n_pairs, n_lo, n_hi, D, p_extra, flag overrides)
CASES = {
    'd64': (10, 24, 20, 60, 64, {}, 0.15),
    'd64_nodrop': (10, 24, 20, 60, 64, dict(dropout=0.0), 0.15),
    'd96_aligned_intended': (10, 20, 30, 90, 96, dict(loss_mode='aligned', ntn_mode='intended'),
                             0.1),
    'd64_sigmoid_final': (8, 16, 10, 64, 64, dict(final_act='sigmoid'), 0.15),
    'd256_sparse': (8, 16, 64, 250, 256, {}, 0.03),
    'd512_web': (5, 6, 200, 512, 512, {}, 0.012),
    'd40_single_node': (10, 24, 1, 40, 40, {}, 0.2),
}


def _problem(name, seed=31):
    G, P, lo, hi, D, ov, pe = CASES[name]
    return small_problem(n_graphs=G, n_pairs=P, seed=seed, n_lo=lo, n_hi=hi, n_max=D,
                         flags_overrides=ov, p_extra=pe)


def _check_grad(g_gpu, g_ref, prob, tol=TOL):
    """Per variable, each against its own largest reference component (_fixtures)."""
    check_grad_per_var(g_gpu, g_ref, prob.layers, prob.d_in, tol)


@pytest.mark.parametrize('name', list(CASES))
def test_web_matches_oracle(gpu, name):
    prob = _problem(name)
    model, batch = prob.make_gpu_web_model(device=gpu)
    seed = 4321
    s = model.pred_sim_without_act(batch, seed=seed).cpu().numpy()
    ref = run_oracle_step(prob, seed)
    np.testing.assert_allclose(s, ref.s, rtol=TOL, atol=TOL)
    s2 = model.test_scores(batch, seed=seed)
    model.fwd_bwd(batch, seed=seed)
    _check_grad(model.grad.cpu().numpy(), ref.grad_mse, prob)
    loss_mse = float(model.loss_buf[0].item())
    assert abs(loss_mse - ref.loss_mse) <= TOL * max(1.0, abs(ref.loss_mse))
    model.apply_adam()
    reg = float(model.reg_buf[0].item())
    assert abs(loss_mse + reg - ref.loss) <= TOL * max(1.0, abs(ref.loss))
    np.testing.assert_allclose(model.params.cpu().numpy(), ref.new_params, rtol=0, atol=2e-5)
    assert np.array_equal(s2.astype(np.float32), s)


def test_web_wide_types_and_k16(gpu):
    """d_in up to 64 (four one-hot type tiles in the gW0 product), K = 16 NTN maps,
    a 512-node graph (the largest instance the kernels take)."""
    ov = dict(layer_3='Padding:max_in_dims=512,padding_value=0',
              layer_4='NTN:input_dim=512,feature_map_dim=16,inneract=relu,dropout=True,bias=True')
    prob = small_problem(n_graphs=4, n_pairs=6, seed=17, n_lo=500, n_hi=512, n_max=512,
                         n_types=60, flags_overrides=ov, p_extra=0.01)
    assert prob.d_in > 48, prob.d_in
    model, batch = prob.make_gpu_web_model(device=gpu)
    ref = run_oracle_step(prob, 99)
    np.testing.assert_allclose(model.pred_sim_without_act(batch, seed=99).cpu().numpy(), ref.s,
                               rtol=TOL, atol=TOL)
    model.fwd_bwd(batch, seed=99)
    _check_grad(model.grad.cpu().numpy(), ref.grad_mse, prob)


def test_web_padding_value(gpu):
    """Non-zero padding_value: the NTN input is non-zero past the graph's nodes, so
    the kernels run the full D extent."""
    ov = dict(layer_3='Padding:max_in_dims=64,padding_value=1',
              layer_4='NTN:input_dim=64,feature_map_dim=10,inneract=relu,dropout=True,bias=True')
    prob = small_problem(n_graphs=8, n_pairs=12, seed=9, n_lo=10, n_hi=50, n_max=64,
                         flags_overrides=ov)
    model, batch = prob.make_gpu_web_model(device=gpu)
    ref = run_oracle_step(prob, 77)
    np.testing.assert_allclose(model.pred_sim_without_act(batch, seed=77).cpu().numpy(), ref.s,
                               rtol=TOL, atol=TOL)
    model.fwd_bwd(batch, seed=77)
    _check_grad(model.grad.cpu().numpy(), ref.grad_mse, prob)


def test_web_chunks_shards_determinism(gpu):
    """Chunked == one chunk (scores bitwise, gradient to fp32 order), sharded forward
    == unsharded, fwd_bwd bitwise reproducible, gradient additive over shards."""
    import torch
    prob = small_problem(n_graphs=24, n_pairs=700, seed=12, n_lo=20, n_hi=128, n_max=128,
                         p_extra=0.05)
    model, full = prob.make_gpu_web_model(device=gpu)
    _, chunked = prob.make_gpu_web_model(device=gpu, chunk=97)
    seed = 5
    s_full = model.pred_sim_without_act(full, seed=seed).cpu().numpy()
    s_ch = model.pred_sim_without_act(chunked, seed=seed).cpu().numpy()
    assert np.array_equal(s_full, s_ch)
    model.fwd_bwd(full, seed=seed)
    g_full, l_full = model.grad.clone(), float(model.loss_buf[0].item())
    model.fwd_bwd(full, seed=seed)
    assert torch.equal(g_full, model.grad), 'sg_web_fwd_bwd is not bitwise reproducible'
    model.fwd_bwd(chunked, seed=seed)
    g = model.grad.cpu().numpy()
    _check_grad(g, g_full.cpu().numpy(), prob, tol=1e-5)
    # shards of the pair list keyed by their global offset
    h = full.n_pairs // 2
    b0 = model.web_batch(full.csr, full.pairs[:h], full.labels[:h], 0, full.n_pairs,
                         y_stats=full.y_stats)
    b1 = model.web_batch(full.csr, full.pairs[h:], full.labels[h:], h, full.n_pairs,
                         y_stats=full.y_stats)
    s0 = model.pred_sim_without_act(b0, seed=seed).cpu().numpy()
    s1 = model.pred_sim_without_act(b1, seed=seed).cpu().numpy()
    assert np.array_equal(np.concatenate([s0, s1]), s_full)
    model.fwd_bwd(b0, seed=seed, add_label_term=True)
    g0, l0 = model.grad.clone(), float(model.loss_buf[0].item())
    model.fwd_bwd(b1, seed=seed, add_label_term=False)
    _check_grad((g0 + model.grad).cpu().numpy(), g_full.cpu().numpy(), prob, tol=1e-5)
    assert abs(l0 + float(model.loss_buf[0].item()) - l_full) <= 1e-5 * max(1.0, abs(l_full))


def test_web_pipeline_is_bitwise_the_serial_sequence(gpu, monkeypatch):
    """The two-stream chunk pipeline (forward instance kernel of chunk c + 1 beside the
    NTN GEMMs of chunk c, two workspace slots) gives the bits of the one-stream sequence:
    scores, gradient and loss, forward and fwd_bwd, over several chunks."""
    import torch
    prob = small_problem(n_graphs=24, n_pairs=700, seed=13, n_lo=20, n_hi=128, n_max=128,
                         p_extra=0.05)
    model, chunked = prob.make_gpu_web_model(device=gpu, chunk=97)
    out = {}
    for mode in ('1', '0'):
        monkeypatch.setenv('SG_WEB_PIPE', mode)
        s = model.pred_sim_without_act(chunked, seed=9).clone()
        model.fwd_bwd(chunked, seed=9)
        torch.cuda.synchronize()
        out[mode] = (s, model.grad.clone(), model.loss_buf.clone())
    for a, b in zip(out['1'], out['0']):
        assert torch.equal(a, b)


def test_web_t_kernel_k_groups_are_bitwise(gpu, monkeypatch):
    """The T GEMM with four feature maps per block (web_t_kernel_kg: the x2 chunk staged once
    for four W[k] planes) keeps web_t_kernel_b3's MFMA order per (k, tile): scores, gradient
    and loss bitwise those of one k per block, K = 10 (groups 4, 4, 2) and K = 16."""
    import torch
    for K in (10, 16):
        ov = dict(layer_3='Padding:max_in_dims=256,padding_value=0',
                  layer_4='NTN:input_dim=256,feature_map_dim={},inneract=relu,dropout=True,'
                          'bias=True'.format(K))
        prob = small_problem(n_graphs=20, n_pairs=600, seed=23, n_lo=20, n_hi=250, n_max=256,
                             flags_overrides=ov, p_extra=0.03)
        model, chunked = prob.make_gpu_web_model(device=gpu, chunk=251)
        out = {}
        for mode in ('1', '0'):
            monkeypatch.setenv('SG_WEB_TKG', mode)
            s = model.pred_sim_without_act(chunked, seed=3).clone()
            model.fwd_bwd(chunked, seed=3)
            torch.cuda.synchronize()
            out[mode] = (s, model.grad.clone(), model.loss_buf.clone())
        for a, b in zip(out['1'], out['0']):
            assert torch.equal(a, b), K


def test_web_xcd_units_match_flat_units(gpu, monkeypatch):
    """The XCD-partitioned unit order (instances of graph g on the blocks of partition
    g % 8) changes only which workgroup runs an instance: scores and loss are bitwise
    those of the plain size-class order, the gradient equal up to the order of the
    per-block sums (and bitwise reproducible)."""
    import torch
    prob = small_problem(n_graphs=40, n_pairs=900, seed=21, n_lo=8, n_hi=128, n_max=128,
                         p_extra=0.05)
    model, chunked = prob.make_gpu_web_model(device=gpu, chunk=301)
    out = {}
    for mode in ('1', '0', '1'):
        monkeypatch.setenv('SG_WEB_XCD', mode)
        s = model.pred_sim_without_act(chunked, seed=5).clone()
        model.fwd_bwd(chunked, seed=5)
        torch.cuda.synchronize()
        r = (s, model.grad.clone(), model.loss_buf.clone())
        if mode in out:
            assert all(torch.equal(a, b) for a, b in zip(out[mode], r))
        out[mode] = r
    (s1, g1, l1), (s0, g0, l0) = out['1'], out['0']
    assert torch.equal(s1, s0)
    assert torch.equal(l1, l0)
    _check_grad(g1.cpu().numpy(), g0.cpu().numpy(), prob, tol=1e-5)


def test_web_empty_batch(gpu):
    prob = _problem('d64')
    model, batch = prob.make_gpu_web_model(device=gpu)
    empty = model.web_batch(batch.csr, batch.pairs[:0], batch.labels[:0], 0, 1,
                            y_stats=batch.y_stats)
    model.fwd_bwd(empty, seed=1)
    assert float(model.grad.abs().max().item()) == 0.0


def test_web_pipeline_streams_per_caller_stream_and_release(gpu):
    """The chunk pipeline's second stream is per (device, caller stream): steps issued on two
    torch streams give the one-stream bits, and sg_web_release (teardown) destroys the
    auxiliary streams, after which a call re-creates them."""
    import torch
    from graphembedding_amd import _lib
    prob = small_problem(n_graphs=24, n_pairs=500, seed=14, n_lo=20, n_hi=128, n_max=128,
                         p_extra=0.05)
    model, chunked = prob.make_gpu_web_model(device=gpu, chunk=97)
    ref = model.pred_sim_without_act(chunked, seed=4).clone()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        s_side = model.pred_sim_without_act(chunked, seed=4)
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    assert torch.equal(s_side, ref)
    _lib.web_release()
    assert torch.equal(model.pred_sim_without_act(chunked, seed=4), ref)
    _lib.web_release()
