"""A 20-step training trajectory of the reference's default loop: train_val's
FLAGS.iters = 20 steps of B = 5 pairs (model/Siamese/train.py:8-44, config.py:70,111),
each step get_feed_dict -> sess.run([opt_op, loss]) with TF Adam (models.py:28-36), on
AIDS80nef-shaped data (52 training graphs, so the sampler wraps and re-shuffles its list
in place many times: samplers.py:24-31, quirk A6), with the B + B² label draws of quirk
A3 (label_stream 'compat').

The one-hot column map is pinned (node_feat_order='sorted'): the reference's set order
(graphs.py:101-104, quirk A7) depends on PYTHONHASHSEED for string atom types, so an
unpinned map trains a different problem in every process.

The GPU runs the device feed (sg_feed_step) -> fused fwd+bwd -> sg_adam_tf, eagerly and
as one captured hipGraph of 20 steps.  Checked per step:
- the device feed equals the host get_feed_dict byte for byte (inputs and labels);
- teacher-forced: the oracle's float64 update from the GPU's own pre-step state (params,
  Adam m and v, β powers) is within 2e-5 of the GPU's update, and the step's loss
  (incl. weight decay) within 1e-4;
- the validation leg (train.py:19-21,88-93): device val feed == host val feed, val loss
  within 1e-4 of the oracle at the post-step parameters with the val seed stream's masks.
After 20 steps, against a FLOAT32 free-running oracle trajectory — the C restatement's
fp32 fwd+bwd (oracle/siamese_cpu.c) plus float32 TF ApplyAdam
(siamese_oracle.adam_tf_step_f32), i.e. the reference's own fp32 training — :
- the parameters within 1e-4;
- the SCORES of the trained model (north_star's quantity) on the reference's test matrix
  (test i x get_orig_train_graph(j) after the in-place shuffles, train.py:47-74) within
  1e-4, pre-activation s and final ŷ = exp(-η s²), dropout on (A4) with the eval seed.
The float64 free-running trajectory is reported beside it (fp32 rounding drift).
Dropout 0 and 0.1."""
import numpy as np
import pytest

from oracle import cpu_ref
from oracle import siamese_oracle as O

pytestmark = pytest.mark.gpu

STEPS = 20


def _setup(gpu, dropout):
    from graphembedding_amd.config import Flags
    from graphembedding_amd.data import synthetic_ged_matrix
    from graphembedding_amd.data_siamese import SiameseModelData
    from graphembedding_amd.device_sampler import DeviceFeed
    from graphembedding_amd.dist_calculator import DistCalculator
    from graphembedding_amd.model_mse import SiameseGCNTNMSE
    f = Flags(dataset='syn_aids80nef', sampler='random', label_stream='compat', batch_size=5,
              dropout=dropout, node_feat_order='sorted')
    assert f.iters == STEPS

    def make():
        data = SiameseModelData(f)
        gs = list(data.orig_train_graphs) + [data.test_data.gs[i].nxgraph for i in range(data.m)]
        return data, DistCalculator.from_matrix(f.dataset, gs, synthetic_ged_matrix(gs))
    data_d, dc_d = make()
    model = SiameseGCNTNMSE(data_d.input_dim(), f, device=gpu)
    assert model.kernel_path == 1
    return f, make, model, data_d, DeviceFeed(model, data_d, dc_d, 'train')


def _oracle_graphs(words, n_max):
    from graphembedding_amd.packer import unpack_host
    r = unpack_host(words, n_max)
    out = ([], [])
    for i in range(words.shape[0]):
        for side in (0, 1):
            n = int(r['n'][i, side])
            out[side].append(O.Graph(adj=r['adj'][i, side, :n, :n].astype(np.float64),
                                     types=r['types'][i, side, :n].astype(np.int64)))
    return out


def _gids(gl):
    return [g.nxgraph.graph['gid'] for g in gl]


@pytest.mark.parametrize('dropout', [0.0, 0.1])
def test_default_loop_20_steps_match_oracle(gpu, dropout):
    import torch
    from graphembedding_amd.device_sampler import DeviceFeed
    from graphembedding_amd.packer import record_words
    f, make, model, data_d, feed = _setup(gpu, dropout)
    data_h, dc_h = make()
    spec = O.OracleSpec(layers=model.layers, d_in=model.input_dim, keep_prob=1.0 - f.dropout,
                        final_act=f.final_act, sim_kernel=f.sim_kernel, yeta=f.yeta,
                        loss_mode=f.loss_mode, ntn_mode=f.ntn_mode,
                        weight_decay=f.weight_decay, dist_norm=f.dist_norm)
    p0 = model.params.cpu().numpy().copy()
    flat = p0.astype(np.float64)            # float64 free-running trajectory (reported)
    st = O.adam_init(flat.size)
    th32 = p0.copy()                        # float32 free-running trajectory (asserted)
    st32 = O.adam_init(th32.size)
    W = record_words(model.n_max, model.record_dtype)
    # the validation leg of train_val (train.py:19-21,88-93): sess.run([loss]) on a val
    # feed after every train step — the loss at the current parameters, no update, with
    # dropout masks from the val seed stream; fed by the device val feed, which must equal
    # the host get_feed_dict(..., 'val') byte for byte
    data_v, dc_v = make()
    vfeed = DeviceFeed(model, data_v, dc_v, 'val')
    steps, worst, vworst = [], 0.0, 0.0
    for step in range(STEPS):
        b = feed.next_batch()
        words = b.records.cpu().numpy().view(np.uint32).reshape(b.n_pairs, W).copy()
        labels = b.labels.cpu().numpy()
        hb = model.get_feed_dict(data_h, dc_h, 'train')     # the host feed, same stream
        assert np.array_equal(hb.records.cpu().numpy().view(np.uint32).reshape(-1, W), words), step
        assert np.array_equal(hb.labels.cpu().numpy(), labels), step
        seed = model._seed(None)
        # the GPU's state before the step (for the teacher-forced one-step check)
        pre = [t.cpu().numpy().astype(np.float64) for t in (model.params, model.adam_m,
                                                            model.adam_v)]
        bp = [float(x) for x in model.beta_powers.cpu().numpy()]
        loss = model.train_step(b)
        g1s, g2s = _oracle_graphs(words, model.n_max)
        # free-running float64 trajectory
        res = O.fwd_bwd(spec, flat, g1s, g2s, labels.astype(np.float64), seed)
        flat = O.adam_tf_step(flat, res.grad, st, lr=f.learning_rate)
        # free-running float32 trajectory: C restatement fwd+bwd, float32 TF Adam; ȳ as the
        # batch's y_stats holds it (float64 mean, stored float32)
        ybar = float(np.float32(labels.astype(np.float64).mean()))
        _, g32, _ = cpu_ref.fwd_bwd_records(words, model.n_max, model.input_dim, th32, seed,
                                            1.0 - f.dropout, f.yeta, ybar)
        th32 = O.adam_tf_step_f32(th32, g32, st32, lr=f.learning_rate,
                                  weight_decay=f.weight_decay)
        # teacher-forced: the oracle's step from the GPU's own pre-step state
        r1 = O.fwd_bwd(spec, pre[0], g1s, g2s, labels.astype(np.float64), seed)
        st1 = O.AdamState(pre[1].copy(), pre[2].copy(), bp[0], bp[1])
        nxt = O.adam_tf_step(pre[0], r1.grad, st1, lr=f.learning_rate)
        one = float(np.abs(model.params.cpu().numpy() - nxt).max())
        worst = max(worst, one)
        assert one <= 2e-5, (step, one)
        assert abs(loss - r1.loss) <= 1e-4 * max(1.0, abs(r1.loss)), (step, loss, r1.loss)
        steps.append((round(loss, 6), round(res.loss, 6)))
        # validation: device val feed == host val feed; loss vs the oracle at 1e-4
        vb = vfeed.next_batch()
        vwords = vb.records.cpu().numpy().view(np.uint32).reshape(vb.n_pairs, W).copy()
        hv = model.get_feed_dict(data_h, dc_h, 'val')
        assert np.array_equal(hv.records.cpu().numpy().view(np.uint32).reshape(-1, W),
                              vwords), ('val feed', step)
        assert np.array_equal(hv.labels.cpu().numpy(), vb.labels.cpu().numpy()), ('val', step)
        vseed = model.val_seed()
        g_before = model.grad_loss.clone()
        vloss = model.val_loss(vb)
        assert torch.equal(g_before, model.grad_loss), 'val_loss must not touch grad | loss'
        v1, v2 = _oracle_graphs(vwords, model.n_max)
        rv = O.fwd_bwd(spec, model.params.cpu().numpy().astype(np.float64), v1, v2,
                       vb.labels.cpu().numpy().astype(np.float64), vseed)
        verr = abs(vloss - rv.loss) / max(1.0, abs(rv.loss))
        vworst = max(vworst, verr)
        assert verr <= 1e-4, ('val loss', step, vloss, rv.loss)
    # the reference's in-place list shuffles (A6), after 20 train and 20 val steps
    feed.sampler.sync_host()
    assert _gids(data_h.train_data.gs) == _gids(feed.sampler.host.gs)
    vfeed.sampler.sync_host()
    assert _gids(data_h.valid_data.gs) == _gids(vfeed.sampler.host.gs)
    got = model.params.cpu().numpy()
    err32 = float(np.abs(got - th32).max())
    err64 = float(np.abs(got.astype(np.float64) - flat).max())
    ref_drift = float(np.abs(th32.astype(np.float64) - flat).max())

    # the trained model's scores on the reference's test matrix (train.py:47-74): test i
    # against get_orig_train_graph(j) of the shuffled lists, one launch, the eval seed
    m, n = data_h.m_n()
    g1s = [data_h.test_data.get_graph(i) for i in range(m) for j in range(n)]
    g2s = [data_h.get_orig_train_graph(j) for i in range(m) for j in range(n)]
    tb = model.make_batch(g1s, g2s)
    tseed = model._seed(None)
    s_gpu = model.test_scores(tb)
    twords = tb.records.cpu().numpy().view(np.uint32).reshape(m * n, W).copy()
    t1, t2 = _oracle_graphs(twords, model.n_max)
    s_ref = O.forward(spec, th32.astype(np.float64), t1, t2, tseed)
    s_64 = O.forward(spec, flat, t1, t2, tseed)
    y_gpu = model.apply_final_act_np(s_gpu)
    y_ref = O.final_act(spec, s_ref)
    s_err = float(np.max(np.abs(s_gpu - s_ref) / np.maximum(1.0, np.abs(s_ref))))
    y_err = float(np.max(np.abs(y_gpu - y_ref)))
    y_err64 = float(np.max(np.abs(y_gpu - O.final_act(spec, s_64))))
    print('dropout {}: teacher-forced max |param err| {:.3g}; after 20 steps max |param err| '
          'vs fp32 oracle {:.3g}, vs fp64 oracle {:.3g} (fp32-vs-fp64 oracle drift {:.3g}); '
          'test-matrix {}x{} max rel |s err| {:.3g}, max |sim err| {:.3g} (vs fp64-trained '
          '{:.3g}); worst val-loss rel err {:.3g}; losses (gpu, oracle) {}'.format(
              dropout, worst, err32, err64, ref_drift, m, n, s_err, y_err, y_err64, vworst,
              steps))
    assert err32 <= 1e-4, err32
    assert s_err <= 1e-4, s_err
    assert y_err <= 1e-4, y_err
    bp = model.beta_powers.cpu().numpy()
    assert bp[0] == np.float32(st.beta1_power) and bp[1] == np.float32(st.beta2_power)

    # the same 20 steps as one captured hipGraph (feed -> fwd_bwd_dseed -> Adam -> seed+1)
    f2, make2, model2, _, feed2 = _setup(gpu, dropout)
    assert np.array_equal(model2.params.cpu().numpy(), p0)
    steps20 = model2.capture_train_steps(feed2, STEPS)
    steps20.replay()
    torch.cuda.synchronize()
    assert torch.equal(model2.params, model.params), 'graph replay != eager steps'
