"""Graph-captured reference training steps (hipGraph replay of DeviceFeed →
sg_fwd_bwd_dseed → Adam → seed advance) == the same steps run eagerly, bitwise:
the fused path sums in a fixed order and the dropout seed comes from the device."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('stack', ['default', 'average'])
def test_graph_steps_equal_eager_steps(gpu, stack):
    import torch
    from _fixtures import AVERAGE_STACK
    from graphembedding_amd.config import Flags
    from graphembedding_amd.data import synthetic_ged_matrix
    from graphembedding_amd.data_siamese import SiameseModelData
    from graphembedding_amd.device_sampler import DeviceFeed
    from graphembedding_amd.dist_calculator import DistCalculator
    from graphembedding_amd.model_mse import SiameseGCNTNMSE
    ov = dict(AVERAGE_STACK) if stack == 'average' else {}
    f = Flags(dataset='syn_aids80nef', node_feat_order='sorted', **ov)

    def make():
        data = SiameseModelData(f)
        gs = list(data.orig_train_graphs) + [data.test_data.gs[i].nxgraph for i in range(data.m)]
        dc = DistCalculator.from_matrix(f.dataset, gs, synthetic_ged_matrix(gs))
        model = SiameseGCNTNMSE(data.input_dim(), f, device=gpu)
        return model, DeviceFeed(model, data, dc, 'train')

    m_e, feed_e = make()
    m_g, feed_g = make()
    assert m_g.kernel_path == 1
    steps = 7
    for _ in range(3 * steps):
        m_e.train_step(feed_e.next_batch(), sync=False)
    g = m_g.capture_train_steps(feed_g, n_steps=steps)
    g.replay(3)
    torch.cuda.synchronize()
    assert m_g.step_count == m_e.step_count == 3 * steps
    for a, b in ((m_e.params, m_g.params), (m_e.adam_m, m_g.adam_m), (m_e.adam_v, m_g.adam_v),
                 (m_e.loss_buf, m_g.loss_buf), (feed_e.sampler.state, feed_g.sampler.state)):
        assert torch.equal(a, b)
    assert not torch.equal(m_g.params, torch.from_numpy(
        np.asarray(m_g.flat_params())).to(gpu) * 0), 'params moved'


def test_graph_capture_refuses_a_grad_hook(gpu):
    """A data-parallel gradient hook is host-driven (torch.distributed): a hipGraph cannot
    record it, so capture_train_steps refuses a model that has one instead of silently
    replaying steps without the exchange."""
    from graphembedding_amd.config import Flags
    from graphembedding_amd.data import synthetic_ged_matrix
    from graphembedding_amd.data_siamese import SiameseModelData
    from graphembedding_amd.device_sampler import DeviceFeed
    from graphembedding_amd.dist_calculator import DistCalculator
    from graphembedding_amd.model_mse import SiameseGCNTNMSE
    f = Flags(dataset='syn_aids80nef', node_feat_order='sorted')
    data = SiameseModelData(f)
    gs = list(data.orig_train_graphs) + [data.test_data.gs[i].nxgraph for i in range(data.m)]
    dc = DistCalculator.from_matrix(f.dataset, gs, synthetic_ged_matrix(gs))
    model = SiameseGCNTNMSE(data.input_dim(), f, device=gpu)
    model.grad_hook = lambda m: None
    with pytest.raises(RuntimeError, match='grad_hook'):
        model.capture_train_steps(DeviceFeed(model, data, dc, 'train'), n_steps=2)
