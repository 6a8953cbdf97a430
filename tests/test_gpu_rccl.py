"""The multi-GPU step's collective on the real RCCL backend (shard.py's all-reduce hook,
as bench.py runs it for N > 1), at world size 1 so it fits a one-GPU box: the in-place
SUM all-reduce of model.grad_loss goes through RCCL on device memory and must leave
the step bitwise unchanged.  World sizes > 1 are covered by the gloo test in
test_distributed.py (shards + all-reduce == the single-process step)."""
import pytest

pytestmark = pytest.mark.gpu


def test_rccl_world1_hook_keeps_step_bitwise(gpu):
    import torch
    import torch.distributed as dist
    from graphembedding_amd.allpairs import AllPairsShard, load_graph_set
    from graphembedding_amd.config import Flags
    from graphembedding_amd.model_mse import SiameseGCNTNMSE
    from graphembedding_amd.shard import make_allreduce_hook

    gs = load_graph_set('syn_aids700nef', n_max=10)
    flags = Flags(dropout=0.1)
    labels = gs.label_matrix(flags.yeta)
    shard = AllPairsShard(gs, labels, 0, 1, device=gpu, n_pairs=6400)
    models = [SiameseGCNTNMSE(gs.d_in, flags, device=gpu, n_max=gs.n_max) for _ in range(2)]
    batches = [shard.batch(m) for m in models]
    assert models[0].grad.data_ptr() == models[0].grad_loss.data_ptr()   # one in-place call
    dist.init_process_group('nccl', store=dist.HashStore(), rank=0, world_size=1,
                            device_id=gpu)
    try:
        assert dist.get_backend() == 'nccl'
        hook = make_allreduce_hook()
        for _ in range(3):
            for k, (m, b) in enumerate(zip(models, batches)):
                m.fwd_bwd(b)
                if k == 0:
                    hook(m)
                m.apply_adam()
                m.step_count += 1
        torch.cuda.synchronize()
    finally:
        dist.destroy_process_group()
    a, b = models
    assert torch.equal(a.grad_loss, b.grad_loss)
    assert torch.equal(a.params, b.params)
    assert float(a.loss_buf[0]) > 0.0


def test_rccl_direct_world1_hook_keeps_step_bitwise(gpu):
    """rccl.RcclComm: ncclAllReduce enqueued on the compute stream (bench.py's default
    collective for N > 1) leaves a world-size-1 step bitwise unchanged."""
    import torch
    import torch.distributed as dist
    from graphembedding_amd.allpairs import AllPairsShard, load_graph_set
    from graphembedding_amd.config import Flags
    from graphembedding_amd.model_mse import SiameseGCNTNMSE
    from graphembedding_amd.rccl import RcclComm
    from graphembedding_amd.shard import make_rccl_hook

    gs = load_graph_set('syn_aids700nef', n_max=10)
    flags = Flags(dropout=0.1)
    labels = gs.label_matrix(flags.yeta)
    shard = AllPairsShard(gs, labels, 0, 1, device=gpu, n_pairs=6400)
    models = [SiameseGCNTNMSE(gs.d_in, flags, device=gpu, n_max=gs.n_max) for _ in range(2)]
    batches = [shard.batch(m) for m in models]
    comm = RcclComm(0, 1, store=dist.HashStore())
    try:
        hook = make_rccl_hook(comm)
        for _ in range(3):
            for k, (m, b) in enumerate(zip(models, batches)):
                m.fwd_bwd(b)
                if k == 0:
                    hook(m)
                m.apply_adam()
                m.step_count += 1
        torch.cuda.synchronize()
    finally:
        comm.destroy()
    a, b = models
    assert torch.equal(a.grad_loss, b.grad_loss)
    assert torch.equal(a.params, b.params)
