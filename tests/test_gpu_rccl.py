"""The multi-GPU step's collective on the real RCCL backend (shard.py's all-reduce hook,
as bench.py runs it for N > 1), at world size 1 so it fits a one-GPU box: the in-place
SUM all-reduce of model.grad_loss goes through RCCL on device memory and must leave
the step bitwise unchanged.  World sizes > 1 are covered by the gloo test in
test_distributed.py (shards + all-reduce == the single-process step), and on a node
with two or more GPUs by the two-rank direct-RCCL sum at the end of this file."""
import os

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
        assert comm.device() == torch.cuda.current_device()
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


def _two_rank_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    torch.cuda.set_device(rank)
    dev = torch.device('cuda', rank)
    dist.init_process_group('nccl', rank=rank, world_size=world, device_id=dev)
    try:
        from graphembedding_amd.rccl import open_rccl
        comm, why = open_rccl(rank, world)
        assert comm is not None, why
        # the init runs on a helper thread, which must have selected this rank's GPU
        assert comm.device() == rank, (rank, comm.device())
        n = 2727   # an odd count: a wrong count or datatype enum would show
        g = torch.Generator().manual_seed(100 + rank)
        x = torch.randn(n, generator=g, dtype=torch.float32).to(dev)
        a, b = x.clone(), x.clone()
        comm.all_reduce_sum_(a)
        dist.all_reduce(b, op=dist.ReduceOp.SUM)
        torch.cuda.synchronize()
        expect = sum(torch.randn(n, generator=torch.Generator().manual_seed(100 + r),
                                 dtype=torch.float32).double() for r in range(world))
        q.put((rank, float((a.cpu().double() - expect).abs().max()),
               bool(torch.equal(a, b))))
        comm.destroy()
    finally:
        dist.destroy_process_group()


@pytest.mark.skipif(__import__('torch').cuda.device_count() < 2,
                    reason='needs two GPUs (the round-end 8-GPU node); a one-GPU box skips it')
def test_rccl_direct_two_ranks_sum(gpu):
    """Two ranks, one GPU each: RcclComm.all_reduce_sum_ (opened by open_rccl) gives the
    exact sum of distinct per-rank buffers and equals torch.distributed's all-reduce."""
    import socket
    import torch.multiprocessing as mp
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    procs = [ctx.Process(target=_two_rank_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, err, same in out:
        assert err <= 1e-5, (rank, err)
        assert same, rank
