"""Data-parallel path (graphembedding_amd/shard.py) on CPU with gloo, world 2:
per-rank pair shards keyed by GLOBAL pair index + one SUM all-reduce of the
flat gradient reproduce the single-process step.  The per-shard arithmetic is
the oracle's C restatement standing in for the GPU kernel."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from graphembedding_amd.shard import make_allreduce_hook, make_rccl_hook, shard_range


def test_shard_range_partitions():
    for n in (0, 1, 7, 490000, 1001):
        for w in (1, 2, 3, 8):
            spans = [shard_range(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [e - s for s, e in spans]
            assert max(sizes) - min(sizes) <= 1


class _FakeModel:
    """grad / loss_buf either separate tensors or views of one grad_loss buffer
    (SiameseGCNTNMSE's layout, reduced by one in-place all-reduce)."""
    def __init__(self, grad, loss, shared=False):
        if shared:
            n = len(grad)
            self.grad_loss = torch.zeros(n + 2, dtype=torch.float32)
            self.grad = self.grad_loss[:n]
            self.loss_buf = self.grad_loss[n:]
            self.grad.copy_(torch.tensor(grad, dtype=torch.float32))
            self.loss_buf[0] = loss
        else:
            self.grad = torch.tensor(grad, dtype=torch.float32)
            self.loss_buf = torch.tensor([loss, 0.0], dtype=torch.float32)


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, shared=False):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        from _fixtures import small_problem
        from oracle import cpu_ref
        prob = small_problem(n_graphs=20, n_pairs=301, seed=31)
        words = prob.store().pack_host(prob.pairs, prob.labels)
        ybar = float(prob.labels.astype(np.float64).mean())   # global label stats
        s0, e0 = shard_range(len(prob.pairs), rank, world)
        _, g, loss = cpu_ref.fwd_bwd_records(words[s0:e0], prob.n_max, prob.d_in, prob.params,
                                             77, 0.9, prob.flags.yeta, ybar, pair_offset=s0,
                                             threads=1)
        m = _FakeModel(g, loss, shared)
        make_allreduce_hook()(m)
        _, g_full, loss_full = cpu_ref.fwd_bwd_records(words, prob.n_max, prob.d_in,
                                                       prob.params, 77, 0.9, prob.flags.yeta,
                                                       ybar, threads=1)
        err = float(np.abs(m.grad.numpy() - g_full).max())
        lerr = abs(float(m.loss_buf[0]) - loss_full)
        q.put((rank, err, lerr, float(np.abs(g_full).max())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('shared', [False, True])
def test_two_rank_gloo_step_equals_single_process(shared):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, shared)) for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, err, lerr, scale in out:
        assert err <= 1e-5 * max(1.0, scale), (rank, err)
        assert lerr <= 1e-4, (rank, lerr)


def test_rccl_hook_reduces_grad_loss_in_place():
    """shard.make_rccl_hook hands the collective exactly grad | loss_mse (one in-place
    call on the shared buffer) and refuses a model whose buffers are not views of it."""
    calls = []

    class _Comm:
        def all_reduce_sum_(self, t):
            calls.append(t)
            t.mul_(2.0)

    m = _FakeModel([1.0, -2.0, 3.0], 0.5, shared=True)
    hook = make_rccl_hook(_Comm())
    hook(m)
    assert len(calls) == 1 and calls[0].numel() == 4
    assert calls[0].data_ptr() == m.grad_loss.data_ptr()
    assert m.grad.tolist() == [2.0, -4.0, 6.0] and float(m.loss_buf[0]) == 1.0
    assert float(m.loss_buf[1]) == 0.0
    with pytest.raises(RuntimeError):
        m2 = _FakeModel([1.0], 0.0, shared=False)
        m2.grad_loss = torch.zeros(3)
        hook(m2)


def _open_worker(rank, world, port, q, case):
    """open_rccl with injected failures (no GPU: the unique id, the communicator init and
    the abort are fakes); reports what each rank ended up with and how long it took."""
    import threading
    import time
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from graphembedding_amd.rccl import open_rccl
        aborted = []

        def uid(lib):
            if case == 'uid_fails' and rank == 0:
                raise RuntimeError('injected ncclGetUniqueId failure')
            return b'u' * 128

        def init(lib, raw, r, w):
            assert raw == b'u' * 128 and w == world
            if r == 1 and case in ('init_fails_peer_hangs', 'init_fails_peer_ok'):
                raise RuntimeError('injected ncclCommInitRank failure')
            if case == 'init_fails_peer_hangs':
                threading.Event().wait(30)   # a peer stuck in init, waiting for rank 1
            return 'comm{}'.format(r)

        t0 = time.time()
        comm, why = open_rccl(rank, world, timeout_s=3.0, _uid=uid, _init=init,
                              _abort=lambda lib, c: aborted.append(c))
        dist.barrier()   # both ranks still talk over the process group afterwards
        q.put((rank, None if comm is None else comm.comm, why, aborted, time.time() - t0))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('case', ['ok', 'uid_fails', 'init_fails_peer_ok',
                                  'init_fails_peer_hangs'])
def test_open_rccl_ranks_agree(case):
    """bench.py's collective choice is the same on every rank: open_rccl returns a
    communicator on both ranks or on neither, whichever rank fails (rank 0's unique id,
    one rank's init while the peer's succeeds, one rank's init while the peer's stalls),
    and no rank waits past the init timeout."""
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_open_worker, args=(r, 2, port, q, case)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    comms = [o[1] for o in out]
    if case == 'ok':
        assert comms == ['comm0', 'comm1']
        assert all(o[2] is None for o in out)
        return
    assert comms == [None, None], out
    assert all(o[2] for o in out), out   # every rank says why it falls back
    assert all(o[4] < 20.0 for o in out), out
    if case == 'init_fails_peer_ok':   # rank 0 held a communicator its peer gave up on
        assert out[0][3] == ['comm0'] and out[1][3] == []


def test_rccl_binding_loads():
    """graphembedding_amd.rccl binds torch's own librccl.so (the symbols the direct
    collective uses) and draws a unique id without touching a GPU."""
    import ctypes
    from graphembedding_amd.rccl import NCCL_UNIQUE_ID_BYTES, _UniqueId, _rccl
    L = _rccl()
    for sym in ('ncclGetUniqueId', 'ncclCommInitRank', 'ncclAllReduce', 'ncclCommDestroy',
                'ncclGetErrorString'):
        assert hasattr(L, sym), sym
    uid = _UniqueId()
    assert L.ncclGetUniqueId(ctypes.byref(uid)) == 0
    assert ctypes.sizeof(uid) == NCCL_UNIQUE_ID_BYTES
    assert any(ctypes.string_at(ctypes.addressof(uid), NCCL_UNIQUE_ID_BYTES))
