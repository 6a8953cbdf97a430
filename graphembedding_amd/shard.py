"""Data parallelism over the pair space.

One process per GPU (torch.distributed; backend "nccl" = RCCL on ROCm, "gloo"
on CPU for tests).  A step's ordered pair range [0, P) is split into
contiguous per-rank shards; dropout masks are keyed by the GLOBAL pair index,
so the sharded step computes exactly the unsharded one.  The only exchange is
one SUM all-reduce of the flat fp32 gradient (+ the loss scalar) per step —
10.9 KB at the default model, latency-bound over xGMI.
"""
from __future__ import annotations

from typing import Tuple


def shard_range(n_items: int, rank: int, world: int) -> Tuple[int, int]:
    base, rem = divmod(int(n_items), int(world))
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def make_allreduce_hook(group=None):
    """Model.grad_hook: sum grad and loss_mse over ranks.  They are adjacent in
    model.grad_loss, so this is one in-place all-reduce (RCCL over xGMI)."""
    import torch.distributed as dist

    def hook(model):
        buf = getattr(model, 'grad_loss', None)
        n = model.grad.numel()
        if (buf is not None and model.grad.data_ptr() == buf.data_ptr()
                and model.loss_buf.data_ptr() == buf[n:].data_ptr()):
            dist.all_reduce(buf[:n + 1], op=dist.ReduceOp.SUM, group=group)
            return
        import torch
        tmp = torch.cat([model.grad, model.loss_buf[:1]])
        dist.all_reduce(tmp, op=dist.ReduceOp.SUM, group=group)
        model.grad.copy_(tmp[:n])
        model.loss_buf[:1].copy_(tmp[n:])

    return hook


def make_rccl_hook(comm):
    """Model.grad_hook over a rccl.RcclComm: the same in-place SUM of grad | loss_mse,
    enqueued by RCCL directly on the compute stream (no side stream, no events)."""

    def hook(model):
        n = model.grad.numel()
        buf = model.grad_loss
        if model.grad.data_ptr() != buf.data_ptr() or model.loss_buf.data_ptr() != buf[n:].data_ptr():
            raise RuntimeError('make_rccl_hook: grad and loss_buf must be views of grad_loss')
        comm.all_reduce_sum_(buf[:n + 1])

    return hook
