"""RCCL called directly on the compute stream (one SUM all-reduce of the
flat gradient per step, over xGMI).

torch.distributed's "nccl" backend (= RCCL) runs every collective on a side stream of
its own, fenced by events against the caller's stream on both sides.  For the
10.9 KB gradient of this model the collective is pure latency, so those two
cross-stream hops are part of every step's fixed cost.  RcclComm opens one RCCL
communicator over the same ranks (the unique id goes through the process group's
store) and enqueues ncclAllReduce on the stream the fused kernels use, in order
with them: no events and no side stream.  The library is the librccl.so torch itself
loaded, so there is one RCCL in the process.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

NCCL_UNIQUE_ID_BYTES = 128   # rccl.h
NCCL_FLOAT32 = 7             # ncclFloat32
NCCL_SUM = 0                 # ncclSum


class _UniqueId(ctypes.Structure):
    _fields_ = [('internal', ctypes.c_char * NCCL_UNIQUE_ID_BYTES)]


_LIB = None


def _rccl():
    global _LIB
    if _LIB is None:
        import torch
        cand = [os.path.join(os.path.dirname(torch.__file__), 'lib', 'librccl.so'),
                'librccl.so.1', 'librccl.so']
        err = None
        for c in cand:
            try:
                _LIB = ctypes.CDLL(c)
                break
            except OSError as e:
                err = e
        if _LIB is None:
            raise RuntimeError('librccl.so not found: {}'.format(err))
        L = _LIB
        L.ncclGetUniqueId.argtypes = [ctypes.POINTER(_UniqueId)]
        L.ncclCommInitRank.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, _UniqueId,
                                       ctypes.c_int]
        L.ncclAllReduce.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                    ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        L.ncclCommDestroy.argtypes = [ctypes.c_void_p]
        L.ncclGetErrorString.argtypes = [ctypes.c_int]
        L.ncclGetErrorString.restype = ctypes.c_char_p
    return _LIB


def _check(rc: int, what: str):
    if rc != 0:
        msg = _rccl().ncclGetErrorString(rc)
        raise RuntimeError('{} failed: {} ({})'.format(what, msg.decode() if msg else '?', rc))


class RcclComm(object):
    """One RCCL communicator over this process group's ranks (one process per GPU;
    call after torch.cuda.set_device).  `store` is any torch.distributed Store reachable
    by every rank; default: the default process group's store."""

    _count = 0   # communicators opened by this process: every rank opens them in the same order

    def __init__(self, rank: int, world: int, store=None, tag: str = None):
        import torch.distributed as dist
        if store is None:
            store = dist.distributed_c10d._get_default_store()
        if tag is None:   # a fresh key per communicator: ranks never read a stale id
            tag = 'sg_rccl_uid_{}'.format(RcclComm._count)
        RcclComm._count += 1
        L = _rccl()
        uid = _UniqueId()
        if rank == 0:
            _check(L.ncclGetUniqueId(ctypes.byref(uid)), 'ncclGetUniqueId')
            store.set(tag, ctypes.string_at(ctypes.addressof(uid), NCCL_UNIQUE_ID_BYTES))
        else:
            raw = store.get(tag)
            ctypes.memmove(ctypes.addressof(uid), raw, NCCL_UNIQUE_ID_BYTES)
        self.comm = ctypes.c_void_p()
        _check(L.ncclCommInitRank(ctypes.byref(self.comm), int(world), uid, int(rank)),
               'ncclCommInitRank')
        self.rank, self.world = int(rank), int(world)

    def all_reduce_sum_(self, t, stream: Optional[int] = None):
        """In-place SUM all-reduce of a contiguous float32 device tensor, enqueued on
        `stream` (default: torch's current stream)."""
        import torch
        if t.dtype != torch.float32 or not t.is_contiguous() or not t.is_cuda:
            raise RuntimeError('RcclComm.all_reduce_sum_: contiguous float32 device tensor')
        if stream is None:
            stream = torch.cuda.current_stream().cuda_stream
        p = t.data_ptr()
        _check(_rccl().ncclAllReduce(p, p, t.numel(), NCCL_FLOAT32, NCCL_SUM, self.comm,
                                     ctypes.c_void_p(int(stream))), 'ncclAllReduce')

    def destroy(self):
        if self.comm:
            _rccl().ncclCommDestroy(self.comm)
            self.comm = ctypes.c_void_p()
