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
        L.ncclCommAbort.argtypes = [ctypes.c_void_p]
        L.ncclCommCuDevice.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]
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
    by every rank; default: the default process group's store.  The constructor is the
    plain path (world 1, tests); multi-rank callers use open_rccl(), under which every
    rank ends up with a communicator or none does."""

    _count = 0   # communicators opened by this process: every rank opens them in the same order

    def __init__(self, rank: int, world: int, store=None, tag: str = None):
        import torch.distributed as dist
        if store is None:
            store = dist.distributed_c10d._get_default_store()
        if tag is None:   # a fresh key per communicator: ranks never read a stale id
            tag = 'sg_rccl_uid_{}'.format(RcclComm._count)
        RcclComm._count += 1
        uid = _UniqueId()
        if rank == 0:
            # always publish a record, a failure marker included, so that no peer waits
            # in store.get for an id that will not come (multi-rank: use open_rccl)
            try:
                L = _rccl()
                _check(L.ncclGetUniqueId(ctypes.byref(uid)), 'ncclGetUniqueId')
            except Exception as e:
                store.set(tag, b'\x00' + str(e).encode()[:200])
                raise
            store.set(tag, b'\x01' + ctypes.string_at(ctypes.addressof(uid), NCCL_UNIQUE_ID_BYTES))
        else:
            raw = store.get(tag)
            if raw[:1] != b'\x01':
                raise RuntimeError('rank 0 published no RCCL unique id: {}'.format(
                    bytes(raw[1:]).decode(errors='replace')))
            L = _rccl()
            ctypes.memmove(ctypes.addressof(uid), bytes(raw[1:]), NCCL_UNIQUE_ID_BYTES)
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

    def device(self) -> int:
        """The GPU the communicator was initialised on (ncclCommCuDevice)."""
        d = ctypes.c_int(-1)
        _check(_rccl().ncclCommCuDevice(self.comm, ctypes.byref(d)), 'ncclCommCuDevice')
        return int(d.value)

    def destroy(self):
        if self.comm:
            _rccl().ncclCommDestroy(self.comm)
            self.comm = ctypes.c_void_p()


def _agree(ok: bool, group=None) -> bool:
    """True on every rank iff `ok` holds on every rank: a MIN all-reduce of a flag through
    the already-initialised process group (CUDA tensor for the nccl backend, CPU for gloo)."""
    import torch
    import torch.distributed as dist
    dev = 'cuda' if dist.get_backend(group) == 'nccl' else 'cpu'
    if dev == 'cuda':
        dev = torch.device('cuda', torch.cuda.current_device())
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(int(t.item()))


def open_rccl(rank: int, world: int, store=None, group=None, timeout_s: float = 120.0,
              _uid=None, _init=None, _abort=None):
    """Open one RcclComm on every rank, or on none: returns (comm, None) on every rank, or
    (None, reason) on every rank, so the caller falls back to torch.distributed together.
    No rank is left waiting on a communicator that another rank abandoned:

    1. rank 0 draws the unique id and ALWAYS publishes a record to the store, a failure
       marker included, so the other ranks never wait in store.get for an id that will
       not come;
    2. the ranks agree (MIN all-reduce over the process group) that every rank has the
       library and the id before any of them enters ncclCommInitRank, a collective;
    3. ncclCommInitRank runs on a helper thread joined with `timeout_s`: a rank whose init
       fails, or stalls because a peer's failed, reports it, and a second agreement
       decides; on a failed agreement the ranks holding a communicator abort it.

    `_uid(lib) -> bytes`, `_init(lib, uid_bytes, rank, world) -> comm pointer` and
    `_abort(lib, comm)` replace the library calls in tests (failure injection)."""
    import threading
    import torch.distributed as dist
    if store is None:
        store = dist.distributed_c10d._get_default_store()
    tag = 'sg_rccl_uid_{}'.format(RcclComm._count)
    RcclComm._count += 1
    lib, reason = None, None
    try:
        lib = _rccl()
    except Exception as e:   # noqa: BLE001 (any load failure means: fall back)
        reason = 'rank {}: {}'.format(rank, e)

    def get_uid():
        if _uid is not None:
            return _uid(lib)
        uid = _UniqueId()
        _check(lib.ncclGetUniqueId(ctypes.byref(uid)), 'ncclGetUniqueId')
        return ctypes.string_at(ctypes.addressof(uid), NCCL_UNIQUE_ID_BYTES)

    raw = None
    if rank == 0:
        rec = b'\x00' + b'no library'
        if lib is not None:
            try:
                raw = get_uid()
                rec = b'\x01' + raw
            except Exception as e:   # noqa: BLE001
                reason = 'rank 0: {}'.format(e)
                rec = b'\x00' + str(e).encode()[:200]
        store.set(tag, rec)
    else:
        rec = store.get(tag)
        if rec[:1] == b'\x01':
            raw = bytes(rec[1:])
        elif reason is None:
            reason = 'rank 0 published no unique id ({})'.format(rec[1:].decode(errors='replace'))
    if not _agree(lib is not None and raw is not None, group):
        return None, reason or 'a peer rank could not load RCCL or get the unique id'

    box = {}
    # HIP keeps the current device per host thread and a new thread starts on device 0:
    # the helper thread must select this rank's GPU before ncclCommInitRank, or every rank
    # would initialise its communicator on GPU 0
    dev = None
    try:
        import torch
        if torch.cuda.is_available():
            dev = torch.cuda.current_device()
    except Exception:   # noqa: BLE001 (CPU-only callers: gloo tests with fake init)
        dev = None
    box['device'] = dev

    def init():
        try:
            if dev is not None:
                import torch
                torch.cuda.set_device(dev)
            if _init is not None:
                box['comm'] = _init(lib, raw, rank, world)
                return
            uid = _UniqueId()
            ctypes.memmove(ctypes.addressof(uid), raw, NCCL_UNIQUE_ID_BYTES)
            c = ctypes.c_void_p()
            _check(lib.ncclCommInitRank(ctypes.byref(c), int(world), uid, int(rank)),
                   'ncclCommInitRank')
            box['comm'] = c
        except Exception as e:   # noqa: BLE001
            box['err'] = str(e)

    th = threading.Thread(target=init, name='sg_rccl_init', daemon=True)
    th.start()
    th.join(timeout_s)
    ok = not th.is_alive() and 'comm' in box
    if not ok:
        reason = 'rank {}: {}'.format(rank, box.get('err', 'ncclCommInitRank did not return '
                                                            'within {} s'.format(timeout_s)))
    if not _agree(ok, group):
        if ok:   # this rank holds a communicator its peers gave up on
            try:
                if _abort is not None:
                    _abort(lib, box['comm'])
                else:
                    lib.ncclCommAbort(box['comm'])
            except Exception:   # noqa: BLE001
                pass
        return None, reason or 'ncclCommInitRank failed on a peer rank'
    comm = RcclComm.__new__(RcclComm)
    comm.comm, comm.rank, comm.world = box['comm'], int(rank), int(world)
    return comm, None
