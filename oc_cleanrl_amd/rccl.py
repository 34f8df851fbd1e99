"""The data-parallel gradient exchange's own RCCL communicator.

ppo_atari_multigpu.py:360-374 all-reduces the flat gradient vector once per minibatch through
torch.distributed. Issued through torch's ProcessGroup, each collective is an eager call with
watchdog bookkeeping between graph replays (three replays and two collectives per minibatch), or,
captured, a collective on the process group's own stream whose watchdog events then live inside
the capture. Here the exchange owns an RCCL communicator (ctypes over the librccl that torch has
already loaded; the process group only bootstraps it: rank 0's unique id is broadcast through
it) and issues ncclAllReduce on the caller's HIP stream, so each epoch's minibatches are captured
with their all-reduces into one hipGraph and nothing of torch's watchdog is in the capture.

Failure: every call's ncclResult is checked (RuntimeError naming the call and RCCL's message);
a peer that never arrives is bounded by the rank watchdog (oc_cleanrl_amd.watch), which exits
the process, since a collective waiting inside a graph replay cannot be interrupted from Python.
"""
from __future__ import annotations

import ctypes
import os

import torch
import torch.distributed as dist

NCCL_FLOAT32 = 7  # ncclFloat32 (rccl.h ncclDataType_t)
NCCL_SUM = 0      # ncclSum (rccl.h ncclRedOp_t)
UNIQUE_ID_BYTES = 128


class _UniqueId(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * UNIQUE_ID_BYTES)]


_LIB = None


def library_path() -> str:
    """The librccl torch links (loaded already in this process: dlopen returns the same copy);
    ROCm's own only when torch ships none."""
    p = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    return p if os.path.exists(p) else "librccl.so"


def _lib():
    global _LIB
    if _LIB is None:
        lib = ctypes.CDLL(library_path())
        vp, i, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
        lib.ncclGetUniqueId.argtypes = [ctypes.POINTER(_UniqueId)]
        lib.ncclCommInitRank.argtypes = [ctypes.POINTER(vp), i, _UniqueId, i]
        lib.ncclAllReduce.argtypes = [vp, vp, sz, i, i, vp, vp]
        lib.ncclCommDestroy.argtypes = [vp]
        lib.ncclCommAbort.argtypes = [vp]
        lib.ncclGetErrorString.argtypes = [i]
        lib.ncclGetErrorString.restype = ctypes.c_char_p
        lib.ncclCommGetAsyncError.argtypes = [vp, ctypes.POINTER(i)]
        for f in ("ncclGetUniqueId", "ncclCommInitRank", "ncclAllReduce", "ncclCommDestroy",
                  "ncclCommAbort", "ncclCommGetAsyncError"):
            getattr(lib, f).restype = i
        _LIB = lib
    return _LIB


def _check(rc: int, what: str):
    if rc != 0:
        msg = _lib().ncclGetErrorString(rc)
        raise RuntimeError(f"{what} failed: ncclResult {rc} "
                           f"({msg.decode() if msg else 'unknown'})")


def unique_id() -> bytes:
    """The library loaded and a fresh ncclUniqueId (rank 0's part of the bootstrap), as its raw
    128 bytes (a c_char array would stop at the first NUL). Local: no collective."""
    lib = _lib()
    uid = _UniqueId()
    _check(lib.ncclGetUniqueId(ctypes.byref(uid)), "ncclGetUniqueId")
    return ctypes.string_at(ctypes.addressof(uid), UNIQUE_ID_BYTES)


class RcclComm:
    """One RCCL communicator over the ranks of the default process group, on this process's
    current HIP device (torch.cuda.set_device before constructing). uid: rank 0's unique_id(),
    or None to draw it here; it is broadcast through the process group either way.

    ncclCommInitRank is itself collective: a rank whose init fails raises, while its peers stay
    inside theirs. Nothing after that point can be agreed on through the group, so the failures
    that can be agreed on (the library, the unique id) are checked before it (trainer._rccl_comm)
    and a failing init is bounded by the rank watchdog (oc_cleanrl_amd.watch)."""

    def __init__(self, rank: int, world: int, group=None, uid: bytes | None = None):
        lib = _lib()
        if rank == 0 and uid is None:
            uid = unique_id()
        box = [uid if rank == 0 else None]
        dist.broadcast_object_list(box, src=0, group=group)
        if box[0] is None or len(box[0]) != UNIQUE_ID_BYTES:
            raise RuntimeError(f"RCCL unique id of {len(box[0] or b'')} bytes")
        raw = _UniqueId()
        ctypes.memmove(ctypes.addressof(raw), box[0], UNIQUE_ID_BYTES)
        comm = ctypes.c_void_p()
        _check(lib.ncclCommInitRank(ctypes.byref(comm), world, raw, rank), "ncclCommInitRank")
        self.comm, self.rank, self.world = comm, rank, world

    def all_reduce_sum(self, t: torch.Tensor, stream=None):
        """In-place SUM over the ranks of the contiguous f32 CUDA tensor `t`, enqueued on `stream`
        (default: the current stream; capturable)."""
        if t.dtype != torch.float32 or not t.is_cuda or not t.is_contiguous():
            raise ValueError("RcclComm.all_reduce_sum: a contiguous f32 CUDA tensor")
        s = stream if stream is not None else torch.cuda.current_stream(t.device)
        _check(_lib().ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), NCCL_FLOAT32, NCCL_SUM,
                                    self.comm, s.cuda_stream), "ncclAllReduce")

    def async_error(self) -> int:
        rc = ctypes.c_int(0)
        _check(_lib().ncclCommGetAsyncError(self.comm, ctypes.byref(rc)), "ncclCommGetAsyncError")
        return rc.value

    def close(self, abort: bool = False):
        if self.comm:
            (_lib().ncclCommAbort if abort else _lib().ncclCommDestroy)(self.comm)
            self.comm = ctypes.c_void_p()


class RcclExchange:
    """trainer.GradExchange's contract (whole / split, the /world either here or in the optimizer)
    over an RcclComm on HIP streams. split(): the tail's all-reduce runs on `side` (forked from
    the current stream once the first backward phase has written the tail) while
    `lower_backward()` fills the head on the current stream; the current stream then joins `side`
    and reduces the head. Both collectives are ordered on the one communicator (the head's is
    issued after the join), as RCCL requires; everything is stream-ordered, so the whole minibatch
    can be captured."""

    def __init__(self, buf, tail_off: int, world: int, scale_in_optimizer: bool, comm: RcclComm,
                 side=None):
        self.buf, self.tail_off, self.world = buf, tail_off, world
        self.scale_in_optimizer, self.comm, self.side = scale_in_optimizer, comm, side

    def _finish(self):
        if not self.scale_in_optimizer:
            self.buf.div_(self.world)

    def whole(self):
        self.comm.all_reduce_sum(self.buf)
        self._finish()

    def split(self, lower_backward):
        cur = torch.cuda.current_stream(self.buf.device)
        self.side.wait_stream(cur)
        self.comm.all_reduce_sum(self.buf[self.tail_off:], self.side)
        lower_backward()
        cur.wait_stream(self.side)
        self.comm.all_reduce_sum(self.buf[:self.tail_off], cur)
        self._finish()
