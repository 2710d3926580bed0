"""Raw RCCL communicators whose collectives run on the caller's HIP stream.

Why not ``torch.distributed`` for the data path: ProcessGroupNCCL runs every collective
on ONE internal stream per device and fences it against the issuing stream with events.
The serving pipeline keeps three steps in flight on three slot streams (plus a result
stream) and HIP maps a process's streams onto 4 hardware queues. Through
torch.distributed at world size 1 the record gather cost 6-10 % and the frame scatter
up to 25 % (profiles/r4_rccl_gather_ab.txt, r5f_rccl_world1_ab.txt), for ~9 us of actual
GPU work per step; through these stream-ordered communicators the gather costs 1.2-2.5 %
and the scatter 3.2-4.5 % (r5f_rccl_world1_ab.txt). On the torch path the collectives of all
three slots funnel through the one internal stream (each slot's scatter waits behind the
previous slot's gather, which waits for that slot's post-processing), and the lazily
created internal stream lands on a hardware queue that one of the slot streams already
uses, so it also queues behind that slot's model kernels.

Here each pipeline slot owns a communicator of its own (``ncclCommInitRank`` over the
same ranks; the unique ids travel over the gloo control group) and every collective is
enqueued directly on the slot's stream with ``ncclScatter`` / ``ncclGather``: ordered
after the upload and before the model on that stream, no extra stream, no cross-slot
dependency. The library is the librccl the torch build links (one RCCL per process).

Reference: the reference has no multi-device code at all; this is the
north-star X1/X2 path over xGMI.
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Optional

import torch

_lib = None

_DT = {torch.float32: 7, torch.uint8: 1, torch.int32: 2, torch.float64: 8, torch.bfloat16: 9,
       torch.float16: 6, torch.int8: 0, torch.int64: 4}


class RcclError(RuntimeError):
    pass


class _UniqueId(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * 128)]


def lib():
    """The RCCL library torch itself uses (already mapped by libtorch_hip)."""
    global _lib
    if _lib is None:
        cands = [os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so"),
                 "librccl.so.1", "/opt/rocm/lib/librccl.so.1"]
        err = None
        for c in cands:
            try:
                if c.startswith("/") and not os.path.exists(c):
                    continue
                L = ctypes.CDLL(c)
                break
            except OSError as e:  # pragma: no cover - image without RCCL
                err = e
        else:
            raise RcclError(f"librccl not found: {err}")
        L.ncclGetErrorString.restype = ctypes.c_char_p
        L.ncclGetUniqueId.argtypes = [ctypes.POINTER(_UniqueId)]
        L.ncclCommInitRank.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, _UniqueId, ctypes.c_int]
        for fn in ("ncclScatter", "ncclGather"):
            getattr(L, fn).argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                       ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        L.ncclCommCount.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]
        L.ncclCommDestroy.argtypes = [ctypes.c_void_p]
        L.ncclCommAbort.argtypes = [ctypes.c_void_p]
        L.ncclCommGetAsyncError.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]
        _lib = L
    return _lib


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise RcclError(f"{what}: {lib().ncclGetErrorString(rc).decode()} ({rc})")


def available() -> bool:
    try:
        lib()
        return True
    except RcclError:
        return False


def uid_bytes(uid: _UniqueId) -> bytes:
    """The id's raw 128 bytes. NOT ``bytes(uid.internal)``: a ``c_char`` array field reads
    (and assigns) as a NUL-terminated string, and the id holds NULs -- an 8-byte magic,
    then the root's sockaddr, whose family field is ``02 00`` -- so the root's address and
    port would arrive zeroed on the other ranks."""
    return ctypes.string_at(ctypes.addressof(uid), ctypes.sizeof(uid))


def uid_from_bytes(raw: bytes) -> _UniqueId:
    if len(raw) != ctypes.sizeof(_UniqueId):
        raise ValueError(f"ncclUniqueId must be {ctypes.sizeof(_UniqueId)} bytes, got {len(raw)}")
    uid = _UniqueId()
    ctypes.memmove(ctypes.addressof(uid), raw, len(raw))
    return uid


def share_uid(ctx, uid: Optional[_UniqueId]) -> _UniqueId:
    """Rank 0's id on every rank, byte for byte, over the host (gloo) group."""
    if ctx.world == 1:
        return uid
    import torch.distributed as dist
    obj = [uid_bytes(uid) if ctx.rank == 0 else None]
    dist.broadcast_object_list(obj, src=0, group=ctx.cpu_group)
    return uid if ctx.rank == 0 else uid_from_bytes(obj[0])


class StreamComm:
    """One RCCL communicator over the ranks of ``ctx``; collectives on a given stream."""

    def __init__(self, ctx, tag: str = "slot"):
        L = lib()
        uid = _UniqueId()
        if ctx.rank == 0:
            _check(L.ncclGetUniqueId(ctypes.byref(uid)), "ncclGetUniqueId")
        uid = share_uid(ctx, uid)
        self.world, self.rank = ctx.world, ctx.rank
        self.device = ctx.device
        self.comm = ctypes.c_void_p()
        with torch.cuda.device(ctx.device):
            _check(L.ncclCommInitRank(ctypes.byref(self.comm), ctx.world, uid, ctx.rank),
                   f"ncclCommInitRank({tag})")
        self.alive = True
        n = ctypes.c_int(0)
        _check(L.ncclCommCount(self.comm, ctypes.byref(n)), "ncclCommCount")
        # the communicator's own view of the group size (bench.py reports it: proof of how
        # many ranks RCCL actually joined)
        self.nranks = int(n.value)
        if self.nranks != ctx.world:
            raise RcclError(f"ncclCommCount({tag}) = {self.nranks}, expected {ctx.world}")

    @staticmethod
    def _stream(stream: Optional[torch.cuda.Stream]) -> ctypes.c_void_p:
        s = stream if stream is not None else torch.cuda.current_stream()
        return ctypes.c_void_p(s.cuda_stream)

    def scatter(self, recv: torch.Tensor, send: Optional[torch.Tensor], root: int = 0,
                stream: Optional[torch.cuda.Stream] = None) -> None:
        """recv [n] on every rank <- rows of send [world, n] on ``root`` (contiguous)."""
        if recv.dtype not in _DT or not recv.is_contiguous():
            raise ValueError("scatter: contiguous tensor of a supported dtype")
        if self.rank == root and (send is None or send.numel() != recv.numel() * self.world
                                  or send.dtype != recv.dtype or not send.is_contiguous()):
            raise ValueError("scatter: root needs a contiguous [world, n] send buffer")
        sp = send.data_ptr() if self.rank == root else 0
        _check(lib().ncclScatter(ctypes.c_void_p(sp), ctypes.c_void_p(recv.data_ptr()), recv.numel(),
                                 _DT[recv.dtype], root, self.comm, self._stream(stream)), "ncclScatter")

    def gather(self, send: torch.Tensor, recv: Optional[torch.Tensor], root: int = 0,
               stream: Optional[torch.cuda.Stream] = None) -> None:
        """recv [world, n] on ``root`` <- send [n] of every rank (contiguous)."""
        if send.dtype not in _DT or not send.is_contiguous():
            raise ValueError("gather: contiguous tensor of a supported dtype")
        if self.rank == root and (recv is None or recv.numel() != send.numel() * self.world
                                  or recv.dtype != send.dtype or not recv.is_contiguous()):
            raise ValueError("gather: root needs a contiguous [world, n] receive buffer")
        rp = recv.data_ptr() if self.rank == root else 0
        _check(lib().ncclGather(ctypes.c_void_p(send.data_ptr()), ctypes.c_void_p(rp), send.numel(),
                                _DT[send.dtype], root, self.comm, self._stream(stream)), "ncclGather")

    def async_error(self) -> int:
        err = ctypes.c_int(0)
        lib().ncclCommGetAsyncError(self.comm, ctypes.byref(err))
        return int(err.value)

    def abort(self) -> None:
        """A peer is gone: free the communicator without waiting for it."""
        if self.alive:
            self.alive = False
            lib().ncclCommAbort(self.comm)

    def destroy(self) -> None:
        if self.alive:
            self.alive = False
            lib().ncclCommDestroy(self.comm)


def slot_comms(ctx, n: int) -> List[StreamComm]:
    """``n`` communicators over ``ctx``'s ranks (one per pipeline slot), created in the
    same order on every rank."""
    return [StreamComm(ctx, f"slot{i}") for i in range(n)]
