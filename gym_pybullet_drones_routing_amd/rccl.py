"""A raw RCCL communicator for the learner hand-off (shard.LearnerHandoff).

torch.distributed's ProcessGroupNCCL wraps every collective in host-side bookkeeping (work objects,
events, a watchdog) that costs tens of microseconds per call - more than the ~5 us env step the
hand-off ships - and that left a process hanging at teardown once its collectives had been captured
in a hipGraph (round-6 probe, scripts/rccl_probe.py).  This module calls RCCL (the ``librccl.so``
torch itself loaded, so one RCCL in the process) through ctypes: ``ncclAllGather`` and grouped
``ncclSend`` / ``ncclRecv`` on the caller's current stream, each a ~1 us host call, capturable into a
hipGraph.  The communicator's unique id travels over the existing torch.distributed group (the
rendezvous: one broadcast at construction).
"""
import ctypes
import os

import torch
import torch.distributed as dist

NCCL_UNIQUE_ID_BYTES = 128
NCCL_UINT8 = 1       # ncclDataType_t (rccl.h)
NCCL_FLOAT32 = 7


class UniqueId(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * NCCL_UNIQUE_ID_BYTES)]


_lib = None
_lib_path = None


def _load():
    global _lib, _lib_path
    if _lib is not None:
        return _lib
    cands = [os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so"), "/opt/rocm/lib/librccl.so"]
    path = next((p for p in cands if os.path.exists(p)), None)
    if path is None:
        raise RuntimeError("librccl.so not found (torch/lib or /opt/rocm/lib)")
    lib = ctypes.CDLL(path)
    vp, ci, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
    sig = {
        "ncclGetUniqueId": [ctypes.POINTER(UniqueId)],
        "ncclCommInitRank": [ctypes.POINTER(vp), ci, UniqueId, ci],
        "ncclCommDestroy": [vp],
        "ncclAllGather": [vp, vp, sz, ci, vp, vp],
        "ncclSend": [vp, sz, ci, ci, vp, vp],
        "ncclRecv": [vp, sz, ci, ci, vp, vp],
        "ncclGroupStart": [],
        "ncclGroupEnd": [],
    }
    for name, args in sig.items():
        fn = getattr(lib, name)
        fn.restype = ci
        fn.argtypes = args
    lib.ncclGetErrorString.restype = ctypes.c_char_p
    lib.ncclGetErrorString.argtypes = [ci]
    _lib, _lib_path = lib, path
    return lib


def _check(lib, name, rc):
    if rc != 0:
        raise RuntimeError(f"{name} failed: {lib.ncclGetErrorString(rc).decode(errors='replace')} ({rc})")


_DT = {torch.uint8: (NCCL_UINT8, 1), torch.float32: (NCCL_FLOAT32, 4)}


class RcclComm:
    """An RCCL communicator over the ranks of the initialised torch.distributed group (one rank
    per GPU, this rank's GPU ``device``).  Collectives on flat contiguous device tensors, enqueued
    on the current stream (so a hipGraph capture records them)."""

    def __init__(self, device):
        self.lib = _load()
        self.lib_path = _lib_path
        self.device = torch.device(device)
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        uid = UniqueId()
        if self.rank == 0:
            _check(self.lib, "ncclGetUniqueId", self.lib.ncclGetUniqueId(ctypes.byref(uid)))
        if self.world > 1:
            box = [bytes(uid.internal) if self.rank == 0 else None]
            dist.broadcast_object_list(box, src=0)
            uid.internal = box[0]
        self.comm = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _check(self.lib, "ncclCommInitRank",
                   self.lib.ncclCommInitRank(ctypes.byref(self.comm), self.world, uid, self.rank))

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    @staticmethod
    def _dt(t):
        if t.dtype not in _DT or not t.is_contiguous() or not t.is_cuda:
            raise ValueError("RCCL hand-off buffers: contiguous uint8 / float32 device tensors")
        return _DT[t.dtype]

    def all_gather(self, send, recv):
        """recv [world * n] <- every rank's send [n], in rank order."""
        dt, _ = self._dt(send)
        n = send.numel()
        if recv.numel() != self.world * n or recv.dtype != send.dtype:
            raise ValueError("all_gather: recv must hold world x send elements of send's dtype")
        _check(self.lib, "ncclAllGather", self.lib.ncclAllGather(
            ctypes.c_void_p(send.data_ptr()), ctypes.c_void_p(recv.data_ptr()), n, dt, self.comm, self._stream()))

    def gather(self, send, recv, root):
        """recv [world * n] on ``root`` <- every rank's send [n] (grouped send / recv; ``recv`` is
        ignored elsewhere)."""
        dt, es = self._dt(send)
        n = send.numel()
        if self.rank == root and (recv is None or recv.numel() != self.world * n or recv.dtype != send.dtype):
            raise ValueError("gather: recv on the root must hold world x send elements of send's dtype")
        st = self._stream()
        lib = self.lib
        _check(lib, "ncclGroupStart", lib.ncclGroupStart())
        ok = False
        try:
            if self.rank == root:
                base = recv.data_ptr()
                for r in range(self.world):
                    _check(lib, "ncclRecv", lib.ncclRecv(ctypes.c_void_p(base + r * n * es), n, dt, r, self.comm, st))
            _check(lib, "ncclSend", lib.ncclSend(ctypes.c_void_p(send.data_ptr()), n, dt, root, self.comm, st))
            ok = True
        finally:
            rc = lib.ncclGroupEnd()     # the group is closed whatever failed inside it
            if ok:
                _check(lib, "ncclGroupEnd", rc)

    def scatter(self, send, recv, root):
        """recv [n] on every rank <- block r of ``root``'s send [world * n] (ignored elsewhere)."""
        dt, es = self._dt(recv)
        n = recv.numel()
        if self.rank == root and (send is None or send.numel() != self.world * n or send.dtype != recv.dtype):
            raise ValueError("scatter: send on the root must hold world x recv elements of recv's dtype")
        st = self._stream()
        lib = self.lib
        _check(lib, "ncclGroupStart", lib.ncclGroupStart())
        ok = False
        try:
            if self.rank == root:
                base = send.data_ptr()
                for r in range(self.world):
                    _check(lib, "ncclSend", lib.ncclSend(ctypes.c_void_p(base + r * n * es), n, dt, r, self.comm, st))
            _check(lib, "ncclRecv", lib.ncclRecv(ctypes.c_void_p(recv.data_ptr()), n, dt, root, self.comm, st))
            ok = True
        finally:
            rc = lib.ncclGroupEnd()
            if ok:
                _check(lib, "ncclGroupEnd", rc)

    def destroy(self):
        if self.comm:
            torch.cuda.synchronize(self.device)
            _check(self.lib, "ncclCommDestroy", self.lib.ncclCommDestroy(self.comm))
            self.comm = ctypes.c_void_p()
