"""Communicators of the sharded LaserMapping (include/loam_core.h, "Sharded LaserMapping").

A sharded mapper (``BatchMapper(..., comm=c)``) splits every mapping stream over ``c.size``
ranks: each rank stores the map points of the 4 m blocks it owns, the 5-NN candidate lists are
all-gathered once per outer round and every Ceres iteration all-reduces the 29 normal-equation
sums.  Transports:

- ``Comm.rccl(rank, size, uid, device)`` — RCCL over xGMI, collectives enqueued on the
  mapper's HIP stream (no host synchronisation).  ``Comm.rccl_unique_id()`` on rank 0, shared
  by the caller (``bench.py`` uses torch.distributed's object broadcast).
- ``Comm.local_group(size, device)`` — ranks as threads of one process on one device: the
  library stages each collective on the device and orders it with events on the ranks' own HIP
  streams (the threads meet only when they enqueue; no device synchronisation).
- ``ThreadGroup(size).comm(rank)`` — ranks as threads of one process (one GPU or several):
  host-buffer callbacks meeting at a barrier, summed in rank order.
- ``TorchDistComm.create()`` — host-buffer callbacks over an initialised torch.distributed group
  (gloo), all-gather + ordered sum so every rank gets bit-identical sums.
- ``TorchDistStagedComm.create()`` — the same collectives behind device-pointer callbacks
  (``host_buffers = 0``: the library hands over HBM pointers and its HIP stream); the callback
  waits for the stream and stages through host memory.  It exercises the device-pointer
  transport path of the C-ABI, which a caller's own device collectives would use.

Every allreduce must give bit-identical results on all ranks (every rank then takes the same
trust-region step and stores points with the same pose); RCCL's ring / tree algorithms reduce
each element once and broadcast it, the Python transports sum in rank order.
"""
import ctypes
import threading

import numpy as np

from ._core import check, lib

DT_F64, DT_I32 = 0, 1
RCCL_ID_BYTES = 128

ALLREDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                ctypes.c_int32, ctypes.c_void_p)
ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                ctypes.c_int64, ctypes.c_void_p)


class CommOps(ctypes.Structure):
    _fields_ = [("user", ctypes.c_void_p), ("host_buffers", ctypes.c_int32),
                ("allreduce_sum", ALLREDUCE_FN), ("allgather", ALLGATHER_FN)]


def _view(buf, count, dtype):
    ct = ctypes.c_double if dtype == DT_F64 else ctypes.c_int32
    return np.ctypeslib.as_array(ctypes.cast(buf, ctypes.POINTER(ct)), shape=(count,))


def _bytes_view(buf, n):
    return np.ctypeslib.as_array(ctypes.cast(buf, ctypes.POINTER(ctypes.c_uint8)), shape=(n,))


class Comm:
    """A loam_comm handle (must outlive the mappers that use it)."""

    def __init__(self, handle, rank, size, keep=()):
        self.h = handle
        self.rank = rank
        self.size = size
        self._keep = keep  # ctypes callbacks referenced by the C side

    @staticmethod
    def rccl_unique_id():
        buf = (ctypes.c_uint8 * RCCL_ID_BYTES)()
        check(lib().loam_comm_rccl_unique_id(buf))
        return bytes(buf)

    @classmethod
    def rccl(cls, rank, size, uid, device=0):
        if len(uid) != RCCL_ID_BYTES:
            raise ValueError("RCCL unique id must be 128 bytes")
        buf = (ctypes.c_uint8 * RCCL_ID_BYTES).from_buffer_copy(uid)
        h = ctypes.c_void_p()
        check(lib().loam_comm_create_rccl(rank, size, buf, device, ctypes.byref(h)))
        return cls(h, rank, size)

    @classmethod
    def from_host_callbacks(cls, rank, size, allreduce, allgather):
        """allreduce(np_array) sums in place over the ranks; allgather(np_uint8_send) -> bytes of
        every rank's send in rank order (written into the returned buffer)."""

        def ar(user, buf, count, dtype, stream):
            try:
                allreduce(_view(buf, count, dtype))
                return 0
            except Exception:  # noqa: BLE001 — reported to the C side as a failed collective
                return 1

        def ag(user, send, recv, nbytes, stream):
            try:
                out = allgather(_bytes_view(send, nbytes))
                _bytes_view(recv, nbytes * size)[:] = out
                return 0
            except Exception:  # noqa: BLE001
                return 1

        ops = CommOps()
        ops.user = None
        ops.host_buffers = 1
        ops.allreduce_sum = ALLREDUCE_FN(ar)
        ops.allgather = ALLGATHER_FN(ag)
        h = ctypes.c_void_p()
        check(lib().loam_comm_create(rank, size, ctypes.byref(ops), ctypes.byref(h)))
        return cls(h, rank, size, keep=(ops, ops.allreduce_sum, ops.allgather, ar, ag))

    @classmethod
    def from_device_callbacks(cls, rank, size, allreduce, allgather):
        """device-pointer callbacks: allreduce(d_buf, count, dtype, hip_stream) sums in place over
        the ranks, allgather(d_send, d_recv, nbytes, hip_stream) fills d_recv with every rank's
        send in rank order; both return 0 on success"""

        def ar(user, buf, count, dtype, stream):
            try:
                return int(allreduce(buf, count, dtype, stream) or 0)
            except Exception:  # noqa: BLE001
                return 1

        def ag(user, send, recv, nbytes, stream):
            try:
                return int(allgather(send, recv, nbytes, stream) or 0)
            except Exception:  # noqa: BLE001
                return 1

        ops = CommOps()
        ops.user = None
        ops.host_buffers = 0
        ops.allreduce_sum = ALLREDUCE_FN(ar)
        ops.allgather = ALLGATHER_FN(ag)
        h = ctypes.c_void_p()
        check(lib().loam_comm_create(rank, size, ctypes.byref(ops), ctypes.byref(h)))
        return cls(h, rank, size, keep=(ops, ops.allreduce_sum, ops.allgather, ar, ag))

    @classmethod
    def local_group(cls, size, device=0):
        """``size`` ranks of this process on one device (one thread and one sharded handle per
        rank): the collectives are ordered on the ranks' HIP streams by events, the threads meet
        only when they enqueue one (loam_comm_create_local)"""
        hs = (ctypes.c_void_p * size)()
        check(lib().loam_comm_create_local(size, device, hs))
        return [cls(ctypes.c_void_p(hs[r]), r, size) for r in range(size)]

    @classmethod
    def single(cls):
        """a one-rank comm: the sharded code path with trivial collectives"""
        h = ctypes.c_void_p()
        check(lib().loam_comm_create(0, 1, None, ctypes.byref(h)))
        return cls(h, 0, 1)

    def close(self):
        if getattr(self, "h", None) and self.h.value:
            lib().loam_comm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class ThreadGroup:
    """Ranks as threads of one process: collectives meet at a barrier (timeout: a rank that
    fails makes the others' collectives fail instead of hanging)."""

    def __init__(self, size, timeout=120.0):
        self.size = size
        self.barrier = threading.Barrier(size, timeout=timeout)
        self.slots = [None] * size

    def _allreduce(self, rank, arr):
        self.slots[rank] = arr.copy()
        self.barrier.wait()
        total = self.slots[0].copy()
        for r in range(1, self.size):
            total += self.slots[r]
        self.barrier.wait()
        arr[:] = total

    def _allgather(self, rank, send):
        self.slots[rank] = send.copy()
        self.barrier.wait()
        out = np.concatenate(self.slots)
        self.barrier.wait()
        return out

    def comm(self, rank):
        return Comm.from_host_callbacks(rank, self.size, lambda a: self._allreduce(rank, a),
                                        lambda s: self._allgather(rank, s))


def dist_allreduce_ordered(arr):
    """in-place sum of a numpy array over the default torch.distributed group, as an
    all-gather + rank-ordered sum: bit-identical on every rank whatever the backend"""
    import torch
    import torch.distributed as dist

    t = torch.from_numpy(np.array(arr, copy=True))
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, t)
    total = parts[0].clone()
    for p in parts[1:]:
        total += p
    arr[:] = total.numpy()


def dist_allgather_bytes(send):
    """every rank's uint8 buffer (same size everywhere), concatenated in rank order"""
    import torch
    import torch.distributed as dist

    t = torch.from_numpy(np.array(send, copy=True))
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, t)
    return torch.cat(parts).numpy()


class TorchDistComm:
    """Host-buffer comm over the default torch.distributed group (e.g. gloo, one process per
    rank), through dist_allreduce_ordered / dist_allgather_bytes."""

    @staticmethod
    def create():
        import torch.distributed as dist

        return Comm.from_host_callbacks(dist.get_rank(), dist.get_world_size(), dist_allreduce_ordered,
                                        dist_allgather_bytes)


class TorchDistStagedComm:
    """Device-pointer callbacks over the default torch.distributed group: wait for the mapper's
    HIP stream, copy the device buffer to host memory, run the ordered gloo collective, copy back.
    The library side is its device-pointer (host_buffers = 0) transport."""

    @staticmethod
    def create():
        import torch.distributed as dist

        hip = ctypes.CDLL("libamdhip64.so")
        hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
        hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        d2h, h2d = 2, 1  # hipMemcpyDeviceToHost, hipMemcpyHostToDevice

        def allreduce(buf, count, dtype, stream):
            if hip.hipStreamSynchronize(stream) != 0:
                return 1
            arr = np.empty(count, dtype=np.float64 if dtype == DT_F64 else np.int32)
            if hip.hipMemcpy(arr.ctypes.data, buf, arr.nbytes, d2h) != 0:
                return 1
            dist_allreduce_ordered(arr)
            return hip.hipMemcpy(buf, arr.ctypes.data, arr.nbytes, h2d)

        def allgather(send, recv, nbytes, stream):
            if hip.hipStreamSynchronize(stream) != 0:
                return 1
            arr = np.empty(nbytes, dtype=np.uint8)
            if nbytes and hip.hipMemcpy(arr.ctypes.data, send, nbytes, d2h) != 0:
                return 1
            out = np.ascontiguousarray(dist_allgather_bytes(arr))
            return hip.hipMemcpy(recv, out.ctypes.data, out.nbytes, h2d) if out.nbytes else 0

        return Comm.from_device_callbacks(dist.get_rank(), dist.get_world_size(), allreduce, allgather)
