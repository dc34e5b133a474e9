"""mpi4py-compatible host control plane (the subset the reference drivers use).

Replaces mpi4py (environment.yaml:7) for the driver-level messages of
test.py:55-57,102-106,121-136,145 and test2.py:22-24,58-61,73-85: pickled
send/recv, buffer Send/Recv (bare ndarray or [buf, MPI.INT|MPI.DOUBLE]),
bcast, Gatherv, Barrier, allreduce.  Transport: torch.distributed over gloo
(host memory), rendezvous from the torchrun environment (RANK, WORLD_SIZE,
MASTER_ADDR=127.0.0.1, MASTER_PORT).  Launched without that environment the
world has one rank.  Device data never goes through here: the solver's halo
and reductions run over RCCL inside libmxsolve.so.
"""
from __future__ import annotations

import atexit
import sys
import os
import pickle

import numpy as np


class Datatype:
    def __init__(self, name: str, dtype):
        self.name, self.dtype = name, np.dtype(dtype)

    def __repr__(self):
        return f"MPI.{self.name}"


INT = Datatype("INT", np.int32)
LONG = Datatype("LONG", np.int64)
INT64_T = Datatype("INT64_T", np.int64)
DOUBLE = Datatype("DOUBLE", np.float64)
FLOAT = Datatype("FLOAT", np.float32)
BYTE = Datatype("BYTE", np.uint8)


class Op:
    def __init__(self, name, fn):
        self.name, self.fn = name, fn

    def __repr__(self):
        return f"MPI.{self.name}"


SUM = Op("SUM", lambda a, b: a + b)
MAX = Op("MAX", lambda a, b: max(a, b))
MIN = Op("MIN", lambda a, b: min(a, b))
PROD = Op("PROD", lambda a, b: a * b)

ANY_SOURCE = -1
ANY_TAG = -1


def _buf(spec):
    """[buf, datatype] / (buf, counts, displs, type) / bare ndarray -> (array, extra)."""
    if isinstance(spec, (list, tuple)):
        arr = spec[0]
        rest = list(spec[1:])
        if rest and isinstance(rest[-1], Datatype):
            dt = rest.pop()
            if arr.dtype != dt.dtype:
                raise TypeError(f"buffer dtype {arr.dtype} does not match {dt}")
        return arr, rest
    return spec, []


_EXIT_ON_EXCEPTION = []


def _note_uncaught(prev):
    """sys.excepthook wrapper: remember that the interpreter is exiting on an
    unhandled exception, so _finalize skips its long barrier."""
    def hook(tp, val, tb):
        _EXIT_ON_EXCEPTION.append(tp)
        prev(tp, val, tb)
    return hook


def _finalize(dist):
    """MPI_Finalize at interpreter exit (mpi4py registers the same): a last
    barrier, then the process group torn down while every rank is still
    there.  Without it a rank could exit while a peer's gloo threads were
    still live, and that peer's teardown died in std::terminate ('terminate
    called without an active exception', about one run in ten).  A rank
    exiting on an unhandled exception skips the barrier (its peers are not
    coming, or are blocked elsewhere): it closes its connections at once so
    the failure reaches them.  MXSOLVE_FINALIZE_TIMEOUT_S bounds the barrier
    (default 300 s)."""
    if not dist.is_initialized():
        return
    try:
        # bounded: a rank that died (or is stuck in another collective) must
        # not hold its peers' exit forever
        import datetime
        if not _EXIT_ON_EXCEPTION:
            t = float(os.environ.get("MXSOLVE_FINALIZE_TIMEOUT_S", "300"))
            dist.monitored_barrier(timeout=datetime.timedelta(seconds=t))
    except Exception:  # noqa: BLE001 -- a peer already gone: tear down anyway
        pass
    try:
        dist.destroy_process_group()
    except Exception:  # noqa: BLE001
        pass


class Comm:
    """COMM_WORLD over torch.distributed (gloo) -- or a world of one."""

    def __init__(self, self_only: bool = False):
        self._dist = None
        size = 1 if self_only else int(os.environ.get("WORLD_SIZE", "1"))
        if size > 1:
            import torch.distributed as dist
            if not dist.is_initialized():
                os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
                dist.init_process_group("gloo")
                sys.excepthook = _note_uncaught(sys.excepthook)
                atexit.register(_finalize, dist)
            self._dist = dist
            self._rank, self._size = dist.get_rank(), dist.get_world_size()
        else:
            self._rank, self._size = 0, 1

    # -- identity -----------------------------------------------------------
    def Get_rank(self) -> int:
        return self._rank

    def Get_size(self) -> int:
        return self._size

    rank = property(Get_rank)
    size = property(Get_size)

    def Barrier(self):
        if self._dist:
            self._dist.barrier()

    barrier = Barrier

    # -- raw transport --------------------------------------------------------
    def _send_bytes(self, data: bytes, dest: int, tag: int):
        import torch
        n = torch.tensor([len(data)], dtype=torch.int64)
        self._dist.send(n, dst=dest, tag=tag)
        if len(data):
            self._dist.send(torch.frombuffer(bytearray(data), dtype=torch.uint8), dst=dest, tag=tag)

    def _recv_bytes(self, source: int, tag: int) -> bytes:
        import torch
        n = torch.zeros(1, dtype=torch.int64)
        self._dist.recv(n, src=source, tag=tag)
        buf = torch.empty(int(n[0]), dtype=torch.uint8)
        if buf.numel():
            self._dist.recv(buf, src=source, tag=tag)
        return buf.numpy().tobytes()

    def _check_peer(self, r, what):
        if not (0 <= r < self._size) or r == self._rank:
            raise ValueError(f"invalid {what} rank {r}")

    # -- pickled objects (test.py:102,121) -------------------------------------
    def send(self, obj, dest: int, tag: int = 0):
        self._check_peer(dest, "dest")
        self._send_bytes(pickle.dumps(obj), dest, tag)

    def recv(self, buf=None, source: int = 0, tag: int = 0, status=None):
        self._check_peer(source, "source")
        return pickle.loads(self._recv_bytes(source, tag))

    def bcast(self, obj, root: int = 0):
        if self._size == 1:
            return obj
        lst = [obj if self._rank == root else None]
        self._dist.broadcast_object_list(lst, src=root)
        return lst[0]

    def allreduce(self, obj, op: Op = SUM):
        vals = self.allgather(obj)
        out = vals[0]
        for v in vals[1:]:
            out = op.fn(out, v)
        return out

    def allgather(self, obj):
        if self._size == 1:
            return [obj]
        lst = [None] * self._size
        self._dist.all_gather_object(lst, obj)
        return lst

    def gather(self, obj, root: int = 0):
        vals = self.allgather(obj)
        return vals if self._rank == root else None

    # -- buffers (test.py:103-106,128-131; test2.py:59-61,78-80) ---------------
    def Send(self, buf, dest: int, tag: int = 0):
        import torch
        self._check_peer(dest, "dest")
        arr, _ = _buf(buf)
        arr = np.ascontiguousarray(arr)
        self._dist.send(torch.from_numpy(arr.reshape(-1).view(np.uint8)), dst=dest, tag=tag)

    def Recv(self, buf, source: int = 0, tag: int = 0, status=None):
        import torch
        self._check_peer(source, "source")
        arr, _ = _buf(buf)
        if not arr.flags.c_contiguous:
            raise ValueError("Recv needs a contiguous buffer")
        t = torch.from_numpy(arr.reshape(-1).view(np.uint8))
        self._dist.recv(t, src=source, tag=tag)

    def Bcast(self, buf, root: int = 0):
        import torch
        if self._size == 1:
            return
        arr, _ = _buf(buf)
        t = torch.from_numpy(arr.reshape(-1).view(np.uint8))
        self._dist.broadcast(t, src=root)

    def Gatherv(self, sendbuf, recvbuf, root: int = 0):
        """test.py:145 passes a bare receive array with no counts; mpi4py would
        split it evenly (and fail when the size does not divide).  Here the
        counts are exchanged, so any row split gathers correctly."""
        sarr, _ = _buf(sendbuf)
        sarr = np.ascontiguousarray(sarr).reshape(-1)
        parts = self.allgather(sarr) if self._size > 1 else [sarr]
        if self._rank == root:
            rarr, rest = _buf(recvbuf)
            counts = [p.size for p in parts]
            displs = np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(int)
            if rest and rest[0] is not None:
                counts = list(rest[0])
                if len(rest) > 1 and rest[1] is not None:
                    displs = list(rest[1])
            flat = rarr.reshape(-1)
            for p, c, d in zip(parts, counts, displs):
                if p.size != c:
                    raise ValueError(f"Gatherv count mismatch: got {p.size}, expected {c}")
                flat[d:d + c] = p
        return None

    def Allreduce(self, sendbuf, recvbuf, op: Op = SUM):
        s, _ = _buf(sendbuf)
        r, _ = _buf(recvbuf)
        vals = self.allgather(np.array(s, copy=True))
        out = vals[0].copy()
        for v in vals[1:]:
            out = op.fn(out, v) if op is not MAX and op is not MIN else (np.maximum(out, v) if op is MAX else np.minimum(out, v))
        r[...] = out

    def Get_processor_name(self):
        import socket
        return socket.gethostname()


COMM_WORLD = Comm()
COMM_SELF = COMM_WORLD if COMM_WORLD.size == 1 else Comm(self_only=True)


def Get_processor_name():
    return COMM_WORLD.Get_processor_name()


def Wtime():
    import time
    return time.perf_counter()
