"""Thin Python handles over the C ABI (include/mxsolve.h).

Device vectors are torch float64 tensors (PyTorch is only the device-memory
and stream plumbing here); every compute call goes through libmxsolve.so.
A communicator's HIP stream is installed as torch's current stream for the
calling thread, so torch copies and library kernels are ordered on one queue.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import numpy as np
import torch

from . import _lib
from ._lib import KSPParams, KSPResult, MatInfo, MxError, call

KSP_TYPES = {"cg": 0, "gmres": 1, "preonly": 2}
PC_TYPES = {"none": 0, "jacobi": 1}
NORM_TYPES = {"default": -1, "none": 0, "preconditioned": 1, "unpreconditioned": 2, "natural": 3}
STENCILS = {"poisson2d": 0, "poisson3d": 1, "poisson3d27": 2, "convdiff3d": 3}


def _ptr(t) -> C.c_void_p:
    if isinstance(t, torch.Tensor):
        if not t.is_cuda or t.dtype != torch.float64 or not t.is_contiguous():
            raise TypeError("device vectors must be contiguous float64 CUDA tensors")
        return C.c_void_p(t.data_ptr())
    if t is None:
        return C.c_void_p(0)
    return C.c_void_p(int(t))


def default_device() -> int:
    n = torch.cuda.device_count()
    if n == 0:
        raise RuntimeError("mxsolve needs a ROCm GPU (no CPU fallback)")
    lr = os.environ.get("LOCAL_RANK")
    return int(lr) % n if lr is not None else 0


def unique_id() -> bytes:
    buf = C.create_string_buffer(128)
    call("mx_get_unique_id", buf, 128)
    return buf.raw


BIG_VECTOR_BYTES = 64 << 20


class _DeviceBuffer:
    """Library-allocated device memory exposed through __cuda_array_interface__;
    the tensor made from it keeps this object (and so the memory) alive."""

    def __init__(self, n: int, device: int):
        self.ptr = C.c_void_p()
        self.device = device
        call("mx_dev_alloc", device, n * 8, C.byref(self.ptr))
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "<f8", "data": (self.ptr.value or 0, False),
                                         "version": 2, "strides": None}

    def __del__(self):
        try:
            if self.ptr:
                _lib.load().mx_dev_free(self.ptr)
                self.ptr = C.c_void_p()
        except Exception:  # noqa: BLE001
            pass


def device_vector(n: int, device: int) -> torch.Tensor:
    """A float64 vector in HBM: large ones from the library's allocator (its
    device buffer cache, mx_dev_alloc), small ones from torch's cache."""
    if n * 8 < BIG_VECTOR_BYTES:
        return torch.empty(n, dtype=torch.float64, device=torch.device("cuda", device))
    buf = _DeviceBuffer(n, device)
    return torch.as_tensor(buf, device=torch.device("cuda", device))


class DeviceComm:
    """One rank's communicator handle (self, RCCL, or in-process local)."""

    def __init__(self, handle: C.c_void_p):
        self.h = handle
        r, s, d = C.c_int(), C.c_int(), C.c_int()
        call("mx_comm_info", handle, C.byref(r), C.byref(s), C.byref(d))
        self.rank, self.size, self.device = r.value, s.value, d.value
        sp = C.c_void_p()
        call("mx_comm_stream", handle, C.byref(sp))
        self.stream_ptr = sp.value
        self.torch_stream = torch.cuda.ExternalStream(self.stream_ptr, device=torch.device("cuda", self.device))
        self.activate()

    def activate(self):
        """Make this comm's stream torch's current stream (thread-local)."""
        torch.cuda.set_device(self.device)
        torch.cuda.set_stream(self.torch_stream)

    @classmethod
    def self_comm(cls, device: int | None = None):
        h = C.c_void_p()
        call("mx_comm_create_self", default_device() if device is None else device, C.byref(h))
        return cls(h)

    @classmethod
    def rccl(cls, rank: int, size: int, uid: bytes, device: int | None = None):
        h = C.c_void_p()
        b = C.create_string_buffer(uid, len(uid))
        call("mx_comm_create_rccl", rank, size, default_device() if device is None else device,
             b, len(uid), C.byref(h))
        return cls(h)

    @classmethod
    def shm(cls, rank: int, size: int, name: str, device: int | None = None, slot_kib: int | None = None):
        """Node-local processes sharing GPUs: payloads staged through POSIX
        shared memory `name` (rank 0 creates it; every rank passes the same name)."""
        h = C.c_void_p()
        kib = slot_kib if slot_kib is not None else int(os.environ.get("MXSOLVE_SHM_KIB", str(64 << 10)))
        call("mx_comm_create_shm", rank, size, default_device() if device is None else device,
             name.encode(), kib, C.byref(h))
        return cls(h)

    def comm_bench(self, what: int, iters: int = 200, mat=None) -> float:
        """Device time per communication op in us: 0 all-reduce of 1 double,
        1 of 3 doubles, 2 the halo exchange of `mat`.  Collective."""
        out = C.c_double()
        call("mx_debug_comm_bench", self.h, mat.h if mat is not None else C.c_void_p(0), what, iters,
             C.byref(out))
        return out.value

    def abort(self):
        if self.h:
            call("mx_comm_abort", self.h)

    def barrier(self):
        call("mx_comm_barrier", self.h)

    def empty(self, n: int) -> torch.Tensor:
        return device_vector(max(int(n), 0), self.device)

    def zeros(self, n: int) -> torch.Tensor:
        return device_vector(max(int(n), 0), self.device).zero_()

    def destroy(self):
        """Destroys the communicator (its stream goes with it): when that
        stream is this thread's current torch stream, the device's default
        stream becomes current again, so later torch work is not enqueued on
        a destroyed stream."""
        if self.h:
            if torch.cuda.current_stream(self.device).cuda_stream == self.stream_ptr:
                torch.cuda.set_stream(torch.cuda.default_stream(self.device))
            call("mx_comm_destroy", self.h)
            self.h = None


def _peer_abort(e) -> bool:
    return isinstance(e, MxError) and "another rank failed" in str(e)


class LocalWorld:
    """P virtual ranks sharing one GPU in one process (one host thread per rank)."""

    def __init__(self, size: int):
        self.h = C.c_void_p()
        call("mx_world_create_local", size, C.byref(self.h))
        self.size = size

    def comm(self, rank: int, device: int = 0) -> DeviceComm:
        h = C.c_void_p()
        call("mx_comm_create_local", self.h, rank, device, C.byref(h))
        return DeviceComm(h)

    def destroy(self):
        if self.h:
            call("mx_world_destroy", self.h)
            self.h = None

    def run(self, fn, device: int = 0):
        """Run fn(comm) on every rank in its own thread; return the results by rank."""
        out, errs = [None] * self.size, [None] * self.size

        def body(r):
            c = self.comm(r, device)
            try:
                out[r] = fn(c)
            except BaseException as e:  # noqa: BLE001
                errs[r] = e
                call("mx_world_abort", self.h)     # release ranks waiting on this one
            finally:
                torch.cuda.synchronize(device)
                c.destroy()

        ts = [threading.Thread(target=body, args=(r,)) for r in range(self.size)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        first = [e for e in errs if e is not None and not _peer_abort(e)]
        for e in first or [e for e in errs if e is not None]:
            raise e
        return out


def layout_split(N: int, P: int) -> np.ndarray:
    r = (C.c_int64 * (P + 1))()
    call("mx_layout_split", N, P, r)
    return np.array(list(r), dtype=np.int64)


class DMat:
    """Assembled row-partitioned AIJ matrix living in HBM."""

    def __init__(self, comm: DeviceComm, handle: C.c_void_p):
        self.comm, self.h = comm, handle
        self._info = None

    # -- construction ---------------------------------------------------
    @classmethod
    def from_csr(cls, comm: DeviceComm, M: int, N: int, indptr, cols, vals, m_local: int = -1,
                 n_local: int = -1, add: bool = False):
        """createAIJ(size=(M,N), csr=(indptr, cols, vals)): local rows, global cols."""
        if isinstance(indptr, torch.Tensor):
            ip, cl, vl = indptr, cols, vals
            for t in (ip, cl):   # read in place by the library: no hidden copies
                if not t.is_cuda or t.dtype not in (torch.int32, torch.int64) or not t.is_contiguous():
                    raise TypeError("device CSR index arrays must be contiguous int32/int64 CUDA tensors")
            _ptr(vl)
            dev = 1
            ipb, clb = ip.element_size(), cl.element_size()
            nnz = cl.numel()
            keep = (ip, cl, vl)
            pi, pc, pv = C.c_void_p(ip.data_ptr()), C.c_void_p(cl.data_ptr()), C.c_void_p(vl.data_ptr())
        else:
            ip = np.ascontiguousarray(indptr)
            if ip.dtype not in (np.int32, np.int64):
                ip = ip.astype(np.int64)
            cl = np.ascontiguousarray(cols)
            if cl.dtype not in (np.int32, np.int64):
                cl = cl.astype(np.int64)
            vl = np.ascontiguousarray(vals, dtype=np.float64)
            dev, ipb, clb, nnz = 0, ip.itemsize, cl.itemsize, cl.size
            keep = (ip, cl, vl)
            pi, pc, pv = (C.c_void_p(a.ctypes.data) for a in keep)
        h = C.c_void_p()
        call("mx_mat_create_csr", comm.h, M, N, m_local, n_local, pi, ipb, pc, clb, pv, nnz,
             int(add), dev, C.byref(h))
        del keep
        return cls(comm, h)

    @classmethod
    def from_coo(cls, comm: DeviceComm, M: int, N: int, rows, cols, vals, m_local: int = -1,
                 n_local: int = -1, add: bool = False):
        r = np.ascontiguousarray(rows, dtype=np.int64)
        c = np.ascontiguousarray(cols, dtype=np.int64)
        v = np.ascontiguousarray(vals, dtype=np.float64)
        h = C.c_void_p()
        call("mx_mat_create_coo", comm.h, M, N, m_local, n_local, C.c_void_p(r.ctypes.data),
             C.c_void_p(c.ctypes.data), C.c_void_p(v.ctypes.data), r.size, int(add), 0, C.byref(h))
        return cls(comm, h)

    @classmethod
    def stencil(cls, comm: DeviceComm, kind: str, nx: int, ny: int | None = None, nz: int | None = None):
        ny = nx if ny is None else ny
        nz = nx if nz is None else nz
        h = C.c_void_p()
        call("mx_mat_create_stencil", comm.h, STENCILS[kind], nx, ny, nz, C.byref(h))
        return cls(comm, h)

    # -- queries ----------------------------------------------------------
    def info(self) -> dict:
        if self._info is None:
            mi = MatInfo()
            call("mx_mat_get_info", self.h, C.byref(mi))
            self._info = {k: getattr(mi, k) for k, _ in MatInfo._fields_}
        return self._info

    @property
    def local_rows(self) -> int:
        return self.info()["m"]

    def csr(self):
        i = self.info()
        nnz = i["nnz_d"] + i["nnz_o"]
        ip = np.zeros(i["m"] + 1, np.int64)
        cl = np.zeros(max(nnz, 1), np.int64)
        vl = np.zeros(max(nnz, 1), np.float64)
        call("mx_mat_get_csr", self.h, C.c_void_p(ip.ctypes.data), C.c_void_p(cl.ctypes.data),
             C.c_void_p(vl.ctypes.data))
        return ip, cl[:nnz], vl[:nnz]

    def split(self) -> dict:
        i = self.info()
        m, nd, no, ng = i["m"], i["nnz_d"], i["nnz_o"], i["nghost"]
        a = dict(dptr=np.zeros(m + 1, np.int64), dcol=np.zeros(max(nd, 1), np.int32),
                 dval=np.zeros(max(nd, 1)), optr=np.zeros(m + 1, np.int64),
                 ocol=np.zeros(max(no, 1), np.int32), oval=np.zeros(max(no, 1)),
                 garray=np.zeros(max(ng, 1), np.int64))
        call("mx_mat_get_split", self.h, *(C.c_void_p(a[k].ctypes.data) for k in
                                          ("dptr", "dcol", "dval", "optr", "ocol", "oval", "garray")))
        a["dcol"], a["dval"] = a["dcol"][:nd], a["dval"][:nd]
        a["ocol"], a["oval"], a["garray"] = a["ocol"][:no], a["oval"][:no], a["garray"][:ng]
        return a

    # -- compute ------------------------------------------------------------
    def mult(self, x: torch.Tensor, y: torch.Tensor):
        call("mx_mat_mult", self.h, _ptr(x), _ptr(y))

    def diagonal(self, out: torch.Tensor):
        call("mx_mat_get_diagonal", self.h, _ptr(out))

    def bench_mult(self, x: torch.Tensor, y: torch.Tensor, iters: int):
        s, m = C.c_double(), C.c_double()
        call("mx_mat_bench_mult", self.h, _ptr(x), _ptr(y), iters, C.byref(s), C.byref(m))
        return s.value, m.value

    def bench_mult_cold(self, x: torch.Tensor, y: torch.Tensor, flush: torch.Tensor, iters: int = 5):
        """Cold-cache MatMult (flush buffer filled before each): median device
        ms of the SpMV kernel alone (one rank; else < 0) and of the MatMult."""
        s, m = C.c_double(), C.c_double()
        call("mx_mat_bench_mult_cold", self.h, _ptr(x), _ptr(y), _ptr(flush), flush.numel(), iters,
             C.byref(s), C.byref(m))
        return s.value, m.value

    def solve(self, b: torch.Tensor, x: torch.Tensor, ksp: str = "cg", pc: str = "jacobi",
              rtol: float = 1e-5, atol: float = 1e-50, dtol: float = 1e5, max_it: int = 10000,
              restart: int = 30, norm: str = "default", guess_nonzero: bool = False,
              history: bool = False, profile: bool = False, poll_every: int = 16) -> dict:
        p = KSPParams()
        _lib.load().mx_ksp_default_params(C.byref(p))
        p.ksp_type, p.pc_type, p.norm_type = KSP_TYPES[ksp], PC_TYPES[pc], NORM_TYPES[norm]
        p.rtol, p.atol, p.dtol, p.max_it, p.restart = rtol, atol, dtol, max_it, restart
        p.guess_nonzero, p.profile, p.poll_every = int(guess_nonzero), int(profile), poll_every   # profile: bool or bits
        r = KSPResult()
        h = np.zeros(max_it + 2) if history else None
        call("mx_ksp_solve", self.h, C.byref(p), _ptr(b), _ptr(x), C.byref(r),
             C.c_void_p(h.ctypes.data) if history else C.c_void_p(0))
        out = {k: getattr(r, k) for k, _ in KSPResult._fields_}
        if history:
            out["history"] = h[: r.its + 1]
        return out

    def ksp_reset(self):
        """KSPDestroy/KSPReset: drop the solver state kept on this operator."""
        if self.h and self.comm.h:          # (the communicator's stream is synced)
            call("mx_ksp_destroy", self.h)

    def destroy(self):
        """MatDestroy.  A matrix must go before its communicator: once the
        communicator is destroyed the device memory is left to process exit
        (the library's matrix refers to the communicator's stream)."""
        if self.h:
            if self.comm.h:
                call("mx_mat_destroy", self.h)
            self.h = None

    def __del__(self):
        try:
            self.destroy()
        except Exception:  # noqa: BLE001
            pass


# ---------------------------------------------------------------- Vec helpers
def vdot(comm: DeviceComm, x, y) -> float:
    out = C.c_double()
    call("mx_vec_dot", comm.h, x.numel(), _ptr(x), _ptr(y), C.byref(out))
    return out.value


def vnorm(comm: DeviceComm, x) -> float:
    out = C.c_double()
    call("mx_vec_norm2", comm.h, x.numel(), _ptr(x), C.byref(out))
    return out.value


def vaxpy(comm, a, x, y):
    call("mx_vec_axpy", comm.h, y.numel(), float(a), _ptr(x), _ptr(y))


def vaypx(comm, a, x, y):
    call("mx_vec_aypx", comm.h, y.numel(), float(a), _ptr(x), _ptr(y))


def vpmult(comm, x, y, w):
    call("mx_vec_pointwise_mult", comm.h, w.numel(), _ptr(x), _ptr(y), _ptr(w))


def vscale(comm, a, x):
    call("mx_vec_scale", comm.h, x.numel(), float(a), _ptr(x))


def vset(comm, a, x):
    call("mx_vec_set", comm.h, x.numel(), float(a), _ptr(x))


def vmdot(comm: DeviceComm, x, ys) -> np.ndarray:
    """VecMDot: [x . y for y in ys] (collective)."""
    arr = (C.c_void_p * max(len(ys), 1))(*[_ptr(y).value for y in ys])
    out = np.zeros(len(ys))
    call("mx_vec_mdot", comm.h, x.numel(), _ptr(x), len(ys), arr, out.ctypes.data_as(C.POINTER(C.c_double)))
    return out


def vmaxpy(comm: DeviceComm, y, alphas, xs):
    """VecMAXPY: y += sum_k alphas[k] xs[k] (PETSc's grouping)."""
    arr = (C.c_void_p * max(len(xs), 1))(*[_ptr(v).value for v in xs])
    a = np.ascontiguousarray(alphas, dtype=np.float64)
    call("mx_vec_maxpy", comm.h, y.numel(), _ptr(y), len(xs), a.ctypes.data_as(C.POINTER(C.c_double)), arr)


DISPATCH_KINDS = ("sell", "sell_cg", "pair_lean", "pair_zm", "pair_zm_split", "pair_zm27", "pair_zm27_split",
                  "pair_zmf64", "pair_zmf64_split", "pair_zmcg", "boundary", "zm_pw", "zm_rupd", "pair_zmc",
                  "pair_zmc_split", "zm_pbw", "zm_pbws", "cb")


def dispatch_counts(reset: bool = False) -> dict:
    """Host-side counts of the MatMult-family launches by kernel kind since the
    last reset (mx_debug_dispatch_counts; replayed graph launches not counted)."""
    out = (C.c_int64 * len(DISPATCH_KINDS))()
    call("mx_debug_dispatch_counts", out, len(DISPATCH_KINDS), int(reset))
    return {k: int(out[i]) for i, k in enumerate(DISPATCH_KINDS)}


ASM_PHASES = ("h2d_ms", "canon_ms", "split_ms", "layout_ms", "halo_ms", "total_ms", "host_bytes", "alloc_ms")


def assembly_times() -> dict:
    """Phase times of this thread's last createAIJ(csr=...) (mx_debug_assembly_times)."""
    out = (C.c_double * len(ASM_PHASES))()
    call("mx_debug_assembly_times", out, len(ASM_PHASES))
    return {k: float(out[i]) for i, k in enumerate(ASM_PHASES)}


def rhs_hash(comm, i0: int, out: torch.Tensor):
    call("mx_vec_rhs_hash", comm.h, i0, out.numel(), _ptr(out))
