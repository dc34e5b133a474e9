"""ctypes wrapper around the C oracle (oracle/petsc_oracle.c).

TEST INFRASTRUCTURE ONLY -- importable from tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg.  The product (libmxsolve.so + mxsolve) never
imports this module.  Parity status: see petsc_oracle.h / DESIGN.md (CG/GMRES
iterates are "parity unpinned" against PETSc itself; pinned against this
restatement and the reference's own fixtures).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liboracle.so")

KSP_TYPES = {"cg": 0, "gmres": 1, "preonly": 2}
PC_TYPES = {"none": 0, "jacobi": 1}
NORM_TYPES = {"default": -1, "none": 0, "preconditioned": 1, "unpreconditioned": 2, "natural": 3}


class KSPParams(C.Structure):
    _fields_ = [("ksp_type", C.c_int), ("pc_type", C.c_int), ("norm_type", C.c_int),
                ("max_it", C.c_int), ("restart", C.c_int), ("guess_nonzero", C.c_int),
                ("rtol", C.c_double), ("atol", C.c_double), ("dtol", C.c_double),
                ("haptol", C.c_double), ("breakdowntol", C.c_double),
                ("axpy_fma", C.c_int), ("nthreads", C.c_int)]


class KSPResult(C.Structure):
    _fields_ = [("its", C.c_int), ("reason", C.c_int), ("rnorm", C.c_double)]


_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        P = C.c_void_p
        i64p = np.ctypeslib.ndpointer(np.int64, flags="C")
        i32p = np.ctypeslib.ndpointer(np.int32, flags="C")
        f64p = np.ctypeslib.ndpointer(np.float64, flags="C")
        L.or_split_ownership.argtypes = [C.c_int64, C.c_int, i64p]
        L.or_mat_create_csr.argtypes = [C.c_int64, C.c_int64, C.c_int, i64p, i64p, f64p, C.c_int, C.POINTER(C.c_int)]
        L.or_mat_create_csr.restype = P
        L.or_mat_create_coo.argtypes = [C.c_int64, C.c_int64, C.c_int, i64p, i64p, i64p, f64p, C.c_int, C.POINTER(C.c_int)]
        L.or_mat_create_coo.restype = P
        L.or_mat_destroy.argtypes = [P]
        L.or_mat_nnz.argtypes = [P]
        L.or_mat_nnz.restype = C.c_int64
        L.or_mat_get_csr.argtypes = [P, i64p, i64p, f64p]
        L.or_mat_block_sizes.argtypes = [P, C.c_int] + [C.POINTER(C.c_int64)] * 4
        L.or_mat_get_block.argtypes = [P, C.c_int, i64p, i32p, f64p, i64p, i32p, f64p, i64p]
        L.or_mat_mult.argtypes = [P, f64p, f64p]
        L.or_mat_get_diagonal.argtypes = [P, f64p]
        L.or_ksp_solve.argtypes = [P, C.POINTER(KSPParams), f64p, f64p, C.POINTER(KSPResult), P]
        L.or_ksp_default_params.argtypes = [C.POINTER(KSPParams)]
        L.or_stencil.argtypes = [C.c_int, C.c_int64, C.c_int64, C.c_int64, P, P, P]
        L.or_stencil.restype = C.c_int64
        L.or_rhs_hash.argtypes = [C.c_int64, C.c_int64, f64p]
        dp = C.POINTER(C.c_double)
        L.or_vec_maxpy.argtypes = [C.c_int64, C.c_int, dp, C.POINTER(dp), dp]
        L.or_vec_mdot.argtypes = [C.c_int64, dp, C.c_int, C.POINTER(dp), dp]
        _lib = L
    return _lib


def split_ownership(N: int, P: int) -> np.ndarray:
    r = np.zeros(P + 1, np.int64)
    lib().or_split_ownership(N, P, r)
    return r


def stash_order(M: int, P: int, per_rank):
    """MatAssemblyEnd's stash delivery, restated: every rank's MatSetValues
    entries (in call order) end up on the owner of their row; the owner applies
    its own entries first and then the stashed ones (PETSc's
    MatAssemblyEnd_MPIAIJ -> MatStashScatterGetMesg loop).  PETSc applies the
    messages in arrival order; the deterministic rule used here (and by the
    device path) is ascending source rank.  Negative rows/columns are dropped
    like MatSetValues does.  Returns (coo_ptr, rows, cols, vals) for
    OracleMat.from_coo.  per_rank: list of P (rows, cols, vals) triples."""
    ranges = split_ownership(M, P)
    seg = [[] for _ in range(P)]
    for q, (r, c, v) in enumerate(per_rank):
        r, c, v = np.asarray(r, np.int64), np.asarray(c, np.int64), np.asarray(v, np.float64)
        keep = (r >= 0) & (c >= 0)
        r, c, v = r[keep], c[keep], v[keep]
        own = np.searchsorted(ranges, r, side="right") - 1
        for o in range(P):
            sel = own == o
            seg[o].append((q, r[sel], c[sel], v[sel]))
    rows, cols, vals, ptr = [], [], [], [0]
    for o in range(P):
        parts = sorted(seg[o], key=lambda t: (t[0] != o, t[0]))   # own entries first, then by rank
        for _, r, c, v in parts:
            rows.append(r); cols.append(c); vals.append(v)
        ptr.append(ptr[-1] + sum(p[1].size for p in parts))
    cat = lambda xs, dt: np.concatenate(xs).astype(dt) if xs else np.zeros(0, dt)
    return np.array(ptr, np.int64), cat(rows, np.int64), cat(cols, np.int64), cat(vals, np.float64)


class OracleMat:
    """P-rank AIJ matrix assembled by the restated PETSc rules."""

    def __init__(self, ptr, M, N, P):
        self.ptr, self.M, self.N, self.P = ptr, M, N, P

    @classmethod
    def from_csr(cls, M, N, indptr, cols, vals, P=1, add=False):
        err = C.c_int(0)
        p = lib().or_mat_create_csr(M, N, P, np.ascontiguousarray(indptr, np.int64),
                                    np.ascontiguousarray(cols, np.int64),
                                    np.ascontiguousarray(vals, np.float64), int(add), C.byref(err))
        if not p:
            raise ValueError(f"oracle assembly failed ({err.value})")
        return cls(p, M, N, P)

    @classmethod
    def from_coo(cls, M, N, coo_ptr, rows, cols, vals, P=1, add=False):
        err = C.c_int(0)
        p = lib().or_mat_create_coo(M, N, P, np.ascontiguousarray(coo_ptr, np.int64),
                                    np.ascontiguousarray(rows, np.int64),
                                    np.ascontiguousarray(cols, np.int64),
                                    np.ascontiguousarray(vals, np.float64), int(add), C.byref(err))
        if not p:
            raise ValueError(f"oracle assembly failed ({err.value})")
        return cls(p, M, N, P)

    def __del__(self):
        if getattr(self, "ptr", None):
            lib().or_mat_destroy(self.ptr)
            self.ptr = None

    @property
    def nnz(self):
        return int(lib().or_mat_nnz(self.ptr))

    def csr(self):
        nnz = self.nnz
        ip = np.zeros(self.M + 1, np.int64)
        c = np.zeros(max(nnz, 1), np.int64)
        v = np.zeros(max(nnz, 1), np.float64)
        lib().or_mat_get_csr(self.ptr, ip, c, v)
        return ip, c[:nnz], v[:nnz]

    def block(self, r):
        m, nd, no, ng = (C.c_int64() for _ in range(4))
        lib().or_mat_block_sizes(self.ptr, r, C.byref(m), C.byref(nd), C.byref(no), C.byref(ng))
        m, nd, no, ng = m.value, nd.value, no.value, ng.value
        dptr = np.zeros(m + 1, np.int64); optr = np.zeros(m + 1, np.int64)
        dcol = np.zeros(max(nd, 1), np.int32); dval = np.zeros(max(nd, 1))
        ocol = np.zeros(max(no, 1), np.int32); oval = np.zeros(max(no, 1))
        g = np.zeros(max(ng, 1), np.int64)
        lib().or_mat_get_block(self.ptr, r, dptr, dcol, dval, optr, ocol, oval, g)
        return dict(dptr=dptr, dcol=dcol[:nd], dval=dval[:nd], optr=optr, ocol=ocol[:no],
                    oval=oval[:no], garray=g[:ng])

    def mult(self, x):
        y = np.zeros(self.M)
        lib().or_mat_mult(self.ptr, np.ascontiguousarray(x, np.float64), y)
        return y

    def diagonal(self):
        d = np.zeros(self.M)
        lib().or_mat_get_diagonal(self.ptr, d)
        return d

    def solve(self, b, x0=None, ksp="cg", pc="jacobi", rtol=1e-5, atol=1e-50, dtol=1e5,
              max_it=10000, restart=30, norm="default", axpy_fma=True, nthreads=1,
              history=False):
        p = KSPParams()
        lib().or_ksp_default_params(C.byref(p))
        p.ksp_type = KSP_TYPES[ksp]; p.pc_type = PC_TYPES[pc]; p.norm_type = NORM_TYPES[norm]
        p.max_it = max_it; p.restart = restart; p.rtol = rtol; p.atol = atol; p.dtol = dtol
        p.axpy_fma = int(axpy_fma); p.nthreads = nthreads
        x = np.zeros(self.M) if x0 is None else np.array(x0, np.float64)
        p.guess_nonzero = int(x0 is not None)
        r = KSPResult()
        h = np.zeros(max_it + 2) if history else None
        rc = lib().or_ksp_solve(self.ptr, C.byref(p), np.ascontiguousarray(b, np.float64), x,
                                C.byref(r), h.ctypes.data_as(C.c_void_p) if history else None)
        if rc:
            raise RuntimeError("oracle solve failed")
        out = dict(x=x, its=r.its, reason=r.reason, rnorm=r.rnorm)
        if history:
            out["history"] = h[: r.its + 1]
        return out


STENCILS = {"poisson2d": 0, "poisson3d": 1, "poisson3d27": 2, "convdiff3d": 3}


def stencil(kind: str, nx: int, ny: int = None, nz: int = None):
    """Canonical global CSR of the synthetic operators."""
    ny = nx if ny is None else ny
    nz = nx if nz is None else nz
    k = STENCILS[kind]
    nnz = lib().or_stencil(k, nx, ny, nz, None, None, None)
    nrow = nx * ny if k == 0 else nx * ny * nz
    ip = np.zeros(nrow + 1, np.int64); c = np.zeros(nnz, np.int64); v = np.zeros(nnz)
    lib().or_stencil(k, nx, ny, nz, ip.ctypes.data_as(C.c_void_p), c.ctypes.data_as(C.c_void_p),
                     v.ctypes.data_as(C.c_void_p))
    return ip, c, v


def rhs_hash(i0: int, n: int) -> np.ndarray:
    b = np.zeros(n)
    lib().or_rhs_hash(i0, n, b)
    return b


def vec_maxpy(y, alphas, xs):
    """VecMAXPY_Seq restated: returns y + sum alphas[k] xs[k] with PETSc's grouping."""
    out = np.ascontiguousarray(y, dtype=np.float64).copy()
    xs = [np.ascontiguousarray(v, dtype=np.float64) for v in xs]
    a = np.ascontiguousarray(alphas, dtype=np.float64)
    f64p = C.POINTER(C.c_double)
    arr = (f64p * max(len(xs), 1))(*[v.ctypes.data_as(f64p) for v in xs])
    lib().or_vec_maxpy(out.size, len(xs), a.ctypes.data_as(f64p), arr, out.ctypes.data_as(f64p))
    return out


def vec_mdot(x, ys):
    """VecMDot, sequential sums."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    ys = [np.ascontiguousarray(v, dtype=np.float64) for v in ys]
    f64p = C.POINTER(C.c_double)
    arr = (f64p * max(len(ys), 1))(*[v.ctypes.data_as(f64p) for v in ys])
    out = np.zeros(len(ys))
    lib().or_vec_mdot(x.size, x.ctypes.data_as(f64p), len(ys), arr, out.ctypes.data_as(f64p))
    return out
