"""KSPPREONLY + PCLU (test.py:38-43,138).

The reference factors with MUMPS; here the distributed system is gathered to
rank 0 over the host control plane (as a centralized MUMPS analysis would) and
solved by libmxsolve's GPU dense LU with partial pivoting (mx_lu_solve_csr);
the solution is scattered back to the owners of the rows.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import core
from . import _lib
from ._lib import call


def lu_solve(A, b, x):
    from .PETSc import _mpi
    mc = _mpi(A.getComm())
    ip, cj, vv = A.getDeviceHandle().csr()
    bl = b.getArray()
    parts = mc.allgather((ip, cj, vv, bl)) if mc.Get_size() > 1 else [(ip, cj, vv, bl)]
    xl = None
    if mc.Get_rank() == 0:
        ips, cjs, vvs, bs = [], [], [], []
        off = 0
        for k, (pi, pc, pv, pb) in enumerate(parts):
            ips.append(pi[(1 if k else 0):] + off)
            off += pi[-1]
            cjs.append(pc); vvs.append(pv); bs.append(pb)
        gip = np.ascontiguousarray(np.concatenate(ips), np.int64)
        gcj = np.ascontiguousarray(np.concatenate(cjs), np.int64)
        gvv = np.ascontiguousarray(np.concatenate(vvs), np.float64)
        gb = np.ascontiguousarray(np.concatenate(bs), np.float64)
        n = gb.size
        gx = np.zeros(n)
        dc = A._dc
        try:
            call("mx_lu_solve_csr", dc.h, n, C.c_void_p(gip.ctypes.data), C.c_void_p(gcj.ctypes.data),
                 C.c_void_p(gvv.ctypes.data), C.c_void_p(gb.ctypes.data), C.c_void_p(gx.ctypes.data))
        except Exception as e:       # every rank raises the same error instead of waiting in bcast
            if mc.Get_size() == 1:
                raise
            chunks = ("error", getattr(e, "code", None), getattr(e, "msg", str(e)))
            err = e
        else:
            counts = [p[3].size for p in parts]
            starts = np.concatenate([[0], np.cumsum(counts)])
            chunks = [gx[starts[r]:starts[r + 1]] for r in range(len(parts))]
    else:
        chunks = None
    if mc.Get_size() > 1:
        chunks = mc.bcast(chunks, root=0)
        if isinstance(chunks, tuple) and chunks[:1] == ("error",):
            if mc.Get_rank() == 0:
                raise err
            if chunks[1] is None:
                raise RuntimeError(chunks[2])
            raise _lib.MxError(chunks[1], chunks[2])
    xl = chunks[mc.Get_rank()]
    x.setArray(xl)
    return x
