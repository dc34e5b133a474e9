"""BASELINE.json configurations at full size on one GPU.

C3 (3D 7-pt 256^3, CG+Jacobi): parity with the oracle's full-size solve
(iteration count equal, rel-L2 <= 1e-10).  C2 (2D 4096^2, CG), C4 (conv-diff
256^3, GMRES(30)) and C5's per-GPU share (27-pt 512x512x64, CG) are too long
for the CPU oracle; they are checked through size-independent properties:
the converged reason, the true preconditioned residual recomputed from x
(agrees with the recurrence's final norm), and assembly identities (nnz
formulas, aligned-offset slices)."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def true_prec_residual(A, b, x, dinv_scalar=None):
    from mxsolve.core import vnorm
    comm = A.comm
    r = comm.empty(b.numel())
    A.mult(x, r)
    r = b - r
    d = comm.empty(b.numel())
    A.diagonal(d)
    z = r / d
    return float(torch.linalg.vector_norm(z)), float(torch.linalg.vector_norm(b / d))


def test_c3_full_parity(selfcomm, oracle_mod):
    from mxsolve.core import DMat, rhs_hash
    n = 256
    A = DMat.stencil(selfcomm, "poisson3d", n)
    info = A.info()
    assert info["nnz_d"] == 7 * n ** 3 - 6 * n ** 2 and info["dia_slices"] == n ** 3 // 64
    M = info["M"]
    b = selfcomm.empty(M)
    rhs_hash(selfcomm, 0, b)
    x = selfcomm.zeros(M)
    r = A.solve(b, x, ksp="cg")
    ip, c, v = oracle_mod.stencil("poisson3d", n)
    O = oracle_mod.OracleMat.from_csr(M, M, ip, c, v)
    del ip, c, v
    o = O.solve(b.cpu().numpy(), ksp="cg", nthreads=min(16, os.cpu_count() or 1))
    assert (r["its"], r["reason"]) == (o["its"], o["reason"]) == (560, 2)
    xr = x.cpu().numpy()
    assert np.linalg.norm(xr - o["x"]) / np.linalg.norm(o["x"]) <= 1e-10


@pytest.mark.parametrize("kind,dims,ksp", [("poisson2d", (4096, 4096, 1), "cg"),
                                          ("convdiff3d", (256, 256, 256), "gmres"),
                                          ("poisson3d27", (512, 512, 64), "cg")])
def test_full_size_properties(selfcomm, kind, dims, ksp):
    from mxsolve.core import DMat, rhs_hash
    nx, ny, nz = dims
    A = DMat.stencil(selfcomm, kind, nx, ny, nz)
    info = A.info()
    M = info["M"]
    nnz = {"poisson2d": 5 * nx * nx - 4 * nx,
           "convdiff3d": 7 * nx ** 3 - 6 * nx ** 2,
           "poisson3d27": (3 * nx - 2) * (3 * ny - 2) * (3 * nz - 2)}[kind]
    assert info["nnz_d"] == nnz
    b = selfcomm.empty(M)
    rhs_hash(selfcomm, 0, b)
    x = selfcomm.zeros(M)
    r = A.solve(b, x, ksp=ksp)
    assert r["reason"] == 2, r                       # CONVERGED_RTOL within max_it
    zr, zb = true_prec_residual(A, b, x)
    # recurrence norm vs recomputed true preconditioned residual: both at the
    # rtol level (CG: ||z||, GMRES: |g_{k+1}| estimate)
    assert zr <= 1.5e-5 * zb, (zr, zb)
    assert abs(zr - r["rnorm"]) <= 0.05 * zr + 1e-12 * zb
    del A
    torch.cuda.empty_cache()
