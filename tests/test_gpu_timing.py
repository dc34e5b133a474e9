"""The KSP's MatMult timing (bench.py's roofline.achieved): on one rank the
events are attached to the kernel's own dispatch (hipExtLaunchKernel,
mx_launch.hpp); with P > 1 they bracket the whole MatMult.  A profiled solve
runs eagerly and must give the graph-replayed solve's bits."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kind,n", [("poisson3d", 64), ("poisson3d", 20)])
def test_profiled_solve_times_every_matmult(selfcomm, kind, n):
    from mxsolve.core import DMat, rhs_hash
    A = DMat.stencil(selfcomm, kind, n)
    m = A.info()["m"]
    b = selfcomm.empty(m)
    rhs_hash(selfcomm, 0, b)
    x0 = selfcomm.zeros(m)
    r0 = A.solve(b, x0, ksp="cg", rtol=0.0, max_it=40)
    x1 = selfcomm.zeros(m)
    r1 = A.solve(b, x1, ksp="cg", rtol=0.0, max_it=40, profile=True)
    assert r0["its"] == r1["its"] == 40
    assert np.array_equal(x0.cpu().numpy().view(np.uint64), x1.cpu().numpy().view(np.uint64))
    assert r1["spmv_count"] == 40
    per = r1["spmv_ms"] / r1["spmv_count"]
    y = selfcomm.empty(m)
    alone, _ = A.bench_mult(b, y, 20)
    assert 0.0 < per < 20 * alone + 0.05, (per, alone)
    A.destroy()


def test_profiled_solve_multirank():
    from mxsolve.core import DMat, LocalWorld, rhs_hash

    def body(comm):
        A = DMat.stencil(comm, "poisson3d", 24)
        info = A.info()
        b = comm.empty(info["m"])
        rhs_hash(comm, info["rstart"], b)
        x = comm.zeros(info["m"])
        r = A.solve(b, x, ksp="cg", rtol=0.0, max_it=20, profile=True)
        A.destroy()
        return r["spmv_count"], r["spmv_ms"]

    w = LocalWorld(2)
    try:
        res = w.run(body)
    finally:
        w.destroy()
    assert all(c == 20 and ms > 0.0 for c, ms in res), res
