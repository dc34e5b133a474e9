"""hipGraph replay of the CG iteration batch, and RCCL collectives inside the
captured graph (one-rank RCCL communicator forced onto the collective path:
unfused partial folds + ncclAllReduce), against eager launches."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def solve(comm, graph, n=24, max_it=10000, kind="poisson3d"):
    from mxsolve import _lib
    from mxsolve.core import DMat, rhs_hash
    L = _lib.load()
    old = L.mx_debug_set(7, graph)
    try:
        A = DMat.stencil(comm, kind, n)
        m = A.info()["m"]
        b = comm.empty(m)
        rhs_hash(comm, 0, b)
        x = comm.zeros(m)
        r = A.solve(b, x, ksp="cg", max_it=max_it, history=True)
        r2 = A.solve(b, x, ksp="cg", max_it=max_it)        # replays the cached graph
        assert (r2["its"], r2["reason"]) == (r["its"], r["reason"])
        out = (r, x.cpu().numpy())
        A.destroy()
        return out
    finally:
        L.mx_debug_set(7, old)


@pytest.mark.parametrize("max_it", [10000, 7, 16, 33])
def test_graph_equals_eager(selfcomm, max_it):
    (re, xe), (rg, xg) = solve(selfcomm, 0, max_it=max_it), solve(selfcomm, 1, max_it=max_it)
    assert (re["its"], re["reason"]) == (rg["its"], rg["reason"])
    assert np.array_equal(xe, xg) and np.array_equal(re["history"], rg["history"])


def test_rccl_collectives_in_graph(selfcomm):
    from mxsolve import _lib
    from mxsolve.core import DeviceComm, unique_id
    L = _lib.load()
    ref, xref = solve(selfcomm, 0)
    rc = DeviceComm.rccl(0, 1, unique_id(), device=0)
    old = L.mx_debug_set(8, 1)
    try:
        for g in (0, 1):
            r, x = solve(rc, g)
            assert (r["its"], r["reason"]) == (ref["its"], ref["reason"])
            assert np.array_equal(x, xref)
    finally:
        L.mx_debug_set(8, old)
        selfcomm.activate()
        rc.destroy()
