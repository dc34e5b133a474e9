"""Failure detection on the RCCL path: host waits on an RCCL
communicator's work poll ncclCommGetAsyncError (an error aborts at once) and
run under deadlines: the KSP poller's wait fails after knob 33 ms WITHOUT
progress (re-armed whenever the device's iteration count moves), the other
waits only past knob 47 ms when it is set (default: none, as with MPI).
Exercised on a one-rank RCCL communicator with bounded device stalls (RCCL
refuses two ranks on one GPU; a real peer failure needs the 8-GPU node)."""
import ctypes as C

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_rccl_wait_deadline_aborts_communicator():
    from mxsolve import _lib
    from mxsolve.core import DMat, DeviceComm, rhs_hash, unique_id
    L = _lib.load()
    rc = DeviceComm.rccl(0, 1, unique_id(), device=0)
    try:
        # the default deadline (600 s) does not trip a 0.3 s wait that observes no progress
        _lib.call("mx_debug_comm_stall", rc.h, 300_000)
        old = L.mx_debug_set(47, 50)              # 50 ms deadline
        try:
            with pytest.raises(_lib.MxError) as ei:
                _lib.call("mx_debug_comm_stall", rc.h, 400_000)   # 0.4 s of device time
            assert ei.value.code == _lib.MX_ERR_COMM and "aborted" in ei.value.msg
        finally:
            L.mx_debug_set(47, old)
        torch.cuda.synchronize()                 # the bounded stall has drained
        # the aborted communicator refuses further collectives
        old8 = L.mx_debug_set(8, 1)              # force the collective path on one rank
        mats = []
        try:
            with pytest.raises(_lib.MxError) as ej:
                mats.append(DMat.stencil(rc, "poisson3d", 8))
                m = mats[0].info()["m"]
                b, x = rc.empty(m), rc.zeros(m)
                rhs_hash(rc, 0, b)
                mats[0].solve(b, x, ksp="cg", pc="jacobi")
            assert ej.value.code == _lib.MX_ERR_COMM
        finally:
            L.mx_debug_set(8, old8)
            for A in mats:                        # before the communicator goes
                A.destroy()
    finally:
        torch.cuda.synchronize()
        rc.destroy()
    # a fresh communicator works again
    rc2 = DeviceComm.rccl(0, 1, unique_id(), device=0)
    _lib.call("mx_debug_comm_stall", rc2.h, 1000)
    rc2.destroy()


def test_rccl_poller_deadline_rearms_on_progress():
    """A poller wait far longer than the no-progress deadline (knob 33 = 40 ms)
    completes: with batches of 2000 iterations the poller waits on a whole
    batch (~70 ms at 128^3), and the deadline re-arms each time the device's
    count of iterations begun moves -- a rank waiting on a slow but live peer
    is not failed."""
    import time
    from mxsolve import _lib
    from mxsolve.core import DMat, DeviceComm, rhs_hash, unique_id
    L = _lib.load()
    rc = DeviceComm.rccl(0, 1, unique_id(), device=0)
    old = {k: L.mx_debug_set(k, v) for k, v in ((8, 1), (7, 0), (33, 40))}   # collective path, eager
    A = None
    try:
        A = DMat.stencil(rc, "poisson3d", 128)
        m = A.info()["m"]
        b, x = rc.empty(m), rc.zeros(m)
        rhs_hash(rc, 0, b)
        t0 = time.perf_counter()
        r = A.solve(b, x, ksp="cg", pc="jacobi", rtol=0.0, atol=0.0, max_it=4000, poll_every=2000)
        dt = time.perf_counter() - t0
        assert r["its"] == 4000 and dt > 0.1, (r, dt)
    finally:
        for k, v in old.items():
            L.mx_debug_set(k, v)
        if A is not None:
            A.destroy()
        torch.cuda.synchronize()
        rc.destroy()


def test_rccl_gmres_readback_deadline():
    """GMRES(30)'s restart read-back waits under the no-progress deadline
    (knob 33): with a 0.4 s device stall before the read-back (knob 61) and a
    50 ms deadline the solve fails with MX_ERR_COMM and the communicator is
    aborted; without the stall the same solve completes (the step kernels keep
    the progress word moving)."""
    from mxsolve import _lib
    from mxsolve.core import DMat, DeviceComm, rhs_hash, unique_id
    L = _lib.load()
    rc = DeviceComm.rccl(0, 1, unique_id(), device=0)
    old = {k: L.mx_debug_set(k, v) for k, v in ((8, 1), (33, 50))}   # collective path, 50 ms
    mats = []
    try:
        A = DMat.stencil(rc, "convdiff3d", 32)
        mats.append(A)
        m = A.info()["m"]
        b, x = rc.empty(m), rc.zeros(m)
        rhs_hash(rc, 0, b)
        r = A.solve(b, x, ksp="gmres", pc="jacobi", rtol=1e-8)
        assert r["reason"] > 0, r
        old61 = L.mx_debug_set(61, 400_000)
        try:
            x.zero_()
            with pytest.raises(_lib.MxError) as ei:
                A.solve(b, x, ksp="gmres", pc="jacobi", rtol=1e-8)
            assert ei.value.code == _lib.MX_ERR_COMM and "no progress" in ei.value.msg, ei.value.msg
        finally:
            L.mx_debug_set(61, old61)
    finally:
        for k, v in old.items():
            L.mx_debug_set(k, v)
        torch.cuda.synchronize()                 # the bounded stall has drained
        for A in mats:
            A.destroy()
        rc.destroy()
