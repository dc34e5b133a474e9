"""Failure detection on the RCCL path: host waits on an RCCL
communicator's work poll ncclCommGetAsyncError under a deadline (knob 33) and
abort the communicator with MX_ERR_COMM instead of hanging.  Exercised on a
one-rank RCCL communicator with a bounded device stall longer than the
deadline (RCCL refuses two ranks on one GPU; a real peer failure needs the
8-GPU node)."""
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
        # a short stall inside the default deadline passes
        _lib.call("mx_debug_comm_stall", rc.h, 2000)
        old = L.mx_debug_set(33, 50)              # 50 ms deadline
        try:
            with pytest.raises(_lib.MxError) as ei:
                _lib.call("mx_debug_comm_stall", rc.h, 400_000)   # 0.4 s of device time
            assert ei.value.code == _lib.MX_ERR_COMM and "aborted" in ei.value.msg
        finally:
            L.mx_debug_set(33, old)
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
