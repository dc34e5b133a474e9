#!/usr/bin/env python3
"""Standalone streaming rates of the vector-pass shapes on 16.8M doubles
(HIP events, back to back): torch copy (1R1W), the library's VecAXPY
(2R1W), VecPointwiseMult (2R1W) and torch's a*x+y into a third vector (2R1W).
    python tools/stream_ab.py"""
import json, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-petsc4py-example_amd"))
import torch  # noqa: E402
from mxsolve.core import DeviceComm, device_vector, vaxpy, vpmult  # noqa: E402

comm = DeviceComm.self_comm(0)
m = 1 << 24
a, b, c = (device_vector(m, 0).fill_(1.0) for _ in range(3))


def t(fn, reps=30):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


out = {}
us = t(lambda: b.copy_(a)); out["copy_1R1W"] = {"us": round(us, 1), "TBps": round(16 * m / us / 1e6, 2)}
us = t(lambda: vaxpy(comm, 0.5, a, b)); out["axpy_2R1W"] = {"us": round(us, 1), "TBps": round(24 * m / us / 1e6, 2)}
us = t(lambda: vpmult(comm, a, b, c)); out["pmult_2R1W"] = {"us": round(us, 1), "TBps": round(24 * m / us / 1e6, 2)}
us = t(lambda: torch.add(a, b, alpha=0.5, out=c)); out["torch_add_2R1W"] = {"us": round(us, 1), "TBps": round(24 * m / us / 1e6, 2)}
us = t(lambda: a.sum()); out["torch_sum_1R"] = {"us": round(us, 1), "TBps": round(8 * m / us / 1e6, 2)}
print(json.dumps(out), flush=True)
