#!/usr/bin/env python3
"""GMRES(30)+Jacobi on conv-diff 256^3 (config C4) for a fixed number of
iterations: a kernel-trace source for the GMRES inner step.
    python tools/gmres_trace.py [n] [its] [knob=value+...]"""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-petsc4py-example_amd"))
import torch  # noqa: E402
from mxsolve import _lib  # noqa: E402
from mxsolve.core import DeviceComm, DMat, rhs_hash  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
its = int(sys.argv[2]) if len(sys.argv) > 2 else 60
for kv in (sys.argv[3].split("+") if len(sys.argv) > 3 else []):
    k, v = kv.split("=")
    _lib.load().mx_debug_set(int(k), int(v))
comm = DeviceComm.self_comm(0)
A = DMat.stencil(comm, "convdiff3d", n)
m = A.info()["m"]
b = comm.empty(m); rhs_hash(comm, 0, b); x = comm.zeros(m)
A.solve(b, x, ksp="gmres", rtol=0.0, max_it=30)
torch.cuda.synchronize(); t0 = time.perf_counter()
r = A.solve(b, x, ksp="gmres", rtol=0.0, max_it=its)
torch.cuda.synchronize()
print({"its": r["its"], "ms_per_it": round((time.perf_counter() - t0) / its * 1e3, 4)}, flush=True)
