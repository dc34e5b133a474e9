#!/usr/bin/env python3
"""C5's per-GPU share (27-point 512x512x64) CG under each knob setting given,
for a rocprofv3 kernel trace (the 27-point z-march's launches are named by
their template arguments, so one trace separates the variants).
    python tools/c5_trace.py [its] [knob=value+... ...]"""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-petsc4py-example_amd"))
import torch  # noqa: E402
from mxsolve import _lib  # noqa: E402
from mxsolve.core import DeviceComm, DMat, rhs_hash  # noqa: E402

L = _lib.load()
its = int(sys.argv[1]) if len(sys.argv) > 1 else 100
comm = DeviceComm.self_comm(0)
A = DMat.stencil(comm, "poisson3d27", 512, 512, 64)
m = A.info()["m"]
b = comm.empty(m); rhs_hash(comm, 0, b); x = comm.zeros(m)
for v in (sys.argv[2:] or [""]):
    old = [(int(k), L.mx_debug_set(int(k), int(val))) for k, val in (kv.split("=") for kv in v.split("+") if kv)]
    A.solve(b, x, ksp="cg", rtol=0.0, max_it=its)
    torch.cuda.synchronize()
    for k, o in old:
        L.mx_debug_set(k, o)
print("done", flush=True)
