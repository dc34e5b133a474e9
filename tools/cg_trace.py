#!/usr/bin/env python3
"""CG on one stencil operator under each knob setting given, for a rocprofv3
kernel trace (variants are told apart by their kernels' template arguments,
or run one after another).
    python tools/cg_trace.py KIND NX,NY,NZ ITS [knob=value+... ...]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-petsc4py-example_amd"))
import torch  # noqa: E402

from mxsolve import _lib  # noqa: E402
from mxsolve.core import DeviceComm, DMat, rhs_hash  # noqa: E402

L = _lib.load()
kind, dims, its = sys.argv[1], [int(t) for t in sys.argv[2].split(",")], int(sys.argv[3])
comm = DeviceComm.self_comm(0)
A = DMat.stencil(comm, kind, *dims)
m = A.info()["m"]
b = comm.empty(m)
rhs_hash(comm, 0, b)
x = comm.zeros(m)
for v in (sys.argv[4:] or [""]):
    old = [(int(k), L.mx_debug_set(int(k), int(val))) for k, val in (kv.split("=") for kv in v.split("+") if kv)]
    A.solve(b, x, ksp="cg", rtol=0.0, max_it=its)
    torch.cuda.synchronize()
    for k, o in old:
        L.mx_debug_set(k, o)
print("done", flush=True)
