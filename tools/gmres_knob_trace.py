#!/usr/bin/env python3
"""GMRES(30)+Jacobi on conv-diff n^3 (config C4), one ITS-iteration solve per
knob setting, in order -- a kernel-trace source for interleaved knob A/B of
the GMRES step's kernels (tools/trace_blocks.py splits the launches by
setting).  python tools/gmres_knob_trace.py N ITS [knob=value+... ...]"""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-petsc4py-example_amd"))
import torch  # noqa: E402
from mxsolve import _lib  # noqa: E402
from mxsolve.core import DeviceComm, DMat, rhs_hash  # noqa: E402

L = _lib.load()
n, its = int(sys.argv[1]), int(sys.argv[2])
comm = DeviceComm.self_comm(0)
A = DMat.stencil(comm, "convdiff3d", n)
m = A.info()["m"]
b = comm.empty(m); rhs_hash(comm, 0, b); x = comm.zeros(m)
A.solve(b, x, ksp="gmres", rtol=0.0, max_it=30)
for v in (sys.argv[3:] or [""]):
    old = [(int(k), L.mx_debug_set(int(k), int(val))) for k, val in (kv.split("=") for kv in v.split("+") if kv)]
    x.zero_()
    torch.cuda.synchronize(); t0 = time.perf_counter()
    A.solve(b, x, ksp="gmres", rtol=0.0, max_it=its)
    torch.cuda.synchronize()
    print(v, round((time.perf_counter() - t0) / its * 1e3, 4), "ms/it", flush=True)
    for k, o in old:
        L.mx_debug_set(k, o)
