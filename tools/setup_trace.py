#!/usr/bin/env python3
"""The first solve on a fresh operator (PCSetUp + KSPSetUp + the graph) and a
repeat, for a rocprofv3 --kernel-trace --hip-runtime-trace timeline:
    python tools/setup_trace.py [n] [ksp]"""
import os, sys, time
T_START = time.perf_counter()
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-petsc4py-example_amd"))
import torch  # noqa: E402
from mxsolve.core import DeviceComm, DMat, rhs_hash  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
ksp = sys.argv[2] if len(sys.argv) > 2 else "cg"
comm = DeviceComm.self_comm(0)
A0 = DMat.stencil(comm, "poisson3d", 8)
b0 = comm.empty(A0.info()["m"]); rhs_hash(comm, 0, b0); x0 = comm.zeros(A0.info()["m"])
A0.solve(b0, x0, ksp=ksp, pc="jacobi", rtol=0.0, max_it=2)
A0.destroy()
A = DMat.stencil(comm, "poisson3d", n)
m = A.info()["m"]
b = comm.empty(m); rhs_hash(comm, 0, b); x = comm.zeros(m)
torch.cuda.synchronize()
for tag in ("first", "repeat"):
    t0 = time.perf_counter()
    A.solve(b, x, ksp=ksp, pc="jacobi", rtol=0.0, max_it=1)
    torch.cuda.synchronize()
    print(tag, round((time.perf_counter() - t0) * 1e3, 3), "ms", flush=True)
print("process", round(time.perf_counter() - T_START, 3), "s", flush=True)
