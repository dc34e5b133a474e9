#!/usr/bin/env python3
"""Kernel timeline of one K-iteration CG solve (run under rocprofv3
--kernel-trace): prints nothing itself; tools/timeline_report.py reads the
trace.  python tools/solve_timeline.py [K] [n]"""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-petsc4py-example_amd"))
import torch  # noqa: E402
from mxsolve.core import DeviceComm, DMat, rhs_hash  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
n = int(sys.argv[2]) if len(sys.argv) > 2 else 256
comm = DeviceComm.self_comm(0)
A = DMat.stencil(comm, "poisson3d", n)
m = A.info()["m"]
b = comm.empty(m); rhs_hash(comm, 0, b); x = comm.zeros(m)
for _ in range(3):
    A.solve(b, x, ksp="cg", rtol=0.0, max_it=K)
torch.cuda.synchronize()
