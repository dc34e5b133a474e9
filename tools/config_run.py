#!/usr/bin/env python3
"""One BASELINE configuration's solve with the library's defaults, for
rocprofv3 passes: KIND NX NY NZ KSP ITS (rtol 0: exactly ITS iterations,
after a 10-iteration warm-up solve).
    python tools/config_run.py poisson3d27 512 512 64 cg 50"""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-petsc4py-example_amd"))
import torch  # noqa: E402
from mxsolve.core import DeviceComm, DMat, rhs_hash  # noqa: E402

kind, nx, ny, nz, ksp, its = sys.argv[1], *map(int, sys.argv[2:5]), sys.argv[5], int(sys.argv[6])
comm = DeviceComm.self_comm(0)
A = DMat.stencil(comm, kind, nx, ny, nz)
m = A.info()["m"]
b = comm.empty(m); rhs_hash(comm, 0, b); x = comm.zeros(m)
A.solve(b, x, ksp=ksp, pc="jacobi", rtol=0.0, max_it=10)
x.zero_()
r = A.solve(b, x, ksp=ksp, pc="jacobi", rtol=0.0, max_it=its)
torch.cuda.synchronize()
print("done", r["its"], r.get("cg_mode"), flush=True)
