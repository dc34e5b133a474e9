#!/usr/bin/env python3
"""Time series of CG iteration time on a fresh process: consecutive 100-iteration
solves at 256^3 (does the device speed up under sustained load?).

    python tools/ramp.py [n] [solves]
"""
import json, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-petsc4py-example_amd"))
import torch  # noqa: E402
from mxsolve.core import DeviceComm, DMat, rhs_hash  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
k = int(sys.argv[2]) if len(sys.argv) > 2 else 40
comm = DeviceComm.self_comm(0)
A = DMat.stencil(comm, "poisson3d", n)
m = A.info()["m"]
b = comm.empty(m); rhs_hash(comm, 0, b); x = comm.zeros(m)
t_start = time.perf_counter()
out = []
for i in range(k):
    torch.cuda.synchronize(); t0 = time.perf_counter()
    A.solve(b, x, ksp="cg", rtol=0.0, max_it=100)
    torch.cuda.synchronize(); t1 = time.perf_counter()
    out.append((round(t1 - t_start, 3), round((t1 - t0) / 100 * 1e6, 1)))
print(json.dumps({"n": n, "t_s_us_per_it": out}), flush=True)
