#!/usr/bin/env python3
"""Interleaved A/B of eager vs hipGraph-replayed CG iterations (256^3, N=1)."""
import json, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-petsc4py-example_amd"))
import numpy as np, torch  # noqa: E401,E402
from mxsolve import _lib  # noqa: E402
from mxsolve.core import DeviceComm, DMat, rhs_hash  # noqa: E402
L = _lib.load()
comm = DeviceComm.self_comm(0)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
A = DMat.stencil(comm, "poisson3d", n)
m = A.info()["m"]
b = comm.empty(m); rhs_hash(comm, 0, b); x = comm.zeros(m)
res = {0: [], 1: []}
for rnd in range(4):
    for g in (0, 1):
        L.mx_debug_set(7, g)
        A.solve(b, x, ksp="cg", rtol=0.0, max_it=32)
        torch.cuda.synchronize(); t0 = time.perf_counter()
        A.solve(b, x, ksp="cg", rtol=0.0, max_it=200)
        torch.cuda.synchronize(); res[g].append((time.perf_counter() - t0) / 200 * 1e3)
L.mx_debug_set(7, 0)
print(json.dumps({"n": n, "eager_ms_per_it": round(float(np.median(res[0])), 4), "graph_ms_per_it": round(float(np.median(res[1])), 4)}))
