#!/usr/bin/env python3
"""Diagnostic: test.py's 100x100 system on P in-process ranks, GMRES(restart)
for max_it iterations; prints its / reason / rnorm per rank."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-petsc4py-example_amd"))
import numpy as np, torch  # noqa: E401,E402
from mxsolve.core import DMat, LocalWorld  # noqa: E402

P, restart, max_it = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
g = np.load(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "reference_systems.npz"))
ip, c, v = g["sys_indptr"].astype(np.int64), g["sys_indices"].astype(np.int64), g["sys_data"]
M = 100
rng = [M * r // P for r in range(P + 1)]
rng = [0] + [sum((M // P) + (1 if i < M % P else 0) for i in range(r)) for r in range(1, P + 1)]


def body(comm):
    r = comm.rank
    r0, r1 = rng[r], rng[r + 1]
    lip = ip[r0:r1 + 1] - ip[r0]
    A = DMat.from_csr(comm, M, M, lip.astype(np.int32), c[ip[r0]:ip[r1]].astype(np.int32), v[ip[r0]:ip[r1]])
    b = torch.from_numpy(g["sys_B"][r0:r1].copy()).cuda()
    x = comm.zeros(r1 - r0)
    res = A.solve(b, x, ksp="gmres", restart=restart, max_it=max_it)
    A.destroy()
    return res["its"], res["reason"], res["rnorm"]


w = LocalWorld(P)
try:
    print(P, restart, max_it, w.run(body), flush=True)
finally:
    w.destroy()
