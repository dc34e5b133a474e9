#!/usr/bin/env python3
"""Per-solve fixed cost vs per-iteration cost of the CG path: wall and device
(HIP-event) time of solves with max_it = K (rtol = 0) for several K; a line
through them gives the per-solve overhead (intercept) and the iteration time.
    python tools/solve_overhead.py [n]"""
import json, os, statistics, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-petsc4py-example_amd"))
import numpy as np, torch  # noqa: E401,E402
from mxsolve.core import DeviceComm, DMat, rhs_hash  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
comm = DeviceComm.self_comm(0)
A = DMat.stencil(comm, "poisson3d", n)
m = A.info()["m"]
b = comm.empty(m); rhs_hash(comm, 0, b); x = comm.zeros(m)
A.solve(b, x, ksp="cg", rtol=0.0, max_it=40)
Ks = [1, 4, 16, 17, 20, 32, 48, 100]
rows = []
for K in Ks:
    wall, dev = [], []
    for _ in range(5):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = A.solve(b, x, ksp="cg", rtol=0.0, max_it=K)
        torch.cuda.synchronize()
        wall.append((time.perf_counter() - t0) * 1e3)
        dev.append(r["solve_ms"])
    rows.append((K, statistics.median(wall), statistics.median(dev)))
    print(json.dumps({"K": K, "wall_ms": round(rows[-1][1], 4), "device_ms": round(rows[-1][2], 4)}), flush=True)
k = np.array([r[0] for r in rows], float)
for j, name in ((1, "wall"), (2, "device")):
    yv = np.array([r[j] for r in rows])
    s, c = np.polyfit(k, yv, 1)
    print(json.dumps({"fit": name, "per_iteration_ms": round(s, 5), "per_solve_ms": round(c, 4)}), flush=True)
