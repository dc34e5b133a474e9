#!/usr/bin/env python3
"""Per-solve cost of short CG solves (max_it = K, rtol = 0) under values of
one knob, interleaved in one process: median wall and device ms per solve.
    python tools/start_ab.py KEY v1,v2,... [K] [n] [reps]"""
import json, os, statistics, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-petsc4py-example_amd"))
import torch  # noqa: E402
from mxsolve import _lib  # noqa: E402
from mxsolve.core import DeviceComm, DMat, rhs_hash  # noqa: E402

key = int(sys.argv[1])
vals = [int(v) for v in sys.argv[2].split(",")]
K = int(sys.argv[3]) if len(sys.argv) > 3 else 20
n = int(sys.argv[4]) if len(sys.argv) > 4 else 256
reps = int(sys.argv[5]) if len(sys.argv) > 5 else 15
L = _lib.load()
comm = DeviceComm.self_comm(0)
A = DMat.stencil(comm, "poisson3d", n)
m = A.info()["m"]
b = comm.empty(m); rhs_hash(comm, 0, b); x = comm.zeros(m)
old = L.mx_debug_set(key, vals[0])
res = {v: ([], []) for v in vals}
for rep in range(reps):
    for v in (vals if rep % 2 == 0 else vals[::-1]):
        L.mx_debug_set(key, v)
        A.solve(b, x, ksp="cg", rtol=0.0, max_it=K)          # settle (graph key may change)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = A.solve(b, x, ksp="cg", rtol=0.0, max_it=K)
        torch.cuda.synchronize()
        res[v][0].append((time.perf_counter() - t0) * 1e3)
        res[v][1].append(r["solve_ms"])
L.mx_debug_set(key, old)
print(json.dumps({"key": key, "K": K, "n": n, **{str(v): {"wall_ms": round(statistics.median(w), 4),
                                                          "device_ms": round(statistics.median(d), 4)}
                                                 for v, (w, d) in res.items()}}))
