#!/usr/bin/env python3
"""Does a short CG solve run slower when the GPU was idle before it?  Wall
time of a K-iteration solve (rtol = 0) after: an idle pause, a long solve,
and back-to-back repeats.   python tools/warm_probe.py [K] [n]"""
import json, os, statistics, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-petsc4py-example_amd"))
import torch  # noqa: E402
from mxsolve.core import DeviceComm, DMat, rhs_hash  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
n = int(sys.argv[2]) if len(sys.argv) > 2 else 256
comm = DeviceComm.self_comm(0)
A = DMat.stencil(comm, "poisson3d", n)
m = A.info()["m"]
b = comm.empty(m); rhs_hash(comm, 0, b); x = comm.zeros(m)
A.solve(b, x, ksp="cg", rtol=0.0, max_it=40)


def timed(k):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = A.solve(b, x, ksp="cg", rtol=0.0, max_it=k)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3, r["solve_ms"]


out = {"idle": [], "after_long": [], "back_to_back": [], "long_per_it": []}
for rep in range(8):
    time.sleep(0.05)
    out["idle"].append(timed(K))
    w, d = timed(400)
    out["long_per_it"].append((w / 400, d / 400))
    out["after_long"].append(timed(K))
    for _ in range(4):
        out["back_to_back"].append(timed(K))
print(json.dumps({"K": K, **{k: {"wall_ms": round(statistics.median(v[0] for v in vals), 4),
                                 "device_ms": round(statistics.median(v[1] for v in vals), 4)}
                             for k, vals in out.items()}}))
