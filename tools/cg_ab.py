#!/usr/bin/env python3
"""Interleaved A/B of CG variants on one operator: every round runs every
variant once (300 iterations, rtol = 0), so slow phases of the device hit all
variants alike.  Variant = comma-free list of knob=value pairs joined by '+'
(mx_debug_set keys), e.g. "9=0" "9=2" "9=1+3=2048".

    python tools/cg_ab.py [kind] [nx,ny,nz] [rounds] variant ...
"""
import json, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-petsc4py-example_amd"))
import numpy as np, torch  # noqa: E401,E402
from mxsolve import _lib  # noqa: E402
from mxsolve.core import DeviceComm, DMat, rhs_hash  # noqa: E402

L = _lib.load()
kind = sys.argv[1] if len(sys.argv) > 1 else "poisson3d"
dims = [int(t) for t in (sys.argv[2] if len(sys.argv) > 2 else "256,256,256").split(",")]
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 5
variants = sys.argv[4:] or ["9=0", "9=2"]
comm = DeviceComm.self_comm(0)
A = DMat.stencil(comm, kind, *dims)
m = A.info()["m"]
b = comm.empty(m); rhs_hash(comm, 0, b); x = comm.zeros(m)


def setv(v):
    old = []
    for kv in v.split("+"):
        k, val = kv.split("=")
        old.append(f"{k}={L.mx_debug_set(int(k), int(val))}")
    return "+".join(old)


res = {v: [] for v in variants}
for rnd in range(rounds):
    for v in (variants if rnd % 2 == 0 else variants[::-1]):
        old = setv(v)
        A.solve(b, x, ksp="cg", rtol=0.0, max_it=32)
        torch.cuda.synchronize(); t0 = time.perf_counter()
        A.solve(b, x, ksp="cg", rtol=0.0, max_it=300)
        torch.cuda.synchronize(); res[v].append((time.perf_counter() - t0) / 300 * 1e6)
        setv(old)
print(json.dumps({"kind": kind, "dims": dims, **{v: {"med_us": round(float(np.median(t)), 1),
                                                   "min_us": round(float(np.min(t)), 1)}
                                                for v, t in res.items()}}), flush=True)
