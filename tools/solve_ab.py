#!/usr/bin/env python3
"""Interleaved A/B of whole CG solves of K iterations (rtol = 0) on one
operator -- the per-solve fixed costs that the 300-iteration tools/cg_ab.py
averages away: wall time between syncs, as bench.py's timed region.
    python tools/solve_ab.py [kind] [nx,ny,nz] [K] [rounds] variant ...   (variant: knob=value+...)"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-petsc4py-example_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mxsolve import _lib  # noqa: E402
from mxsolve.core import DeviceComm, DMat, rhs_hash  # noqa: E402

L = _lib.load()
kind = sys.argv[1] if len(sys.argv) > 1 else "poisson3d"
dims = [int(t) for t in (sys.argv[2] if len(sys.argv) > 2 else "256,256,256").split(",")]
K = int(sys.argv[3]) if len(sys.argv) > 3 else 20
rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 20
variants = sys.argv[5:] or ["67=0", "67=1"]
comm = DeviceComm.self_comm(0)
A = DMat.stencil(comm, kind, *dims)
m = A.info()["m"]
b = comm.empty(m)
rhs_hash(comm, 0, b)
x = comm.zeros(m)


def setv(v):
    return [(int(k), L.mx_debug_set(int(k), int(val))) for k, val in (kv.split("=") for kv in v.split("+") if kv)]


res = {v: [] for v in variants}
for v in variants:                       # warm: graphs, work space
    old = setv(v)
    A.solve(b, x, ksp="cg", rtol=0.0, max_it=K)
    for k, o in old:
        L.mx_debug_set(k, o)
for rnd in range(rounds):
    for v in (variants if rnd % 2 == 0 else variants[::-1]):
        old = setv(v)
        A.solve(b, x, ksp="cg", rtol=0.0, max_it=5)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        A.solve(b, x, ksp="cg", rtol=0.0, max_it=K)
        torch.cuda.synchronize()
        res[v].append((time.perf_counter() - t0) * 1e3)
        for k, o in old:
            L.mx_debug_set(k, o)
print(json.dumps({"kind": kind, "dims": dims, "K": K, **{v: {"med_ms": round(float(np.median(t)), 4),
                                                               "min_ms": round(float(np.min(t)), 4)}
                                                           for v, t in res.items()}}), flush=True)
