#!/usr/bin/env python3
"""Interleaved A/B of GMRES(30) variants (knob sets) on conv-diff n^3, one operator.
    python tools/gmres_ab.py [n] [rounds] variant ...   (variant: "77=512+..." knob=value)"""
import json, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-petsc4py-example_amd"))
import numpy as np, torch  # noqa: E401,E402
from mxsolve import _lib  # noqa: E402
from mxsolve.core import DeviceComm, DMat, rhs_hash  # noqa: E402

L = _lib.load()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
variants = sys.argv[3:] or ["", "77=512"]
comm = DeviceComm.self_comm(0)
A = DMat.stencil(comm, "convdiff3d", n)
m = A.info()["m"]
b = comm.empty(m); rhs_hash(comm, 0, b); x = comm.zeros(m)


def setv(v):
    old = []
    for kv in filter(None, v.split("+")):   # "" = the defaults
        k, val = kv.split("=")
        old.append(f"{k}={L.mx_debug_set(int(k), int(val))}")
    return "+".join(old)


res = {v: [] for v in variants}
for rnd in range(rounds):
    for v in (variants if rnd % 2 == 0 else variants[::-1]):
        old = setv(v)
        torch.cuda.synchronize(); t0 = time.perf_counter()
        r = A.solve(b, x, ksp="gmres", rtol=0.0, max_it=60)
        torch.cuda.synchronize(); res[v].append((time.perf_counter() - t0) / 60 * 1e3)
        setv(old)
print(json.dumps({"n": n, **{v: {"med_ms": round(float(np.median(t)), 4), "min_ms": round(float(np.min(t)), 4)}
                             for v, t in res.items()}}), flush=True)
