#!/usr/bin/env python3
"""Interleaved A/B of run-time knob settings on one operator's standalone
MatMult (bench_mult: device time per launch), products checked bitwise equal.
    python tools/mult_ab.py kind NXxNYxNZ rounds "42=1" "40=6" ..."""
import json, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-petsc4py-example_amd"))
import numpy as np, torch  # noqa: E401,E402
from mxsolve import _lib  # noqa: E402
from mxsolve.core import DeviceComm, DMat, rhs_hash  # noqa: E402

L = _lib.load()
kind, dims, rounds = sys.argv[1], [int(t) for t in sys.argv[2].split("x")], int(sys.argv[3])
variants = ["base"] + sys.argv[4:]
comm = DeviceComm.self_comm(0)
A = DMat.stencil(comm, kind, *dims)
m = A.info()["m"]
x = comm.empty(m); rhs_hash(comm, 0, x)
ref = comm.empty(m); A.mult(x, ref)
y = comm.empty(m)


def setv(v):
    old = []
    for kv in (v.split("+") if v != "base" else []):
        k, val = kv.split("=")
        old.append((int(k), L.mx_debug_set(int(k), int(val))))
    return old


res = {v: [] for v in variants}
for r in range(rounds):
    for v in (variants if r % 2 == 0 else variants[::-1]):
        old = setv(v)
        res[v].append(A.bench_mult(x, y, 30)[0] * 1e3)
        if r == 0:
            assert torch.equal(y.view(torch.int64), ref.view(torch.int64)), v
        for k, o in old:
            L.mx_debug_set(k, o)
print(json.dumps({"kind": kind, "dims": dims, **{v: round(float(np.median(t)), 2) for v, t in res.items()}}), flush=True)
