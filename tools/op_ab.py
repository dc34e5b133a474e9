#!/usr/bin/env python3
"""Operators assembled under different knob settings (e.g. format choices read
at assembly), side by side in one process: interleaved CG and standalone
MatMult timing, products checked bitwise equal.
    python tools/op_ab.py kind n rounds "19=1" "19=0" ...   (n: an edge, or NXxNYxNZ)"""
import json, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-petsc4py-example_amd"))
import numpy as np, torch  # noqa: E401,E402
from mxsolve import _lib  # noqa: E402
from mxsolve.core import DeviceComm, DMat, rhs_hash  # noqa: E402

L = _lib.load()
kind, n, rounds = sys.argv[1], sys.argv[2], int(sys.argv[3])
dims = [int(t) for t in n.split("x")]
variants = sys.argv[4:]
comm = DeviceComm.self_comm(0)


def setv(v):
    old = []
    for kv in v.split("+"):
        k, val = kv.split("=")
        old.append(f"{k}={L.mx_debug_set(int(k), int(val))}")
    return "+".join(old)


ops = {}
for v in variants:
    old = setv(v)
    A = DMat.stencil(comm, kind, *dims)
    m = A.info()["m"]
    b = comm.empty(m); rhs_hash(comm, 0, b); x = comm.zeros(m); y = comm.empty(m)
    A.solve(b, x, ksp="cg", rtol=0.0, max_it=20)
    A.mult(b, y)
    ops[v] = (A, b, x, y)
    setv(old)
ys = [o[3] for o in ops.values()]
assert all(torch.equal(ys[0].view(torch.int64), t.view(torch.int64)) for t in ys[1:])
res = {v: {"cg": [], "mult": []} for v in variants}
for rnd in range(rounds):
    for v in (variants if rnd % 2 == 0 else variants[::-1]):
        A, b, x, y = ops[v]
        old = setv(v)          # run-time knobs apply to the measurement as well
        A.solve(b, x, ksp="cg", rtol=0.0, max_it=32)
        torch.cuda.synchronize(); t0 = time.perf_counter()
        A.solve(b, x, ksp="cg", rtol=0.0, max_it=300)
        torch.cuda.synchronize(); res[v]["cg"].append((time.perf_counter() - t0) / 300 * 1e6)
        res[v]["mult"].append(A.bench_mult(b, y, 30)[0] * 1e3)
        setv(old)
print(json.dumps({"kind": kind, "n": n, **{v: {"cg_us": round(float(np.median(r["cg"])), 1),
                                              "mult_us": round(float(np.median(r["mult"])), 1)}
                                           for v, r in res.items()}}), flush=True)
