#!/usr/bin/env python3
"""CG iteration time at 256^3 vs the placement of the vectors: the skew
between the KSP work vectors (knob 11, doubles) and the offsets of x and b
inside one torch buffer (doubles).  Interleaved rounds, one operator.

    python tools/skew_ab.py [n] [skews] [x offsets]
"""
import json, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-petsc4py-example_amd"))
import numpy as np, torch  # noqa: E401,E402
from mxsolve import _lib  # noqa: E402
from mxsolve.core import DeviceComm, DMat, rhs_hash  # noqa: E402

L = _lib.load()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
skews = [int(t) for t in (sys.argv[2] if len(sys.argv) > 2 else "0,32,512,4128").split(",")]
xoffs = [int(t) for t in (sys.argv[3] if len(sys.argv) > 3 else "0").split(",")]
comm = DeviceComm.self_comm(0)
A = DMat.stencil(comm, "poisson3d", n)
m = A.info()["m"]
buf = comm.empty(2 * m + 2 * max(xoffs) + 64)
res = {}
for rnd in range(3):
    for sk in skews:
        for xo in xoffs:
            x = buf[xo: xo + m]
            b = buf[m + 2 * xo + 32: 2 * m + 2 * xo + 32]
            rhs_hash(comm, 0, b)
            x.zero_()
            old = L.mx_debug_set(11, sk)
            A.solve(b, x, ksp="cg", rtol=0.0, max_it=32)
            torch.cuda.synchronize(); t0 = time.perf_counter()
            A.solve(b, x, ksp="cg", rtol=0.0, max_it=300)
            torch.cuda.synchronize()
            res.setdefault(f"skew{sk}_x{xo}", []).append(round((time.perf_counter() - t0) / 300 * 1e6, 1))
            L.mx_debug_set(11, old)
print(json.dumps({"n": n, **res}), flush=True)
