#!/usr/bin/env python3
"""P in-process ranks (LocalComm) on one GPU running CG on 256^3: a kernel
trace source for the per-rank launches of the N > 1 iteration (halo pack,
split MatMult, boundary launch, folds).  Host-ordered transport: read kernel
durations from rocprofv3, not wall time.

    python tools/local_trace.py [P] [its] [knob=value+...]
"""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-petsc4py-example_amd"))
import torch  # noqa: E402
from mxsolve import _lib  # noqa: E402
from mxsolve.core import LocalWorld, DMat, rhs_hash  # noqa: E402

P = int(sys.argv[1]) if len(sys.argv) > 1 else 8
its = int(sys.argv[2]) if len(sys.argv) > 2 else 40
L = _lib.load()
if len(sys.argv) > 3:
    for kv in sys.argv[3].split("+"):
        k, v = kv.split("=")
        L.mx_debug_set(int(k), int(v))
w = LocalWorld(P)


def body(comm):
    A = DMat.stencil(comm, "poisson3d", 256)
    info = A.info()
    b = comm.empty(info["m"])
    rhs_hash(comm, info["rstart"], b)
    x = comm.zeros(info["m"])
    r = A.solve(b, x, ksp="cg", rtol=0.0, max_it=its)
    A.destroy()
    return r["its"]


print(w.run(body), flush=True)
w.destroy()
