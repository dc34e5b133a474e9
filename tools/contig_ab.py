#!/usr/bin/env python3
"""Two operators in one process, one in physically contiguous allocations
(knob 18), one in plain hipMalloc: interleaved CG timing at 256^3.
    python tools/contig_ab.py [first: contig|plain] [rounds]"""
import json, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-petsc4py-example_amd"))
import numpy as np, torch  # noqa: E401,E402
from mxsolve import _lib  # noqa: E402
from mxsolve.core import DeviceComm, DMat, rhs_hash  # noqa: E402

L = _lib.load()
first = sys.argv[1] if len(sys.argv) > 1 else "contig"
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 4
comm = DeviceComm.self_comm(0)
order = ["contig", "plain"] if first == "contig" else ["plain", "contig"]
ops = {}
for kind in order:
    L.mx_debug_set(18, 1 if kind == "contig" else 0)
    A = DMat.stencil(comm, "poisson3d", 256)
    m = A.info()["m"]
    b = comm.empty(m); rhs_hash(comm, 0, b); x = comm.zeros(m)
    A.solve(b, x, ksp="cg", rtol=0.0, max_it=20)      # KSP work space allocated now
    ops[kind] = (A, b, x)
L.mx_debug_set(18, 0)
res = {k: [] for k in ops}
for rnd in range(rounds):
    for k in (order if rnd % 2 == 0 else order[::-1]):
        A, b, x = ops[k]
        A.solve(b, x, ksp="cg", rtol=0.0, max_it=32)
        torch.cuda.synchronize(); t0 = time.perf_counter()
        A.solve(b, x, ksp="cg", rtol=0.0, max_it=300)
        torch.cuda.synchronize(); res[k].append(round((time.perf_counter() - t0) / 300 * 1e6, 1))
print(json.dumps({"first": first, **res}), flush=True)
