#!/usr/bin/env python3
"""Sequential CG solves of one operator under several knob variants (a kernel
trace source: run it under rocprofv3 --kernel-trace and split the launches by
kernel name and grid).  Variant = knob=value pairs joined by '+'.

    python tools/knob_runs.py kind nx,ny,nz its variant ...
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-petsc4py-example_amd"))
import torch  # noqa: E402

from mxsolve import _lib  # noqa: E402
from mxsolve.core import DeviceComm, DMat, rhs_hash  # noqa: E402

L = _lib.load()
kind, dims, its = sys.argv[1], [int(t) for t in sys.argv[2].split(",")], int(sys.argv[3])
comm = DeviceComm.self_comm(0)
A = DMat.stencil(comm, kind, *dims)
m = A.info()["m"]
b = comm.empty(m)
rhs_hash(comm, 0, b)
x = comm.zeros(m)
for var in sys.argv[4:]:
    old = [(int(k), L.mx_debug_set(int(k), int(v))) for k, v in (kv.split("=") for kv in var.split("+"))]
    A.solve(b, x, ksp="cg", rtol=0.0, max_it=20)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = A.solve(b, x, ksp="cg", rtol=0.0, max_it=its)
    torch.cuda.synchronize()
    print(json.dumps({"variant": var, "us_per_it": round((time.perf_counter() - t0) / its * 1e6, 1),
                      "cg_mode": r["cg_mode"]}), flush=True)
    for k, v in old:
        L.mx_debug_set(k, v)
A.destroy()
comm.destroy()
