#!/usr/bin/env python3
"""MatMult only (for per-kernel PMC passes): one operator, `iters` back-to-back
products.   python tools/spmv_only.py [kind] [n | nxXnyXnz] [iters] [knob=value+...]"""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-petsc4py-example_amd"))
import torch  # noqa: E402
from mxsolve import _lib  # noqa: E402
from mxsolve.core import DeviceComm, DMat, rhs_hash  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "poisson3d"
dims = [int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "256").split("x")]
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 20
L = _lib.load()
if len(sys.argv) > 4:
    for kv in sys.argv[4].split("+"):
        k, v = kv.split("=")
        L.mx_debug_set(int(k), int(v))
comm = DeviceComm.self_comm(0)
A = DMat.stencil(comm, kind, *dims)
m = A.info()["m"]
x = comm.empty(m); rhs_hash(comm, 0, x); y = comm.empty(m)
s, mm = A.bench_mult(x, y, iters)
torch.cuda.synchronize()
print(f"spmv {s * 1e3:.1f} us  matmult {mm * 1e3:.1f} us  codes {A.info()['value_codes']}", flush=True)
