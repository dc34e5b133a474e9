#!/usr/bin/env python3
"""In-solve time of the streamed-values MatMult (bench.py's spmv_general leg:
variable-coefficient 7-point n^3 through createAIJ(csr=...)) against the
placement of the KSP work vectors: one operator, a profiled 100-iteration CG
per work-vector skew (knob 11, doubles between consecutive vectors), the
skews interleaved over two rounds.
    python tools/general_place.py [n] [skew ...]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-petsc4py-example_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402
from mxsolve import _lib  # noqa: E402
from mxsolve.core import DeviceComm, DMat, rhs_hash  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
skews = [int(v) for v in sys.argv[2:]] or [0, 2, 64, 256, 512, 2048, 8192, 65536]
L = _lib.load()
comm = DeviceComm.self_comm(0)
N, ip, cj, vv = bench.varcoef_csr(n)
A = DMat.from_csr(comm, N, N, ip, cj, vv)
del ip, cj, vv
m = A.info()["m"]
b = comm.empty(m); rhs_hash(comm, 0, b); x = comm.zeros(m)
A.solve(b, x, ksp="cg", pc="jacobi", rtol=0.0, max_it=20)
for rnd in range(2):
    for sk in skews:
        old = L.mx_debug_set(11, sk)
        x.zero_()
        r = A.solve(b, x, ksp="cg", pc="jacobi", rtol=0.0, max_it=100, profile=1)
        L.mx_debug_set(11, old)
        print(f"round {rnd} skew {sk:6d}: in-solve MatMult {r['spmv_ms'] / max(r['spmv_count'], 1) * 1e3:7.1f} us", flush=True)
