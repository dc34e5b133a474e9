#!/usr/bin/env python3
"""Interleaved A/B of the CG iteration with and without the fused MatMult
(knob 9) over SpMV grid sizes (knob 3): ms per iteration and the
HIP-event mean of the MatMult launches.  python tools/cgfuse_ab.py [n] [kind]"""
import json, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-petsc4py-example_amd"))
import numpy as np, torch  # noqa: E401,E402
from mxsolve import _lib  # noqa: E402
from mxsolve.core import DeviceComm, DMat, rhs_hash  # noqa: E402
L = _lib.load()
comm = DeviceComm.self_comm(0)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
kind = sys.argv[2] if len(sys.argv) > 2 else "poisson3d"
A = DMat.stencil(comm, kind, n)
m = A.info()["m"]
b = comm.empty(m); rhs_hash(comm, 0, b); x = comm.zeros(m)
# variant = fusion(knob 9):grid(knob 3)
variants = [tuple(int(t) for t in v.split(":")[:2])
            for v in (sys.argv[3] if len(sys.argv) > 3 else "0:8192,1:8192,2:8192,3:8192").split(",")]
res = {v: [] for v in variants}
spmv = {v: [] for v in variants}
for rnd in range(4):
    for v in variants:
        L.mx_debug_set(9, v[0]); L.mx_debug_set(3, v[1])
        A.solve(b, x, ksp="cg", rtol=0.0, max_it=32)
        torch.cuda.synchronize(); t0 = time.perf_counter()
        A.solve(b, x, ksp="cg", rtol=0.0, max_it=200)
        torch.cuda.synchronize(); res[v].append((time.perf_counter() - t0) / 200 * 1e3)
        r = A.solve(b, x, ksp="cg", rtol=0.0, max_it=50, profile=True)
        spmv[v].append(r["spmv_ms"] / max(r["spmv_count"], 1))
L.mx_debug_set(9, 3); L.mx_debug_set(3, 8192)
print(json.dumps({"n": n, "kind": kind, **{f"fuse{v[0]}_grid{v[1]}": {"ms_it": round(float(np.median(res[v])), 4),
                                                      "matmult_ms": round(float(np.median(spmv[v])), 4)}
                                   for v in variants}}))
