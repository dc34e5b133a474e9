#!/usr/bin/env python3
"""Interleaved knob A/B on bench.py's streamed-values leg (variable-coefficient
7-point n^3 through createAIJ(csr=...), CG + Jacobi, mode 2): one operator, a
profiled 100-iteration CG per setting per round, printing the in-solve MatMult
time and the iteration time.
    python tools/general_knob_ab.py N ROUNDS knob=value[+...] ..."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-petsc4py-example_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402
from mxsolve import _lib  # noqa: E402
from mxsolve.core import DeviceComm, DMat, rhs_hash  # noqa: E402

n, rounds = int(sys.argv[1]), int(sys.argv[2])
settings = sys.argv[3:] or [""]
L = _lib.load()
comm = DeviceComm.self_comm(0)
N, ip, cj, vv = bench.varcoef_csr(n)
A = DMat.from_csr(comm, N, N, ip, cj, vv)
del ip, cj, vv
m = A.info()["m"]
b = comm.empty(m); rhs_hash(comm, 0, b); x = comm.zeros(m)
A.solve(b, x, ksp="cg", pc="jacobi", rtol=0.0, max_it=20)
for rnd in range(rounds):
    for v in settings:
        old = [(int(k), L.mx_debug_set(int(k), int(val))) for k, val in (kv.split("=") for kv in v.split("+") if kv)]
        x.zero_()
        r = A.solve(b, x, ksp="cg", pc="jacobi", rtol=0.0, max_it=100, profile=1)
        x.zero_()
        torch.cuda.synchronize(); t0 = time.perf_counter()
        A.solve(b, x, ksp="cg", pc="jacobi", rtol=0.0, max_it=200)
        torch.cuda.synchronize(); dt = (time.perf_counter() - t0) / 200
        for k, o in old:
            L.mx_debug_set(k, o)
        print(f"round {rnd} {v or 'default':12s} MatMult {r['spmv_ms'] / max(r['spmv_count'], 1) * 1e3:7.1f} us"
              f"  iteration {dt * 1e6:7.1f} us  mode {r['cg_mode']}", flush=True)
