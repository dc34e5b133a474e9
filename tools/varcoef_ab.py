#!/usr/bin/env python3
"""Interleaved knob A/B on the variable-coefficient 7-point 256^3 leg (fp64
aligned-offset SELL, tools/bench_general.py varcoef): one operator, CG
iterations and the standalone MatMult under launch-time knob settings.
    python tools/varcoef_ab.py rounds "26=6" "26=4" ..."""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-petsc4py-example_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import numpy as np, torch  # noqa: E401,E402
from mxsolve import _lib  # noqa: E402
from mxsolve.core import DeviceComm, DMat, rhs_hash  # noqa: E402
from bench_general import varcoef_csr  # noqa: E402

L = _lib.load()
rounds, variants = int(sys.argv[1]), sys.argv[2:]
comm = DeviceComm.self_comm(0)
N, ip, c, v = varcoef_csr(256)
A = DMat.from_csr(comm, N, N, ip, c, v)
b = comm.empty(N); rhs_hash(comm, 0, b); x = comm.zeros(N); y = comm.empty(N)


def setv(s):
    return "+".join(f"{k}={L.mx_debug_set(int(k), int(val))}" for k, val in (kv.split("=") for kv in s.split("+")))


res = {vv: {"cg": [], "mult": []} for vv in variants}
for rnd in range(rounds):
    for vv in (variants if rnd % 2 == 0 else variants[::-1]):
        old = setv(vv)
        A.solve(b, x, ksp="cg", rtol=0.0, max_it=32)
        torch.cuda.synchronize(); t0 = time.perf_counter()
        A.solve(b, x, ksp="cg", rtol=0.0, max_it=200)
        torch.cuda.synchronize(); res[vv]["cg"].append((time.perf_counter() - t0) / 200 * 1e6)
        res[vv]["mult"].append(A.bench_mult(b, y, 30)[0] * 1e3)
        setv(old)
print(json.dumps({vv: {"cg_us": round(float(np.median(r["cg"])), 1), "mult_us": round(float(np.median(r["mult"])), 1)}
                  for vv, r in res.items()}), flush=True)
