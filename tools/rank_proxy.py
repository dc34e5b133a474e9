#!/usr/bin/env python3
"""One GPU, one interior rank of the north-star partition: 3D 7-point
256 x 256 x (Z + 2) over 3 in-process ranks (LocalComm) owning 1 / Z / 1
planes, so rank 1 is an interior rank of 256^3 over 256 / Z GPUs (Z = 32:
P = 8, 2,097,152 rows; Z = 64: P = 4), a ghost plane on each side, and the
end ranks add little work (PLANES=Z in the environment, default 32).  Interleaved A/B of CG
variants (knob=value lists joined by '+'), median wall us per iteration of
the whole 3-rank solve (LocalComm's host-synchronous all-reduces included --
compare variants, not absolute numbers; kernel durations come from a
rocprofv3 trace of the same run).

    python tools/rank_proxy.py [rounds] [its] variant ...
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-petsc4py-example_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle  # noqa: E402
from mxsolve import _lib  # noqa: E402
from mxsolve.core import DMat, LocalWorld, rhs_hash  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
its = int(sys.argv[2]) if len(sys.argv) > 2 else 200
variants = sys.argv[3:] or ["9=1", "9=2", "9=5"]
L = _lib.load()
nx, nz = 256, int(os.environ.get("PLANES", "32")) + 2
ip, c, v = oracle.stencil("poisson3d", nx, nx, nz)
M = ip.size - 1
plane = nx * nx
bounds = [0, plane, plane * (nz - 1), M]


def setv(var):
    old = []
    for kv in var.split("+"):
        k, val = kv.split("=")
        old.append(f"{k}={L.mx_debug_set(int(k), int(val))}")
    return "+".join(old)


res = {var: [] for var in variants}
w = LocalWorld(3)


def body(comm):
    r = comm.rank
    r0, r1 = bounds[r], bounds[r + 1]
    lip = ip[r0:r1 + 1] - ip[r0]
    A = DMat.from_csr(comm, M, M, lip, c[ip[r0]:ip[r1]], v[ip[r0]:ip[r1]], m_local=r1 - r0, n_local=r1 - r0)
    m = A.info()["m"]
    b = comm.empty(m)
    rhs_hash(comm, r0, b)
    x = comm.zeros(m)
    out = {}
    for rnd in range(rounds):
        for var in (variants if rnd % 2 == 0 else variants[::-1]):
            comm.barrier()
            if r == 0:
                setv(var)
            comm.barrier()
            A.solve(b, x, ksp="cg", rtol=0.0, max_it=32)
            torch.cuda.synchronize()
            comm.barrier()
            t0 = time.perf_counter()
            rr = A.solve(b, x, ksp="cg", rtol=0.0, max_it=its)
            torch.cuda.synchronize()
            comm.barrier()
            out.setdefault(var, []).append(((time.perf_counter() - t0) / its * 1e6, rr["cg_mode"]))
    A.destroy()
    return out


defaults = {var: setv(var) for var in variants[:1]}   # remember the defaults of the first variant's knobs
outs = w.run(body)
w.destroy()
for var, old in defaults.items():
    setv(old)
rec = {"proxy": f"256x256x{nz} over 3 ranks (1/{nz - 2}/1 planes): a P={256 // (nz - 2)} interior rank of 256^3",
       "its": its}
for var in variants:
    t = [u for u, _ in outs[1][var]]
    rec[var] = {"med_us": round(float(np.median(t)), 1), "min_us": round(float(np.min(t)), 1),
                "cg_mode": outs[1][var][0][1]}
print(json.dumps(rec), flush=True)
