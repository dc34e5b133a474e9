#!/usr/bin/env python3
"""CG iteration time on one GPU by communicator kind, interleaved: the self
communicator, a one-rank RCCL communicator on the fused single-rank path, and
the same on the collective path (knob 8).  Each round rebuilds the operator.

    python tools/comm_ab.py [n] [rounds]
"""
import json, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-petsc4py-example_amd"))
import numpy as np, torch  # noqa: E401,E402
from mxsolve import _lib  # noqa: E402
from mxsolve.core import DeviceComm, DMat, rhs_hash, unique_id  # noqa: E402

L = _lib.load()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
comms = {"self": (DeviceComm.self_comm(0), 0), "rccl": (DeviceComm.rccl(0, 1, unique_id(), device=0), 0)}
comms["rccl_coll"] = (comms["rccl"][0], 1)
res = {k: [] for k in comms}
for rnd in range(rounds):
    order = list(comms) if rnd % 2 == 0 else list(reversed(list(comms)))
    for k in order:
        comm, coll = comms[k]
        comm.activate()
        A = DMat.stencil(comm, "poisson3d", n)
        m = A.info()["m"]
        b = comm.empty(m); rhs_hash(comm, 0, b); x = comm.zeros(m)
        o8 = L.mx_debug_set(8, coll)
        A.solve(b, x, ksp="cg", rtol=0.0, max_it=48)
        torch.cuda.synchronize(); t0 = time.perf_counter()
        A.solve(b, x, ksp="cg", rtol=0.0, max_it=300)
        torch.cuda.synchronize(); res[k].append((time.perf_counter() - t0) / 300 * 1e6)
        L.mx_debug_set(8, o8)
        A.destroy(); del b, x
print(json.dumps({"n": n, **{k: [round(v, 1) for v in vs] for k, vs in res.items()}}), flush=True)
comms["self"][0].activate()
comms["rccl"][0].destroy()
