#!/usr/bin/env python3
"""Device assembly time of one stencil operator in a fresh process, after the
process start-up cost (code-object load, first pools) is paid on an 8^3
operator: python tools/asm_time.py kind nx ny nz"""
import json, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-petsc4py-example_amd"))
import torch  # noqa: E402
from mxsolve.core import DeviceComm, DMat, rhs_hash  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "poisson3d27"
dims = [int(v) for v in sys.argv[2:5]] if len(sys.argv) > 4 else [512, 512, 64]
comm = DeviceComm.self_comm(0)
t0 = time.perf_counter()
A0 = DMat.stencil(comm, "poisson3d", 8)
b0 = comm.empty(A0.info()["m"]); rhs_hash(comm, 0, b0); x0 = comm.zeros(A0.info()["m"])
A0.solve(b0, x0, ksp="cg", max_it=2, rtol=0.0)
A0.destroy()
torch.cuda.synchronize()
t_init = time.perf_counter() - t0
ts = []
for rep in range(3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    A = DMat.stencil(comm, kind, *dims)
    torch.cuda.synchronize()
    ts.append(time.perf_counter() - t0)
    A.destroy()
print(json.dumps({"kind": kind, "dims": dims, "process_init_s": round(t_init, 4),
                  "assembly_s": [round(t, 4) for t in ts]}), flush=True)
