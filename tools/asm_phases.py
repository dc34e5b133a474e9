#!/usr/bin/env python3
"""Device assembly of the stencil operators by phase, after the process
start-up cost is paid on an 8^3 operator: for each configuration, REPS
assemblies in the same process, each with its wall time and
mx_debug_assembly_times' phases (canonicalisation, split, layouts, halo).
python tools/asm_phases.py [REPS] [kind:nx:ny:nz ...]"""
import json, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-petsc4py-example_amd"))
import torch  # noqa: E402
from mxsolve.core import DeviceComm, DMat, rhs_hash, assembly_times  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
cfgs = [a.split(":") for a in sys.argv[2:]] or [["poisson3d27", "512", "512", "64"], ["poisson3d", "256", "256", "256"]]
comm = DeviceComm.self_comm(0)
A0 = DMat.stencil(comm, "poisson3d", 8)
b0 = comm.empty(A0.info()["m"]); rhs_hash(comm, 0, b0); x0 = comm.zeros(A0.info()["m"])
A0.solve(b0, x0, ksp="cg", max_it=2, rtol=0.0)
A0.destroy()
torch.cuda.synchronize()
for kind, *d in cfgs:
    dims = [int(v) for v in d]
    for rep in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        A = DMat.stencil(comm, kind, *dims)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        ph = assembly_times()
        info = A.info()
        A.destroy()
        print(json.dumps({"kind": kind, "dims": dims, "rep": rep, "wall_ms": round(wall * 1e3, 3),
                          "nnz": info["nnz_d"] + info["nnz_o"],
                          **{k: round(v, 3) for k, v in ph.items() if k.endswith("_ms")}}), flush=True)
