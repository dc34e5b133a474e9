#!/usr/bin/env python3
"""Device assembly time of one stencil operator in a fresh process, after the
process start-up cost (code-object load, first pools) is paid on an 8^3
operator: python tools/asm_time.py kind nx ny nz [knob=value+... ...]
(several knob variants: interleaved, 3 assemblies each per round, 3 rounds)"""
import json, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-petsc4py-example_amd"))
import torch  # noqa: E402
from mxsolve import _lib  # noqa: E402
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
variants = sys.argv[5:] or [""]
L = _lib.load()
ts = {v: [] for v in variants}
for rnd in range(3 if len(variants) > 1 else 1):
    for v in (variants if rnd % 2 == 0 else variants[::-1]):
        old = [(int(k), L.mx_debug_set(int(k), int(val))) for k, val in (kv.split("=") for kv in v.split("+") if kv)]
        for rep in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            A = DMat.stencil(comm, kind, *dims)
            torch.cuda.synchronize()
            ts[v].append(time.perf_counter() - t0)
            A.destroy()
        for k, o in old:
            L.mx_debug_set(k, o)
print(json.dumps({"kind": kind, "dims": dims, "process_init_s": round(t_init, 4),
                  **{"assembly_s" + (f"[{v}]" if v else ""): [round(t, 4) for t in t_v] for v, t_v in ts.items()}}),
      flush=True)
