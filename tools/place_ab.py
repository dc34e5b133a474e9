#!/usr/bin/env python3
"""Placement sensitivity of the MatMult: the same operator applied to x/y
vectors from different allocations (library contiguous vs torch/hipMalloc),
standalone MatMult time (HIP events) per allocation.
    python tools/place_ab.py [n] [count]"""
import json, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-petsc4py-example_amd"))
import torch  # noqa: E402
from mxsolve import _lib  # noqa: E402
from mxsolve.core import DeviceComm, DMat, rhs_hash, device_vector  # noqa: E402

L = _lib.load()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
cnt = int(sys.argv[2]) if len(sys.argv) > 2 else 6
comm = DeviceComm.self_comm(0)
A = DMat.stencil(comm, "poisson3d", n)
m = A.info()["m"]
xs = {"lib": [device_vector(m, 0) for _ in range(cnt)],
      "torch": [torch.empty(m, dtype=torch.float64, device="cuda") for _ in range(cnt)]}
for v in xs.values():
    for t in v:
        rhs_hash(comm, 0, t)
y = device_vector(m, 0)
out = {}
for kind, v in xs.items():
    out[kind + "_x"] = [round(A.bench_mult(t, y, 30)[0] * 1e3, 1) for t in v]
x0 = xs["lib"][0]
out["lib_y"] = [round(A.bench_mult(x0, t, 30)[0] * 1e3, 1) for t in xs["lib"][1:]]
out["torch_y"] = [round(A.bench_mult(x0, t, 30)[0] * 1e3, 1) for t in xs["torch"]]
out["ptr_mod_2M"] = [(t.data_ptr() >> 21) & 1023 for t in xs["lib"]]
print(json.dumps(out), flush=True)
