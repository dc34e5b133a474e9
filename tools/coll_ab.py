#!/usr/bin/env python3
"""Per-iteration cost of the collective CG path on one GPU.

A one-rank RCCL communicator with knob 8 (force_coll) runs exactly the
multi-rank iteration minus the halo: partial folds + ncclAllReduce per inner
product instead of the single-rank fused folds.  Run on a rank's share of the
256^3 problem at P = 2/4/8 (256 x 256 x 128/64/32) to see the fixed
per-iteration overhead the strong-scaling runs pay.

    python tools/coll_ab.py [nz,...] [mode:fold,...]   (knob 9 : knob 10)
"""
import json, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-petsc4py-example_amd"))
import numpy as np, torch  # noqa: E401,E402
from mxsolve import _lib  # noqa: E402
from mxsolve.core import DeviceComm, DMat, rhs_hash, unique_id  # noqa: E402

L = _lib.load()
nzs = [int(t) for t in (sys.argv[1] if len(sys.argv) > 1 else "32,64").split(",")]
variants = [tuple(int(u) for u in t.split(":")) for t in (sys.argv[2] if len(sys.argv) > 2 else "0:1,1:1").split(",")]
if os.environ.get("MX_GRID"):                 # SpMV grid (knob 3)
    L.mx_debug_set(3, int(os.environ["MX_GRID"]))
if os.environ.get("MX_GRAPH"):                # graph replay policy (knob 7)
    L.mx_debug_set(7, int(os.environ["MX_GRAPH"]))
self_c = DeviceComm.self_comm(0)
rc = DeviceComm.rccl(0, 1, unique_id(), device=0)


def run(comm, coll, variant, nz, its=400):
    mode, fold = variant
    comm.activate()
    A = DMat.stencil(comm, "poisson3d", 256, 256, nz)
    m = A.info()["m"]
    b = comm.empty(m); rhs_hash(comm, 0, b); x = comm.zeros(m)
    o8, o9, o10 = L.mx_debug_set(8, coll), L.mx_debug_set(9, mode), L.mx_debug_set(10, fold)
    try:
        ts = []
        A.solve(b, x, ksp="cg", rtol=0.0, max_it=48)
        for _ in range(3):
            torch.cuda.synchronize(); t0 = time.perf_counter()
            A.solve(b, x, ksp="cg", rtol=0.0, max_it=its)
            torch.cuda.synchronize(); ts.append((time.perf_counter() - t0) / its * 1e6)
        r = A.solve(b, x, ksp="cg", rtol=0.0, max_it=64, profile=True)
        return {"us_it": round(float(np.median(ts)), 2),
                "matmult_us": round(r["spmv_ms"] / max(r["spmv_count"], 1) * 1e3, 2)}
    finally:
        L.mx_debug_set(8, o8); L.mx_debug_set(9, o9); L.mx_debug_set(10, o10)
        A.destroy()


out = {}
for nz in nzs:
    for v in variants:
        out[f"nz{nz}_m{v[0]}f{v[1]}_self"] = run(self_c, 0, v, nz)
        out[f"nz{nz}_m{v[0]}f{v[1]}_coll"] = run(rc, 1, v, nz)
print(json.dumps(out), flush=True)
self_c.activate()
rc.destroy()
