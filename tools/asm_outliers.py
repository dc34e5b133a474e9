#!/usr/bin/env python3
"""Repeated assemblies of one stencil operator, each followed by a short CG
solve (as bench.py's legs do), with the phase times of every assembly; lists
the ones slower than 3x the median.  Knob variants alternate per round.
    python tools/asm_outliers.py kind nx ny nz reps [knob=value+... ...]"""
import json, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-petsc4py-example_amd"))
import numpy as np, torch  # noqa: E401,E402
from mxsolve import _lib  # noqa: E402
from mxsolve.core import DeviceComm, DMat, assembly_times, rhs_hash  # noqa: E402

kind = sys.argv[1]
dims = [int(v) for v in sys.argv[2:5]]
reps = int(sys.argv[5])
variants = sys.argv[6:] or [""]
L = _lib.load()
comm = DeviceComm.self_comm(0)
rows = {v: [] for v in variants}
for rep in range(reps):
    for v in (variants if rep % 2 == 0 else variants[::-1]):
        old = [(int(k), L.mx_debug_set(int(k), int(val))) for k, val in (kv.split("=") for kv in v.split("+") if kv)]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        A = DMat.stencil(comm, kind, *dims)
        torch.cuda.synchronize()
        t = (time.perf_counter() - t0) * 1e3
        ph = assembly_times()
        m = A.info()["m"]
        b = comm.empty(m); rhs_hash(comm, 0, b); x = comm.zeros(m)
        A.solve(b, x, ksp="cg", rtol=0.0, max_it=20)
        torch.cuda.synchronize()
        A.destroy(); del b, x
        for k, o in old:
            L.mx_debug_set(k, o)
        free_gb = torch.cuda.mem_get_info(0)[0] / 2**30
        rows[v].append({"ms": round(t, 2), **{k: round(ph[k], 2) for k in ("canon_ms", "split_ms", "layout_ms")},
                        "free_gb": round(free_gb, 2)})
        print(json.dumps({"rep": rep, "variant": v, **rows[v][-1]}), flush=True)
for v, r in rows.items():
    ms = np.array([e["ms"] for e in r])
    med = float(np.median(ms))
    print(json.dumps({"variant": v, "median_ms": med, "max_ms": float(ms.max()),
                      "outliers": [e for e in r if e["ms"] > 3 * med]}), flush=True)
