#!/usr/bin/env python3
"""createAIJ(csr=...) from fresh host arrays (256^3 7-point, 1.47 GB): the
host-to-device phase under each registration-thread / chunk-size setting
(MX_H2D_THR / MX_H2D_CH / MX_H2D_CH0: read per call by a temporary sweep
build of h2d_pinned, not the committed library, which fixes 4 / 64 / 4).
"warm": one 128^3 createAIJ before the timed calls."""
import os, sys, itertools
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "mpi-petsc4py-example_amd"))
import numpy as np  # noqa: E402
import bench  # noqa: E402
from mxsolve.core import DeviceComm, DMat, assembly_times  # noqa: E402
comm = DeviceComm.self_comm(0)
n = 256
res = {}
ip0, cj0, vv0 = bench.host_csr_stencil(n, n, n)
grid = [(4, 64, 4)]
if len(sys.argv) > 1 and sys.argv[1] == "warm":      # one smaller createAIJ through the pipeline first
    w = bench.host_csr_stencil(128, 128, 128)
    Aw = DMat.from_csr(comm, w[0].size - 1, w[0].size - 1, *w)
    print(f"warm 128^3: h2d {assembly_times()['h2d_ms']:.2f} ms", flush=True)
    Aw.destroy()
for rep in range(4):
    for thr, ch, ch0 in grid:
        os.environ.update(MX_H2D_THR=str(thr), MX_H2D_CH=str(ch), MX_H2D_CH0=str(ch0))
        ip, cj, vv = ip0.copy(), cj0.copy(), vv0.copy()       # fresh (touched, never registered) pages
        A = DMat.from_csr(comm, ip.size - 1, ip.size - 1, ip, cj, vv)
        t = assembly_times()
        A.destroy()
        del ip, cj, vv
        res.setdefault((thr, ch, ch0), []).append(t["h2d_ms"])
        print(f"rep {rep} thr {thr} ch {ch} ch0 {ch0}: h2d {t['h2d_ms']:.2f} ms = {t['host_bytes'] / t['h2d_ms'] / 1e6:.1f} GB/s",
              flush=True)
for k, v in res.items():
    print("median", k, round(float(np.median(v)), 2), "ms", [round(x, 2) for x in v])
