#!/usr/bin/env python3
"""P in-process ranks, random CSR: MatMult with the column-block path
(key 84 = 2) and the one-pass kernel (0) against the oracle; prints where
each differs (rank, rows, values)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-petsc4py-example_amd")); sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np, torch  # noqa: E402
import oracle  # noqa: E402
from mxsolve import _lib  # noqa: E402
from mxsolve.core import LocalWorld, DMat  # noqa: E402
from test_gpu_cb import _random_csr  # noqa: E402
P = int(sys.argv[1]) if len(sys.argv) > 1 else 2
N = 1 << 12
ip, c, v = _random_csr(N, 7, 23)
ranges = oracle.split_ownership(N, P)
xh = np.random.default_rng(8).standard_normal(N)
yo = oracle.OracleMat.from_csr(N, N, ip, c, v, P=P).mult(xh)
L = _lib.load()


def body(comm):
    r0, r1 = ranges[comm.rank], ranges[comm.rank + 1]
    A = DMat.from_csr(comm, N, N, ip[r0:r1 + 1] - ip[r0], c[ip[r0]:ip[r1]], v[ip[r0]:ip[r1]])
    info = A.info()
    y = comm.empty(r1 - r0)
    A.mult(torch.from_numpy(xh[r0:r1].copy()).cuda(), y)
    A.destroy()
    return info["cb_blocks"], info["nghost"], y.cpu().numpy()


for cb in (2, 0):
    old = L.mx_debug_set(84, cb)
    w = LocalWorld(P)
    try:
        out = w.run(body)
    finally:
        L.mx_debug_set(84, old)
        w.destroy()
    for r, (nb, ng, y) in enumerate(out):
        e = yo[ranges[r]:ranges[r + 1]]
        bad = np.nonzero(y.view(np.uint64) != e.view(np.uint64))[0]
        print(f"cb={cb} rank {r}: cb_blocks {nb} nghost {ng} bad {bad.size}", bad[:8], y[bad[:4]], e[bad[:4]], flush=True)
