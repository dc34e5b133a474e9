#!/usr/bin/env python3
"""test_fused_equals_separate_ranks' case (poisson3d 14^3, in-process ranks)
under the current MXSOLVE_KNOBS, printing where the fused modes' x differs
from the separate passes' (rank, count, first rows, values).  Written for a
poisoned-reuse allocator build (not in the library).
    python tools/poison_probe.py [P] [n]"""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-petsc4py-example_amd"))
import numpy as np  # noqa: E402
from mxsolve import _lib  # noqa: E402
from mxsolve.core import DMat, LocalWorld, rhs_hash  # noqa: E402

L = _lib.load()
P = int(sys.argv[1]) if len(sys.argv) > 1 else 2
n = int(sys.argv[2]) if len(sys.argv) > 2 else 14
old27 = L.mx_debug_set(27, 0)


def solve(comm):
    A = DMat.stencil(comm, "poisson3d", n)
    info = A.info()
    b = comm.empty(info["m"]); rhs_hash(comm, info["rstart"], b)
    x = comm.zeros(info["m"])
    r = A.solve(b, x, ksp="cg", history=True)
    A.destroy()
    return r["its"], r["reason"], np.array(r["history"]), x.cpu().numpy()


outs = {}
for fuse in (1, 2, 0):
    w = LocalWorld(P)
    old = L.mx_debug_set(9, fuse)
    try:
        outs[fuse] = w.run(solve)
    finally:
        L.mx_debug_set(9, old)
        w.destroy()
for mode in (1, 2):
    for rk, (a, b) in enumerate(zip(outs[mode], outs[0])):
        dx = np.nonzero(a[3].view(np.uint64) != b[3].view(np.uint64))[0]
        dh = np.nonzero(a[2].view(np.uint64) != b[2].view(np.uint64))[0] if a[2].shape == b[2].shape else "shape"
        print(f"mode {mode} rank {rk}: its {a[0]}/{b[0]} reason {a[1]}/{b[1]} hist diffs {dh} "
              f"x diffs {dx.size} of {a[3].size}", flush=True)
        for i in dx[:8]:
            print(f"    row {i}: {a[3][i]!r} vs {b[3][i]!r}", flush=True)
L.mx_debug_set(27, old27)
