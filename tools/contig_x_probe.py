#!/usr/bin/env python3
"""test_fused_equals_separate_ranks' failing case under MXSOLVE_KNOBS (CG
modes 1, 2, 0 on P in-process ranks, poisson3d 14^3): for every rank, the
solution x as the host sees it through the copy engine (x.cpu()) against the
same x summed and copied by kernels (torch.sum, x.clone().cpu()) -- a write a
kernel made that the copy does not see (or the reverse) shows up as a
difference.  Prints the rows where the modes' x differ.
    MXSOLVE_KNOBS=81=1+82=1024 python tools/contig_x_probe.py [P]"""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-petsc4py-example_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from mxsolve import _lib  # noqa: E402
from mxsolve.core import DMat, LocalWorld, rhs_hash  # noqa: E402

L = _lib.load()
P = int(sys.argv[1]) if len(sys.argv) > 1 else 2
old27 = L.mx_debug_set(27, 0)


def solve(comm):
    A = DMat.stencil(comm, "poisson3d", 14)
    info = A.info()
    b = comm.empty(info["m"]); rhs_hash(comm, info["rstart"], b)
    x = comm.zeros(info["m"])
    r = A.solve(b, x, ksp="cg", history=True)
    A.destroy()
    ksum = float(torch.sum(x))                       # a reduction kernel
    kcopy = x.clone()                                # a copy kernel, then the copy engine
    torch.cuda.synchronize()
    xh = x.cpu().numpy()
    return {"its": r["its"], "x": xh, "ksum": ksum, "kcopy": kcopy.cpu().numpy(), "ptr": x.data_ptr()}


outs = {}
for fuse in (1, 2, 0):
    w = LocalWorld(P)
    old = L.mx_debug_set(9, fuse)
    try:
        outs[fuse] = w.run(solve)
    finally:
        L.mx_debug_set(9, old)
        w.destroy()
for fuse in (1, 2, 0):
    for rk, o in enumerate(outs[fuse]):
        zeros = int(np.sum(o["x"] == 0.0))
        print(f"mode {fuse} rank {rk}: its {o['its']} x@{o['ptr']:#x} host-copy sum {o['x'].sum()!r} kernel sum "
              f"{o['ksum']!r} clone-copy sum {o['kcopy'].sum()!r} zeros {zeros}", flush=True)
for mode in (1, 2):
    for rk, (a, b) in enumerate(zip(outs[mode], outs[0])):
        d = np.nonzero(a["x"].view(np.uint64) != b["x"].view(np.uint64))[0]
        if d.size:
            print(f"mode {mode} vs 0, rank {rk}: {d.size} rows differ, rows {d[0]}..{d[-1]}", flush=True)
L.mx_debug_set(27, old27)
