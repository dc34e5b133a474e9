#!/usr/bin/env python3
"""Repeated 8-rank assemblies of one stencil operator on in-process ranks
(LocalComm, one GPU), each followed by a short solve when DIAG_SOLVE is set:
every rank's assembly summary is compared with the first round's, and any
difference is printed -- the race check behind the device synchronisation at
the start of assemble() (mx_assembly.hip).
    python tools/asm_race.py KIND N REPS [knob=value ...]"""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-petsc4py-example_amd")); sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np, torch
from mxsolve import _lib
from mxsolve.core import DMat, DeviceComm
from test_gpu_multirank import run_ranks
self_c = DeviceComm.self_comm(0)
L = _lib.load()
kind, n, reps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
knobs = [tuple(int(v) for v in kv.split("=")) for kv in sys.argv[4:]]
for k, v in knobs: L.mx_debug_set(k, v)
KEYS = ("nnz_d", "nnz_o", "nghost", "sell_slots_d", "sell_slots_o", "dia_slices", "value_codes", "code_bytes",
        "pair_shape", "pair_units", "pair_blocks", "pair_code", "pair_lean", "nsend", "nrecv")
def body(comm):
    A = DMat.stencil(comm, kind, n)
    info = dict(A.info())
    if os.environ.get("DIAG_SOLVE"):
        from mxsolve.core import rhs_hash
        b = comm.empty(info["m"]); rhs_hash(comm, info["rstart"], b); x = comm.zeros(info["m"])
        A.solve(b, x, ksp="gmres" if kind == "convdiff3d" else "cg", pc="jacobi", max_it=50)
    A.destroy()
    return {k: info.get(k) for k in KEYS}
ref = None
nbad = 0
for i in range(reps):
    r = run_ranks(8, body)
    if ref is None: ref = r
    for q in range(8):
        if r[q] != ref[q]:
            nbad += 1
            print(i, "rank", q, "DIFF", {k: (ref[q][k], r[q][k]) for k in KEYS if r[q][k] != ref[q][k]}, flush=True)
print("ref rank0", ref[0], flush=True)
print("done", reps, "bad", nbad, flush=True)
