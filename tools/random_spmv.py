#!/usr/bin/env python3
"""Standalone MatMult of the random-pattern general-AIJ leg (2^24 rows, the
diagonal + 6 uniform random columns, column-index SELL) under knob variants,
interleaved in one process: median HIP-event time per launch.
    python tools/random_spmv.py [log2 rows] variant ...   (variant: "k=v+k=v", "" = defaults)"""
import json, os, statistics, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-petsc4py-example_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402
from mxsolve import _lib  # noqa: E402
from mxsolve.core import DeviceComm, DMat  # noqa: E402
from bench_general import random_csr  # noqa: E402

lg = int(sys.argv[1]) if len(sys.argv) > 1 else 24
variants = sys.argv[2:] or [""]
L = _lib.load()
comm = DeviceComm.self_comm(0)
N, ip, c, v = random_csr(1 << lg)
A = DMat.from_csr(comm, N, N, ip, c, v)
del ip, c, v
x = torch.rand(N, dtype=torch.float64, device="cuda")
y = torch.empty_like(x)


def setv(s):
    old = []
    for kv in filter(None, s.split("+")):
        k, val = kv.split("=")
        old.append((int(k), L.mx_debug_set(int(k), int(val))))
    return old


res = {s: [] for s in variants}
for rnd in range(5):
    for s in (variants if rnd % 2 == 0 else variants[::-1]):
        old = setv(s)
        ms, _ = A.bench_mult(x, y, 10)
        res[s].append(ms * 1e3)
        for k, o in old:
            L.mx_debug_set(k, o)
info = A.info()
print(json.dumps({"rows": N, "nnz": info["nnz_d"], "slots": info["sell_slots_d"],
                  **{(s or "default"): round(statistics.median(t), 1) for s, t in res.items()}}))
