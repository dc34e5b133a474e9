#!/usr/bin/env python3
"""Two builds of libmxsolve.so side by side in ONE process (ctypes loads each
RTLD_LOCAL, so each keeps its own kernels and knobs): interleaved CG rounds
on the same device, so placement, clocks and neighbours hit both alike.

    python tools/lib_ab.py libA.so,libB.so[,...] [n] [rounds] [knob=value+...]
AB_KIND (stencil kind, default 1 = 3D 7-pt; 3 = conv-diff) and AB_KSP
(0 = CG, 1 = GMRES(30)) select the operator and the method.
"""
import ctypes as C, json, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-petsc4py-example_amd"))
import numpy as np, torch  # noqa: E401,E402
from mxsolve._lib import KSPParams, KSPResult  # noqa: E402

paths = sys.argv[1].split(",")          # the same path twice: two operators of one build
n = int(sys.argv[2]) if len(sys.argv) > 2 else 256
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 5
kind = int(os.environ.get("AB_KIND", "1"))
ksp = int(os.environ.get("AB_KSP", "0"))
knobs = [tuple(int(u) for u in kv.split("=")) for kv in sys.argv[4].split("+")] if len(sys.argv) > 4 else []
torch.cuda.init()
libs = []
for pth in paths:
    L = C.CDLL(os.path.abspath(pth), mode=os.RTLD_LOCAL)
    for k, v in knobs:
        L.mx_debug_set(k, v)
    comm, A = C.c_void_p(), C.c_void_p()
    assert L.mx_comm_create_self(0, C.byref(comm)) == 0
    s = C.c_void_p()
    assert L.mx_comm_stream(comm, C.byref(s)) == 0
    torch.cuda.set_stream(torch.cuda.ExternalStream(s.value))
    assert L.mx_mat_create_stencil(comm, kind, C.c_int64(n), C.c_int64(n), C.c_int64(n), C.byref(A)) == 0
    m = n ** 3
    b = torch.rand(m, dtype=torch.float64, device="cuda")
    x = torch.zeros(m, dtype=torch.float64, device="cuda")
    libs.append((L, comm, A, b, x, s.value))
torch.cuda.synchronize()


def solve(lib, its):
    L, comm, A, b, x, st = lib
    torch.cuda.set_stream(torch.cuda.ExternalStream(st))
    p = KSPParams()
    L.mx_ksp_default_params(C.byref(p))
    p.ksp_type, p.pc_type, p.max_it, p.rtol = ksp, 1, its, 0.0
    r = KSPResult()
    assert L.mx_ksp_solve(A, C.byref(p), C.c_void_p(b.data_ptr()), C.c_void_p(x.data_ptr()), C.byref(r), None) == 0
    return r


res = [[] for _ in libs]
for rnd in range(rounds):
    for j in (range(len(libs)) if rnd % 2 == 0 else reversed(range(len(libs)))):
        solve(libs[j], 32)
        torch.cuda.synchronize(); t0 = time.perf_counter()
        solve(libs[j], 300)
        torch.cuda.synchronize(); res[j].append((time.perf_counter() - t0) / 300 * 1e6)
print(json.dumps({"n": n, "kind": kind, "ksp": ksp, "knobs": sys.argv[4] if len(sys.argv) > 4 else "",
                  **{f"{j}:{os.path.basename(p)}": {"med_us": round(float(np.median(t)), 1),
                                                    "all": [round(v, 1) for v in t]}
                     for j, (p, t) in enumerate(zip(paths, res))}}), flush=True)
