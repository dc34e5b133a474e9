"""One rank of a multi-process solve on a shared GPU (tests/test_gpu_shm.py):
the shared-memory transport between processes, against the oracle.

    RANK=.. WORLD_SIZE=.. MASTER_ADDR=127.0.0.1 MASTER_PORT=.. python tests/_shm_worker.py kind n ksp name
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-petsc4py-example_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from mxsolve.core import DeviceComm, DMat, rhs_hash  # noqa: E402


def main():
    kind, n, ksp, name = sys.argv[1], int(sys.argv[2]), sys.argv[3], sys.argv[4]
    dist.init_process_group("gloo")
    rank, P = dist.get_rank(), dist.get_world_size()
    comm = DeviceComm.shm(rank, P, name, device=0, slot_kib=1)   # 1 KiB slots: exchanges take several rounds
    A = DMat.stencil(comm, kind, n)
    info = A.info()
    b = comm.empty(info["m"])
    rhs_hash(comm, info["rstart"], b)
    x = comm.zeros(info["m"])
    r = A.solve(b, x, ksp=ksp, pc="jacobi", history=True)
    parts = [None] * P
    dist.all_gather_object(parts, (info["rstart"], x.cpu().numpy(), A.csr()))
    if rank == 0:
        import oracle
        xs = np.concatenate([p[1] for p in sorted(parts, key=lambda t: t[0])])
        ip, c, v = oracle.stencil(kind, n)
        M = ip.size - 1
        O = oracle.OracleMat.from_csr(M, M, ip, c, v, P=P)
        o = O.solve(oracle.rhs_hash(0, M), ksp=ksp, pc="jacobi")
        rel = float(np.linalg.norm(xs - o["x"]) / np.linalg.norm(o["x"]))
        # assembled rows, in global numbering, equal the oracle's CSR
        rows_ok = True
        for r0, _, (lip, lc, lv) in parts:
            m = lip.size - 1
            g0, g1 = ip[r0], ip[r0 + m]
            rows_ok &= bool(np.array_equal(lip, ip[r0:r0 + m + 1] - g0) and np.array_equal(lc, c[g0:g1])
                            and np.array_equal(lv.view(np.uint64), v[g0:g1].view(np.uint64)))
        print(json.dumps({"its": r["its"], "reason": r["reason"], "oracle_its": o["its"],
                          "oracle_reason": o["reason"], "rel": rel, "rows_ok": rows_ok}), flush=True)
    A.destroy()
    comm.destroy()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
