"""One rank of the shared-memory collective stress test (tests/test_gpu_shm.py):
barrier() immediately followed by all-reduces and exchanges, with skewed
rank timing, many times; and (mode "lu_singular") the preonly+LU path on a
singular matrix, where every rank must raise the same PETSc.Error.

    RANK=.. WORLD_SIZE=.. MASTER_ADDR=127.0.0.1 MASTER_PORT=.. python tests/_shm_stress_worker.py mode name
"""
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-petsc4py-example_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def barrier_loop(name):
    from mxsolve.core import DeviceComm, DMat, vdot
    dist.init_process_group("gloo")
    rank, P = dist.get_rank(), dist.get_world_size()
    comm = DeviceComm.shm(rank, P, name, device=0, slot_kib=1)
    A = DMat.stencil(comm, "poisson3d", 8)
    m = A.info()["m"]
    x = comm.empty(m)
    x.fill_(1.0)
    y = comm.empty(m)
    rng = random.Random(rank)
    total = 0.0
    for it in range(200):
        if rng.random() < 0.5:
            time.sleep(rng.random() * 1e-3)
        comm.barrier()
        total += vdot(comm, x, x)
        if it % 10 == 0:
            comm.barrier()
            A.mult(x, y)            # halo exchange right after a barrier
    torch.cuda.synchronize()
    out = {"rank": rank, "total": total, "expect": 200.0 * 8 ** 3}
    A.destroy()
    comm.destroy()
    dist.destroy_process_group()
    return out


def lu_singular():
    sys.path.insert(0, os.path.join(ROOT, "mpi-petsc4py-example_amd", "compat"))
    from petsc4py import PETSc
    import numpy as np
    comm = PETSc.COMM_WORLD
    n = 8
    rs, re = (0, 4) if comm.rank == 0 else (4, 8)
    ip = np.arange(0, (re - rs) + 1, dtype=np.int64)
    cj = np.arange(rs, re, dtype=np.int64)
    vv = np.ones(re - rs)
    if rs <= 5 < re:
        vv[5 - rs] = 0.0                  # a zero row: exactly singular
    A = PETSc.Mat().createAIJ(size=((re - rs, n), (re - rs, n)), csr=(ip, cj, vv), comm=comm)
    A.assemble()
    b, x = A.getVecs()
    b.set(1.0)
    ksp = PETSc.KSP().create(comm)
    ksp.setOperators(A)
    ksp.setType("preonly")
    ksp.getPC().setType("lu")
    try:
        ksp.solve(b, x)
    except PETSc.Error as e:
        return {"rank": comm.rank, "raised": True, "ierr": e.ierr}
    return {"rank": comm.rank, "raised": False}


if __name__ == "__main__":
    mode = sys.argv[1]
    res = barrier_loop(sys.argv[2]) if mode == "barrier" else lu_singular()
    print(json.dumps(res), flush=True)
