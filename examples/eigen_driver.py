"""Counterpart of the reference's test2.py call sequence (test2.py:1-101),
written from scratch: rank 0 builds the 100x100 tridiagonal matrix with
A[i,j] = i+j+1 for |i-j| <= 1 (test2.py:6-18), distributes CSR row blocks,
every rank calls the helper createPETScMat (petsc_funcs.py:5-10) and
solveSLEPcEigenvalues (petsc_funcs.py:13-20), rank 0 prints the converged
eigenvalues.

    python examples/eigen_driver.py [-eps_nev 3]
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "mpi-petsc4py-example_amd", "compat"))
sys.path.insert(0, os.path.join(HERE, "..", "mpi-petsc4py-example_amd"))

import numpy as np  # noqa: E402
import petsc4py  # noqa: E402

petsc4py.init(sys.argv)
from mpi4py import MPI  # noqa: E402

from mxsolve import petsc_funcs as pet  # noqa: E402


def create(nsize):
    ip = [0]
    cols, vals = [], []
    for i in range(nsize):
        for j in (i - 1, i, i + 1):
            if 0 <= j < nsize:
                cols.append(j)
                vals.append(float(i + j + 1))
        ip.append(len(cols))
    return np.array(ip, np.int32), np.array(cols, np.int32), np.array(vals)


def main():
    comm = MPI.COMM_WORLD
    rank, nprocs = comm.Get_rank(), comm.Get_size()
    if rank == 0:
        nsize = 100
        ip, cj, vv = create(nsize)
        shape = (nsize, nsize)
        q, r = divmod(nsize, nprocs)
        count = [q + 1 if i < r else q for i in range(nprocs)]
        displ = [sum(count[:i]) for i in range(nprocs)]
        for i in range(1, nprocs):
            rs, re = displ[i], displ[i] + count[i]
            a = (ip[rs:re + 1] - ip[rs]).astype(np.int32)
            b = cj[ip[rs]:ip[re]]
            c = vv[ip[rs]:ip[re]]
            comm.send({"CSR_indptr": a.size, "CSR_indices": b.size, "CSR_data": c.size}, dest=i)
            comm.Send([a, MPI.INT], dest=i)
            comm.Send([np.ascontiguousarray(b), MPI.INT], dest=i)
            comm.Send([np.ascontiguousarray(c), MPI.DOUBLE], dest=i)
        rs, re = displ[0], displ[0] + count[0]
        CSR = (ip[rs:re + 1] - ip[rs], cj[ip[rs]:ip[re]], vv[ip[rs]:ip[re]])
    else:
        lengths = comm.recv(source=0)
        a = np.empty(lengths["CSR_indptr"], dtype=np.int32)
        b = np.empty(lengths["CSR_indices"], dtype=np.int32)
        c = np.empty(lengths["CSR_data"], dtype=np.double)
        comm.Recv([a, MPI.INT], source=0)
        comm.Recv([b, MPI.INT], source=0)
        comm.Recv([c, MPI.DOUBLE], source=0)
        CSR = (a, b, c)
        shape = None
    shape = comm.bcast(shape, root=0)
    A = pet.createPETScMat(comm, shape, CSR)
    E = pet.solveSLEPcEigenvalues(comm, A)
    nconv = E.getConverged()
    vr, wr = A.getVecs()
    vi, wi = A.getVecs()
    if rank == 0:
        for i in range(nconv):
            k = E.getEigenpair(i, vr, vi)
            print("Eigenvalue: ", k)


if __name__ == "__main__":
    main()
