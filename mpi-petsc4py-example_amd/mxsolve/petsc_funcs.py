"""The reference helper signatures (petsc_funcs.py:5-20), written for mxsolve.

createPETScMat(comm, shape, csr) -> Mat   (petsc_funcs.py:5-10)
solveSLEPcEigenvalues(comm, A)  -> EPS   (petsc_funcs.py:13-20)
"""
from . import PETSc, SLEPc


def createPETScMat(comm, shape, csr):
    """createAIJ(comm, size=shape, csr=csr) + assemble(): GPU assembly."""
    A = PETSc.Mat().createAIJ(comm=comm, size=shape, csr=csr)
    A.assemble()
    return A


def solveSLEPcEigenvalues(comm, A):
    """EPS(HEP) with options from the database (-eps_nev, -eps_tol, ...)."""
    E = SLEPc.EPS().create(comm=comm)
    E.setOperators(A)
    E.setProblemType(SLEPc.EPS.ProblemType.HEP)
    E.setFromOptions()
    E.solve()
    return E
