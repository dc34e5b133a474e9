"""mxsolve -- MI355X-native hot path of the mpi-petsc4py-example workflow.

createAIJ(csr=...) assembly -> MatMult (VecScatter halo + SpMV) -> KSPSolve
CG / GMRES with Jacobi, in hand-written gfx950 HIP kernels behind the C ABI
of libmxsolve.so (include/mxsolve.h).  Submodules:

  core        handles over the C ABI (communicators, matrices, vectors)
  PETSc       petsc4py-compatible operator API (Mat, Vec, KSP, PC, Options)
  MPI         mpi4py-compatible host control plane (torch.distributed gloo)
  SLEPc       slepc4py-compatible EPS (import surface for petsc_funcs)
  petsc_funcs the reference helper signatures (createPETScMat, solveSLEPcEigenvalues)
"""
__version__ = "0.1.0"
