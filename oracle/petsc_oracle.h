/*
 * petsc_oracle.h -- CPU restatement of the PETSc algorithms on the hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the checker
 * / CPU baseline.  The product path (libmxsolve.so) never links or calls it.
 *
 * Parity status (see DESIGN.md "Oracle"):
 *   - assembly (canonical CSR, INSERT/ADD, diag/offdiag split, garray) is
 *     pinned by the reference's own inputs: test.py's seed-42 CSR and
 *     test2.py's tridiagonal CSR are canonical, so PETSc's MatGetRow output
 *     equals the input byte-for-byte (tests/golden/reference_systems.npz).
 *   - the preonly+LU end-to-end result is pinned by test.py:149
 *     (allclose(X, X_actual)).
 *   - CG/GMRES+Jacobi iteration counts and iterates: PARITY UNPINNED against
 *     PETSc itself (no PETSc in this image); they are pinned
 *     against this restatement of PETSc's documented algorithm plus
 *     known-answer properties (exact solves, SPD convergence, residual checks).
 *
 * The reference's numerics live in un-vendored PETSc (conda-forge petsc4py,
 * unpinned, environment.yaml:6; ~3.22 at the 2025-03-14 snapshot).  Each
 * function below cites the reference call site that reaches it and the PETSc
 * routine whose published algorithm it restates.
 */
#ifndef PETSC_ORACLE_H
#define PETSC_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* KSP / PC enums: values follow PETSc's KSPConvergedReason. */
enum { OR_KSP_CG = 0, OR_KSP_GMRES = 1, OR_KSP_PREONLY = 2 };
enum { OR_PC_NONE = 0, OR_PC_JACOBI = 1 };
enum { OR_NORM_DEFAULT = -1, OR_NORM_NONE = 0, OR_NORM_PRECONDITIONED = 1,
       OR_NORM_UNPRECONDITIONED = 2, OR_NORM_NATURAL = 3 };

typedef struct {
  int ksp_type;      /* OR_KSP_* */
  int pc_type;       /* OR_PC_* */
  int norm_type;     /* OR_NORM_* */
  int max_it;        /* default 10000 */
  int restart;       /* GMRES restart, default 30 */
  int guess_nonzero; /* 0: x <- 0 before solve */
  double rtol, atol, dtol; /* 1e-5, 1e-50, 1e5 */
  double haptol;     /* GMRES happy-breakdown tol, 1e-30 */
  double breakdowntol; /* GMRES restart consistency tol, 0.1 */
  int axpy_fma;      /* VecAXPY through an FMA BLAS (OpenBLAS Haswell/Zen kernels) */
  int nthreads;      /* OpenMP threads for the CPU baseline (0 = 1) */
} or_ksp_params;

typedef struct {
  int its;
  int reason;
  double rnorm;
} or_ksp_result;

typedef struct or_mat or_mat;

/* PetscSplitOwnership (test.py:68-74): ranges[P+1]. */
void or_split_ownership(int64_t N, int P, int64_t *ranges);

/* createAIJ(csr=...) on P ranks (petsc_funcs.py:6, test.py:24).  indptr/cols/vals
 * hold the concatenation of every rank's local CSR (rank r owns rows
 * [ranges[r], ranges[r+1])), global column ids.  insert_mode: 0 INSERT, 1 ADD.
 * Returns NULL and sets *err (negative: column out of range = -1,
 * bad indptr = -2). */
or_mat *or_mat_create_csr(int64_t M, int64_t N, int P, const int64_t *indptr,
                          const int64_t *cols, const double *vals, int insert_mode,
                          int *err);
/* MatSetValuesCOO-style: entries (rows[k], cols[k], vals[k]) in any order,
 * rows must be owned by the rank block they are listed in: entries
 * [coo_ptr[r], coo_ptr[r+1]) belong to rank r. Negative indices are skipped. */
or_mat *or_mat_create_coo(int64_t M, int64_t N, int P, const int64_t *coo_ptr,
                          const int64_t *rows, const int64_t *cols, const double *vals,
                          int insert_mode, int *err);
void or_mat_destroy(or_mat *A);
int64_t or_mat_nnz(const or_mat *A);
/* Global canonical CSR as MatGetRow/getValuesCSR return it (global cols, sorted). */
void or_mat_get_csr(const or_mat *A, int64_t *indptr, int64_t *cols, double *vals);
/* Per-rank split: sizes then arrays. */
void or_mat_block_sizes(const or_mat *A, int r, int64_t *m, int64_t *nnz_d, int64_t *nnz_o,
                        int64_t *nghost);
void or_mat_get_block(const or_mat *A, int r, int64_t *dptr, int32_t *dcol, double *dval,
                      int64_t *optr, int32_t *ocol, double *oval, int64_t *garray);
/* MatMult_MPIAIJ order: y_r = A_d x_r, then y_r += A_o lvec (global vectors). */
void or_mat_mult(const or_mat *A, const double *x, double *y);
void or_mat_get_diagonal(const or_mat *A, double *d);
/* KSPSolve (test.py:50). history may be NULL, else max_it+2 doubles. */
int or_ksp_solve(const or_mat *A, const or_ksp_params *p, const double *b, double *x,
                 or_ksp_result *res, double *history);
void or_ksp_default_params(or_ksp_params *p);

/* Synthetic stencil operators as canonical global CSR;
 * kind 0: 2D 5-pt (n x n), 1: 3D 7-pt (n^3), 2: 3D 27-pt (nx*ny*nz),
 * 3: 3D convection-diffusion 7-pt.  Two-call protocol: with indptr==NULL
 * returns nnz. */
int64_t or_stencil(int kind, int64_t nx, int64_t ny, int64_t nz, int64_t *indptr,
                   int64_t *cols, double *vals);
/* b_i = (splitmix64(i + 42*phi) >> 11) * 2^-53 for i in [i0, i0+n). */
void or_rhs_hash(int64_t i0, int64_t n, double *b);

/* VecMAXPY_Seq (PETSc's grouping) and a sequential VecMDot, for the Vec ABI tests */
void or_vec_maxpy(int64_t n, int nv, const double *alpha, double *const *x, double *y);
void or_vec_mdot(int64_t n, const double *x, int nv, const double *const *y, double *out);

#ifdef __cplusplus
}
#endif
#endif
