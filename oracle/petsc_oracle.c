/*
 * petsc_oracle.c -- CPU restatement of the PETSc algorithms that the
 * reference's hot path reaches (see petsc_oracle.h for scope and pinning).
 *
 * TEST INFRASTRUCTURE ONLY: loaded by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py.  Never linked into libmxsolve.so.
 *
 * Build: oracle/Makefile (gcc -O2 -fopenmp -ffp-contract=off).  No FMA is
 * contracted: conda-forge builds PETSc for -march=nocona, so PETSc's own C
 * loops (MatMult_SeqAIJ, VecAYPX_Seq, VecMAXPY_Seq) round every multiply and
 * add separately; VecAXPY goes through BLAS daxpy, whose OpenBLAS
 * Haswell/Zen kernel is a fused multiply-add (params.axpy_fma).
 */
#include "petsc_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------------ */
/* Layout                                                                    */
/* ------------------------------------------------------------------------ */

/* PetscSplitOwnership: m = N/P + (N%P > rank); identical to the driver's
 * divmod split at test.py:68-74 and test2.py:33-37. */
void or_split_ownership(int64_t N, int P, int64_t *ranges) {
  int64_t q = N / P, r = N % P;
  ranges[0] = 0;
  for (int i = 0; i < P; ++i) ranges[i + 1] = ranges[i] + q + (i < r ? 1 : 0);
}

/* ------------------------------------------------------------------------ */
/* Assembly: MatMPIAIJSetPreallocationCSR -> MatSetValues(INSERT|ADD) ->     */
/* MatAssemblyEnd -> MatSetUpMultiply_MPIAIJ                                  */
/* (reached from petsc_funcs.py:6-7 and test.py:24-28)                        */
/* ------------------------------------------------------------------------ */

typedef struct {
  int64_t m, rstart, cstart, cend;
  int64_t *dptr; int32_t *dcol; double *dval; /* diagonal block, local cols */
  int64_t *optr; int32_t *ocol; double *oval; /* off-diag block, ghost index */
  int64_t nghost; int64_t *garray;            /* sorted global ghost cols */
  double *diag;                               /* MatGetDiagonal */
} or_block;

struct or_mat {
  int P;
  int64_t M, N;
  int64_t *ranges, *cranges;
  or_block *blk;
};

typedef struct { int64_t col; int64_t pos; double val; } entry_t;

static int cmp_entry(const void *a, const void *b) {
  const entry_t *x = (const entry_t *)a, *y = (const entry_t *)b;
  if (x->col != y->col) return x->col < y->col ? -1 : 1;
  return x->pos < y->pos ? -1 : (x->pos > y->pos);
}

static int cmp_i64(const void *a, const void *b) {
  int64_t x = *(const int64_t *)a, y = *(const int64_t *)b;
  return x < y ? -1 : (x > y);
}

/* Canonicalise one row in input order (MatSetValues_SeqAIJ semantics):
 * negative columns are ignored, columns are kept sorted, an existing entry is
 * overwritten (INSERT: last wins) or accumulated in input order (ADD: the
 * first occurrence is stored, later ones are added), explicit zeros are kept
 * (MAT_IGNORE_ZERO_ENTRIES is off by default).  Returns entries kept. */
static int64_t canon_row(entry_t *e, int64_t n, int add) {
  qsort(e, (size_t)n, sizeof(entry_t), cmp_entry);
  int64_t k = 0;
  for (int64_t j = 0; j < n; ++j) {
    if (e[j].col < 0) continue;
    if (k > 0 && e[k - 1].col == e[j].col) {
      if (add) e[k - 1].val = e[k - 1].val + e[j].val;
      else e[k - 1].val = e[j].val;
    } else {
      e[k++] = e[j];
    }
  }
  return k;
}

/* Split one rank's canonical rows into A_d / A_o and build garray
 * (MatSetUpMultiply_MPIAIJ: garray = sorted unique off-process columns, A_o
 * columns renumbered into [0, nghost) in garray order). */
static int build_block(or_block *B, int64_t m, entry_t **rows, const int64_t *rowlen) {
  int64_t nd = 0, no = 0;
  for (int64_t i = 0; i < m; ++i)
    for (int64_t j = 0; j < rowlen[i]; ++j) {
      int64_t c = rows[i][j].col;
      if (c >= B->cstart && c < B->cend) nd++; else no++;
    }
  B->m = m;
  B->dptr = (int64_t *)calloc((size_t)m + 1, sizeof(int64_t));
  B->optr = (int64_t *)calloc((size_t)m + 1, sizeof(int64_t));
  B->dcol = (int32_t *)malloc((size_t)(nd ? nd : 1) * sizeof(int32_t));
  B->dval = (double *)malloc((size_t)(nd ? nd : 1) * sizeof(double));
  B->ocol = (int32_t *)malloc((size_t)(no ? no : 1) * sizeof(int32_t));
  B->oval = (double *)malloc((size_t)(no ? no : 1) * sizeof(double));
  int64_t *gtmp = (int64_t *)malloc((size_t)(no ? no : 1) * sizeof(int64_t));
  int64_t pd = 0, po = 0;
  for (int64_t i = 0; i < m; ++i) {
    for (int64_t j = 0; j < rowlen[i]; ++j) {
      int64_t c = rows[i][j].col;
      if (c >= B->cstart && c < B->cend) {
        B->dcol[pd] = (int32_t)(c - B->cstart); B->dval[pd++] = rows[i][j].val;
      } else {
        gtmp[po] = c; B->oval[po++] = rows[i][j].val;
      }
    }
    B->dptr[i + 1] = pd; B->optr[i + 1] = po;
  }
  /* garray */
  int64_t *g = (int64_t *)malloc((size_t)(no ? no : 1) * sizeof(int64_t));
  memcpy(g, gtmp, (size_t)no * sizeof(int64_t));
  qsort(g, (size_t)no, sizeof(int64_t), cmp_i64);
  int64_t ng = 0;
  for (int64_t j = 0; j < no; ++j) if (ng == 0 || g[ng - 1] != g[j]) g[ng++] = g[j];
  B->nghost = ng; B->garray = g;
  for (int64_t j = 0; j < no; ++j) {
    int64_t lo = 0, hi = ng - 1, c = gtmp[j];
    while (lo < hi) { int64_t mid = (lo + hi) / 2; if (g[mid] < c) lo = mid + 1; else hi = mid; }
    B->ocol[j] = (int32_t)lo;
  }
  free(gtmp);
  /* diagonal (global row rstart+i, global col rstart+i) */
  B->diag = (double *)calloc((size_t)m ? (size_t)m : 1, sizeof(double));
  for (int64_t i = 0; i < m; ++i) {
    int64_t lc = B->rstart + i - B->cstart;
    for (int64_t j = B->dptr[i]; j < B->dptr[i + 1]; ++j)
      if (B->dcol[j] == lc) { B->diag[i] = B->dval[j]; break; }
  }
  return 0;
}

static or_mat *mat_alloc(int64_t M, int64_t N, int P) {
  or_mat *A = (or_mat *)calloc(1, sizeof(or_mat));
  A->P = P; A->M = M; A->N = N;
  A->ranges = (int64_t *)malloc(((size_t)P + 1) * sizeof(int64_t));
  A->cranges = (int64_t *)malloc(((size_t)P + 1) * sizeof(int64_t));
  or_split_ownership(M, P, A->ranges);
  or_split_ownership(N, P, A->cranges);
  A->blk = (or_block *)calloc((size_t)P, sizeof(or_block));
  for (int r = 0; r < P; ++r) {
    A->blk[r].rstart = A->ranges[r];
    A->blk[r].cstart = A->cranges[r];
    A->blk[r].cend = A->cranges[r + 1];
  }
  return A;
}

or_mat *or_mat_create_csr(int64_t M, int64_t N, int P, const int64_t *indptr,
                          const int64_t *cols, const double *vals, int insert_mode,
                          int *err) {
  *err = 0;
  if (indptr[0] != 0) { *err = -2; return NULL; }
  for (int64_t i = 0; i < M; ++i) if (indptr[i + 1] < indptr[i]) { *err = -2; return NULL; }
  for (int64_t k = 0; k < indptr[M]; ++k) if (cols[k] >= N) { *err = -1; return NULL; }
  or_mat *A = mat_alloc(M, N, P);
  for (int r = 0; r < P; ++r) {
    or_block *B = &A->blk[r];
    int64_t r0 = A->ranges[r], m = A->ranges[r + 1] - r0;
    entry_t **rows = (entry_t **)malloc(((size_t)m + 1) * sizeof(entry_t *));
    int64_t *len = (int64_t *)malloc(((size_t)m + 1) * sizeof(int64_t));
    for (int64_t i = 0; i < m; ++i) {
      int64_t a = indptr[r0 + i], n = indptr[r0 + i + 1] - a;
      rows[i] = (entry_t *)malloc((size_t)(n ? n : 1) * sizeof(entry_t));
      for (int64_t j = 0; j < n; ++j) {
        rows[i][j].col = cols[a + j]; rows[i][j].pos = j; rows[i][j].val = vals[a + j];
      }
      len[i] = canon_row(rows[i], n, insert_mode);
    }
    build_block(B, m, rows, len);
    for (int64_t i = 0; i < m; ++i) free(rows[i]);
    free(rows); free(len);
  }
  return A;
}

or_mat *or_mat_create_coo(int64_t M, int64_t N, int P, const int64_t *coo_ptr,
                          const int64_t *rowsg, const int64_t *cols, const double *vals,
                          int insert_mode, int *err) {
  *err = 0;
  or_mat *A = mat_alloc(M, N, P);
  for (int r = 0; r < P; ++r) {
    int64_t r0 = A->ranges[r], m = A->ranges[r + 1] - r0;
    for (int64_t k = coo_ptr[r]; k < coo_ptr[r + 1]; ++k) {
      if (rowsg[k] < 0 || cols[k] < 0) continue;
      if (rowsg[k] < r0 || rowsg[k] >= r0 + m || cols[k] >= N) { *err = -1; or_mat_destroy(A); return NULL; }
    }
  }
  for (int r = 0; r < P; ++r) {
    or_block *B = &A->blk[r];
    int64_t r0 = A->ranges[r], m = A->ranges[r + 1] - r0;
    int64_t *cnt = (int64_t *)calloc((size_t)m + 1, sizeof(int64_t));
    for (int64_t k = coo_ptr[r]; k < coo_ptr[r + 1]; ++k)
      if (rowsg[k] >= 0 && cols[k] >= 0) cnt[rowsg[k] - r0]++;
    entry_t **rows = (entry_t **)malloc(((size_t)m + 1) * sizeof(entry_t *));
    int64_t *len = (int64_t *)calloc((size_t)m + 1, sizeof(int64_t));
    for (int64_t i = 0; i < m; ++i) rows[i] = (entry_t *)malloc((size_t)(cnt[i] ? cnt[i] : 1) * sizeof(entry_t));
    for (int64_t k = coo_ptr[r]; k < coo_ptr[r + 1]; ++k) {
      if (rowsg[k] < 0 || cols[k] < 0) continue;   /* MatSetValues skips negative indices */
      int64_t i = rowsg[k] - r0;
      entry_t *e = &rows[i][len[i]];
      e->col = cols[k]; e->pos = k; e->val = vals[k];
      len[i]++;
    }
    for (int64_t i = 0; i < m; ++i) len[i] = canon_row(rows[i], len[i], insert_mode);
    build_block(B, m, rows, len);
    for (int64_t i = 0; i < m; ++i) free(rows[i]);
    free(rows); free(len); free(cnt);
  }
  return A;
}

void or_mat_destroy(or_mat *A) {
  if (!A) return;
  for (int r = 0; r < A->P; ++r) {
    or_block *B = &A->blk[r];
    free(B->dptr); free(B->dcol); free(B->dval); free(B->optr); free(B->ocol);
    free(B->oval); free(B->garray); free(B->diag);
  }
  free(A->blk); free(A->ranges); free(A->cranges); free(A);
}

int64_t or_mat_nnz(const or_mat *A) {
  int64_t n = 0;
  for (int r = 0; r < A->P; ++r) n += A->blk[r].dptr[A->blk[r].m] + A->blk[r].optr[A->blk[r].m];
  return n;
}

/* MatGetRow_MPIAIJ: merges A_o (cols < cstart), A_d, A_o (cols >= cend) into
 * one globally sorted row -- what petsc4py's getValuesCSR returns. */
void or_mat_get_csr(const or_mat *A, int64_t *indptr, int64_t *cols, double *vals) {
  int64_t p = 0, row = 0;
  indptr[0] = 0;
  for (int r = 0; r < A->P; ++r) {
    const or_block *B = &A->blk[r];
    for (int64_t i = 0; i < B->m; ++i, ++row) {
      int64_t o = B->optr[i], oe = B->optr[i + 1];
      for (; o < oe && B->garray[B->ocol[o]] < B->cstart; ++o) { cols[p] = B->garray[B->ocol[o]]; vals[p++] = B->oval[o]; }
      for (int64_t d = B->dptr[i]; d < B->dptr[i + 1]; ++d) { cols[p] = B->dcol[d] + B->cstart; vals[p++] = B->dval[d]; }
      for (; o < oe; ++o) { cols[p] = B->garray[B->ocol[o]]; vals[p++] = B->oval[o]; }
      indptr[row + 1] = p;
    }
  }
}

void or_mat_block_sizes(const or_mat *A, int r, int64_t *m, int64_t *nnz_d, int64_t *nnz_o,
                        int64_t *nghost) {
  const or_block *B = &A->blk[r];
  *m = B->m; *nnz_d = B->dptr[B->m]; *nnz_o = B->optr[B->m]; *nghost = B->nghost;
}

void or_mat_get_block(const or_mat *A, int r, int64_t *dptr, int32_t *dcol, double *dval,
                      int64_t *optr, int32_t *ocol, double *oval, int64_t *garray) {
  const or_block *B = &A->blk[r];
  memcpy(dptr, B->dptr, ((size_t)B->m + 1) * sizeof(int64_t));
  memcpy(optr, B->optr, ((size_t)B->m + 1) * sizeof(int64_t));
  memcpy(dcol, B->dcol, (size_t)B->dptr[B->m] * sizeof(int32_t));
  memcpy(dval, B->dval, (size_t)B->dptr[B->m] * sizeof(double));
  memcpy(ocol, B->ocol, (size_t)B->optr[B->m] * sizeof(int32_t));
  memcpy(oval, B->oval, (size_t)B->optr[B->m] * sizeof(double));
  memcpy(garray, B->garray, (size_t)B->nghost * sizeof(int64_t));
}

/* ------------------------------------------------------------------------ */
/* MatMult_MPIAIJ: VecScatter x -> lvec; y = A_d x (MatMult_SeqAIJ: per row, */
/* sum = 0, sum += a_j * x_cj in ascending column order); y += A_o lvec      */
/* (MatMultAdd_SeqAIJ: sum = y_i, then the same sequential loop).  Inode     */
/* routines are not used: PETSc disables them when it finds > 0.8 m nodes,   */
/* which holds for every pattern in scope (no two consecutive rows alike).   */
/* ------------------------------------------------------------------------ */

static void block_mult(const or_mat *A, int r, const double *x, double *y) {
  const or_block *B = &A->blk[r];
  const double *xl = x + B->cstart;
  double *yl = y + B->rstart;
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < B->m; ++i) {
    double sum = 0.0;
    for (int64_t j = B->dptr[i]; j < B->dptr[i + 1]; ++j) sum += B->dval[j] * xl[B->dcol[j]];
    for (int64_t j = B->optr[i]; j < B->optr[i + 1]; ++j) sum += B->oval[j] * x[B->garray[B->ocol[j]]];
    yl[i] = sum;
  }
}

void or_mat_mult(const or_mat *A, const double *x, double *y) {
  for (int r = 0; r < A->P; ++r) block_mult(A, r, x, y);
}

void or_mat_get_diagonal(const or_mat *A, double *d) {
  for (int r = 0; r < A->P; ++r) memcpy(d + A->blk[r].rstart, A->blk[r].diag, (size_t)A->blk[r].m * sizeof(double));
}

/* ------------------------------------------------------------------------ */
/* Vec kernels (VecDot/VecNorm = local sums + MPI_Allreduce: summed here per */
/* rank, ranks in order)                                                      */
/* ------------------------------------------------------------------------ */

static double vdot(const or_mat *A, const double *x, const double *y) {
  double tot = 0.0;
  for (int r = 0; r < A->P; ++r) {
    const or_block *B = &A->blk[r];
    double s = 0.0;
#pragma omp parallel for reduction(+ : s) schedule(static)
    for (int64_t i = B->rstart; i < B->rstart + B->m; ++i) s += x[i] * y[i];
    tot += s;
  }
  return tot;
}

static double vnorm(const or_mat *A, const double *x) { return sqrt(vdot(A, x, x)); }

/* VecAXPY: y += a x through BLAS daxpy */
static void vaxpy(int64_t n, double a, const double *x, double *y, int usefma) {
  if (a == 0.0) return;
  if (usefma) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) y[i] = fma(a, x[i], y[i]);
  } else {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) y[i] = y[i] + a * x[i];
  }
}

/* VecAYPX_Seq: y = x + a y (C loop; a == 0 copies, a == 1 is VecAXPY, a == -1 is x - y) */
static void vaypx(int64_t n, double a, const double *x, double *y, int usefma) {
  if (a == 0.0) { memcpy(y, x, (size_t)n * sizeof(double)); return; }
  if (a == 1.0) { vaxpy(n, 1.0, x, y, usefma); return; }
  if (a == -1.0) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) y[i] = x[i] - y[i];
    return;
  }
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) y[i] = x[i] + a * y[i];
}

/* PCApply_Jacobi: y = dinv .* x */
static void pc_apply(int pc, int64_t n, const double *dinv, const double *x, double *y) {
  if (pc == OR_PC_JACOBI) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) y[i] = x[i] * dinv[i];
  } else {
    memcpy(y, x, (size_t)n * sizeof(double));
  }
}

/* VecMAXPY_Seq: the first nv%4 vectors in one PetscKernelAXPY{,2,3} pass, then
 * groups of four, each group U += ((a0 p0 + a1 p1) + a2 p2) + a3 p3. */
static void vmaxpy(int64_t n, int nv, const double *alpha, double *const *V, double *y) {
  int rem = nv & 3;
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) {
    double u = y[i];
    int j = 0;
    if (rem == 1) { u = alpha[0] * V[0][i] + u; j = 1; }
    else if (rem == 2) { u = u + (alpha[0] * V[0][i] + alpha[1] * V[1][i]); j = 2; }
    else if (rem == 3) { u = u + ((alpha[0] * V[0][i] + alpha[1] * V[1][i]) + alpha[2] * V[2][i]); j = 3; }
    for (; j < nv; j += 4)
      u = u + (((alpha[j] * V[j][i] + alpha[j + 1] * V[j + 1][i]) + alpha[j + 2] * V[j + 2][i]) + alpha[j + 3] * V[j + 3][i]);
    y[i] = u;
  }
}

static void vscale(int64_t n, double a, double *x) {
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) x[i] = a * x[i];
}

/* ------------------------------------------------------------------------ */
/* KSP                                                                       */
/* ------------------------------------------------------------------------ */

enum {
  R_ITERATING = 0, R_CONVERGED_RTOL = 2, R_CONVERGED_ATOL = 3, R_CONVERGED_ITS = 4,
  R_DIVERGED_NULL = -2, R_DIVERGED_ITS = -3, R_DIVERGED_DTOL = -4, R_DIVERGED_BREAKDOWN = -5,
  R_DIVERGED_INDEFINITE_PC = -8, R_DIVERGED_NANORINF = -9, R_DIVERGED_INDEFINITE_MAT = -10
};

void or_ksp_default_params(or_ksp_params *p) {
  memset(p, 0, sizeof(*p));
  p->ksp_type = OR_KSP_GMRES; p->pc_type = OR_PC_JACOBI; p->norm_type = OR_NORM_DEFAULT;
  p->max_it = 10000; p->restart = 30; p->guess_nonzero = 0;
  p->rtol = 1e-5; p->atol = 1e-50; p->dtol = 1e5; p->haptol = 1e-30; p->breakdowntol = 0.1;
  p->axpy_fma = 1; p->nthreads = 1;
}

typedef struct { double rnorm0, ttol; } conv_t;

/* KSPConvergedDefault (n = iteration, rnorm = current norm). snorm0 is the
 * norm used for rnorm0 when the guess is nonzero (computed by the caller as
 * PETSc does: the preconditioned / natural / plain norm of b). */
static int converged(const or_ksp_params *p, conv_t *c, int n, double rnorm, int normtype,
                     int guess_zero, double snorm) {
  /* KSP_NORM_NONE installs KSPConvergedSkip: CONVERGED_ITS once n >= max_it */
  if (normtype == OR_NORM_NONE) return n >= p->max_it ? R_CONVERGED_ITS : R_ITERATING;
  if (n == 0) {
    if (!guess_zero) {
      if (snorm == 0.0) snorm = rnorm;
      c->rnorm0 = snorm;
    } else {
      c->rnorm0 = rnorm;
    }
    c->ttol = fmax(p->rtol * c->rnorm0, p->atol);
  }
  if (isnan(rnorm) || isinf(rnorm)) return R_DIVERGED_NANORINF;
  if (rnorm <= c->ttol) return rnorm < p->atol ? R_CONVERGED_ATOL : R_CONVERGED_RTOL;
  if (rnorm >= p->dtol * c->rnorm0) return R_DIVERGED_DTOL;
  return R_ITERATING;
}

static double *vnew(int64_t n) { return (double *)calloc((size_t)(n ? n : 1), sizeof(double)); }

/* KSP initial-norm helper for a nonzero guess (KSPConvergedDefault n == 0). */
static double rhs_norm(const or_mat *A, const or_ksp_params *p, const double *dinv,
                       const double *b, int normtype) {
  int64_t n = A->M;
  if (normtype == OR_NORM_UNPRECONDITIONED) return vnorm(A, b);
  double *z = vnew(n);
  pc_apply(p->pc_type, n, dinv, b, z);
  double s = (normtype == OR_NORM_NATURAL) ? sqrt(fabs(vdot(A, b, z))) : vnorm(A, z);
  free(z);
  return s;
}

/* KSPSolve_CG (Hestenes-Stiefel, src/ksp/ksp/impls/cg/cg.c), reached from
 * ksp.solve at test.py:50 under -ksp_type cg. */
static int solve_cg(const or_mat *A, const or_ksp_params *p, const double *dinv, const double *b,
                    double *x, or_ksp_result *res, double *hist) {
  int64_t n = A->M;
  int normtype = p->norm_type == OR_NORM_DEFAULT ? OR_NORM_PRECONDITIONED : p->norm_type;
  double *R = vnew(n), *Z = vnew(n), *P = vnew(n), *W = vnew(n);
  double dp = 0.0, beta = 0.0, betaold = 0.0, dpi = 0.0, dpiold = 0.0, a, bb;
  conv_t c = {0, 0};
  int reason = 0, i;
  int guess_zero = !p->guess_nonzero;
  res->its = 0;
  if (!guess_zero) {
    or_mat_mult(A, x, R);
    vaypx(n, -1.0, b, R, p->axpy_fma);       /* r <- b - Ax */
  } else {
    memcpy(R, b, (size_t)n * sizeof(double));
  }
  switch (normtype) {
  case OR_NORM_PRECONDITIONED: pc_apply(p->pc_type, n, dinv, R, Z); dp = vnorm(A, Z); break;
  case OR_NORM_UNPRECONDITIONED: dp = vnorm(A, R); break;
  case OR_NORM_NATURAL: pc_apply(p->pc_type, n, dinv, R, Z); beta = vdot(A, Z, R); dp = sqrt(fabs(beta)); break;
  default: dp = 0.0;
  }
  if (isnan(dp) || isinf(dp)) { reason = R_DIVERGED_NANORINF; goto done; }
  if (hist) hist[0] = dp;
  res->rnorm = dp;
  {
    double snorm = guess_zero ? 0.0 : rhs_norm(A, p, dinv, b, normtype);
    reason = converged(p, &c, 0, dp, normtype, guess_zero, snorm);
  }
  if (reason) goto done;
  if (normtype != OR_NORM_PRECONDITIONED && normtype != OR_NORM_NATURAL) pc_apply(p->pc_type, n, dinv, R, Z);
  if (normtype != OR_NORM_NATURAL) beta = vdot(A, Z, R);
  if (isnan(beta) || isinf(beta)) { reason = R_DIVERGED_NANORINF; goto done; }
  i = 0;
  do {
    res->its = i + 1;
    if (beta == 0.0) { reason = R_CONVERGED_ATOL; break; }
    else if (i > 0 && beta * betaold < 0.0) { reason = R_DIVERGED_INDEFINITE_PC; break; }
    if (!i) {
      memcpy(P, Z, (size_t)n * sizeof(double));
      bb = 0.0;
    } else {
      bb = beta / betaold;
      vaypx(n, bb, Z, P, p->axpy_fma);       /* p <- z + b p */
    }
    dpiold = dpi;
    or_mat_mult(A, P, W);                    /* w <- A p */
    dpi = vdot(A, P, W);
    if (isnan(dpi) || isinf(dpi)) { reason = R_DIVERGED_NANORINF; break; }
    betaold = beta;
    if (dpi == 0.0 || (i > 0 && ((dpi > 0) - (dpi < 0)) * ((dpiold > 0) - (dpiold < 0)) < 0)) {
      reason = R_DIVERGED_INDEFINITE_MAT; break;
    }
    a = beta / dpi;
    vaxpy(n, a, P, x, p->axpy_fma);          /* x <- x + a p */
    vaxpy(n, -a, W, R, p->axpy_fma);         /* r <- r - a w */
    if (normtype == OR_NORM_PRECONDITIONED) { pc_apply(p->pc_type, n, dinv, R, Z); dp = vnorm(A, Z); }
    else if (normtype == OR_NORM_UNPRECONDITIONED) dp = vnorm(A, R);
    else if (normtype == OR_NORM_NATURAL) { pc_apply(p->pc_type, n, dinv, R, Z); beta = vdot(A, Z, R); dp = sqrt(fabs(beta)); }
    else dp = 0.0;
    if (isnan(dp) || isinf(dp)) { res->rnorm = dp; reason = R_DIVERGED_NANORINF; break; }
    res->rnorm = dp;
    if (hist) hist[i + 1] = dp;
    reason = converged(p, &c, i + 1, dp, normtype, guess_zero, 0.0);
    if (reason) break;
    if (normtype != OR_NORM_PRECONDITIONED && normtype != OR_NORM_NATURAL) pc_apply(p->pc_type, n, dinv, R, Z);
    if (normtype != OR_NORM_NATURAL) beta = vdot(A, Z, R);
    if (isnan(beta) || isinf(beta)) { reason = R_DIVERGED_NANORINF; break; }
    i++;
  } while (i < p->max_it);
  if (!reason && i >= p->max_it) reason = R_DIVERGED_ITS;
done:
  res->reason = reason;
  free(R); free(Z); free(P); free(W);
  return 0;
}

/* KSPSolve_GMRES / KSPGMRESCycle with classical Gram-Schmidt, no refinement
 * (src/ksp/ksp/impls/gmres/gmres.c, borthog2.c), left preconditioning,
 * preconditioned residual norm. */
static int solve_gmres(const or_mat *A, const or_ksp_params *p, const double *dinv,
                       const double *b, double *x, or_ksp_result *res, double *hist) {
  int64_t n = A->M;
  int max_k = p->restart > 0 ? p->restart : 30;
  int ld = max_k + 2;
  double **VV = (double **)malloc(((size_t)max_k + 1) * sizeof(double *));
  for (int k = 0; k <= max_k; ++k) VV[k] = vnew(n);
  double *TEMP = vnew(n), *TMAT = vnew(n);
  double *hh = (double *)calloc((size_t)ld * (max_k + 1), sizeof(double));
  double *hes = (double *)calloc((size_t)ld * (max_k + 1), sizeof(double));
  double *grs = (double *)calloc((size_t)max_k + 2, sizeof(double));
  double *cc = (double *)calloc((size_t)max_k + 1, sizeof(double));
  double *ss = (double *)calloc((size_t)max_k + 1, sizeof(double));
  double *lhh = (double *)calloc((size_t)max_k + 1, sizeof(double));
#define HH(a, b) hh[(b) * ld + (a)]
#define HES(a, b) hes[(b) * ld + (a)]
  int reason = 0, its = 0, itcount = 0, guess_zero = !p->guess_nonzero;
  double ksp_rnorm = -1.0, gm_rnorm0 = 0.0;
  conv_t c = {0, 0};
  while (!reason) {
    /* KSPInitialResidual: vv0 = B (b - A x) */
    if (!guess_zero) {
      or_mat_mult(A, x, TMAT);
      memcpy(TEMP, b, (size_t)n * sizeof(double));
      vaxpy(n, -1.0, TMAT, TEMP, p->axpy_fma);
      pc_apply(p->pc_type, n, dinv, TEMP, VV[0]);
    } else {
      pc_apply(p->pc_type, n, dinv, b, VV[0]);
    }
    /* KSPGMRESCycle */
    int it = 0, hapend = 0;
    double resn = vnorm(A, VV[0]), tt;
    if (resn != 0.0) vscale(n, 1.0 / resn, VV[0]);       /* VecNormalize */
    if (isnan(resn) || isinf(resn)) { reason = R_DIVERGED_NANORINF; break; }
    if (ksp_rnorm > 0.0 && fabs(resn - ksp_rnorm) > p->breakdowntol * gm_rnorm0) {
      reason = R_DIVERGED_BREAKDOWN; break;
    }
    grs[0] = gm_rnorm0 = resn;
    ksp_rnorm = resn;
    if (hist && its == 0) hist[0] = resn;
    if (resn == 0.0) { reason = R_CONVERGED_ATOL; break; }
    {
      double snorm = (its == 0 && !guess_zero) ? rhs_norm(A, p, dinv, b, OR_NORM_PRECONDITIONED) : 0.0;
      reason = converged(p, &c, its, resn, OR_NORM_PRECONDITIONED, its == 0 ? guess_zero : 1, snorm);
    }
    while (!reason && it < max_k && its < p->max_it) {
      /* KSP_PCApplyBAorAB: vv[it+1] = B A vv[it] */
      or_mat_mult(A, VV[it], TMAT);
      pc_apply(p->pc_type, n, dinv, TMAT, VV[it + 1]);
      /* KSPGMRESClassicalGramSchmidtOrthogonalization */
      for (int j = 0; j <= it; ++j) { HH(j, it) = 0.0; HES(j, it) = 0.0; }
      for (int j = 0; j <= it; ++j) lhh[j] = vdot(A, VV[it + 1], VV[j]);
      int bad = 0;
      for (int j = 0; j <= it; ++j) { if (isnan(lhh[j]) || isinf(lhh[j])) bad = 1; lhh[j] = -lhh[j]; }
      if (bad) { reason = R_DIVERGED_NANORINF; break; }
      vmaxpy(n, it + 1, lhh, VV, VV[it + 1]);
      for (int j = 0; j <= it; ++j) { HH(j, it) -= lhh[j]; HES(j, it) -= lhh[j]; }
      /* VecNormalize(vv[it+1]) */
      tt = vnorm(A, VV[it + 1]);
      if (tt != 0.0) vscale(n, 1.0 / tt, VV[it + 1]);
      if (isnan(tt) || isinf(tt)) { reason = R_DIVERGED_NANORINF; break; }
      HH(it + 1, it) = tt; HES(it + 1, it) = tt;
      double hapbnd = fabs(tt / grs[it]);
      if (hapbnd > p->haptol) hapbnd = p->haptol;
      if (tt < hapbnd) hapend = 1;
      /* KSPGMRESUpdateHessenberg */
      {
        double *h = &HH(0, it), *cp = cc, *sp = ss, t;
        for (int j = 1; j <= it; ++j) {
          t = *h;
          *h = (*cp) * t + (*sp) * h[1];
          h++;
          *h = (*cp++) * (*h) - ((*sp++) * t);
        }
        if (!hapend) {
          t = sqrt((*h) * (*h) + h[1] * h[1]);
          if (t == 0.0) { reason = R_DIVERGED_NULL; break; }
          cc[it] = *h / t;
          ss[it] = h[1] / t;
          grs[it + 1] = -(ss[it] * grs[it]);
          grs[it] = cc[it] * grs[it];
          *h = cc[it] * (*h) + ss[it] * h[1];
          resn = fabs(grs[it + 1]);
        } else {
          resn = 0.0;
        }
      }
      it++;
      its++;
      ksp_rnorm = resn;
      if (hist) hist[its] = resn;
      reason = converged(p, &c, its, resn, OR_NORM_PRECONDITIONED, 1, 0.0);
      if (hapend && !reason) { reason = R_DIVERGED_BREAKDOWN; break; }
    }
    /* KSPGMRESBuildSoln(GRS(0), x, x, ksp, it - 1) */
    if (it > 0 && reason != R_DIVERGED_NANORINF) {
      int last = it - 1;
      double *nrs = grs;
      if (HH(last, last) != 0.0) {
        nrs[last] = grs[last] / HH(last, last);
        int ok = 1;
        for (int ii = 1; ii <= last; ++ii) {
          int k = last - ii;
          double t = grs[k];
          for (int j = k + 1; j <= last; ++j) t = t - HH(k, j) * nrs[j];
          if (HH(k, k) == 0.0) { reason = R_DIVERGED_BREAKDOWN; ok = 0; break; }
          nrs[k] = t / HH(k, k);
        }
        if (ok) {
          memset(TEMP, 0, (size_t)n * sizeof(double));
          vmaxpy(n, last + 1, nrs, VV, TEMP);
          vaxpy(n, 1.0, TEMP, x, p->axpy_fma);
        }
      } else {
        reason = R_DIVERGED_BREAKDOWN;
      }
    }
    itcount += it;
    if (itcount >= p->max_it) { if (!reason) reason = R_DIVERGED_ITS; break; }
    guess_zero = 0;
  }
#undef HH
#undef HES
  res->its = its; res->reason = reason; res->rnorm = ksp_rnorm;
  for (int k = 0; k <= max_k; ++k) free(VV[k]);
  free(VV); free(TEMP); free(TMAT); free(hh); free(hes); free(grs); free(cc); free(ss); free(lhh);
  return 0;
}

int or_ksp_solve(const or_mat *A, const or_ksp_params *p, const double *b, double *x,
                 or_ksp_result *res, double *history) {
#ifdef _OPENMP
  omp_set_num_threads(p->nthreads > 0 ? p->nthreads : 1);
#endif
  int64_t n = A->M;
  memset(res, 0, sizeof(*res));
  /* PCSetUp_Jacobi: dinv = 1/diag, exact zero -> 1 */
  double *dinv = vnew(n);
  or_mat_get_diagonal(A, dinv);
  for (int64_t i = 0; i < n; ++i) dinv[i] = dinv[i] == 0.0 ? 1.0 : 1.0 / dinv[i];
  if (!p->guess_nonzero) memset(x, 0, (size_t)n * sizeof(double));
  int rc = 0;
  if (p->ksp_type == OR_KSP_CG) rc = solve_cg(A, p, dinv, b, x, res, history);
  else if (p->ksp_type == OR_KSP_GMRES) rc = solve_gmres(A, p, dinv, b, x, res, history);
  else if (p->ksp_type == OR_KSP_PREONLY) {   /* KSPSolve_PREONLY: x = B b, its = 1 */
    pc_apply(p->pc_type, n, dinv, b, x);
    res->its = 1; res->reason = R_CONVERGED_ITS;
  } else rc = -1;
  free(dinv);
  return rc;
}

/* ------------------------------------------------------------------------ */
/* Synthetic inputs                                           */
/* ------------------------------------------------------------------------ */

static double kappa(int64_t a, int64_t b, int64_t c) {
  int64_t t = ((a + 2 * b + 3 * c) % 4 + 4) % 4;
  return 1.0 + (double)t * 0.25;
}

int64_t or_stencil(int kind, int64_t nx, int64_t ny, int64_t nz, int64_t *indptr,
                   int64_t *cols, double *vals) {
  int64_t nrow = (kind == 0) ? nx * ny : nx * ny * nz;
  int64_t p = 0;
  if (indptr) indptr[0] = 0;
  for (int64_t row = 0; row < nrow; ++row) {
    int64_t i = row % nx, j = (row / nx) % ny, k = (kind == 0) ? 0 : row / (nx * ny);
    if (kind == 0) {
      int64_t nb[5][2] = {{0, -1}, {-1, 0}, {0, 0}, {1, 0}, {0, 1}};
      for (int t = 0; t < 5; ++t) {
        int64_t ii = i + nb[t][0], jj = j + nb[t][1];
        if (ii < 0 || ii >= nx || jj < 0 || jj >= ny) continue;
        if (indptr) { cols[p] = ii + nx * jj; vals[p] = (t == 2) ? 4.0 : -1.0; }
        p++;
      }
    } else if (kind == 1 || kind == 3) {
      int64_t nb[7][3] = {{0, 0, -1}, {0, -1, 0}, {-1, 0, 0}, {0, 0, 0}, {1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
      double diag = 0.0;
      if (kind == 3) {
        diag = kappa(i - 1, j, k) + kappa(i, j, k) + kappa(i, j - 1, k) + kappa(i, j, k) +
               kappa(i, j, k - 1) + kappa(i, j, k) + 0.5;
      }
      for (int t = 0; t < 7; ++t) {
        int64_t ii = i + nb[t][0], jj = j + nb[t][1], kk = k + nb[t][2];
        if (ii < 0 || ii >= nx || jj < 0 || jj >= ny || kk < 0 || kk >= nz) continue;
        if (indptr) {
          cols[p] = ii + nx * (jj + ny * kk);
          if (kind == 1) vals[p] = (t == 3) ? 6.0 : -1.0;
          else {
            double v;
            if (t == 3) v = diag;
            else {
              /* face between this cell and the neighbour; lower cell = min */
              int64_t la = i < ii ? i : ii, lb = j < jj ? j : jj, lc = k < kk ? k : kk;
              v = -kappa(la, lb, lc);
              if (t == 2) v = v - 0.5;   /* upwind convection, beta = 0.5 in +x */
            }
            vals[p] = v;
          }
        }
        p++;
      }
    } else {
      for (int dk = -1; dk <= 1; ++dk)
        for (int dj = -1; dj <= 1; ++dj)
          for (int di = -1; di <= 1; ++di) {
            int64_t ii = i + di, jj = j + dj, kk = k + dk;
            if (ii < 0 || ii >= nx || jj < 0 || jj >= ny || kk < 0 || kk >= nz) continue;
            if (indptr) {
              cols[p] = ii + nx * (jj + ny * kk);
              vals[p] = (di == 0 && dj == 0 && dk == 0) ? 26.0 : -1.0;
            }
            p++;
          }
    }
    if (indptr) indptr[row + 1] = p;
  }
  return p;
}

static uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

void or_rhs_hash(int64_t i0, int64_t n, double *b) {
  const uint64_t seed = 42ULL * 0x9E3779B97F4A7C15ULL;
  for (int64_t i = 0; i < n; ++i)
    b[i] = (double)(splitmix64((uint64_t)(i0 + i) + seed) >> 11) * 0x1.0p-53;
}

/* exported forms of the VecMAXPY_Seq restatement above and of VecMDot (plain
 * sequential sums: PETSc leaves the dot order to BLAS) */
void or_vec_maxpy(int64_t n, int nv, const double *alpha, double *const *x, double *y) { vmaxpy(n, nv, alpha, x, y); }

void or_vec_mdot(int64_t n, const double *x, int nv, const double *const *y, double *out) {
  for (int k = 0; k < nv; ++k) {
    double s = 0.0;
    for (int64_t i = 0; i < n; ++i) s += x[i] * y[k][i];
    out[k] = s;
  }
}
