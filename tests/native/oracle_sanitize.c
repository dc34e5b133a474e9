/* The CPU oracle (oracle/petsc_oracle.c) exercised under AddressSanitizer +
 * UndefinedBehaviorSanitizer (tests/test_cpu_sanitizers.py): every entry
 * point the parity tests use -- stencil generation, CSR and COO assembly with
 * duplicates (INSERT / ADD), empty and long rows, P-rank splits, MatMult,
 * CG / GMRES solves with and without Jacobi, MAXPY / MDot -- plus the
 * argument-error paths.  Exits nonzero on any wrong answer; the sanitizers
 * abort on any memory or UB error. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "petsc_oracle.h"

static int fails = 0;
#define CHECK(c, msg) do { if (!(c)) { printf("FAIL %s\n", msg); fails++; } } while (0)

static or_mat *stencil_mat(int kind, int64_t nx, int64_t ny, int64_t nz, int P, int64_t *M_out) {
  const int64_t nnz = or_stencil(kind, nx, ny, nz, NULL, NULL, NULL);
  const int64_t M = kind == 0 ? nx * ny : nx * ny * nz;
  int64_t *ip = malloc(sizeof(int64_t) * (M + 1)), *c = malloc(sizeof(int64_t) * nnz);
  double *v = malloc(sizeof(double) * nnz);
  or_stencil(kind, nx, ny, nz, ip, c, v);
  int err = 0;
  or_mat *A = or_mat_create_csr(M, M, P, ip, c, v, 0, &err);
  CHECK(A && err == 0, "stencil assembly");
  free(ip); free(c); free(v);
  *M_out = M;
  return A;
}

static void solve_case(int kind, int64_t n, int P, int ksp, int pc) {
  int64_t M;
  or_mat *A = stencil_mat(kind, n, n, n, P, &M);
  double *b = malloc(sizeof(double) * M), *x = calloc((size_t)M, sizeof(double)), *r = malloc(sizeof(double) * M);
  or_rhs_hash(0, M, b);
  or_ksp_params p;
  or_ksp_default_params(&p);
  p.ksp_type = ksp; p.pc_type = pc; p.nthreads = 2;
  or_ksp_result res;
  double *hist = malloc(sizeof(double) * (p.max_it + 2));
  or_ksp_solve(A, &p, b, x, &res, hist);
  CHECK(res.reason > 0, "solve converged");
  or_mat_mult(A, x, r);
  double rn = 0, bn = 0;
  for (int64_t i = 0; i < M; ++i) { rn += (b[i] - r[i]) * (b[i] - r[i]); bn += b[i] * b[i]; }
  CHECK(sqrt(rn / bn) < 1e-3, "true residual");
  free(b); free(x); free(r); free(hist);
  or_mat_destroy(A);
}

int main(void) {
  /* stencils, every kind, P = 1 and 3 */
  for (int kind = 0; kind < 4; ++kind)
    for (int P = 1; P <= 3; P += 2) {
      int64_t M;
      or_mat *A = stencil_mat(kind, kind == 0 ? 17 : 7, kind == 0 ? 17 : 7, 7, P, &M);
      for (int r = 0; r < P; ++r) {
        int64_t m, nd, no, ng;
        or_mat_block_sizes(A, r, &m, &nd, &no, &ng);
        int64_t *dptr = malloc(sizeof(int64_t) * (m + 1)), *optr = malloc(sizeof(int64_t) * (m + 1));
        int32_t *dcol = malloc(sizeof(int32_t) * (nd + 1)), *ocol = malloc(sizeof(int32_t) * (no + 1));
        double *dval = malloc(sizeof(double) * (nd + 1)), *oval = malloc(sizeof(double) * (no + 1));
        int64_t *garray = malloc(sizeof(int64_t) * (ng + 1));
        or_mat_get_block(A, r, dptr, dcol, dval, optr, ocol, oval, garray);
        for (int64_t k = 1; k < ng; ++k) CHECK(garray[k] > garray[k - 1], "garray sorted");
        free(dptr); free(optr); free(dcol); free(ocol); free(dval); free(oval); free(garray);
      }
      or_mat_destroy(A);
    }
  /* CSR with duplicates, an empty row and a long row; INSERT and ADD */
  {
    const int64_t M = 6;
    int64_t ip[7] = {0, 3, 3, 4, 10, 12, 14};
    int64_t c[14] = {2, 0, 2, 1, 5, 4, 3, 2, 1, 0, 5, 5, 0, 4};
    double v[14] = {1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14};
    for (int mode = 0; mode < 2; ++mode) {
      int err = 0;
      or_mat *A = or_mat_create_csr(M, M, 2, ip, c, v, mode, &err);
      CHECK(A && !err, "dup assembly");
      const int64_t nnz = or_mat_nnz(A);
      int64_t *gp = malloc(sizeof(int64_t) * (M + 1)), *gc = malloc(sizeof(int64_t) * nnz);
      double *gv = malloc(sizeof(double) * nnz);
      or_mat_get_csr(A, gp, gc, gv);
      CHECK(gp[1] - gp[0] == 2, "row 0 dedup");
      CHECK(gv[1] == (mode ? 4.0 : 3.0), "row 0 col 2 insert/add");
      free(gp); free(gc); free(gv);
      or_mat_destroy(A);
    }
    int64_t bad[14];
    memcpy(bad, c, sizeof bad);
    bad[5] = 99;
    int err = 0;
    CHECK(or_mat_create_csr(M, M, 1, ip, bad, v, 0, &err) == NULL && err < 0, "column out of range");
  }
  /* COO across ranks, negative indices skipped */
  {
    int64_t ptr[3] = {0, 4, 7};
    int64_t r[7] = {0, 1, -1, 0, 3, 2, 3}, c[7] = {0, 1, 2, 0, 3, 2, 1};
    double v[7] = {1, 2, 3, 4, 5, 6, 7};
    int err = 0;
    or_mat *A = or_mat_create_coo(4, 4, 2, ptr, r, c, v, 1, &err);
    CHECK(A && !err, "coo assembly");
    double x[4] = {1, 1, 1, 1}, y[4];
    or_mat_mult(A, x, y);
    CHECK(y[0] == 5 && y[1] == 2 && y[2] == 6 && y[3] == 12, "coo mult");
    or_mat_destroy(A);
  }
  /* solves */
  solve_case(1, 12, 1, OR_KSP_CG, OR_PC_JACOBI);
  solve_case(1, 10, 3, OR_KSP_CG, OR_PC_NONE);
  solve_case(3, 9, 2, OR_KSP_GMRES, OR_PC_JACOBI);
  solve_case(2, 8, 1, OR_KSP_CG, OR_PC_JACOBI);
  /* MAXPY / MDot */
  {
    enum { N = 1000, NV = 7 };
    double *xs[NV], y[N], a[NV], out[NV];
    for (int k = 0; k < NV; ++k) {
      xs[k] = malloc(sizeof(double) * N);
      for (int i = 0; i < N; ++i) xs[k][i] = (double)((i * 7 + k) % 13) - 6.0;
      a[k] = 0.5 * (k + 1);
    }
    for (int i = 0; i < N; ++i) y[i] = 1.0;
    or_vec_maxpy(N, NV, a, xs, y);
    or_vec_mdot(N, y, NV, (const double *const *)xs, out);
    CHECK(isfinite(out[0]), "mdot finite");
    for (int k = 0; k < NV; ++k) free(xs[k]);
  }
  printf(fails ? "FAIL (%d)\n" : "OK\n", fails);
  return fails ? 1 : 0;
}
