// mx_ksp.hip -- KSPSolve on gfx950: CG, GMRES(restart) and PREONLY with Jacobi.
//
// Replaces ksp.solve(b, x) (test.py:50) under -ksp_type cg|gmres|preonly
// -pc_type jacobi|none.  The algorithms,
// scalar recurrences, stopping rule (KSPConvergedDefault) and breakdown checks
// are PETSc's, restated in oracle/petsc_oracle.c (solve_cg, solve_gmres,
// converged).
//
// MI355X design: the whole solve stays on the device.  Every scalar of the
// recurrence (alpha, beta, Hessenberg, Givens rotations, the convergence test
// and the KSPConvergedReason) lives in device memory and is updated by one
// thread right after the reduction that feeds it, so the host never waits on
// the GPU inside an iteration.  Kernels read a `done` flag and become no-ops
// once the solve has stopped; the host polls that flag every `poll_every`
// iterations one batch behind (the GPU never idles) and stops enqueueing.
// The iteration count is therefore exactly PETSc's.  With P > 1 each
// reduction is one ncclAllReduce of 1-3 (CG) or k+1 (GMRES MDot) doubles on
// the same stream, and the halo is the grouped send/recv of halo_begin().
//
// Fused vector passes (bytes per row of the CG iteration: SpMV + 88 B):
//   cg_p_kernel      z = d.*r recomputed, p = z + (beta/betaold) p   (r,d,p -> p)
//   SpMV + dot       w = A p and p.w partials in one pass
//   cg_update_kernel x += a p (fma), r -= a w (fma), z = d.*r, [z.z, z.r, r.r]
//   A uniform Jacobi diagonal (every d_i equal, e.g. constant-coefficient
//   stencils) is applied as one scalar: the same products bit for bit, 8 B per
//   row less per application (72 B/row instead of 88 B/row per CG iteration).
//   GMRES: SpMV with the Jacobi scaling fused, MDot of k+1 vectors in one pass,
//          MAXPY + norm in one pass.
#include <cmath>
#include <cstring>
#include <initializer_list>

#include "mx_device.hpp"
#include "mx_internal.hpp"

namespace mx {

enum {
  R_ITERATING = 0, R_CONVERGED_RTOL = 2, R_CONVERGED_ATOL = 3, R_CONVERGED_ITS = 4,
  R_DIVERGED_NULL = -2, R_DIVERGED_ITS = -3, R_DIVERGED_DTOL = -4, R_DIVERGED_BREAKDOWN = -5,
  R_DIVERGED_INDEFINITE_PC = -8, R_DIVERGED_NANORINF = -9, R_DIVERGED_INDEFINITE_MAT = -10
};

constexpr int MAX_RESTART = 1000;

// Device-resident solver state (one allocation, zeroed then parameterised).
struct KspState {
  double red[8];
  double beta, betaold, dpi, dpiold, alpha, dp, rnorm0, ttol;
  double rtol, atol, dtol, haptol, breakdowntol;
  double res, ksp_rnorm, gm_rnorm0, scale;
  int its, reason, done, max_it;
  int normtype, guess_zero, inner_stop, it;
  int itcount, max_k, nv, xi;
  // fused CG (SPMV_CG): {b, xa, xpend} read by the MatMult -- p_i = z + b p_{i-1},
  // x += xa p_{xi} pending while xpend != 0 (CgFuse::coef points at pb)
  double pb, xa, xpend;
};

// ------------------------------------------------------------------ shared scalar logic
__device__ __forceinline__ bool not_finite(double v) { return isnan(v) || isinf(v); }

// KSPConvergedDefault (KSPConvergedSkip when the norm type is NONE).
__device__ int dev_converged(KspState *s, int n, double rnorm, bool guess_zero, double snorm) {
  if (s->normtype == MX_NORM_NONE) return n >= s->max_it ? R_CONVERGED_ITS : R_ITERATING;
  if (n == 0) {
    if (!guess_zero) {
      if (snorm == 0.0) snorm = rnorm;
      s->rnorm0 = snorm;
    } else {
      s->rnorm0 = rnorm;
    }
    s->ttol = fmax(s->rtol * s->rnorm0, s->atol);
  }
  if (not_finite(rnorm)) return R_DIVERGED_NANORINF;
  if (rnorm <= s->ttol) return rnorm < s->atol ? R_CONVERGED_ATOL : R_CONVERGED_RTOL;
  if (rnorm >= s->dtol * s->rnorm0) return R_DIVERGED_DTOL;
  return R_ITERATING;
}

__device__ __forceinline__ void stop(KspState *s, int reason) {
  s->reason = reason;
  s->done = 1;
  s->inner_stop = 1;
}

// Either one thread after an all-reduce (P > 1), or a fused single block that
// first folds the per-block partials itself (P == 1, no collective between).
template <int NV>
__device__ __forceinline__ bool gather_red(KspState *s, const double *partials, int nblocks,
                                           bool fused) {
  if (fused) {
    for (int v = 0; v < NV; ++v) {
      const double t = block_sum_array(partials + (size_t)v * nblocks, nblocks);
      if (threadIdx.x == 0) s->red[v] = t;
    }
  }
  return threadIdx.x == 0;
}

// ------------------------------------------------------------------ PCSetUp_Jacobi
__global__ void jacobi_setup_kernel(int64_t n, const double *__restrict__ diag, double *__restrict__ dinv) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const double d = diag[i];
    dinv[i] = d == 0.0 ? 1.0 : 1.0 / d;   // zero diagonal entries use 1
  }
}

// per-block min / max of dinv and a flag for values that forbid the scalar
// form (non-finite, or a zero whose sign differs from d[0]); setup only
__global__ void __launch_bounds__(256) diag_range_kernel(int64_t n, const double *__restrict__ d,
                                                         double *__restrict__ out) {
  __shared__ double smin[256], smax[256], sbad[256];
  const double d0 = d[0];
  double lo = d0, hi = d0, bad = 0.0;
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    const double v = d[i];
    if (isnan(v) || isinf(v)) bad = 1.0;
    if (v == 0.0 && signbit(v) != signbit(d0)) bad = 1.0;
    lo = fmin(lo, v);
    hi = fmax(hi, v);
  }
  smin[threadIdx.x] = lo; smax[threadIdx.x] = hi; sbad[threadIdx.x] = bad;
  __syncthreads();
  for (int s2 = 128; s2 > 0; s2 >>= 1) {
    if (threadIdx.x < s2) {
      smin[threadIdx.x] = fmin(smin[threadIdx.x], smin[threadIdx.x + s2]);
      smax[threadIdx.x] = fmax(smax[threadIdx.x], smax[threadIdx.x + s2]);
      sbad[threadIdx.x] = fmax(sbad[threadIdx.x], sbad[threadIdx.x + s2]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    out[3 * blockIdx.x] = smin[0]; out[3 * blockIdx.x + 1] = smax[0]; out[3 * blockIdx.x + 2] = sbad[0];
  }
}

// ------------------------------------------------------------------ CG kernels
// partials of [z.z, z.r, r.r] (z = d.*r) and, when b != null, the same of b
// for the nonzero-guess rnorm0 (KSPConvergedDefault n == 0).
template <int NV>
__global__ void __launch_bounds__(256) cg_norms_kernel(int64_t n, const double *__restrict__ r,
                                                      const double *__restrict__ b, const Jac jac,
                                                      double *__restrict__ partials) {
  double v[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) v[k] = 0.0;
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    const double ri = r[i];
    const double zi = papply(jac, ri, i);
    v[0] += zi * zi; v[1] += zi * ri; v[2] += ri * ri;
    if (NV == 6) {
      const double bi = b[i];
      const double zb = papply(jac, bi, i);
      v[3 % NV] += zb * zb; v[4 % NV] += bi * zb; v[5 % NV] += bi * bi;
    }
  }
  block_sum_to_partials<NV>(v, partials, gridDim.x);
}

// after the initial norms: dp, rnorm0/ttol, beta, checks for iteration 0
template <int NV>
__global__ void __launch_bounds__(256) cg_init_kernel(KspState *s, const double *partials, int nblocks,
                                                      int fused, double *hist) {
  if (!gather_red<NV>(s, partials, nblocks, fused)) return;
  const double zz = s->red[0], zr = s->red[1], rr = s->red[2];
  double dp;
  switch (s->normtype) {
    case MX_NORM_PRECONDITIONED: dp = sqrt(zz); break;
    case MX_NORM_UNPRECONDITIONED: dp = sqrt(rr); break;
    case MX_NORM_NATURAL: dp = sqrt(fabs(zr)); break;
    default: dp = 0.0;
  }
  s->its = 0;
  s->beta = zr;
  s->dp = dp;
  if (hist) hist[0] = dp;
  if (not_finite(dp)) { stop(s, R_DIVERGED_NANORINF); return; }
  double snorm = 0.0;
  if (!s->guess_zero && NV == 6) {
    const double bz = s->red[3 % NV], bzr = s->red[4 % NV], bb = s->red[5 % NV];
    snorm = s->normtype == MX_NORM_UNPRECONDITIONED ? sqrt(bb)
            : s->normtype == MX_NORM_NATURAL        ? sqrt(fabs(bzr))
                                                    : sqrt(bz);
  }
  const int reason = dev_converged(s, 0, dp, s->guess_zero, snorm);
  if (reason) { stop(s, reason); return; }
  if (not_finite(s->beta)) { stop(s, R_DIVERGED_NANORINF); return; }
  s->its = 1;                                   // top of iteration 0
  s->pb = 0.0;                                  // i == 0: p = z
  if (s->beta == 0.0) { stop(s, R_CONVERGED_ATOL); return; }
}

// p = z + (beta/betaold) p  (i == 0: p = z), z = d.*r recomputed.  The
// iteration index comes from the device state (its = i + 1 at the top of
// iteration i), so every iteration is the same launch sequence (graph replay).
__global__ void cg_p_kernel(int64_t n, const KspState *__restrict__ s, const double *__restrict__ r,
                            const Jac jac, double *__restrict__ p) {
  if (s->done) return;
  const int i = s->its - 1;
  const double b = i == 0 ? 0.0 : s->beta / s->betaold;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += stride) {
    const double z = papply(jac, r[k], k);
    p[k] = (b == 0.0) ? z : z + b * p[k];       // VecAYPX_Seq (b == 0 copies)
  }
}

// cg_p_kernel plus the previous iteration's deferred x step, read from the
// same p_{i-1} before it is overwritten: x += xa p_{i-1}; p = z + b p_{i-1}
__global__ void cg_px_kernel(int64_t n, const KspState *__restrict__ s, const double *__restrict__ r,
                             const Jac jac, double *__restrict__ p, double *__restrict__ x) {
  if (s->done) return;
  const int i = s->its - 1;
  const double b = i == 0 ? 0.0 : s->beta / s->betaold;
  const bool xp = s->xpend != 0.0;
  const double a = s->xa;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += stride) {
    const double po = p[k];
    const double z = papply(jac, r[k], k);
    if (xp) x[k] = fma(a, po, x[k]);            // VecAXPY(X, a, P) of iteration i-1
    p[k] = (b == 0.0) ? z : z + b * po;         // VecAYPX_Seq (b == 0 copies)
  }
}

// dpi = p.w, indefiniteness checks, alpha = beta/dpi
// fused_cg: this iteration's MatMult has applied the pending x step; the
// step of this iteration becomes pending (applied by the next MatMult or by
// cg_finish_x_kernel) -- the same x += a p, one iteration later.
__global__ void __launch_bounds__(256) cg_alpha_kernel(KspState *s, const double *partials,
                                                       int nblocks, int fused, int fused_cg) {
  if (s->done) return;
  const int i = s->its - 1;
  if (!gather_red<1>(s, partials, nblocks, fused)) return;
  if (fused_cg) s->xpend = 0.0;
  s->dpiold = s->dpi;
  s->dpi = s->red[0];
  if (not_finite(s->dpi)) { stop(s, R_DIVERGED_NANORINF); return; }
  s->betaold = s->beta;
  const double dpi = s->dpi, dpo = s->dpiold;
  const int sg = (dpi > 0) - (dpi < 0), sgo = (dpo > 0) - (dpo < 0);
  if (dpi == 0.0 || (i > 0 && sg * sgo < 0)) { stop(s, R_DIVERGED_INDEFINITE_MAT); return; }
  s->alpha = s->beta / s->dpi;
  if (fused_cg) { s->xa = s->alpha; s->xpend = 1.0; s->xi = i; }
}

// x += a p, r -= a w (BLAS daxpy = fma), z = d.*r, partials [z.z, z.r, r.r]
__global__ void __launch_bounds__(256) cg_update_kernel(int64_t n, const KspState *__restrict__ s,
                                                        const double *__restrict__ p,
                                                        const double *__restrict__ w,
                                                        double *__restrict__ x, double *__restrict__ r,
                                                        const Jac jac, double *__restrict__ partials) {
  if (s->done) return;
  const double a = s->alpha;
  double v[3] = {0.0, 0.0, 0.0};
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    if (x) x[i] = fma(a, p[i], x[i]);            // x == null: deferred into the next MatMult
    const double ri = fma(-a, w[i], r[i]);
    r[i] = ri;
    const double zi = papply(jac, ri, i);
    v[0] += zi * zi; v[1] += zi * ri; v[2] += ri * ri;
  }
  block_sum_to_partials<3>(v, partials, gridDim.x);
}

// dp, history, convergence at its = i+1, beta for the next iteration
__global__ void __launch_bounds__(256) cg_conv_kernel(KspState *s, const double *partials,
                                                      int nblocks, int fused, double *hist) {
  if (s->done) return;
  const int i = s->its - 1;
  if (!gather_red<3>(s, partials, nblocks, fused)) return;
  const double zz = s->red[0], zr = s->red[1], rr = s->red[2];
  double dp;
  switch (s->normtype) {
    case MX_NORM_PRECONDITIONED: dp = sqrt(zz); break;
    case MX_NORM_UNPRECONDITIONED: dp = sqrt(rr); break;
    case MX_NORM_NATURAL: dp = sqrt(fabs(zr)); break;
    default: dp = 0.0;
  }
  s->dp = dp;
  if (not_finite(dp)) { stop(s, R_DIVERGED_NANORINF); return; }
  if (hist) hist[i + 1] = dp;
  const int reason = dev_converged(s, i + 1, dp, true, 0.0);
  if (reason) { stop(s, reason); return; }
  s->beta = zr;
  if (not_finite(zr)) { stop(s, R_DIVERGED_NANORINF); return; }
  if (i + 1 >= s->max_it) { stop(s, R_DIVERGED_ITS); return; }
  s->its = i + 2;                               // top of iteration i+1
  s->pb = s->beta / s->betaold;                 // VecAYPX coefficient of iteration i+1
  if (s->beta == 0.0) { stop(s, R_CONVERGED_ATOL); return; }
  if (s->beta * s->betaold < 0.0) { stop(s, R_DIVERGED_INDEFINITE_PC); return; }
}

// the x step still pending when the solve stopped (fused CG)
__global__ void cg_finish_x_kernel(int64_t n, const KspState *__restrict__ s, const double *__restrict__ p0,
                                   const double *__restrict__ p1, double *__restrict__ x) {
  if (s->xpend == 0.0) return;
  const double a = s->xa;
  const double *__restrict__ p = (s->xi & 1) ? p1 : p0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) x[i] = fma(a, p[i], x[i]);
}

// ------------------------------------------------------------------ GMRES kernels
__global__ void gm_resid_kernel(int64_t n, const double *__restrict__ b, const double *__restrict__ ax,
                                const Jac jac, double *__restrict__ v0) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const double t = ax ? fma(-1.0, ax[i], b[i]) : b[i];   // VecCopy + VecAXPY(-1)
    v0[i] = papply(jac, t, i);                               // PCApply
  }
}

__global__ void __launch_bounds__(256) sumsq_kernel(int64_t n, const double *__restrict__ x,
                                                    double *__restrict__ partials, const int *__restrict__ stop_flag) {
  if (stop_flag && *stop_flag) return;
  double v[1] = {0.0};
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) v[0] += x[i] * x[i];
  block_sum_to_partials<1>(v, partials, gridDim.x);
}

// cycle start: VecNormalize(vv0), restart consistency check, convergence test
__global__ void __launch_bounds__(256) gm_start_kernel(KspState *s, const double *partials, int nblocks,
                                                       int fused, double *grs, double *hist, double snorm) {
  if (!gather_red<1>(s, partials, nblocks, fused)) return;
  const double res = sqrt(s->red[0]);
  s->it = 0;
  s->res = res;
  s->scale = res != 0.0 ? 1.0 / res : 1.0;
  if (not_finite(res)) { stop(s, R_DIVERGED_NANORINF); return; }
  if (s->ksp_rnorm > 0.0 && fabs(res - s->ksp_rnorm) > s->breakdowntol * s->gm_rnorm0) {
    stop(s, R_DIVERGED_BREAKDOWN); return;
  }
  grs[0] = res;
  s->gm_rnorm0 = res;
  s->ksp_rnorm = res;
  if (hist && s->its == 0) hist[0] = res;
  if (res == 0.0) { stop(s, R_CONVERGED_ATOL); return; }
  const int reason = dev_converged(s, s->its, res, s->its == 0 ? s->guess_zero : true, snorm);
  if (reason) { stop(s, reason); return; }
  s->inner_stop = (s->its >= s->max_it) ? 1 : 0;
}

__global__ void scale_by_state_kernel(int64_t n, const KspState *__restrict__ s, double *__restrict__ x,
                                      int expect_it) {
  if (s->done && expect_it < 0) return;
  if (expect_it >= 0 && s->it != expect_it) return;
  if (s->res == 0.0 && expect_it < 0) return;
  const double a = s->scale;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) x[i] = a * x[i];
}

// VecMDot: h_j = w . v_j for j in [j0, j0+NV), one pass over w
template <int NV>
__global__ void __launch_bounds__(256) mdot_kernel(int64_t n, const double *__restrict__ w,
                                                   const double *__restrict__ V, int64_t ldv, int j0,
                                                   double *__restrict__ partials, const int *__restrict__ stop_flag) {
  if (*stop_flag) return;
  double acc[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) acc[k] = 0.0;
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    const double wi = w[i];
#pragma unroll
    for (int k = 0; k < NV; ++k) acc[k] += wi * V[(int64_t)(j0 + k) * ldv + i];
  }
  block_sum_to_partials<NV>(acc, partials + (size_t)j0 * gridDim.x, gridDim.x);
}

__global__ void __launch_bounds__(256) gm_orth_kernel(KspState *s, int k, double *red_k, double *lhh,
                                                      double *hh, int ld) {
  if (s->inner_stop) return;
  if (threadIdx.x != 0) return;
  for (int j = 0; j <= k; ++j) {
    if (not_finite(red_k[j])) { stop(s, R_DIVERGED_NANORINF); return; }
    lhh[j] = -red_k[j];
  }
  for (int j = 0; j <= k; ++j) hh[(size_t)k * ld + j] = 0.0 - lhh[j];
}

// VecMAXPY_Seq grouping (first nv%4 vectors, then groups of four), then ||w||^2
__global__ void __launch_bounds__(256) maxpy_norm_kernel(int64_t n, double *__restrict__ w,
                                                         const double *__restrict__ V, int64_t ldv, int nv,
                                                         const double *__restrict__ alpha,
                                                         double *__restrict__ partials,
                                                         const int *__restrict__ stop_flag) {
  if (*stop_flag) return;
  __shared__ double a[MAX_RESTART + 1];
  for (int j = threadIdx.x; j < nv; j += 256) a[j] = alpha[j];
  __syncthreads();
  const int rem = nv & 3;
  double v[1] = {0.0};
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    double u = w[i];
    int j = 0;
    if (rem == 1) { u = a[0] * V[i] + u; j = 1; }
    else if (rem == 2) { u = u + (a[0] * V[i] + a[1] * V[ldv + i]); j = 2; }
    else if (rem == 3) { u = u + ((a[0] * V[i] + a[1] * V[ldv + i]) + a[2] * V[2 * ldv + i]); j = 3; }
    for (; j < nv; j += 4)
      u = u + (((a[j] * V[(int64_t)j * ldv + i] + a[j + 1] * V[(int64_t)(j + 1) * ldv + i]) +
                a[j + 2] * V[(int64_t)(j + 2) * ldv + i]) + a[j + 3] * V[(int64_t)(j + 3) * ldv + i]);
    w[i] = u;
    v[0] += u * u;
  }
  block_sum_to_partials<1>(v, partials, gridDim.x);
}

// normalise vv[k+1], happy breakdown, KSPGMRESUpdateHessenberg, convergence
__global__ void __launch_bounds__(256) gm_step_kernel(KspState *s, int k, const double *partials, int nblocks,
                                                      int fused, double *hh, int ld, double *grs, double *cc,
                                                      double *ss, double *hist) {
  if (s->inner_stop) return;
  if (!gather_red<1>(s, partials, nblocks, fused)) return;
  const double tt = sqrt(s->red[0]);
  s->scale = tt != 0.0 ? 1.0 / tt : 1.0;
  if (not_finite(tt)) { stop(s, R_DIVERGED_NANORINF); return; }
  double *h = hh + (size_t)k * ld;   // column k
  h[k + 1] = tt;
  double hapbnd = fabs(tt / grs[k]);
  if (hapbnd > s->haptol) hapbnd = s->haptol;
  const bool hapend = tt < hapbnd;
  // apply the previous rotations to column k
  for (int j = 1; j <= k; ++j) {
    const double t = h[j - 1];
    h[j - 1] = cc[j - 1] * t + ss[j - 1] * h[j];
    h[j] = cc[j - 1] * h[j] - (ss[j - 1] * t);
  }
  double res;
  if (!hapend) {
    const double t = sqrt(h[k] * h[k] + h[k + 1] * h[k + 1]);
    if (t == 0.0) { stop(s, R_DIVERGED_NULL); return; }
    cc[k] = h[k] / t;
    ss[k] = h[k + 1] / t;
    grs[k + 1] = -(ss[k] * grs[k]);
    grs[k] = cc[k] * grs[k];
    h[k] = cc[k] * h[k] + ss[k] * h[k + 1];
    res = fabs(grs[k + 1]);
  } else {
    res = 0.0;
  }
  s->it = k + 1;
  s->its += 1;
  s->ksp_rnorm = res;
  s->res = tt;          // the scale kernel reads s->scale; res kept nonzero for it
  if (hist) hist[s->its] = res;
  int reason = dev_converged(s, s->its, res, true, 0.0);
  if (hapend && !reason) reason = R_DIVERGED_BREAKDOWN;
  if (reason) { stop(s, reason); return; }
  if (s->it >= s->max_k || s->its >= s->max_it) s->inner_stop = 1;
}

// KSPGMRESBuildSoln: back substitution into grs (in place)
__global__ void gm_buildsoln_kernel(KspState *s, const double *hh, int ld, double *grs) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  s->nv = 0;
  const int it = s->it - 1;
  if (it < 0 || s->reason == R_DIVERGED_NULL || s->reason == R_DIVERGED_NANORINF) return;
  if (s->reason == R_DIVERGED_BREAKDOWN && s->ksp_rnorm > 0.0 && s->it == 0) return;
#define HHd(a, b) hh[(size_t)(b) * ld + (a)]
  if (HHd(it, it) == 0.0) { s->reason = R_DIVERGED_BREAKDOWN; s->done = 1; return; }
  grs[it] = grs[it] / HHd(it, it);
  for (int ii = 1; ii <= it; ++ii) {
    const int k = it - ii;
    double t = grs[k];
    for (int j = k + 1; j <= it; ++j) t = t - HHd(k, j) * grs[j];
    if (HHd(k, k) == 0.0) { s->reason = R_DIVERGED_BREAKDOWN; s->done = 1; return; }
    grs[k] = t / HHd(k, k);
  }
#undef HHd
  s->nv = it + 1;
}

// x += sum_j nrs_j v_j  (VecMAXPY from zero, then VecAXPY(x, 1, TEMP))
__global__ void __launch_bounds__(256) gm_update_x_kernel(int64_t n, const KspState *__restrict__ s,
                                                          const double *__restrict__ V, int64_t ldv,
                                                          const double *__restrict__ nrs, double *__restrict__ x) {
  const int nv = s->nv;
  if (nv == 0) return;
  __shared__ double a[MAX_RESTART + 1];
  for (int j = threadIdx.x; j < nv; j += 256) a[j] = nrs[j];
  __syncthreads();
  const int rem = nv & 3;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    double u = 0.0;
    int j = 0;
    if (rem == 1) { u = a[0] * V[i] + u; j = 1; }
    else if (rem == 2) { u = u + (a[0] * V[i] + a[1] * V[ldv + i]); j = 2; }
    else if (rem == 3) { u = u + ((a[0] * V[i] + a[1] * V[ldv + i]) + a[2] * V[2 * ldv + i]); j = 3; }
    for (; j < nv; j += 4)
      u = u + (((a[j] * V[(int64_t)j * ldv + i] + a[j + 1] * V[(int64_t)(j + 1) * ldv + i]) +
                a[j + 2] * V[(int64_t)(j + 2) * ldv + i]) + a[j + 3] * V[(int64_t)(j + 3) * ldv + i]);
    x[i] = fma(1.0, u, x[i]);
  }
}

__global__ void gm_cycle_end_kernel(KspState *s) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  s->itcount += s->it;
  if (s->itcount >= s->max_it && !s->reason) s->reason = R_DIVERGED_ITS;
  if (s->reason) s->done = 1;
  s->guess_zero = 0;
}

// ------------------------------------------------------------------ host drivers
namespace {

struct Poller {
  hipStream_t st;
  int *pinned = nullptr;
  hipEvent_t ev[2];
  int pending = 0;  // batches enqueued
  explicit Poller(hipStream_t s) : st(s) {
    HIPCHECK(hipHostMalloc(reinterpret_cast<void **>(&pinned), 2 * sizeof(int), hipHostMallocDefault));
    pinned[0] = pinned[1] = 0;
    HIPCHECK(hipEventCreateWithFlags(&ev[0], hipEventDisableTiming));
    HIPCHECK(hipEventCreateWithFlags(&ev[1], hipEventDisableTiming));
  }
  ~Poller() {
    (void)hipStreamSynchronize(st);
    (void)hipHostFree(pinned);
    (void)hipEventDestroy(ev[0]);
    (void)hipEventDestroy(ev[1]);
  }
  // enqueue the flag copy for this batch; return true if the PREVIOUS batch saw done
  bool batch(const int *dev_done) {
    const int slot = pending & 1;
    HIPCHECK(hipMemcpyAsync(&pinned[slot], dev_done, sizeof(int), hipMemcpyDeviceToHost, st));
    HIPCHECK(hipEventRecord(ev[slot], st));
    ++pending;
    if (pending >= 2) {
      const int prev = (pending - 2) & 1;
      HIPCHECK(hipEventSynchronize(ev[prev]));
      if (pinned[prev]) return true;
    }
    return false;
  }
};

struct SpmvTimer {
  bool on = false;
  std::vector<hipEvent_t> ev;
  size_t used = 0;
  hipStream_t st;
  SpmvTimer(bool enable, hipStream_t s, int maxpairs) : on(enable), st(s) {
    if (!on) return;
    ev.resize(2 * (size_t)maxpairs);
    for (auto &e : ev) HIPCHECK(hipEventCreate(&e));
  }
  ~SpmvTimer() { for (auto &e : ev) (void)hipEventDestroy(e); }
  void begin() { if (on && used + 2 <= ev.size()) HIPCHECK(hipEventRecord(ev[used], st)); }
  void end() { if (on && used + 2 <= ev.size()) { HIPCHECK(hipEventRecord(ev[used + 1], st)); used += 2; } }
  void collect(double &ms, int &count) {
    ms = 0.0; count = 0;
    if (!on) return;
    HIPCHECK(hipStreamSynchronize(st));
    for (size_t k = 0; k + 1 < used; k += 2) {
      float t = 0.f;
      HIPCHECK(hipEventElapsedTime(&t, ev[k], ev[k + 1]));
      ms += t; count++;
    }
  }
};

struct Events {
  hipEvent_t a, b;
  Events() { HIPCHECK(hipEventCreate(&a)); HIPCHECK(hipEventCreate(&b)); }
  ~Events() { (void)hipEventDestroy(a); (void)hipEventDestroy(b); }
};

void init_state(KspState &h, const mx_ksp_params &p, int normtype) {
  std::memset(&h, 0, sizeof(h));
  h.rtol = p.rtol; h.atol = p.atol; h.dtol = p.dtol; h.haptol = p.haptol;
  h.breakdowntol = p.breakdowntol; h.max_it = p.max_it; h.normtype = normtype;
  h.guess_zero = !p.guess_nonzero; h.max_k = p.restart; h.ksp_rnorm = -1.0;
}

void read_state(hipStream_t st, const KspState *d, KspState &h) {
  HIPCHECK(hipMemcpyAsync(&h, d, sizeof(KspState), hipMemcpyDeviceToHost, st));
  HIPCHECK(hipStreamSynchronize(st));
}

}  // namespace

// KSPSetUp work space: one device allocation per operator, grown on demand
// and reused by later solves (no hipMalloc/hipFree inside a solve).
struct Carve {
  double *base;
  size_t off = 0;
  explicit Carve(double *b) : base(b) {}
  double *take(size_t n) { double *p = base + off; off += (n + 31) / 32 * 32; return p; }
};
static size_t carve_size(std::initializer_list<size_t> parts) {
  size_t t = 0;
  for (size_t n : parts) t += (n + 31) / 32 * 32;
  return t;
}
static double *workspace(Mat *A, size_t nd) {
  if (A->ksp_ws.n < nd) A->ksp_ws.alloc(nd);
  return A->ksp_ws.p;
}
static KspState *state_buf(Mat *A) {
  if (!A->ksp_state.p) A->ksp_state.alloc(sizeof(KspState));
  return reinterpret_cast<KspState *>(A->ksp_state.p);
}

static void cg_solve(Mat *A, const mx_ksp_params &p, const Jac dinv, const double *b, double *x,
                     mx_ksp_result &res, double *hist_host) {
  Comm *c = A->comm;
  hipStream_t st = c->stream;
  const int64_t n = A->m;
  const bool fused = c->size == 1 && !g_knobs.force_coll;
  int normtype = p.norm_type == MX_NORM_DEFAULT ? MX_NORM_PRECONDITIONED : p.norm_type;
  const size_t nv = (size_t)std::max<int64_t>(n, 1);
  const size_t npart = (size_t)std::max(spmv_blocks(A) + 64, RED_BLOCKS) * 6 + 64;
  const size_t nhist = hist_host ? (size_t)p.max_it + 2 : 1;
  Carve cv(workspace(A, carve_size({nv, nv, nv, nv, npart, nhist})));
  struct { double *p; } r{cv.take(nv)}, pv{cv.take(nv)}, w{cv.take(nv)}, part{cv.take(npart)}, hist{cv.take(nhist)};
  double *pv2 = cv.take(nv);   // fused CG: p_i alternates between pv (i even) and pv2
  struct { KspState *p; } sd{state_buf(A)};
  KspState hs;
  init_state(hs, p, normtype);
  HIPCHECK(hipMemcpyAsync(sd.p, &hs, sizeof(hs), hipMemcpyHostToDevice, st));
  Events ev;
  SpmvTimer timer(p.profile != 0, st, std::min(p.max_it, 4096));
  HIPCHECK(hipEventRecord(ev.a, st));

  // r = b - A x  (or b)
  if (p.guess_nonzero) {
    mat_mult(A, x, r.p);
    vec_aypx(st, n, -1.0, b, r.p);
  } else {
    vec_set(st, n, 0.0, x);
    HIPCHECK(hipMemcpyAsync(r.p, b, sizeof(double) * n, hipMemcpyDeviceToDevice, st));
  }
  KspState *s = sd.p;
  double *red = reinterpret_cast<double *>(s);   // red[] is the first member
  const int nv0 = p.guess_nonzero ? 6 : 3;
  if (nv0 == 6) cg_norms_kernel<6><<<RED_BLOCKS, 256, 0, st>>>(n, r.p, b, dinv, part.p);
  else cg_norms_kernel<3><<<RED_BLOCKS, 256, 0, st>>>(n, r.p, b, dinv, part.p);
  HIPCHECK(hipGetLastError());
  if (!fused) { finish_reduce(part.p, RED_BLOCKS, nv0, red, st); c->allreduce_sum(red, nv0); }
  if (nv0 == 6) cg_init_kernel<6><<<1, 256, 0, st>>>(s, part.p, RED_BLOCKS, fused, hist_host ? hist.p : nullptr);
  else cg_init_kernel<3><<<1, 256, 0, st>>>(s, part.p, RED_BLOCKS, fused, hist_host ? hist.p : nullptr);
  HIPCHECK(hipGetLastError());

  const int poll = p.poll_every > 0 ? p.poll_every : 16;
  Poller poller(st);
  int i = 0;
  const unsigned egrid = grid_for(n, 256, 8192);
  int *done = &s->done;
  double *hist_d = hist_host ? hist.p : nullptr;
  // fused: the direction update and the previous x step ride in the MatMult
  // (SPMV_CG); p ping-pongs between two buffers since neighbours read p_{i-1}
  // 1: direction update + x step inside the MatMult (SPMV_CG)
  // 2: x step deferred into the next direction update (cg_px_kernel)
  // 3 (auto): 1 while r and p of the rank fit the 256 MB MALL (measured:
  // -14% per iteration at 128^3, -8% at 64^3), else 0 (at 256^3 the
  // two-vector gathers of mode 1 overflow the per-XCD L2, +10%, and mode 2's
  // saved pass is repaid by a slower MatMult behind its two-vector writes)
  const int fmode = g_knobs.cg_fuse == 3 ? (n <= (int64_t(8) << 20) ? 1 : 0) : g_knobs.cg_fuse;
  const bool fuse_cg = fmode == 1;
  const bool defer_x = fmode != 0;
  // p_{-1} = -0.0: iteration 0's z + (+0)(-0) is exactly z (VecCopy)
  if (fuse_cg) vec_set(st, n, -0.0, pv2);
  auto iteration = [&](int it) {
    int nb_spmv;
    if (fuse_cg) {
      CgFuse cg;
      cg.r = r.p; cg.pold = (it & 1) ? pv.p : pv2; cg.pnew = (it & 1) ? pv2 : pv.p;
      cg.x = x; cg.coef = &s->pb; cg.jac = dinv;
      timer.begin();
      nb_spmv = matmult_overlap(A, nullptr, w.p, SPMV_CG, Jac{}, part.p, done, &cg);
      timer.end();
    } else {
      if (defer_x) cg_px_kernel<<<egrid, 256, 0, st>>>(n, s, r.p, dinv, pv.p, x);
      else cg_p_kernel<<<egrid, 256, 0, st>>>(n, s, r.p, dinv, pv.p);
      timer.begin();
      nb_spmv = matmult_overlap(A, pv.p, w.p, SPMV_DOT, Jac{}, part.p, done);
      timer.end();
    }
    if (!fused) { finish_reduce(part.p, nb_spmv, 1, red, st, done); c->allreduce_sum(red, 1); }
    cg_alpha_kernel<<<1, 256, 0, st>>>(s, part.p, nb_spmv, fused, defer_x);
    const double *pcur = fuse_cg ? ((it & 1) ? pv2 : pv.p) : pv.p;
    cg_update_kernel<<<RED_BLOCKS, 256, 0, st>>>(n, s, pcur, w.p, defer_x ? nullptr : x, r.p, dinv, part.p);
    if (!fused) { finish_reduce(part.p, RED_BLOCKS, 3, red, st, done); c->allreduce_sum(red, 3); }
    cg_conv_kernel<<<1, 256, 0, st>>>(s, part.p, RED_BLOCKS, fused, hist_d);
    HIPCHECK(hipGetLastError());
  };
  // a captured batch must start on an even iteration when p ping-pongs
  bool graph = g_knobs.graph && c->capturable && !p.profile && (!fuse_cg || (poll & 1) == 0) &&
               !A->cg_graph_failed;
  std::vector<uintptr_t> key;
  if (graph) {
    key = {(uintptr_t)x, (uintptr_t)r.p, (uintptr_t)hist_d, (uintptr_t)dinv.mode, (uintptr_t)dinv.d, 0,
           (uintptr_t)poll, (uintptr_t)g_knobs.overlap, (uintptr_t)g_knobs.spmv_nt, (uintptr_t)g_knobs.spmv_grid,
           (uintptr_t)g_knobs.force_coll, (uintptr_t)fmode};
    std::memcpy(&key[5], &dinv.c, sizeof(double));
  }
  bool use_graph = graph && A->cg_graph && A->cg_key == key;
  // Eager until a graph for exactly this configuration exists: the first
  // batch of the first solve also warms every RCCL connection it uses, so the
  // capture that follows records only steady-state collective calls.
  for (; i < p.max_it;) {
    if (use_graph) {
      HIPCHECK(hipGraphLaunch(A->cg_graph, st));
      i += poll;
    } else {
      for (int k = 0; k < poll && i < p.max_it; ++k, ++i) iteration(i);
    }
    if (poller.batch(done)) break;
    if (graph && !use_graph && i < p.max_it) {
      if (A->cg_graph) { HIPCHECK(hipGraphExecDestroy(A->cg_graph)); A->cg_graph = nullptr; }
      // A capture that fails (a runtime or collective library that cannot
      // record some call) leaves the iterations un-run: drop the graph for
      // this operator and carry on eagerly from the same state.
      hipGraph_t g = nullptr;
      try {
        HIPCHECK(hipStreamBeginCapture(st, hipStreamCaptureModeRelaxed));
        for (int k = 0; k < poll; ++k) iteration(i + k);
        HIPCHECK(hipStreamEndCapture(st, &g));
        HIPCHECK(hipGraphInstantiate(&A->cg_graph, g, nullptr, nullptr, 0));
        HIPCHECK(hipGraphDestroy(g));
        A->cg_key = key;
        use_graph = true;
      } catch (const Error &) {
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(st, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone) {
          hipGraph_t junk = nullptr;
          (void)hipStreamEndCapture(st, &junk);
          if (junk) (void)hipGraphDestroy(junk);
        }
        if (g) (void)hipGraphDestroy(g);
        if (A->cg_graph) { (void)hipGraphExecDestroy(A->cg_graph); A->cg_graph = nullptr; }
        (void)hipGetLastError();
        A->cg_graph_failed = true;
        graph = false;
      }
    }
  }
  if (defer_x) {   // p is in place for mode 2: both buffer slots are pv
    cg_finish_x_kernel<<<egrid, 256, 0, st>>>(n, s, pv.p, fuse_cg ? pv2 : pv.p, x);
    HIPCHECK(hipGetLastError());
  }
  HIPCHECK(hipEventRecord(ev.b, st));
  read_state(st, s, hs);
  float ms = 0.f;
  HIPCHECK(hipEventElapsedTime(&ms, ev.a, ev.b));
  res.its = hs.its;
  res.reason = hs.reason;
  res.rnorm = hs.dp;
  res.solve_ms = ms;
  res.launched_its = i;
  timer.collect(res.spmv_ms, res.spmv_count);
  if (hist_host) HIPCHECK(hipMemcpy(hist_host, hist.p, sizeof(double) * ((size_t)hs.its + 1), hipMemcpyDeviceToHost));
}

template <int NV>
static void launch_mdot(hipStream_t st, int64_t n, const double *w, const double *V, int64_t ldv, int j0,
                        double *partials, const int *stop_flag) {
  mdot_kernel<NV><<<RED_BLOCKS, 256, 0, st>>>(n, w, V, ldv, j0, partials, stop_flag);
}

static void mdot(hipStream_t st, int64_t n, const double *w, const double *V, int64_t ldv, int nv,
                 double *partials, const int *stop_flag) {
  for (int j0 = 0; j0 < nv; j0 += 8) {
    const int k = std::min(8, nv - j0);
    switch (k) {
      case 1: launch_mdot<1>(st, n, w, V, ldv, j0, partials, stop_flag); break;
      case 2: launch_mdot<2>(st, n, w, V, ldv, j0, partials, stop_flag); break;
      case 3: launch_mdot<3>(st, n, w, V, ldv, j0, partials, stop_flag); break;
      case 4: launch_mdot<4>(st, n, w, V, ldv, j0, partials, stop_flag); break;
      case 5: launch_mdot<5>(st, n, w, V, ldv, j0, partials, stop_flag); break;
      case 6: launch_mdot<6>(st, n, w, V, ldv, j0, partials, stop_flag); break;
      case 7: launch_mdot<7>(st, n, w, V, ldv, j0, partials, stop_flag); break;
      default: launch_mdot<8>(st, n, w, V, ldv, j0, partials, stop_flag); break;
    }
    HIPCHECK(hipGetLastError());
  }
}

// per-value finish into out[] (one block per value), used for MDot (k+1 values)
__global__ void __launch_bounds__(256) finish_many_kernel(const double *__restrict__ partials, int nblocks,
                                                          double *__restrict__ out, const int *__restrict__ stop_flag) {
  if (*stop_flag) return;
  const double t = block_sum_array(partials + (size_t)blockIdx.x * nblocks, nblocks);
  if (threadIdx.x == 0) out[blockIdx.x] = t;
}

static void gmres_solve(Mat *A, const mx_ksp_params &p, const Jac dinv, const double *b, double *x,
                        mx_ksp_result &res, double *hist_host) {
  Comm *c = A->comm;
  hipStream_t st = c->stream;
  const int64_t n = A->m;
  const int max_k = p.restart > 0 ? p.restart : 30;
  if (max_k > MAX_RESTART) fail(MX_ERR_UNSUPPORTED, "GMRES restart above 1000");
  const int ld = max_k + 2;
  const int64_t ldv = (std::max<int64_t>(n, 1) + 31) / 32 * 32;
  const size_t nV = (size_t)ldv * (max_k + 1), nh = (size_t)ld * (max_k + 1);
  const size_t npart = (size_t)RED_BLOCKS * (max_k + 2) + (size_t)spmv_blocks(A) + 128;
  const size_t nhist = hist_host ? (size_t)p.max_it + 2 : 1;
  const size_t k1 = (size_t)max_k + 1, k2 = (size_t)max_k + 2;
  Carve cv(workspace(A, carve_size({nV, (size_t)ldv, nh, k2, k1, k1, k1, k2, npart, nhist})));
  struct B { double *p; size_t n; };
  B V{cv.take(nV), nV}, tmat{cv.take(ldv), (size_t)ldv}, hh{cv.take(nh), nh}, grs{cv.take(k2), k2},
      cc{cv.take(k1), k1}, ss{cv.take(k1), k1}, lhh{cv.take(k1), k1}, red{cv.take(k2), k2},
      part{cv.take(npart), npart}, hist{cv.take(nhist), nhist};
  HIPCHECK(hipMemsetAsync(hh.p, 0, sizeof(double) * hh.n, st));
  struct { KspState *p; } sd{state_buf(A)};
  KspState hs;
  init_state(hs, p, MX_NORM_PRECONDITIONED);
  if (p.norm_type != MX_NORM_DEFAULT && p.norm_type != MX_NORM_PRECONDITIONED)
    fail(MX_ERR_UNSUPPORTED, "GMRES with left preconditioning supports the preconditioned norm only");
  hs.max_k = max_k;
  HIPCHECK(hipMemcpyAsync(sd.p, &hs, sizeof(hs), hipMemcpyHostToDevice, st));
  KspState *s = sd.p;
  double *sred = reinterpret_cast<double *>(s);
  const bool fused = c->size == 1;
  double *hist_d = hist_host ? hist.p : nullptr;
  Events ev;
  SpmvTimer timer(p.profile != 0, st, std::min(p.max_it, 4096));
  HIPCHECK(hipEventRecord(ev.a, st));
  const unsigned egrid = grid_for(n, 256, 8192);
  if (!p.guess_nonzero) vec_set(st, n, 0.0, x);
  // snorm for a nonzero first guess: || B b ||
  double snorm = 0.0;
  if (p.guess_nonzero) {
    gm_resid_kernel<<<egrid, 256, 0, st>>>(n, b, nullptr, dinv, tmat.p);
    sumsq_kernel<<<RED_BLOCKS, 256, 0, st>>>(n, tmat.p, part.p, nullptr);
    finish_reduce(part.p, RED_BLOCKS, 1, red.p, st);
    c->allreduce_sum(red.p, 1);
    HIPCHECK(hipMemcpyAsync(&snorm, red.p, sizeof(double), hipMemcpyDeviceToHost, st));
    HIPCHECK(hipStreamSynchronize(st));
    snorm = std::sqrt(snorm);
  }
  int first = 1, launched = 0;
  int *istop = &s->inner_stop;
  while (true) {
    // KSPInitialResidual: vv0 = B (b - A x)
    if (first && !p.guess_nonzero) {
      gm_resid_kernel<<<egrid, 256, 0, st>>>(n, b, nullptr, dinv, V.p);
    } else {
      mat_mult(A, x, tmat.p);
      gm_resid_kernel<<<egrid, 256, 0, st>>>(n, b, tmat.p, dinv, V.p);
    }
    sumsq_kernel<<<RED_BLOCKS, 256, 0, st>>>(n, V.p, part.p, nullptr);
    if (!fused) { finish_reduce(part.p, RED_BLOCKS, 1, sred, st); c->allreduce_sum(sred, 1); }
    gm_start_kernel<<<1, 256, 0, st>>>(s, part.p, RED_BLOCKS, fused, grs.p, hist_d, first ? snorm : 0.0);
    scale_by_state_kernel<<<egrid, 256, 0, st>>>(n, s, V.p, -1);
    HIPCHECK(hipGetLastError());
    first = 0;
    for (int k = 0; k < max_k; ++k) {
      double *vk = V.p + (int64_t)k * ldv, *vk1 = V.p + (int64_t)(k + 1) * ldv;
      timer.begin();
      matmult_overlap(A, vk, vk1, dinv.mode ? SPMV_JACOBI : SPMV_PLAIN, dinv, nullptr, istop);
      timer.end();
      mdot(st, n, vk1, V.p, ldv, k + 1, part.p, istop);
      finish_many_kernel<<<k + 1, 256, 0, st>>>(part.p, RED_BLOCKS, red.p, istop);
      c->allreduce_sum(red.p, k + 1);
      gm_orth_kernel<<<1, 64, 0, st>>>(s, k, red.p, lhh.p, hh.p, ld);
      maxpy_norm_kernel<<<RED_BLOCKS, 256, 0, st>>>(n, vk1, V.p, ldv, k + 1, lhh.p, part.p, istop);
      if (!fused) { finish_reduce(part.p, RED_BLOCKS, 1, sred, st, istop); c->allreduce_sum(sred, 1); }
      gm_step_kernel<<<1, 256, 0, st>>>(s, k, part.p, RED_BLOCKS, fused, hh.p, ld, grs.p, cc.p, ss.p, hist_d);
      scale_by_state_kernel<<<egrid, 256, 0, st>>>(n, s, vk1, k + 1);
      HIPCHECK(hipGetLastError());
      ++launched;
    }
    gm_buildsoln_kernel<<<1, 64, 0, st>>>(s, hh.p, ld, grs.p);
    gm_update_x_kernel<<<egrid, 256, 0, st>>>(n, s, V.p, ldv, grs.p, x);
    gm_cycle_end_kernel<<<1, 64, 0, st>>>(s);
    HIPCHECK(hipGetLastError());
    read_state(st, s, hs);
    if (hs.done) break;
  }
  HIPCHECK(hipEventRecord(ev.b, st));
  HIPCHECK(hipEventSynchronize(ev.b));
  float ms = 0.f;
  HIPCHECK(hipEventElapsedTime(&ms, ev.a, ev.b));
  res.its = hs.its;
  res.reason = hs.reason;
  res.rnorm = hs.ksp_rnorm;
  res.solve_ms = ms;
  res.launched_its = launched;
  timer.collect(res.spmv_ms, res.spmv_count);
  if (hist_host) HIPCHECK(hipMemcpy(hist_host, hist.p, sizeof(double) * ((size_t)hs.its + 1), hipMemcpyDeviceToHost));
}

void ksp_solve(Mat *A, const mx_ksp_params &p, const double *b, double *x, mx_ksp_result &r,
               double *hist) {
  std::memset(&r, 0, sizeof(r));
  if (A->M != A->N || A->m != A->n) fail(MX_ERR_UNSUPPORTED, "KSPSolve needs a square matrix with matching row/column layouts");
  if (p.max_it < 1) fail(MX_ERR_ARG, "max_it must be positive");
  hipStream_t st = A->comm->stream;
  const int64_t n = A->m;
  Jac dv;
  if (p.pc_type == MX_PC_JACOBI) {
    if (A->jac_mode < 0) {   // PCSetUp_Jacobi, once per operator
      A->jac_dinv.alloc((size_t)std::max<int64_t>(n, 1));
      A->jac_mode = 1;
      if (n) {
        jacobi_setup_kernel<<<grid_for(n, 256, 8192), 256, 0, st>>>(n, A->diag.p, A->jac_dinv.p);
        HIPCHECK(hipGetLastError());
        if (g_knobs.jac_const) {
          // uniform diagonal -> one scalar (same products bit for bit)
          constexpr int NB = 256;
          DBuf<double> mm(3 * NB);
          diag_range_kernel<<<NB, 256, 0, st>>>(n, A->jac_dinv.p, mm.p);
          HIPCHECK(hipGetLastError());
          std::vector<double> h(3 * NB);
          HIPCHECK(hipMemcpyAsync(h.data(), mm.p, sizeof(double) * 3 * NB, hipMemcpyDeviceToHost, st));
          HIPCHECK(hipStreamSynchronize(st));
          double lo = h[0], hi = h[1], bad = h[2];
          for (int b = 1; b < NB; ++b) { lo = std::fmin(lo, h[3 * b]); hi = std::fmax(hi, h[3 * b + 1]); bad = std::fmax(bad, h[3 * b + 2]); }
          if (bad == 0.0 && lo == hi) { A->jac_mode = 2; A->jac_c = lo; }
        }
      }
    }
    dv.mode = A->jac_mode;
    dv.d = A->jac_dinv.p;
    dv.c = A->jac_c;
  } else if (p.pc_type != MX_PC_NONE) {
    fail(MX_ERR_UNSUPPORTED, "unsupported PC type");
  }
  switch (p.ksp_type) {
    case MX_KSP_CG: cg_solve(A, p, dv, b, x, r, hist); break;
    case MX_KSP_GMRES: gmres_solve(A, p, dv, b, x, r, hist); break;
    case MX_KSP_PREONLY:   // KSPSolve_PREONLY: x = B b, its = 1, CONVERGED_ITS
      if (dv.mode) vec_pmult(st, n, b, A->jac_dinv.p, x);
      else if (n) HIPCHECK(hipMemcpyAsync(x, b, sizeof(double) * n, hipMemcpyDeviceToDevice, st));
      HIPCHECK(hipStreamSynchronize(st));
      r.its = 1; r.reason = R_CONVERGED_ITS;
      break;
    default: fail(MX_ERR_UNSUPPORTED, "unsupported KSP type");
  }
  HIPCHECK(hipStreamSynchronize(st));
}

}  // namespace mx
