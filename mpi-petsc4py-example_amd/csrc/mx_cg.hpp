// mx_cg.hpp -- device-resident Krylov state and the CG scalar recurrence
// shared by the CG kernels (mx_ksp.hip) and the CG-fused MatMult (mx_spmv.hip).
//
// KSPSolve_CG's scalar steps (PETSc src/ksp/ksp/impls/cg/cg.c, restated in
// oracle/petsc_oracle.c solve_cg) are evaluated at the START of the kernel
// that consumes them, by every workgroup from inputs no kernel of that launch
// writes, so no separate one-block scalar kernel sits between the vector
// passes:
//   * cg_top  (first kernel of iteration i >= 1): the end of iteration i-1 --
//     dp from [z.z, z.r, r.r], KSPConvergedDefault(n = i), beta_i = z.r, the
//     max_it test -- and the top of iteration i (beta == 0, indefinite PC),
//     giving b = beta_i / beta_{i-1};
//   * cg_alpha (the update pass of iteration i): dpi = p.w, the indefinite-
//     matrix test and alpha = beta_i / dpi.
// Workgroup 0 of the committing kernel writes the results; values read by the
// other workgroups of the same launch live in parity slots (beta and dpi by
// iteration parity, the iteration index in two fields written by alternate
// kernels), so the launch has no read/write race.
#pragma once

#include <hip/hip_runtime.h>

#include <cmath>

#include "mx_device.hpp"
#include "mxsolve.h"

namespace mx {

enum {
  R_ITERATING = 0, R_CONVERGED_RTOL = 2, R_CONVERGED_ATOL = 3, R_CONVERGED_ITS = 4,
  R_DIVERGED_NULL = -2, R_DIVERGED_ITS = -3, R_DIVERGED_DTOL = -4, R_DIVERGED_BREAKDOWN = -5,
  R_DIVERGED_INDEFINITE_PC = -8, R_DIVERGED_NANORINF = -9, R_DIVERGED_INDEFINITE_MAT = -10
};

// What every workgroup of a CG iteration's first kernel reads (cg_top), kept
// together so one batch of scalar loads brings it in.
struct CgTopIn {
  int done, it_u, normtype, max_it;
  double red3[3];           // [z.z, z.r, r.r] of the last update pass (folded, all-reduced)
  double betas[2];          // parity slots: beta_i in betas[i & 1]
  double ttol, atol, dtol, rnorm0;
  double xa, xpend;         // deferred x step (CG modes 1/2): x += xa p_{xi} while xpend != 0
  // mode 2 with batched x steps (knob 29 = B > 1): the steps of directions
  // [xlo, xhi) are pending, alpha_j in xal[j % B], p_j in buffer j % B
  double xal[8];
  int xlo, xhi;
};

// Device-resident solver state (one allocation, zeroed then parameterised at
// every solve, which also clears the in-launch fold counters).
struct KspState {
  double red[8];
  double beta, betaold, dpi, dpiold, alpha, dp;
  double rtol, haptol, breakdowntol;
  double res, ksp_rnorm, gm_rnorm0, scale;
  int its, reason, inner_stop, it;
  int itcount, max_k, nv, xi;
  int guess_zero;
  long long t_start;        // wall_clock64() when the solve's first kernel ran (CG)
  int it_k;                 // current CG iteration, written by the iteration's first kernel
                            // (top.it_u: the next one, written by the update pass)
  double pb;
  double red1;              // CG p.w (folded, then all-reduced)
  double dpis[2];           // parity slots: dpi_i in dpis[i & 1]
  alignas(128) CgTopIn top;
  // in-launch fold counters (Fold, mx_device.hpp), one 256-B line each: the
  // p.w partials of the MatMult and the update pass's [z.z, z.r, r.r]
  alignas(256) unsigned fold_dot[9 * FOLD_STRIDE];
  alignas(256) unsigned fold_upd[9 * FOLD_STRIDE];
};

__device__ __forceinline__ bool not_finite(double v) { return isnan(v) || isinf(v); }

// PCApply_Jacobi by form (JM: 0 none, 1 vector d, 2 uniform scalar c)
template <int JM> __device__ __forceinline__ double jac1(double r, double d, double c) {
  if constexpr (JM == 1) return r * d;
  else if constexpr (JM == 2) return r * c;
  else return r;
}
// the direction update p = z + b p_{i-1} (VecAYPX_Seq; b == 0 copies z): one
// expression for every kernel that forms p (cg_pb_kernel, the fused
// direction + p.Ap pass), so they give the same bits; a multiply and an add
// (the library builds with -ffp-contract=off), as VecAYPX_Seq's loop
__device__ __forceinline__ double cg_dir(double z, double b, double po) { return (b == 0.0) ? z : z + b * po; }

struct CgTop {
  int i;          // iteration about to run
  int reason;     // != 0: the solve stops here
  int its;        // KSP its to report (i, or i + 1 for the top-of-iteration stops)
  bool logged;    // dp enters the residual history (finite dp)
  double dp, beta, b;
};

// End of iteration i-1 and top of iteration i, from red3 and the parity slots.
// The caller copies KspState::top first (one batch of scalar loads: the
// prologue's latency is paid by every workgroup generation of the launch).
__device__ __forceinline__ CgTop cg_top(const CgTopIn &in) {
  const int i = in.it_u, normtype = in.normtype, max_it = in.max_it;
  const double zz = in.red3[0], zr = in.red3[1], rr = in.red3[2];
  const double b0 = in.betas[0], b1 = in.betas[1];
  const double ttol = in.ttol, atol = in.atol, dtol = in.dtol, rnorm0 = in.rnorm0;
  CgTop t;
  t.i = i;
  t.reason = R_ITERATING;
  t.its = i + 1;
  t.logged = false;
  t.dp = 0.0;
  t.b = 0.0;
  t.beta = 0.0;
  if (i == 0) return t;                         // cg_init tested iteration 0; p = z
  double dp;
  switch (normtype) {
    case MX_NORM_PRECONDITIONED: dp = sqrt(zz); break;
    case MX_NORM_UNPRECONDITIONED: dp = sqrt(rr); break;
    case MX_NORM_NATURAL: dp = sqrt(fabs(zr)); break;
    default: dp = 0.0;
  }
  t.dp = dp;
  t.its = i;
  if (not_finite(dp)) { t.reason = R_DIVERGED_NANORINF; return t; }
  t.logged = true;
  // KSPConvergedDefault(n = i): rnorm0 / ttol were fixed at n == 0;
  // KSPConvergedSkip when the norm type is NONE
  int reason = R_ITERATING;
  if (normtype == MX_NORM_NONE) reason = i >= max_it ? R_CONVERGED_ITS : R_ITERATING;
  else if (dp <= ttol) reason = dp < atol ? R_CONVERGED_ATOL : R_CONVERGED_RTOL;
  else if (dp >= dtol * rnorm0) reason = R_DIVERGED_DTOL;
  if (reason) { t.reason = reason; return t; }
  t.beta = zr;
  if (not_finite(zr)) { t.reason = R_DIVERGED_NANORINF; return t; }
  if (i >= max_it) { t.reason = R_DIVERGED_ITS; return t; }
  t.its = i + 1;                                // top of iteration i
  const double bo = (i & 1) ? b0 : b1;          // beta_{i-1}
  t.b = zr / bo;                                // VecAYPX coefficient
  if (zr == 0.0) { t.reason = R_CONVERGED_ATOL; return t; }
  if (zr * bo < 0.0) { t.reason = R_DIVERGED_INDEFINITE_PC; return t; }
  return t;
}

// one thread of the committing kernel
__device__ __forceinline__ void cg_commit_top(KspState *s, const CgTop &t, double *hist) {
  s->it_k = t.i;
  if (t.i == 0) return;
  s->dp = t.dp;
  if (t.logged && hist) hist[t.i] = t.dp;
  s->its = t.its;
  if (t.reason) {
    s->reason = t.reason;
    s->top.done = 1;
    s->inner_stop = 1;
    return;
  }
  s->top.betas[t.i & 1] = t.beta;
  s->beta = t.beta;
  s->pb = t.b;
}

// The CG update pass's helpers, shared by cg_update_kernel (mx_ksp.hip) and
// CG mode 5's residual-update MatMult (mx_spmv_pair.hip).
__device__ __forceinline__ void stop(KspState *s, int reason) {
  s->reason = reason;
  s->top.done = 1;
  s->inner_stop = 1;
}

// Words of pinned host memory the CG kernels write with system-scope stores
// (Mat::poll_pinned): the done flag and the iteration count the host's poller
// spins on, and the result the tail pass publishes (no device-to-host copy).
enum { HW_DONE = 0, HW_PROGRESS = 1, HW_ITS = 2, HW_REASON = 3, HW_DP = 4 /* double: words 4-5 */, HW_TICKS = 6 /* int64: 6-7 */,
       HW_WORDS = 8 };

__device__ __forceinline__ void host_store(int *w, int v) {
  __hip_atomic_store(w, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// dpi = p.w (red1), the indefinite-matrix test, alpha = beta_i / dpi.
// Read-only; cg_update_kernel's workgroup 0 commits it.
struct CgAlpha { int i, reason; double dpi, alpha; };
__device__ __forceinline__ CgAlpha cg_alpha(const KspState *s, double dpi) {
  // every input loaded before the first branch
  const int i = s->it_k;
  const double d0 = s->dpis[0], d1 = s->dpis[1];
  const double b0 = s->top.betas[0], b1 = s->top.betas[1];
  CgAlpha a;
  a.i = i;
  a.reason = R_ITERATING;
  a.dpi = dpi;
  a.alpha = 0.0;
  if (not_finite(dpi)) { a.reason = R_DIVERGED_NANORINF; return a; }
  const double dpo = i > 0 ? ((i & 1) ? d0 : d1) : 0.0;     // dpi_{i-1}
  const int sg = (dpi > 0) - (dpi < 0), sgo = (dpo > 0) - (dpo < 0);
  if (dpi == 0.0 || (i > 0 && sg * sgo < 0)) { a.reason = R_DIVERGED_INDEFINITE_MAT; return a; }
  a.alpha = ((i & 1) ? b1 : b0) / dpi;                        // beta_i / dpi
  return a;
}

// workgroup 0, thread 0 of the update pass: commit alpha (or the stop), the
// deferred / batched x step bookkeeping and the host words
__device__ __forceinline__ void cg_commit_alpha(KspState *s, const CgAlpha &al, double pw, int xb, bool xu,
                                                int *hw) {
  s->dpi = al.dpi;
  s->red1 = pw;
  s->top.xpend = 0.0;            // a deferred step of i-1 was applied by this iteration's first kernel
  // batched x steps: this iteration's cg_pb applied [i - B, i) when i % B == 0
  // (also when this pass stops the solve, so the finish pass does not repeat them)
  if (xb > 1 && al.i % xb == 0) s->top.xlo = al.i;
  if (al.reason) {
    stop(s, al.reason);
    if (hw) host_store(hw + HW_DONE, 1);
  } else {
    if (hw) host_store(hw + HW_PROGRESS, al.i + 1);
    s->dpis[al.i & 1] = al.dpi;
    s->alpha = al.alpha;
    if (!xu) { s->top.xa = al.alpha; s->top.xpend = 1.0; s->xi = al.i; }
    if (xb > 1) {                // the step of direction i joins the pending batch
      s->top.xal[al.i % xb] = al.alpha;
      s->top.xhi = al.i + 1;
    }
    s->top.it_u = al.i + 1;
  }
}

}  // namespace mx
