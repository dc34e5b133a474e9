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
#include <type_traits>

#include "mx_cg.hpp"
#include "mx_device.hpp"
#include "mx_internal.hpp"
#include "mx_launch.hpp"

namespace mx {

constexpr int MAX_RESTART = 1000;
constexpr int64_t CG_FUSE_MAX_ROWS = int64_t(3) << 20;   // auto CG fusion: mode 1 up to here
constexpr int64_t CG_UNROLL_MAX_ROWS = int64_t(6) << 20;  // auto 4-step load batching up to here

// ------------------------------------------------------------------ shared scalar logic
// KSPConvergedDefault (KSPConvergedSkip when the norm type is NONE).
__device__ int dev_converged(KspState *s, int n, double rnorm, bool guess_zero, double snorm) {
  if (s->top.normtype == MX_NORM_NONE) return n >= s->top.max_it ? R_CONVERGED_ITS : R_ITERATING;
  if (n == 0) {
    if (!guess_zero) {
      if (snorm == 0.0) snorm = rnorm;
      s->top.rnorm0 = snorm;
    } else {
      s->top.rnorm0 = rnorm;
    }
    s->top.ttol = fmax(s->rtol * s->top.rnorm0, s->top.atol);
  }
  if (not_finite(rnorm)) return R_DIVERGED_NANORINF;
  if (rnorm <= s->top.ttol) return rnorm < s->top.atol ? R_CONVERGED_ATOL : R_CONVERGED_RTOL;
  if (rnorm >= s->top.dtol * s->top.rnorm0) return R_DIVERGED_DTOL;
  return R_ITERATING;
}

// The solver parameters a solve starts from (KspState's parameter fields).
struct KspInit {
  double rtol, atol, dtol, haptol, breakdowntol;
  int max_it, normtype, guess_zero, max_k;
};
// KspState for a new solve, written on the device (no host-to-device copy):
// zero everything -- which also clears the fold counters -- then the
// parameters; stamps the solve's start on the device clock.
__global__ void __launch_bounds__(256) ksp_state_init_kernel(KspState *__restrict__ s, const KspInit in) {
  auto *w = reinterpret_cast<unsigned long long *>(s);
  static_assert(sizeof(KspState) % 8 == 0, "KspState is cleared in 8-byte words");
  for (size_t k = threadIdx.x; k < sizeof(KspState) / 8; k += blockDim.x) w[k] = 0ull;
  __syncthreads();
  if (threadIdx.x != 0) return;
  s->t_start = wall_clock64();
  s->rtol = in.rtol; s->top.atol = in.atol; s->top.dtol = in.dtol; s->haptol = in.haptol;
  s->breakdowntol = in.breakdowntol; s->top.max_it = in.max_it; s->top.normtype = in.normtype;
  s->guess_zero = in.guess_zero; s->max_k = in.max_k; s->ksp_rnorm = -1.0;
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
// after the initial norms (red[0..NV)): dp, rnorm0/ttol, beta, checks for
// iteration 0; one thread
template <int NV>
__device__ void cg_init_body(KspState *s, double *hist);

// partials of [z.z, z.r, r.r] (z = d.*r) and, when NV == 6, the same of b
// for the nonzero-guess rnorm0 (KSPConvergedDefault n == 0).
// START (zero initial guess, unbatched x steps): one pass reads b and writes
// r = b and x = 0 (VecSet + VecCopy + the norms: 3 passes in one); batched x
// steps read b as r_0 and write nothing here.  Eight (NV 6: four) rows'
// loads per thread are issued together (the per-thread sum order is the plain strided loop's).
// fin.cnt != null (one rank): the last workgroup folds the partials in-launch
// into s->red and runs cg_init (no separate init launch).
template <int NV, bool START = false, bool XZERO = true>
__global__ void __launch_bounds__(256) cg_norms_kernel(int64_t n, const double *__restrict__ r,
                                                      const double *__restrict__ b, const Jac jac,
                                                      double *__restrict__ partials,
                                                      double *__restrict__ r_out, double *__restrict__ x_out,
                                                      const Fold fin, KspState *__restrict__ s,
                                                      double *__restrict__ hist) {
  double v[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) v[k] = 0.0;
  auto row = [&](double ri, double bi, int64_t i) {
    const double zi = papply(jac, ri, i);
    v[0] += zi * zi; v[1] += zi * ri; v[2] += ri * ri;
    if (NV == 6) {
      const double zb = papply(jac, bi, i);
      v[3 % NV] += zb * zb; v[4 % NV] += bi * zb; v[5 % NV] += bi * bi;
    }
  };
  const int64_t stride = (int64_t)gridDim.x * 256;
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  constexpr int U = NV == 6 ? 4 : 8;
  for (; i + (U - 1) * stride < n; i += U * stride) {
    double rr[U], bb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      rr[u] = START ? b[i + u * stride] : r[i + u * stride];
      bb[u] = NV == 6 ? b[i + u * stride] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if constexpr (START) {
        r_out[i + u * stride] = rr[u];
        if constexpr (XZERO) x_out[i + u * stride] = 0.0;
      }
      row(rr[u], bb[u], i + u * stride);
    }
  }
  for (; i < n; i += stride) {
    const double ri = START ? b[i] : r[i];
    if constexpr (START) {
      r_out[i] = ri;
      if constexpr (XZERO) x_out[i] = 0.0;
    }
    row(ri, NV == 6 ? b[i] : 0.0, i);
  }
  if (!fin.cnt) {
    block_sum_to_partials<NV>(v, partials, gridDim.x);
    return;
  }
  if (block_fold<NV>(v, partials, fin) && threadIdx.x == 0) cg_init_body<NV>(s, hist);
}

template <int NV>
__global__ void __launch_bounds__(256) cg_init_kernel(KspState *s, const double *partials, int nblocks,
                                                      int fused, double *hist) {
  if (gather_red<NV>(s, partials, nblocks, fused)) cg_init_body<NV>(s, hist);
}

template <int NV>
__device__ void cg_init_body(KspState *s, double *hist) {
  const double zz = s->red[0], zr = s->red[1], rr = s->red[2];
  double dp;
  switch (s->top.normtype) {
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
    snorm = s->top.normtype == MX_NORM_UNPRECONDITIONED ? sqrt(bb)
            : s->top.normtype == MX_NORM_NATURAL        ? sqrt(fabs(bzr))
                                                    : sqrt(bz);
  }
  const int reason = dev_converged(s, 0, dp, s->guess_zero, snorm);
  if (reason) { stop(s, reason); return; }
  if (not_finite(s->beta)) { stop(s, R_DIVERGED_NANORINF); return; }
  s->its = 1;                                   // top of iteration 0
  s->pb = 0.0;                                  // i == 0: p = z
  s->top.betas[0] = s->beta;
  s->top.it_u = 0;
  if (s->beta == 0.0) { stop(s, R_CONVERGED_ATOL); return; }
}

// ---- CG vector passes.  Rows go in pairs (16-B accesses when every vector
// is 16-B aligned, VEC; the same arithmetic on scalars otherwise), and each
// thread issues the loads of two pairs before the first use, so a workgroup
// keeps enough bytes in flight to stream at HBM rate.  Every row's result is
// the same expression as PETSc's loop; the order of the per-thread partial
// sums (update pass) is fixed by the pair walk, independent of VEC.
typedef double dbl2 __attribute__((ext_vector_type(2)));
template <bool VEC> __device__ __forceinline__ dbl2 ld2(const double *__restrict__ v, int64_t k) {
  if constexpr (VEC) return reinterpret_cast<const dbl2 *>(v)[k];
  else return dbl2{v[2 * k], v[2 * k + 1]};
}
template <bool VEC> __device__ __forceinline__ void st2(double *__restrict__ v, int64_t k, dbl2 t) {
  if constexpr (VEC) reinterpret_cast<dbl2 *>(v)[k] = t;
  else { v[2 * k] = t.x; v[2 * k + 1] = t.y; }
}
constexpr int CG_VEC_BLOCKS = 4096;   // grid of the paired vector passes (grid-stride)
constexpr int CG_MAX_VEC_GRID = 65536;  // cap on any vector-pass grid (partials buffer sizing)
// store flavour of the row walk (knob 14): plain, or non-temporal (streamed past the caches)
__device__ __forceinline__ void st1(double *q, double v, int nts) {
  if (nts) __builtin_nontemporal_store(v, q);
  else *q = v;
}

// p = z + b p  (i == 0: p = z), z = d.*r recomputed, b = beta_i / beta_{i-1}
// from the iteration's scalar top (cg_top), which this launch commits.  Every
// iteration is the same launch sequence (graph replay): the index comes from
// the device state.  XD: also the previous iteration's deferred x step, read
// from the same p_{i-1} before it is overwritten (mode 2).
template <int JM, bool XD, bool VEC>
__global__ void __launch_bounds__(256) cg_p_kernel(int64_t n, KspState *__restrict__ s, const double *__restrict__ r,
                                                   const double *__restrict__ dv, const double dc,
                                                   double *__restrict__ p, double *__restrict__ x,
                                                   double *__restrict__ hist, const int nts, const int unr) {
  const CgTopIn top = s->top;
  if (top.done) return;
  const CgTop t = cg_top(top);
  if (blockIdx.x == 0 && threadIdx.x == 0) cg_commit_top(s, t, hist);
  if (t.reason) return;
  const double b = t.b;
  const bool xp = XD && top.xpend != 0.0;
  const double a = top.xa;
  auto pnew = [&](double rr, double dd, double po) {
    const double z = jac1<JM>(rr, dd, dc);
    return (b == 0.0) ? z : z + b * po;          // VecAYPX_Seq (b == 0 copies; i == 0: b = 0)
  };
  auto xnew = [&](double po, double xx) { return fma(a, po, xx); };   // VecAXPY(X, a, P) of i-1
  if constexpr (!VEC) {          // row walk: one row per thread per step
    const int64_t stride = (int64_t)gridDim.x * 256;
    if (unr) {                   // knob 21: four steps' loads issued together
      int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
      for (; i + 3 * stride < n; i += 4 * stride) {
        double po[4], rr[4], dd[4], xx[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          po[u] = p[i + u * stride];
          rr[u] = r[i + u * stride];
          dd[u] = JM == 1 ? dv[i + u * stride] : 0.0;
          xx[u] = XD && xp ? x[i + u * stride] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          if (XD && xp) st1(x + i + u * stride, xnew(po[u], xx[u]), nts);
          st1(p + i + u * stride, pnew(rr[u], dd[u], po[u]), nts);
        }
      }
      for (; i < n; i += stride) {
        const double po = p[i];
        const double z = pnew(r[i], JM == 1 ? dv[i] : 0.0, po);
        if (XD && xp) st1(x + i, xnew(po, x[i]), nts);
        st1(p + i, z, nts);
      }
      return;
    }
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
      const double po = p[i];
      const double z = pnew(r[i], JM == 1 ? dv[i] : 0.0, po);
      if (XD && xp) st1(x + i, xnew(po, x[i]), nts);
      st1(p + i, z, nts);
    }
    return;
  }
  const int64_t np = n >> 1, stride = (int64_t)gridDim.x * 256;
  int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  for (; k < np; k += 2 * stride) {
    const int64_t k2 = k + stride;
    const bool two = k2 < np;
    const dbl2 r0 = ld2<VEC>(r, k), p0 = ld2<VEC>(p, k);
    const dbl2 d0 = JM == 1 ? ld2<VEC>(dv, k) : dbl2{0.0, 0.0};
    const dbl2 x0 = XD && xp ? ld2<VEC>(x, k) : dbl2{0.0, 0.0};
    dbl2 r1 = {0.0, 0.0}, p1 = {0.0, 0.0}, d1 = {0.0, 0.0}, x1 = {0.0, 0.0};
    if (two) {
      r1 = ld2<VEC>(r, k2); p1 = ld2<VEC>(p, k2);
      if (JM == 1) d1 = ld2<VEC>(dv, k2);
      if (XD && xp) x1 = ld2<VEC>(x, k2);
    }
    st2<VEC>(p, k, dbl2{pnew(r0.x, d0.x, p0.x), pnew(r0.y, d0.y, p0.y)});
    if (XD && xp) st2<VEC>(x, k, dbl2{xnew(p0.x, x0.x), xnew(p0.y, x0.y)});
    if (two) {
      st2<VEC>(p, k2, dbl2{pnew(r1.x, d1.x, p1.x), pnew(r1.y, d1.y, p1.y)});
      if (XD && xp) st2<VEC>(x, k2, dbl2{xnew(p1.x, x1.x), xnew(p1.y, x1.y)});
    }
  }
  if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {     // odd last row
    const int64_t i = n - 1;
    const double po = p[i];
    if (XD && xp) x[i] = xnew(po, x[i]);
    p[i] = pnew(r[i], JM == 1 ? dv[i] : 0.0, po);
  }
}

// Mode 2 with the x steps batched over B iterations (knob 29): direction p_i
// lives in buffer i % B, so p_{i-1} .. p_{i-B} are all still in memory when
// p_i is formed; every B-th iteration (i % B == 0) applies the B pending steps
// x = fma(a_{i-1}, p_{i-1}, ... fma(a_{i-B}, p_{i-B}, x)) -- the same FMAs in
// the same order as one VecAXPY per iteration -- before p_i overwrites p_{i-B}.
// x is read and written once per B iterations instead of every iteration.
#ifndef CG_X_NTS
#define CG_X_NTS 1   // batched x steps: x stored non-temporally (with knob 32 bit 0)
#endif
struct PBufs { double *b[8]; };
template <int JM, int B>
__global__ void __launch_bounds__(256) cg_pb_kernel(int64_t n, KspState *__restrict__ s, const double *__restrict__ r,
                                                    const double *__restrict__ dv, const double dc,
                                                    double *pb, const int64_t ps,
                                                    double *__restrict__ x, double *__restrict__ hist, const int unr,
                                                    const double *__restrict__ r0, double *__restrict__ npart,
                                                    const Fold fin) {
  const CgTopIn top = s->top;
  if (top.done) return;
  const CgTop t = cg_top(top);
  if (blockIdx.x == 0 && threadIdx.x == 0) cg_commit_top(s, t, hist);
  if (t.reason) return;
  const int i = t.i;
  const double b = t.b;
  // the B direction buffers lie ps doubles apart from pb (one carve): p_j in
  // buffer j % B at pb + (j % B) ps -- scalar arithmetic (an indexed pointer
  // array went through scratch and serialised the loop; eight pointer
  // arguments spilled SGPRs)
  auto pick = [&](int k) -> double * { return pb + k * ps; };
  auto row = [&](double rr, double dd, double po) { return cg_dir(jac1<JM>(rr, dd, dc), b, po); };
  const int64_t stride = (int64_t)gridDim.x * 256;
  int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  // the pending steps are exactly [i - B, i) when i % B == 0 (the update pass
  // keeps that invariant): p_{i-B+q} sits in buffer q, alpha in xal[q].  p_{i-B}
  // is read through the output pointer before p_i is stored over it, so every
  // pointer is distinct and __restrict__ holds
  if ((i % B) == 0 && top.xhi == i && top.xlo == i - B) {
    double al[B];
#pragma unroll
    for (int q = 0; q < B; ++q) al[q] = top.xal[q];
    // B = 8: the eight step lengths held in VGPRs (an empty asm pins them;
    // as SGPRs beside the eight buffer pointers they spilled)
    if constexpr (B == 8) {
#pragma unroll
      for (int q = 0; q < B; ++q) asm volatile("" : "+v"(al[q]));
    }
    // the first batch ([0, B)) of a zero-guess solve is x's first write: x
    // is the +0.0 the solve started from, so it is not read (nor zeroed at
    // the start); fma(a, p, +0.0) is what the read would have given
    const bool xz = top.xlo == 0 && s->guess_zero;
    double *__restrict__ pout = pb;
    const double *__restrict__ pprev = pick(B - 1);
    const double *__restrict__ p1 = pick(1), *__restrict__ p2 = pick(2), *__restrict__ p3 = pick(3);
    const double *__restrict__ p4 = pick(4), *__restrict__ p5 = pick(5), *__restrict__ p6 = pick(6);
    auto batch = [&](auto ntc) __attribute__((always_inline)) {   // non-temporal reads: see walk below
      constexpr bool NTL = decltype(ntc)::value;
      auto ldv = [&](const double *q) __attribute__((always_inline)) -> double {
        if constexpr (NTL) return __builtin_nontemporal_load(q);
        else return *q;
      };
      for (; k < n; k += stride) {
        const double po = ldv(pprev + k);
        double xx = fma(al[0], ldv(pout + k), xz ? 0.0 : ldv(x + k));   // x += a_{i-B} p_{i-B}, oldest first
        if constexpr (B >= 4) {
          xx = fma(al[1], ldv(p1 + k), xx);
          xx = fma(al[2], ldv(p2 + k), xx);
        }
        if constexpr (B == 8) {
          xx = fma(al[3], ldv(p3 + k), xx);
          xx = fma(al[4], ldv(p4 + k), xx);
          xx = fma(al[5], ldv(p5 + k), xx);
          xx = fma(al[6], ldv(p6 + k), xx);
        }
        // ... x += a_{i-1} p_{i-1}; x is next read B iterations on, so with
        // CG_X_NTS its store bypasses the memory-side cache (p_i keeps it)
        const double xn = fma(al[B - 1], po, xx);
        if constexpr (NTL && CG_X_NTS) __builtin_nontemporal_store(xn, x + k);
        else x[k] = xn;
        pout[k] = row(ldv(r + k), JM == 1 ? dv[k] : 0.0, po);
      }
    };
    if (unr & 2) batch(std::true_type{});
    else batch(std::false_type{});
    return;
  }
  const double *__restrict__ pprev = pick((i + B - 1) % B);   // p_{i-1} (unused at i = 0: b = 0)
  double *__restrict__ pout = pick(i % B);
  // unr bit 1 (knob 32): r and p_{i-1} read non-temporally, so the memory-side
  // cache keeps more of the p_i just written for the MatMult that reads it next
  // (rs: r, or b at iteration 0 of a zero-guess solve -- r_0 = b is not
  // copied into r at the start; iteration 0's update pass writes r_1.  Passed
  // as an argument so the common call keeps r's own aliasing facts)
  // NRM (iteration 0 of a zero-guess solve on one rank, fin.cnt set): the
  // initial norms [z.z, z.r, r.r] of r_0 = b ride in this pass -- the same
  // rows per thread in the same order as cg_norms_kernel on this grid, so the
  // same bits -- folded in-launch, the last workgroup running cg_init
  double nv[3] = {0.0, 0.0, 0.0};
  // NP (b == 0: iteration 0, or a restart of the direction): p_i = z, so
  // p_{i-1} is not read at all (VecAYPX_Seq with b == 0 copies) -- iteration
  // 0 of every solve used to stream the unused buffer (+20 us at 256^3)
  auto walk = [&](auto ntc, const double *__restrict__ rs, auto nrmc, auto npc) __attribute__((always_inline)) {
    constexpr bool NTL = decltype(ntc)::value;
    constexpr bool NRM = decltype(nrmc)::value;
    constexpr bool NP = decltype(npc)::value;
    auto ldv = [&](const double *q) __attribute__((always_inline)) -> double {
      if constexpr (NTL) return __builtin_nontemporal_load(q);
      else return *q;
    };
    auto norms = [&](double rr, double dd) __attribute__((always_inline)) {
      if constexpr (NRM) {
        const double z = jac1<JM>(rr, dd, dc);
        nv[0] += z * z; nv[1] += z * rr; nv[2] += rr * rr;
      }
    };
    if (unr & 1) {                               // four steps' loads issued together
      for (; k + 3 * stride < n; k += 4 * stride) {
        double po[4], rr[4], dd[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          po[u] = NP ? 0.0 : ldv(pprev + k + u * stride);
          rr[u] = ldv(rs + k + u * stride);
          dd[u] = JM == 1 ? dv[k + u * stride] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          pout[k + u * stride] = row(rr[u], dd[u], po[u]);
          norms(rr[u], dd[u]);
        }
      }
    }
    for (; k < n; k += stride) {
      const double rr = ldv(rs + k), dd = JM == 1 ? dv[k] : 0.0;
      pout[k] = row(rr, dd, NP ? 0.0 : ldv(pprev + k));
      norms(rr, dd);
    }
  };
  const std::true_type T{};
  const std::false_type F{};
  if (r0 && i == 0) {                            // (b == 0 at iteration 0)
    if (fin.cnt) {
      if (unr & 2) walk(T, r0, T, T);
      else walk(F, r0, T, T);
      if (block_fold<3>(nv, npart, fin) && threadIdx.x == 0) cg_init_body<3>(s, hist);
    } else if (unr & 2) walk(T, r0, F, T);
    else walk(F, r0, F, T);
  } else if (b == 0.0) {                          // wave-uniform
    if (unr & 2) walk(T, r, F, T);
    else walk(F, r, F, T);
  } else if (unr & 2) walk(T, r, F, F);
  else walk(F, r, F, F);
}

// x += a p, r -= a w (BLAS daxpy = fma), z = d.*r, [z.z, z.r, r.r] folded
// into red3 inside the launch.  XU false: the x step is deferred (modes 1/2:
// applied by the next iteration's first kernel, or by cg_finish_x_kernel).
template <int JM, bool XU, bool VEC>
__global__ void __launch_bounds__(256) cg_update_kernel(int64_t n, KspState *__restrict__ s,
                                                        const double *__restrict__ p,
                                                        const double *__restrict__ w,
                                                        double *__restrict__ x, double *__restrict__ r,
                                                        const double *__restrict__ dv, const double dc,
                                                        double *__restrict__ partials, const Fold fold,
                                                        const int nts, const double *__restrict__ dot_part,
                                                        const int ndot, const int unr, const int xb,
                                                        const double *__restrict__ r0, int *__restrict__ hw) {
  // the host's words (Poller): done, stored by every pass that finds the
  // solve stopped and by the pass that stops it; else the iterations begun
  if (s->top.done) {
    if (hw && blockIdx.x == 0 && threadIdx.x == 0) host_store(hw + HW_DONE, 1);
    return;
  }
  // p.w: folded and all-reduced before this launch, or (one rank) folded here
  // by every workgroup from the MatMult's partials, in fold_kernel's order
  const double pw = ndot > 0 ? block_sum_array<16>(dot_part, ndot) : s->red1;
  const CgAlpha al = cg_alpha(s, pw);
  if (blockIdx.x == 0 && threadIdx.x == 0) cg_commit_alpha(s, al, pw, xb, XU, hw);
  if (al.reason) return;
  const double a = al.alpha;
  double v[3] = {0.0, 0.0, 0.0};
  auto rnew = [&](double ww, double rr, double dd) {   // r - a w, then the partial sums
    const double ri = fma(-a, ww, rr);
    const double zi = jac1<JM>(ri, dd, dc);
    v[0] += zi * zi; v[1] += zi * ri; v[2] += ri * ri;
    return ri;
  };
  // rin: r_i -- r, or b at iteration 0 of a zero-guess solve (see cg_pb_kernel)
  auto body = [&](const double *__restrict__ rin) __attribute__((always_inline)) {
    if constexpr (!VEC) {          // row walk: one row per thread per step
      const int64_t stride = (int64_t)gridDim.x * 256;
      int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
      // unr bit 1 (knob 32): w and r read non-temporally, so the memory-side
      // cache keeps the r written here for the direction update that reads it
      auto walk = [&](auto ntc) __attribute__((always_inline)) {
        constexpr bool NTL = decltype(ntc)::value;
        auto ldv = [&](const double *q) __attribute__((always_inline)) -> double {
          if constexpr (NTL) return __builtin_nontemporal_load(q);
          else return *q;
        };
        if (unr & 1) {             // knob 21: four steps' loads issued together, same sum order
          for (; i + 3 * stride < n; i += 4 * stride) {
            double pp[4], xx[4], ww[4], rr[4], dd[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              ww[u] = ldv(w + i + u * stride);
              rr[u] = ldv(rin + i + u * stride);
              pp[u] = XU ? p[i + u * stride] : 0.0;
              xx[u] = XU ? x[i + u * stride] : 0.0;
              dd[u] = JM == 1 ? dv[i + u * stride] : 0.0;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              if (XU) st1(x + i + u * stride, fma(a, pp[u], xx[u]), nts);
              st1(r + i + u * stride, rnew(ww[u], rr[u], dd[u]), nts);
            }
          }
        }
        for (; i < n; i += stride) {
          if (XU) st1(x + i, fma(a, p[i], x[i]), nts);
          st1(r + i, rnew(ldv(w + i), ldv(rin + i), JM == 1 ? dv[i] : 0.0), nts);
        }
      };
      if (unr & 2) walk(std::true_type{});
      else walk(std::false_type{});
      return;
    }
    const int64_t np = n >> 1, stride = (int64_t)gridDim.x * 256;
    int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
    for (; k < np; k += 2 * stride) {
      const int64_t k2 = k + stride;
      const bool two = k2 < np;
      const dbl2 w0 = ld2<VEC>(w, k);
      const dbl2 r0v = ld2<VEC>(rin, k);
      const dbl2 p0 = XU ? ld2<VEC>(p, k) : dbl2{0.0, 0.0};
      const dbl2 x0 = XU ? ld2<VEC>(x, k) : dbl2{0.0, 0.0};
      const dbl2 d0 = JM == 1 ? ld2<VEC>(dv, k) : dbl2{0.0, 0.0};
      dbl2 w1 = {0.0, 0.0}, r1 = {0.0, 0.0}, p1 = {0.0, 0.0}, x1 = {0.0, 0.0}, d1 = {0.0, 0.0};
      if (two) {
        w1 = ld2<VEC>(w, k2); r1 = ld2<VEC>(rin, k2);
        if (XU) { p1 = ld2<VEC>(p, k2); x1 = ld2<VEC>(x, k2); }
        if (JM == 1) d1 = ld2<VEC>(dv, k2);
      }
      if (XU) st2<VEC>(x, k, dbl2{fma(a, p0.x, x0.x), fma(a, p0.y, x0.y)});
      {
        const double ra = rnew(w0.x, r0v.x, d0.x);
        const double rb = rnew(w0.y, r0v.y, d0.y);
        st2<VEC>(r, k, dbl2{ra, rb});
      }
      if (two) {
        if (XU) st2<VEC>(x, k2, dbl2{fma(a, p1.x, x1.x), fma(a, p1.y, x1.y)});
        const double ra = rnew(w1.x, r1.x, d1.x);
        const double rb = rnew(w1.y, r1.y, d1.y);
        st2<VEC>(r, k2, dbl2{ra, rb});
      }
    }
    if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {     // odd last row
      const int64_t i = n - 1;
      if (XU) x[i] = fma(a, p[i], x[i]);
      r[i] = rnew(w[i], rin[i], JM == 1 ? dv[i] : 0.0);
    }
  };
  if (r0 && al.i == 0) body(r0);
  else body(r);
  block_partials<3>(v, partials, gridDim.x, fold);
}

// one-block fold of per-workgroup partials (block_sum_array's order, the same
// bits as an in-launch fold)
template <int NV>
__global__ void __launch_bounds__(256) fold_kernel(const double *__restrict__ partials, int nblocks,
                                                   double *__restrict__ out, const int *__restrict__ done) {
  if (*done) return;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const double t = block_sum_array<16>(partials + (size_t)k * nblocks, nblocks);
    if (threadIdx.x == 0) out[k] = t;
  }
}

// the scalar top after the last launched iteration (max_it reached without a stop)
__global__ void cg_tail_kernel(KspState *s, double *hist, int *hw) {
  if (threadIdx.x != 0) return;
  const long long t_end = wall_clock64();   // the solve's last kernel: its device time ends here
  if (!s->top.done) cg_commit_top(s, cg_top(s->top), hist);
  // the result, straight into the host's words
  host_store(hw + HW_ITS, s->its);
  host_store(hw + HW_REASON, s->reason);
  const unsigned long long dp = __builtin_bit_cast(unsigned long long, s->dp);
  __hip_atomic_store(reinterpret_cast<unsigned long long *>(hw + HW_DP), dp, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(reinterpret_cast<long long *>(hw + HW_TICKS), t_end - s->t_start, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_SYSTEM);
}

// the x step still pending when the solve stopped (fused CG)
__global__ void cg_finish_x_kernel(int64_t n, const KspState *__restrict__ s, const double *__restrict__ p0,
                                   const double *__restrict__ p1, double *__restrict__ x) {
  if (s->top.xpend == 0.0) return;
  const double a = s->top.xa;
  const double *__restrict__ p = (s->xi & 1) ? p1 : p0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) x[i] = fma(a, p[i], x[i]);
}

// the batched x steps still pending when the solve stopped, oldest first
// (a zero-guess solve that stopped before its first batch has never written
// x: the pending steps start from +0.0, or x is set to 0 when there are none).
// The pending count picks a straight-line body (16-byte row pairs, the NP
// directions' pairs loaded together): round 4's generic loop over eight
// guarded pointers ran at 5.3 TB/s.
template <int NP>
__device__ __forceinline__ void finish_xb_rows(int64_t n, const double *pb, int64_t ps, int B, int j0, bool xz,
                                               const double *__restrict__ xal, double *__restrict__ x) {
  const double *p[NP];
  double a[NP];
#pragma unroll
  for (int q = 0; q < NP; ++q) {
    const int j = (j0 + q) % B;
    p[q] = pb + j * ps;
    a[q] = xal[j];
  }
  const int64_t n2 = n >> 1, stride = (int64_t)gridDim.x * blockDim.x;
  if (reinterpret_cast<uintptr_t>(x) & 15) {     // the caller's x off 16-byte alignment: one row per step
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
      double xx = xz ? 0.0 : x[i];
#pragma unroll
      for (int q = 0; q < NP; ++q) xx = fma(a[q], p[q][i], xx);
      x[i] = xx;
    }
    return;
  }
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n2; k += stride) {
    dbl2 t[NP];
#pragma unroll
    for (int q = 0; q < NP; ++q) t[q] = __builtin_nontemporal_load(reinterpret_cast<const dbl2 *>(p[q]) + k);
    dbl2 xx = xz ? dbl2{0.0, 0.0} : __builtin_nontemporal_load(reinterpret_cast<const dbl2 *>(x) + k);
#pragma unroll
    for (int q = 0; q < NP; ++q) xx = dbl2{fma(a[q], t[q].x, xx.x), fma(a[q], t[q].y, xx.y)};
    reinterpret_cast<dbl2 *>(x)[k] = xx;
  }
  if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {   // odd last row
    const int64_t i = n - 1;
    double xx = xz ? 0.0 : x[i];
#pragma unroll
    for (int q = 0; q < NP; ++q) xx = fma(a[q], p[q][i], xx);
    x[i] = xx;
  }
}

// pb: the B direction buffers, ps doubles apart (one carve, cg_solve)
__global__ void __launch_bounds__(256) cg_finish_xb_kernel(int64_t n, const KspState *__restrict__ s,
                                                           const double *pb, int64_t ps, int B,
                                                           double *__restrict__ x) {
  const int j0 = s->top.xlo, np = s->top.xhi - s->top.xlo;
  const bool xz = j0 == 0 && s->guess_zero;
  if (np <= 0) {
    if (xz) {
      const int64_t stride = (int64_t)gridDim.x * blockDim.x;
      for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) x[i] = 0.0;
    }
    return;
  }
  const double *xal = s->top.xal;
  switch (np) {
    case 1: finish_xb_rows<1>(n, pb, ps, B, j0, xz, xal, x); break;
    case 2: finish_xb_rows<2>(n, pb, ps, B, j0, xz, xal, x); break;
    case 3: finish_xb_rows<3>(n, pb, ps, B, j0, xz, xal, x); break;
    case 4: finish_xb_rows<4>(n, pb, ps, B, j0, xz, xal, x); break;
    case 5: finish_xb_rows<5>(n, pb, ps, B, j0, xz, xal, x); break;
    case 6: finish_xb_rows<6>(n, pb, ps, B, j0, xz, xal, x); break;
    case 7: finish_xb_rows<7>(n, pb, ps, B, j0, xz, xal, x); break;
    default: finish_xb_rows<8>(n, pb, ps, B, j0, xz, xal, x);
  }
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
                                                       int fused, double *grs, double *hist, double snorm,
                                                       double *vscale) {
  if (!gather_red<1>(s, partials, nblocks, fused)) return;
  const double res = sqrt(s->red[0]);
  s->it = 0;
  s->res = res;
  s->scale = res != 0.0 ? 1.0 / res : 1.0;
  vscale[0] = s->scale;       // VecNormalize(vv0), applied where vv0 is read
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
  s->inner_stop = (s->its >= s->top.max_it) ? 1 : 0;
}

// Basis-vector reads of MDot and MAXPY (GM_NTL): non-temporal, so the
// memory-side cache keeps w -- written by the MatMult and read by the MDot,
// then rewritten by the MAXPY and read by the next MatMult -- instead of the
// basis, which is far larger than that cache anyway
#ifndef GM_NTL
#define GM_NTL 1
#endif
__device__ __forceinline__ double gm_ld(const double *q) {
  if constexpr (GM_NTL) return __builtin_nontemporal_load(q);
  else return *q;
}

// VecMDot: h_j = w . v_j for j in [j0, j0 + nv), nv <= NV, one pass over w
// (restart 30: every step's k+1 dots in one launch)
// The basis vectors are stored unnormalised: v_j = vscale[j] * V_j, applied
// at every read (fl(a * x), the bits VecScale would have stored)
template <int NV>
__global__ void __launch_bounds__(256) mdot_kernel(int64_t n, const double *__restrict__ w,
                                                   const double *__restrict__ V, int64_t ldv, int j0, int nv,
                                                   const double *__restrict__ vscale,
                                                   double *__restrict__ partials, const int *__restrict__ stop_flag) {
  if (*stop_flag) return;
  double acc[NV], sc[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    acc[k] = 0.0;
    sc[k] = k < nv ? vscale[j0 + k] : 0.0;
  }
  // branch-free: all NV loads of a row in flight together (a per-vector
  // `if (k < nv)` compiled to a branch and a full wait around every load --
  // the pass ran at 3.6 TB/s); vectors past nv re-read vector nv - 1 (cached
  // lines) and their sums are dropped below
  const double *__restrict__ vk[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) vk[k] = V + (int64_t)(j0 + (k < nv ? k : nv - 1)) * ldv;
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    const double wi = w[i];
    double v[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] = gm_ld(vk[k] + i);
#pragma unroll
    for (int k = 0; k < NV; ++k) acc[k] += wi * (sc[k] * v[k]);
  }
#pragma unroll
  for (int k = 0; k < NV; ++k)
    if (k >= nv) acc[k] = 0.0;
  block_sum_to_partials<NV>(acc, partials + (size_t)j0 * gridDim.x, gridDim.x);
}

// Four lane-distributed partials a0..a3 summed over the wave together: the
// xor-32 step exchanges two values, the xor-16 step one, then four plain
// steps -- lanes 16 q .. 16 q + 15 end with value q = 2 (l >> 5 & 1) + (l >> 4 & 1)'s total
__device__ __forceinline__ double red4(double a0, double a1, double a2, double a3, int lane) {
  const bool b5 = lane & 32, b4 = lane & 16;
  const double c0 = (b5 ? a2 : a0) + __shfl_xor(b5 ? a0 : a2, 32, 64);
  const double c1 = (b5 ? a3 : a1) + __shfl_xor(b5 ? a1 : a3, 32, 64);
  double c = (b4 ? c1 : c0) + __shfl_xor(b4 ? c0 : c1, 16, 64);
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  return c;
}

// VecMDot in one pass over w, chunk form (nv <= 32): a workgroup holds 4096
// rows of w in registers (WP = 8 16-byte pairs per thread) and walks the basis
// vectors one at a time, reading a 32 KB piece of each contiguously (few DRAM
// streams at once), the next vector's loads issued before the current one's
// sums; the four lane partials of a group of four vectors are reduced
// together (red4) and vector j's chunk total is added to one lane's running
// total (one accumulator register instead of nv).  Measured in round 4
// against four vectors in flight per wave (0.8316 -> 0.803 ms per GMRES(30)
// step at 256^3) and round 3's groups of four (126 SGPR spills);
// tools/mdot_probe.hip rates the walk at the plain read ceiling.
// partials[j * gridDim.x + blockIdx.x] as mdot_kernel.
__global__ void __launch_bounds__(256) mdot_chunk_kernel(int64_t n, const double *__restrict__ w,
                                                         const double *__restrict__ V, int64_t ldv, int nv,
                                                         const double *__restrict__ vscale,
                                                         double *__restrict__ partials,
                                                         const int *__restrict__ stop_flag) {
  constexpr int NVX = 32, WP = 8;
  if (*stop_flag) return;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  double acc = 0.0;                                // lane j: vector j's running total
  const dbl2 *__restrict__ w2 = reinterpret_cast<const dbl2 *>(w);
  const int64_t n2 = n >> 1, csz = 256 * WP, nfull = n2 / csz;
  auto chunk = [&](int64_t c0, auto fullc) __attribute__((always_inline)) {
    constexpr bool FULL = decltype(fullc)::value;
    dbl2 wr[WP];
#pragma unroll
    for (int k = 0; k < WP; ++k) {
      const int64_t i = c0 + k * 256 + threadIdx.x;
      wr[k] = (FULL || i < n2) ? w2[i] : dbl2{0.0, 0.0};
    }
    auto vload = [&](int j, dbl2 (&t)[WP]) __attribute__((always_inline)) {
      const dbl2 *__restrict__ vq = reinterpret_cast<const dbl2 *>(V + (int64_t)j * ldv);
#pragma unroll
      for (int k = 0; k < WP; ++k) {
        const int64_t i = c0 + k * 256 + threadIdx.x;
        t[k] = (FULL || i < n2) ? __builtin_nontemporal_load(vq + i) : dbl2{0.0, 0.0};
      }
    };
    dbl2 ta[WP], tb[WP];
    vload(0, ta);
    for (int j = 0; j < nv; j += 4) {            // wave-uniform
      double a[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        dbl2 (&cur)[WP] = (q & 1) ? tb : ta;
        dbl2 (&nxt)[WP] = (q & 1) ? ta : tb;
        if (j + q + 1 < nv) vload(j + q + 1, nxt);
        a[q] = 0.0;
        if (j + q < nv) {
          const double sj = vscale[j + q];
#pragma unroll
          for (int k = 0; k < WP; ++k) {
            a[q] += wr[k].x * (sj * cur[k].x);
            a[q] += wr[k].y * (sj * cur[k].y);
          }
        }
      }
      const double r = red4(a[0], a[1], a[2], a[3], lane);
      if ((lane & 15) == (j >> 2)) acc += r;
    }
  };
  for (int64_t c = blockIdx.x; c < nfull; c += gridDim.x) chunk(c * csz, std::true_type{});
  if (nfull * csz < n2 && (int64_t)blockIdx.x == nfull % gridDim.x) chunk(nfull * csz, std::false_type{});
  // lane l keeps vector 4 (l & 15) + 2 (l >> 5 & 1) + (l >> 4 & 1)
  const int vj = 4 * (lane & 15) + 2 * ((lane >> 5) & 1) + ((lane >> 4) & 1);
  const bool mine = (lane & 15) < NVX / 4 && vj < nv;
  if ((n & 1) && blockIdx.x == 0 && wid == 0 && mine)   // odd length: the last row, vector vj's term
    acc += w[n - 1] * (vscale[vj] * V[(int64_t)vj * ldv + n - 1]);
  __shared__ double sh[NVX][4];
  if (mine) sh[vj][wid] = acc;
  __syncthreads();
  if ((int)threadIdx.x < nv)
    partials[(size_t)threadIdx.x * gridDim.x + blockIdx.x] =
        (sh[threadIdx.x][0] + sh[threadIdx.x][1]) + (sh[threadIdx.x][2] + sh[threadIdx.x][3]);
}

// KSPGMRESClassicalGramSchmidtOrthogonalization after the MDot: the
// coefficients -h_j (h = w.v_j, folded and all-reduced), the Hessenberg
// column (hh[k][j] = 0 - (-h_j)) and the non-finite check, evaluated by every
// workgroup (workgroup 0 commits), then VecMAXPY_Seq's grouping (first nv%4
// vectors, then groups of four) and ||w||^2, folded in-launch (fold.cnt) or
// as plain partials.
// Chunk form, as mdot_chunk_kernel: a workgroup holds 512 MAXPY_WP rows of w
// in registers and walks the basis vectors one at a time, a contiguous piece
// of each, the next vector's loads issued before the current one's products.
// A group's terms gather in a per-row accumulator g (g = a_j v_j, g = g +
// a_j v_j, then u = u + g): each row's expression is VecMAXPY_Seq's,
// u + (((a0 v0 + a1 v1) + a2 v2) + a3 v3), bit for bit.  The one-row-per-lane
// form read all k + 2 vectors at once across the chip and fell from 0.85 of
// peak at k = 2 to 0.73 at k = 29 (C4 256^3, profiles/r06o); MDot's walk
// holds 0.80 there.
#ifndef MAXPY_WP
#define MAXPY_WP 8
#endif
__global__ void __launch_bounds__(256) maxpy_norm_kernel(int64_t n, double *__restrict__ w,
                                                         const double *__restrict__ V, int64_t ldv, int nv,
                                                         KspState *__restrict__ s, const double *__restrict__ red_k,
                                                         const double *__restrict__ vscale,
                                                         double *__restrict__ hh, int ld,
                                                         double *__restrict__ partials, const Fold fold) {
  constexpr int WP = MAXPY_WP;
  if (s->inner_stop) return;
  __shared__ double a[MAX_RESTART + 1], sc[MAX_RESTART + 1];
  __shared__ int bad;
  if (threadIdx.x == 0) bad = 0;
  __syncthreads();
  for (int j = threadIdx.x; j < nv; j += 256) {
    const double h = red_k[j];
    if (not_finite(h)) bad = 1;
    a[j] = -h;                                   // lhh[j] = -h_j
    sc[j] = vscale[j];
  }
  __syncthreads();
  if (bad) {
    if (blockIdx.x == 0 && threadIdx.x == 0) stop(s, R_DIVERGED_NANORINF);
    return;
  }
  if (blockIdx.x == 0)
    for (int j = threadIdx.x; j < nv; j += 256) hh[(size_t)(nv - 1) * ld + j] = 0.0 - a[j];
  const int rem = nv & 3;
  double v[1] = {0.0};
  dbl2 *__restrict__ w2 = reinterpret_cast<dbl2 *>(w);
  const int64_t n2 = n >> 1, csz = 256 * WP, nfull = n2 / csz, ldv2 = ldv >> 1;   // ldv: a multiple of 32
  auto chunk = [&](int64_t c0, auto fullc) __attribute__((always_inline)) {
    constexpr bool FULL = decltype(fullc)::value;
    dbl2 u[WP], g[WP];
#pragma unroll
    for (int k = 0; k < WP; ++k) {
      const int64_t i = c0 + k * 256 + threadIdx.x;
      u[k] = (FULL || i < n2) ? w2[i] : dbl2{0.0, 0.0};
    }
    auto vload = [&](int j, dbl2 (&t)[WP]) __attribute__((always_inline)) {
      const dbl2 *__restrict__ vq = reinterpret_cast<const dbl2 *>(V) + (int64_t)j * ldv2;
#pragma unroll
      for (int k = 0; k < WP; ++k) {
        const int64_t i = c0 + k * 256 + threadIdx.x;
        t[k] = (FULL || i < n2) ? __builtin_nontemporal_load(vq + i) : dbl2{0.0, 0.0};
      }
    };
    dbl2 ta[WP], tb[WP];
    vload(0, ta);
    // j's place in its group: the first nv % 4 vectors form the first group
    for (int j = 0; j < nv; j += 2) {            // wave-uniform
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int jj = j + q;
        if (jj >= nv) break;
        dbl2 (&cur)[WP] = q ? tb : ta;
        dbl2 (&nxt)[WP] = q ? ta : tb;
        if (jj + 1 < nv) vload(jj + 1, nxt);
        const bool first = jj < rem ? jj == 0 : ((jj - rem) & 3) == 0;
        const bool last = jj < rem ? jj == rem - 1 : ((jj - rem) & 3) == 3;
        const double aj = a[jj], sj = sc[jj];
#pragma unroll
        for (int k = 0; k < WP; ++k) {
          const double px = aj * (sj * cur[k].x), py = aj * (sj * cur[k].y);
          g[k].x = first ? px : g[k].x + px;
          g[k].y = first ? py : g[k].y + py;
          if (last) { u[k].x = u[k].x + g[k].x; u[k].y = u[k].y + g[k].y; }
        }
      }
    }
#pragma unroll
    for (int k = 0; k < WP; ++k) {
      const int64_t i = c0 + k * 256 + threadIdx.x;
      if (FULL || i < n2) {
        w2[i] = u[k];
        v[0] += u[k].x * u[k].x;
        v[0] += u[k].y * u[k].y;
      }
    }
  };
  for (int64_t c = blockIdx.x; c < nfull; c += gridDim.x) chunk(c * csz, std::true_type{});
  if (nfull * csz < n2 && (int64_t)blockIdx.x == nfull % gridDim.x) chunk(nfull * csz, std::false_type{});
  if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {   // odd length: the last row
    const int64_t i = n - 1;
    double u = w[i];
    int j = 0;
    auto vj = [&](int j) { return sc[j] * gm_ld(V + (int64_t)j * ldv + i); };
    if (rem == 1) { u = a[0] * vj(0) + u; j = 1; }
    else if (rem == 2) { u = u + (a[0] * vj(0) + a[1] * vj(1)); j = 2; }
    else if (rem == 3) { u = u + ((a[0] * vj(0) + a[1] * vj(1)) + a[2] * vj(2)); j = 3; }
    for (; j < nv; j += 4)
      u = u + (((a[j] * vj(j) + a[j + 1] * vj(j + 1)) + a[j + 2] * vj(j + 2)) + a[j + 3] * vj(j + 3));
    w[i] = u;
    v[0] += u * u;
  }
  block_partials<1>(v, partials, gridDim.x, fold);
}

// normalise vv[k+1], happy breakdown, KSPGMRESUpdateHessenberg, convergence
// The column and the rotations are staged in LDS by the whole workgroup
// (coalesced loads) and thread 0 works there: the rotation loop's dependent
// global loads took ~20 us per step at k ~ 15 (the same operations in the
// same order, so the same bits).
__global__ void __launch_bounds__(256) gm_step_kernel(KspState *s, int k, const double *partials, int nblocks,
                                                      int fused, double *hh, int ld, double *grs, double *cc,
                                                      double *ss, double *hist, double *vscale, int *hw,
                                                      int step) {
  // the host's progress word: this launch (a no-op after a stop too) ran --
  // the restart read-back's wait re-arms its no-progress deadline on it
  if (hw && threadIdx.x == 0) host_store(hw + HW_PROGRESS, step);
  if (s->inner_stop) return;
  (void)gather_red<1>(s, partials, nblocks, fused);   // every thread: the fold syncs the workgroup
  __shared__ double hs[MAX_RESTART + 2], cs[MAX_RESTART + 1], sn[MAX_RESTART + 1];
  __shared__ int wb;
  double *h = hh + (size_t)k * ld;   // column k
  for (int j = threadIdx.x; j <= k + 1; j += blockDim.x) hs[j] = h[j];
  for (int j = threadIdx.x; j < k; j += blockDim.x) {
    cs[j] = cc[j];
    sn[j] = ss[j];
  }
  if (threadIdx.x == 0) wb = 0;
  __syncthreads();
  if (threadIdx.x == 0) {
    [&] {
      const double tt = sqrt(s->red[0]);
      s->scale = tt != 0.0 ? 1.0 / tt : 1.0;
      vscale[k + 1] = s->scale;   // VecScale(vv[k+1], 1/tt), applied where it is read
      if (not_finite(tt)) { stop(s, R_DIVERGED_NANORINF); return; }
      wb = 1;
      hs[k + 1] = tt;
      double hapbnd = fabs(tt / grs[k]);
      if (hapbnd > s->haptol) hapbnd = s->haptol;
      const bool hapend = tt < hapbnd;
      // apply the previous rotations to column k
      for (int j = 1; j <= k; ++j) {
        const double t = hs[j - 1];
        hs[j - 1] = cs[j - 1] * t + sn[j - 1] * hs[j];
        hs[j] = cs[j - 1] * hs[j] - (sn[j - 1] * t);
      }
      double res;
      if (!hapend) {
        const double t = sqrt(hs[k] * hs[k] + hs[k + 1] * hs[k + 1]);
        if (t == 0.0) { stop(s, R_DIVERGED_NULL); return; }
        const double ck = hs[k] / t, sk = hs[k + 1] / t;
        cc[k] = ck;
        ss[k] = sk;
        const double g = grs[k];
        grs[k + 1] = -(sk * g);
        grs[k] = ck * g;
        hs[k] = ck * hs[k] + sk * hs[k + 1];
        res = fabs(grs[k + 1]);
      } else {
        res = 0.0;
      }
      s->it = k + 1;
      s->its += 1;
      s->ksp_rnorm = res;
      s->res = tt;
      if (hist) hist[s->its] = res;
      int reason = dev_converged(s, s->its, res, true, 0.0);
      if (hapend && !reason) reason = R_DIVERGED_BREAKDOWN;
      if (reason) { stop(s, reason); return; }
      if (s->it >= s->max_k || s->its >= s->top.max_it) s->inner_stop = 1;
    }();
  }
  __syncthreads();
  if (wb)
    for (int j = threadIdx.x; j <= k + 1; j += blockDim.x) h[j] = hs[j];
}

// KSPGMRESBuildSoln: back substitution into grs (in place).  Up to restart
// 63 the workgroup stages the Hessenberg block and grs in LDS first (thread 0
// then runs the same operations there: the same bits, without a dependent
// global load per term).
constexpr int GM_LDS_K = 64;
__global__ void __launch_bounds__(256) gm_buildsoln_kernel(KspState *s, const double *hh, int ld, double *grs) {
  if (blockIdx.x != 0) return;
  const int it = s->it - 1;
  const bool stage = it >= 0 && it < GM_LDS_K && ld <= GM_LDS_K + 1;
  __shared__ double hl[GM_LDS_K * (GM_LDS_K + 1)], gl[GM_LDS_K];
  if (stage) {
    for (int q = threadIdx.x; q < (it + 1) * ld; q += blockDim.x) hl[q] = hh[q];   // columns 0 .. it
    for (int q = threadIdx.x; q <= it; q += blockDim.x) gl[q] = grs[q];
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  s->nv = 0;
  if (it < 0 || s->reason == R_DIVERGED_NULL || s->reason == R_DIVERGED_NANORINF) return;
  if (s->reason == R_DIVERGED_BREAKDOWN && s->ksp_rnorm > 0.0 && s->it == 0) return;
  const double *H = stage ? hl : hh;
  double *G = stage ? gl : grs;
#define HHd(a, b) H[(size_t)(b) * ld + (a)]
  if (HHd(it, it) == 0.0) { s->reason = R_DIVERGED_BREAKDOWN; s->top.done = 1; return; }
  G[it] = G[it] / HHd(it, it);
  for (int ii = 1; ii <= it; ++ii) {
    const int k = it - ii;
    double t = G[k];
    for (int j = k + 1; j <= it; ++j) t = t - HHd(k, j) * G[j];
    if (HHd(k, k) == 0.0) {
      if (stage) for (int q = 0; q <= it; ++q) grs[q] = gl[q];
      s->reason = R_DIVERGED_BREAKDOWN; s->top.done = 1; return;
    }
    G[k] = t / HHd(k, k);
  }
#undef HHd
  if (stage) for (int q = 0; q <= it; ++q) grs[q] = gl[q];
  s->nv = it + 1;
}

// x += sum_j nrs_j v_j  (VecMAXPY from zero, then VecAXPY(x, 1, TEMP))
__global__ void __launch_bounds__(256) gm_update_x_kernel(int64_t n, const KspState *__restrict__ s,
                                                          const double *__restrict__ V, int64_t ldv,
                                                          const double *__restrict__ vscale,
                                                          const double *__restrict__ nrs, double *__restrict__ x) {
  const int nv = s->nv;
  if (nv == 0) return;
  __shared__ double a[MAX_RESTART + 1], sc[MAX_RESTART + 1];
  for (int j = threadIdx.x; j < nv; j += 256) {
    a[j] = nrs[j];
    sc[j] = vscale[j];
  }
  __syncthreads();
  const int rem = nv & 3;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    double u = 0.0;
    int j = 0;
    auto vj = [&](int j) { return sc[j] * gm_ld(V + (int64_t)j * ldv + i); };
    if (rem == 1) { u = a[0] * vj(0) + u; j = 1; }
    else if (rem == 2) { u = u + (a[0] * vj(0) + a[1] * vj(1)); j = 2; }
    else if (rem == 3) { u = u + ((a[0] * vj(0) + a[1] * vj(1)) + a[2] * vj(2)); j = 3; }
    for (; j < nv; j += 4)
      u = u + (((a[j] * vj(j) + a[j + 1] * vj(j + 1)) + a[j + 2] * vj(j + 2)) + a[j + 3] * vj(j + 3));
    x[i] = fma(1.0, u, x[i]);
  }
}

__global__ void gm_cycle_end_kernel(KspState *s) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  s->itcount += s->it;
  if (s->itcount >= s->top.max_it && !s->reason) s->reason = R_DIVERGED_ITS;
  if (s->reason) s->top.done = 1;
  s->guess_zero = 0;
}

// ------------------------------------------------------------------ host drivers
namespace {

// wall_clock64() ticks per ms on this device (100 MHz on gfx9)
static double wall_clock_khz(int dev) {
  static int khz[64] = {};
  const int d = dev >= 0 && dev < 64 ? dev : 0;
  if (!khz[d] && (hipDeviceGetAttribute(&khz[d], hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz[d] <= 0))
    khz[d] = 100000;
  return (double)khz[d];
}

// the operator's pinned flag slots and events (Mat::poll_*), made once
static void solve_resources(Mat *A) {
  if (A->poll_pinned) return;
  HIPCHECK(hipHostMalloc(reinterpret_cast<void **>(&A->poll_pinned), HW_WORDS * sizeof(int),
                         hipHostMallocCoherent | hipHostMallocMapped));
  std::memset(A->poll_pinned, 0, HW_WORDS * sizeof(int));
  HIPCHECK(hipHostMalloc(&A->state_pinned, sizeof(KspState), hipHostMallocDefault));
  for (auto &e : A->poll_ev) HIPCHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  for (auto &e : A->solve_ev) HIPCHECK(hipEventCreate(&e));
}

// Done-flag polling, one batch behind, without device-side markers: the
// update pass stores the count of iterations begun and, once the solve has
// stopped, a done flag into pinned host words (HW_*); after enqueuing batch k
// the host spins until batch k-1's last iteration has begun (or done), so at
// most about two batches are in flight and a stopped solve is seen one batch
// late.  (An event record + device-to-host flag copy per batch left the GPU
// idle ~14 us per batch.)
struct Poller {
  hipStream_t st;
  Comm *c;
  int *hw;
  int pending = 0;    // batches enqueued
  int prev_end = 0;   // iteration count at the end of the previous batch
  Poller(Mat *A, hipStream_t s) : st(s), c(A->comm) {
    solve_resources(A);
    hw = A->poll_pinned;
    for (int k = 0; k < HW_WORDS; ++k) reinterpret_cast<volatile int *>(hw)[k] = 0;
  }
  ~Poller() { (void)hipStreamSynchronize(st); }
  int word(int k) const { return reinterpret_cast<const volatile int *>(hw)[k]; }
  // the batch ending at iteration `end` is enqueued; true once done was seen
  bool batch(int end) {
    const int target = prev_end;
    prev_end = end;
    if (++pending < 2) return false;
    c->wait_until([&] { return word(HW_DONE) != 0 || word(HW_PROGRESS) >= target; }, st,
                  [&] { return (long long)word(HW_PROGRESS); }, 0);   // the words are zeroed per solve
    return word(HW_DONE) != 0;
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
  // ext: one-rank solves time the main SpMV kernel by its own dispatch
  // timestamps (g_ext_timing); otherwise events bracket the whole MatMult
  // (halo, interior and boundary launches)
  bool ext = false;
  void begin() {
    if (!on || used + 2 > ev.size()) return;
    if (ext) g_ext_timing = ExtTiming{ev[used], ev[used + 1], true, false};
    else HIPCHECK(hipEventRecord(ev[used], st));
  }
  void end() {
    if (!on || used + 2 > ev.size()) return;
    if (ext) {
      if (g_ext_timing.used) used += 2;   // a launch took the events
      g_ext_timing = ExtTiming{};
      return;
    }
    HIPCHECK(hipEventRecord(ev[used + 1], st));
    used += 2;
  }
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
  explicit Events(Mat *A) { solve_resources(A); a = A->solve_ev[0]; b = A->solve_ev[1]; }
};

void init_state(KspState &h, const mx_ksp_params &p, int normtype) {
  std::memset(&h, 0, sizeof(h));
  h.rtol = p.rtol; h.top.atol = p.atol; h.top.dtol = p.dtol; h.haptol = p.haptol;
  h.breakdowntol = p.breakdowntol; h.top.max_it = p.max_it; h.top.normtype = normtype;
  h.guess_zero = !p.guess_nonzero; h.max_k = p.restart; h.ksp_rnorm = -1.0;
}

// device state -> host through the operator's pinned staging buffer (a
// pageable copy is staged and synchronous in the runtime)
[[maybe_unused]] void read_state(Mat *A, hipStream_t st, const KspState *d, KspState &h) {
  solve_resources(A);
  HIPCHECK(hipMemcpyAsync(A->state_pinned, d, sizeof(KspState), hipMemcpyDeviceToHost, st));
  A->comm->wait_stream(st);
  std::memcpy(&h, A->state_pinned, sizeof(KspState));
}
void write_state(Mat *A, hipStream_t st, KspState *d, const KspState &h) {
  solve_resources(A);
  std::memcpy(A->state_pinned, &h, sizeof(KspState));
  HIPCHECK(hipMemcpyAsync(d, A->state_pinned, sizeof(KspState), hipMemcpyHostToDevice, st));
}

}  // namespace

void Mat::release_ksp() {
  if (cg_graph) (void)hipGraphExecDestroy(cg_graph);
  cg_graph = nullptr;
  cg_key.clear();
  cg_graph_failed = false;
  ksp_ws = DBuf<double>();
  ksp_state = DBuf<char>();
  jac_dinv = DBuf<double>();
  jac_mode = -1;
  if (poll_pinned) (void)hipHostFree(poll_pinned);
  poll_pinned = nullptr;
  if (state_pinned) (void)hipHostFree(state_pinned);
  state_pinned = nullptr;
  for (auto &e : poll_ev) { if (e) (void)hipEventDestroy(e); e = nullptr; }
  for (auto &e : solve_ev) { if (e) (void)hipEventDestroy(e); e = nullptr; }
}

// KSPSetUp work space: one device allocation per operator, grown on demand
// and reused by later solves (no hipMalloc/hipFree inside a solve).
// Consecutive vectors are skewed by g_knobs.ws_skew doubles so that equal
// indices of different vectors do not sit at the same offset modulo the
// large powers of two the HBM channel interleave repeats on.
// The skew is rounded up to an even count: the direction buffers are read and
// written as 16-byte pairs (cg_pb_kernel's batch carve, spmv_pair_pbw_kernel).
static size_t carve_step(size_t n) { return (n + 31) / 32 * 32 + ((size_t)std::max(g_knobs.ws_skew, 0) + 1) / 2 * 2; }
struct Carve {
  double *base;
  size_t off = 0;
  explicit Carve(double *b) : base(b) {}
  double *take(size_t n) { double *p = base + off; off += carve_step(n); return p; }
};
static size_t carve_size(std::initializer_list<size_t> parts) {
  size_t t = 0;
  for (size_t n : parts) t += carve_step(n);
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

static bool aligned16(std::initializer_list<const void *> ptrs) {
  for (const void *q : ptrs)
    if (reinterpret_cast<uintptr_t>(q) & 15) return false;
  return true;
}
// grid of a CG vector pass: the row walk by default (knob 13 = 0), the paired
// walk (16-B accesses, knob 13 = 1) only when every vector is aligned
static unsigned cg_vec_grid(int64_t n, bool paired, int dflt) {
  const int cap = std::min(g_knobs.cg_vec_grid > 0 ? g_knobs.cg_vec_grid : dflt, CG_MAX_VEC_GRID);
  return grid_for(paired ? cdiv(n, 2) : n, 256, cap);
}

// four-step load batches in the row walk (knob 21): 2 = auto, on up to
// CG_UNROLL_MAX_ROWS rows (-3% per iteration at 2M rows/rank; +5% at 256^3)
static int cg_unroll(int64_t n) {
  return g_knobs.cg_unroll == 2 ? (n <= CG_UNROLL_MAX_ROWS ? 1 : 0) : g_knobs.cg_unroll;
}

// direction update (+ the deferred x step when x != null)
static void cg_p_launch(hipStream_t st, int64_t n, KspState *s, const double *r, const Jac &j, double *p,
                        double *x, double *hist) {
  const bool vec = g_knobs.cg_vec && aligned16({r, p, x, j.d});
  const unsigned g = cg_vec_grid(n, vec, vec ? CG_VEC_BLOCKS : 8192);
  const int unr = cg_unroll(n);
#define CGP(JM, XD, V) cg_p_kernel<JM, XD, V><<<g, 256, 0, st>>>(n, s, r, j.d, j.c, p, x, hist, g_knobs.cg_nts, unr)
#define CGP_J(JM) do { if (x) { if (vec) CGP(JM, true, true); else CGP(JM, true, false); } \
                       else { if (vec) CGP(JM, false, true); else CGP(JM, false, false); } } while (0)
  switch (j.mode) { case 1: CGP_J(1); break; case 2: CGP_J(2); break; default: CGP_J(0); }
#undef CGP_J
#undef CGP
  HIPCHECK(hipGetLastError());
}

// the direction-update grid (row walk); the zero-guess norms pass runs on
// the same grid so that its partial sums equal the fused iteration-0 ones.
// Mode 5 (wide): 12288 workgroups (256^3: 185.8 -> 177.6 us per iteration with
// x batches of 4, against 180.6 at 8192; profiles/r03_ab.jsonl)
static unsigned cg_pb_grid(int64_t n, bool wide = false) { return cg_vec_grid(n, false, wide ? 12288 : 8192); }

static void cg_pb_launch(hipStream_t st, int64_t n, KspState *s, const double *r, const Jac &j, const PBufs &pb,
                         int B, double *x, double *hist, const double *r0, double *npart, const Fold &fin_in,
                         bool wide) {
  const unsigned g = cg_pb_grid(n, wide);
  Fold fin = fin_in;
  fin.ntotal = fin.ncount = (int)g;
  const int unr = (cg_unroll(n) ? 1 : 0) | ((g_knobs.cg_ntl & 1) ? 2 : 0);
  const int64_t ps = pb.b[1] - pb.b[0];   // (the buffers are carved consecutively, cg_solve)
#define CGPB(JM, BB) launch_timed(&cg_pb_kernel<JM, BB>, (int)g, st, n, s, r, j.d, j.c, pb.b[0], ps, x, hist, unr, r0, \
                                     npart, fin)
#define CGPB_J(JM) do { if (B == 8) CGPB(JM, 8); else if (B == 4) CGPB(JM, 4); else CGPB(JM, 2); } while (0)
  switch (j.mode) { case 1: CGPB(1, 2); break; case 2: CGPB_J(2); break; default: CGPB_J(0); }
#undef CGPB_J
#undef CGPB
  HIPCHECK(hipGetLastError());
}

// update pass; returns its grid (= partials per value)
static int cg_update_launch(hipStream_t st, int64_t n, KspState *s, const double *p, const double *w, double *x,
                            double *r, const Jac &j, double *partials, const Fold &fold_in,
                            const double *dot_part, int ndot, int xb, const double *r0, int *hw) {
  const bool vec = g_knobs.cg_vec && aligned16({p, w, x, r, j.d});
  const unsigned g = g_knobs.cg_upd_grid > 0 ? grid_for(n, 256, g_knobs.cg_upd_grid)
                                             : cg_vec_grid(n, vec, vec ? CG_VEC_BLOCKS : RED_BLOCKS);
  Fold f = fold_in;
  f.ntotal = f.ncount = (int)g;
  const int unr = (cg_unroll(n) ? 1 : 0) | ((g_knobs.cg_ntl & 2) ? 2 : 0);
  f.base = 0;
#define CGU(JM, XU, V) cg_update_kernel<JM, XU, V><<<g, 256, 0, st>>>(n, s, p, w, x, r, j.d, j.c, partials, f, \
                                                                        g_knobs.cg_nts, dot_part, ndot, unr, xb, r0, \
                                                                        hw)
#define CGU_J(JM) do { if (x) { if (vec) CGU(JM, true, true); else CGU(JM, true, false); } \
                       else { if (vec) CGU(JM, false, true); else CGU(JM, false, false); } } while (0)
  switch (j.mode) { case 1: CGU_J(1); break; case 2: CGU_J(2); break; default: CGU_J(0); }
#undef CGU_J
#undef CGU
  HIPCHECK(hipGetLastError());
  return (int)g;
}

static void cg_solve(Mat *A, const mx_ksp_params &p, const Jac dinv, const double *b, double *x,
                     mx_ksp_result &res, double *hist_host) {
  Comm *c = A->comm;
  hipStream_t st = c->stream;
  const int64_t n = A->m;
  const bool fused = c->size == 1 && !g_knobs.force_coll;
  int normtype = p.norm_type == MX_NORM_DEFAULT ? MX_NORM_PRECONDITIONED : p.norm_type;
  const size_t nv = (size_t)std::max<int64_t>(n, 1);
  // MatMult partials (+ boundary launch), then the update pass's 3 per workgroup
  const size_t npart = (size_t)std::max({spmv_blocks(A) + 64, RED_BLOCKS, g_knobs.norm_grid, (int)cg_pb_grid(n, true)}) * 6 +
                       3 * (size_t)CG_MAX_VEC_GRID + 128;
  const size_t nhist = hist_host ? (size_t)p.max_it + 2 : 1;
  // mode 2 batches B x steps (knob 29; 2 or 4 p buffers) when the batch of
  // launched iterations (poll) is a multiple of B; 1 = the x step every iteration
  const int poll = p.poll_every > 0 ? p.poll_every : 16;
  // auto (3): mode 5 on one rank where it applies (a lean 5/7-point z-march);
  // on P > 1 ranks mode 2 where the z-march applies (the interior-rank proxy,
  // tools/rank_proxy.py, round 3: kernel time per iteration at 2 M rows/rank
  // mode 1 53.8 / 2 52.6 / 5 54.6 us, and mode 2 ahead at 4 M and 8 M rows);
  // otherwise (the general SELL kernel) 1 up to CG_FUSE_MAX_ROWS local rows, else 2
  int fmode = g_knobs.cg_fuse;
  if (fmode == 3) {
    // mode 5 on one rank; on P > 1 ranks where the direction update fuses
    // into the split p.Ap pass (knob 80): the N = 2 rehearsal ran 1659 it/s
    // against mode 2's 1573 (profiles/r05x_shm2_n2.json), the interior-rank
    // proxy's kernels 63.4 us per iteration against mode 5's separate passes'
    // 67.2 (round 5, gpurun_out/r5w)
    if (pair_cg5_applies(A, dinv.mode) && (fused || pair_cg5_pbws_applies(A, dinv.mode, 4))) fmode = 5;
    else if (pair_lean_kind(A) > 0 && pair_zm_applies(A)) fmode = 2;
    else fmode = n <= CG_FUSE_MAX_ROWS ? 1 : 2;
  }
  if (fmode == 4) fmode = 2;   // round 2's mode 4 (the direction update inside the MatMult) is retired
  // mode 5 (knob 9 = 5): mode 2 whose MatMult stores no product -- a p.Ap
  // pass, then the update pass recomputes A p (mx_spmv_pair.hip SPMV_PW /
  // SPMV_RUPD) -- one rank, a lean 5/7-point z-march layout, no or uniform
  // Jacobi; otherwise 2
  if (fmode == 5 && !pair_cg5_applies(A, dinv.mode)) fmode = 2;
  // x-step batch (knob 29; 0 = auto: 4 in mode 5 -- 256^3: -2.8% per iteration
  // against 2 -- else 2)
  // mode 5 on a symmetric 5/7-point operator: the forward-half p.Ap pass
  // (checked once per operator, before any capture)
  if (fmode == 5) pair_sym_prepare(A);
  // (batches of 4 only with no or a uniform Jacobi: the vector-Jacobi
  // direction update with four p buffers spilled SGPRs and is not on any
  // default path -- mode 5, the only one batching by 4, needs a uniform one)
  const int xbk = g_knobs.cg_xbatch == 0 ? (fmode == 5 ? 4 : 2)
                  : ((g_knobs.cg_xbatch == 4 || g_knobs.cg_xbatch == 8) && dinv.mode == 1) ? 2 : g_knobs.cg_xbatch;
  const int xb = ((fmode == 2 || fmode == 5) && (xbk == 2 || xbk == 4 || xbk == 8) && poll % xbk == 0) ? xbk : 1;
  const bool wide_pb = fmode == 5;
  const size_t nx = xb >= 4 ? nv : 0, nx8 = xb == 8 ? nv : 0;
  Carve cv(workspace(A, carve_size({nv, nv, npart, nhist, nv, nv, nx, nx, nx8, nx8, nx8, nx8})));
  struct { double *p; } r{cv.take(nv)}, w{cv.take(nv)}, part{cv.take(npart)}, hist{cv.take(nhist)}, pv{cv.take(nv)};
  // a history entry no kernel writes (a solve that stops on an exactly zero
  // residual) reads as 0.0, as PETSc's, not as an earlier solve's value left
  // in the reused work space
  if (hist_host) HIPCHECK(hipMemsetAsync(hist.p, 0, sizeof(double) * nhist, st));
  double *pv2 = cv.take(nv);   // fused CG: p_i alternates between pv (i even) and pv2
  // x batches of B: p_j in buffer j % B, the B buffers carved consecutively
  // (equally spaced: the kernels address them from pv; unused slots repeat
  // the first two)
  PBufs pbs{{pv.p, pv2, pv.p, pv2, pv.p, pv2, pv.p, pv2}};
  for (int q = 2; q < xb; ++q) pbs.b[q] = cv.take(nv);
  double *pv3 = pbs.b[2], *pv4 = pbs.b[3];
  struct { KspState *p; } sd{state_buf(A)};
  const KspInit kin{p.rtol, p.atol, p.dtol, p.haptol, p.breakdowntol, p.max_it, normtype, !p.guess_nonzero, p.restart};
  ksp_state_init_kernel<<<1, 256, 0, st>>>(sd.p, kin);
  HIPCHECK(hipGetLastError());
  SpmvTimer timer((p.profile & 1) != 0, st, std::min(p.max_it, 4096));
  timer.ext = c->size == 1;
  SpmvTimer utimer((p.profile & 2) != 0, st, std::min(p.max_it, 4096));   // mode 5's residual update
  utimer.ext = c->size == 1;
  SpmvTimer ptimer((p.profile & 4) != 0, st, std::min(p.max_it, 4096));   // the batched direction update
  ptimer.ext = c->size == 1;
  SpmvTimer wtimer((p.profile & 8) != 0, st, std::min(p.max_it, 4096));   // the fused direction + p.Ap pass
  wtimer.ext = c->size == 1;

  // r = b - A x  (or b)
  if (p.guess_nonzero) {
    mat_mult(A, x, r.p);
    vec_aypx(st, n, -1.0, b, r.p);
  }
  KspState *s = sd.p;
  double *red = s->red;
  const int nv0 = p.guess_nonzero ? 6 : 3;
  double *hist0 = hist_host ? hist.p : nullptr;
  // Zero guess, batched x steps, one rank: iteration 0's direction update
  // reads b as r_0 and also forms the initial norms, folds them and runs
  // cg_init (cg_pb_kernel NRM) -- no separate pass over b.  Otherwise the
  // norms pass runs on the direction update's grid (knob 34 overrides), so
  // both give the same bits, then folds in-launch and runs cg_init (one rank)
  // or leaves partials for the all-reduce.
  // knob 69: the direction update rides in mode 5's p.Ap pass (the initial
  // norms then take their own pass over b -- the same bits, see above)
  const bool pbw = fmode == 5 && fused && pair_cg5_pbw_applies(A, dinv.mode, xb);
  // knob 80: the same on P > 1 ranks, into the split p.Ap pass (the halo pack
  // forms the ghost planes' p_i)
  const bool pbws = fmode == 5 && !fused && xb > 1 && pair_cg5_pbws_applies(A, dinv.mode, xb);
  const bool norms_in_pb = fused && xb > 1 && !p.guess_nonzero && !pbw;
  const int ngrid = g_knobs.norm_grid > 0 ? g_knobs.norm_grid : (int)cg_pb_grid(n, wide_pb);
  Fold fin;
  if (fused) { fin.cnt = s->fold_upd; fin.out = red; fin.ntotal = fin.ncount = ngrid; }
#define CGN(...) cg_norms_kernel<__VA_ARGS__><<<ngrid, 256, 0, st>>>
  if (nv0 == 6) CGN(6)(n, r.p, b, dinv, part.p, nullptr, nullptr, fin, s, hist0);
  // x = 0 and r = b; with batched x steps neither is written here: iteration 0
  // reads b as r_0 and the first batch (or the finish pass) writes x first
  else if (xb > 1) { if (!norms_in_pb) CGN(3)(n, b, b, dinv, part.p, nullptr, nullptr, fin, s, hist0); }
  else CGN(3, true)(n, r.p, b, dinv, part.p, r.p, x, fin, s, hist0);
#undef CGN
  HIPCHECK(hipGetLastError());
  if (!fused) {
    finish_reduce(part.p, ngrid, nv0, red, st);
    c->allreduce_sum(red, nv0);
    if (nv0 == 6) cg_init_kernel<6><<<1, 256, 0, st>>>(s, part.p, ngrid, 0, hist0);
    else cg_init_kernel<3><<<1, 256, 0, st>>>(s, part.p, ngrid, 0, hist0);
    HIPCHECK(hipGetLastError());
  }
  Fold fpb;                                   // iteration 0's fused norms (norms_in_pb)
  if (norms_in_pb) { fpb.cnt = s->fold_upd; fpb.out = red; }

  Poller poller(A, st);
  int i = 0;
  const unsigned egrid = grid_for(n, 256, 8192);
  int *done = &s->top.done;
  double *hist_d = hist_host ? hist.p : nullptr;
  // zero-guess batched solves read b as r_0 (nothing copies b into r)
  const double *r0 = (xb > 1 && !p.guess_nonzero) ? b : nullptr;
  // fused: the direction update and the previous x step ride in the MatMult
  // (SPMV_CG); p ping-pongs between two buffers since neighbours read p_{i-1}
  // 1: direction update + x step inside the MatMult (SPMV_CG)
  // 2: x step deferred into the next direction update (cg_p_kernel<XD = true>)
  // 3 (auto): 1 up to CG_FUSE_MAX_ROWS local rows, else 2.  Measured per
  // iteration on 256 x 256 x nz ranks (tools/cg_ab.py, interleaved): nz 32
  // modes 0/1/2 within 1.3% (1 best); nz 128: 2 -3.4% and 1 +3.8% vs 0;
  // 256^3: 2 -6%, 1 +2%.  Mode 1's two-vector gathers overflow the per-XCD
  // L2 at large ranks.  With the row-pair MatMult (value codes): nz 32 mode 1
  // 55.6 / mode 2 56.8 us, nz 64 88.1 / 83.3, nz 128 151.5 / 137.0, 256^3
  // 304 / 268 -- hence the 3M-row threshold
  const bool fuse_cg = fmode == 1;
  const bool defer_x = fmode != 0;
  // p_{-1} = -0.0: iteration 0's z + (+0)(-0) is exactly z (VecCopy)
  if (fuse_cg) vec_set(st, n, -0.0, pv2);
  // in-launch folds: p.w into red1 (MatMult), [z.z, z.r, r.r] into red3 (update)
  Fold fdot, fupd;
  fdot.cnt = s->fold_dot; fdot.out = &s->red1;
  fupd.cnt = s->fold_upd; fupd.out = s->top.red3;
  // 0: fold kernels; 1 (default): the update pass folds in-launch, and so does
  // the MatMult's halo-boundary launch when the product splits (a single
  // workgroup generation, unlike the 8192-block interior launch); 2: always
  const int fold_at = g_knobs.cg_fold;
  const Fold *fdot_p = (fold_at >= 2 || (fold_at >= 1 && matmult_splits(A))) ? &fdot : nullptr;
  if (fold_at < 1) fupd.cnt = nullptr;
  // per iteration: [first kernel: scalar top + p] -> MatMult (+ p.w) -> all-reduce
  // -> update (alpha + x, r, z norms) -> all-reduce; the scalars are
  // evaluated inside the vector kernels (mx_cg.hpp), no one-block kernels
  auto iteration = [&](int it) {
    int nb_spmv;
    if (fuse_cg) {
      CgFuse cg;
      cg.r = r.p; cg.pold = (it & 1) ? pv.p : pv2; cg.pnew = (it & 1) ? pv2 : pv.p;
      cg.x = x; cg.st = s; cg.hist = hist_d; cg.jac = dinv;
      timer.begin();
      nb_spmv = matmult_overlap(A, nullptr, w.p, SPMV_CG, Jac{}, part.p, done, &cg, fdot_p);
      timer.end();
    } else {
      double *pi = xb > 1 ? pbs.b[it % xb] : pv.p;
      // knob 69: the iterations between x-step batches (it % xb != 0; the
      // host's it is the device's i) fuse the direction update into the PW pass
      const bool fuse_pw = pbw && it % xb != 0, fuse_pws = pbws && it % xb != 0;
      if (fuse_pws) {
        wtimer.begin();
        nb_spmv = cg5_pbws_matmult(A, s, r.p, pbs.b, xb, it, hist_d, dinv, w.p, part.p, done, fdot_p);
        wtimer.end();
        if (!nb_spmv) fail(MX_ERR_INTERNAL, "CG without its direction + p.Ap pass");
      } else if (fuse_pw) {
        wtimer.begin();
        nb_spmv = pair_cg5_pbw_launch(A, s, r.p, r0, pbs.b, xb, hist_d, dinv.mode, dinv.c, part.p,
                                      fdot_p ? *fdot_p : Fold{}, st);
        wtimer.end();
        if (!nb_spmv) fail(MX_ERR_INTERNAL, "CG without its direction + p.Ap pass");
      } else if (xb > 1) {
        ptimer.begin();
        cg_pb_launch(st, n, s, r.p, dinv, pbs, xb, x, hist_d, r0, part.p, fpb, wide_pb);
        ptimer.end();
      } else cg_p_launch(st, n, s, r.p, dinv, pv.p, defer_x ? x : nullptr, hist_d);
      if (!fuse_pw && !fuse_pws) {
        timer.begin();
        nb_spmv = matmult_overlap(A, pi, w.p, fmode == 5 ? SPMV_PW : SPMV_DOT, Jac{}, part.p, done, nullptr, fdot_p);
        timer.end();
        if (!nb_spmv) fail(MX_ERR_INTERNAL, "CG without its MatMult");
      }
    }
    // one rank: the update pass folds the MatMult's partials itself (knob 10
    // = 3; mode 5's residual update by default, knob 46)
    const bool fold_in_update = !fdot_p && fused && (fold_at == 3 || (fmode == 5 && g_knobs.cg5_fold));
    if (!fdot_p && !fold_in_update) fold_kernel<1><<<1, 256, 0, st>>>(part.p, nb_spmv, &s->red1, done);
    if (!fused) c->allreduce_sum(&s->red1, 1);
    const double *pcur = fuse_cg ? ((it & 1) ? pv2 : pv.p) : xb > 1 ? pbs.b[it % xb] : pv.p;
    // the update's own partials go after the MatMult's when it folds those
    double *upart = fold_in_update ? part.p + ((nb_spmv + 63) / 64) * 64 : part.p;
    if (fmode == 5) utimer.begin();
    const int nb_upd =
        fmode == 5 ? pair_cg5_rupd_launch(A, s, pcur, w.p, r.p, xb > 1 ? r0 : nullptr, dinv.mode, dinv.c, upart, fupd,
                                          fold_in_update ? part.p : nullptr, fold_in_update ? nb_spmv : 0, xb,
                                          poller.hw, st)
                   : cg_update_launch(st, n, s, pcur, w.p, defer_x ? nullptr : x, r.p, dinv, upart, fupd,
                                      fold_in_update ? part.p : nullptr, fold_in_update ? nb_spmv : 0, xb,
                                      xb > 1 ? r0 : nullptr, poller.hw);
    if (fmode == 5) utimer.end();
    if (!nb_upd) fail(MX_ERR_INTERNAL, "CG without its update pass");
    if (!fupd.cnt) fold_kernel<3><<<1, 256, 0, st>>>(upart, nb_upd, s->top.red3, done);
    if (!fused) c->allreduce_sum(s->top.red3, 3);
    HIPCHECK(hipGetLastError());
  };
  // a captured batch must start on an even iteration when p ping-pongs
  // graph replay: single-rank communicators by default (knob 7 = 1); with
  // multi-rank RCCL communicators only when asked (knob 7 = 2) -- a batch of
  // eager launches keeps the GPU busy there as well (measured within 2% of
  // replay on one rank), and eager RCCL calls are the well-trodden path
  bool graph = (g_knobs.graph >= 2 || (g_knobs.graph == 1 && c->size == 1)) && c->capturable && !p.profile &&
               (!fuse_cg || (poll & 1) == 0) && !A->cg_graph_failed;
  std::vector<uintptr_t> key;
  if (graph) {
    // the whole knob block is part of the key: every knob a captured kernel
    // could have baked in (template choice, launch geometry, argument) counts
    key = {(uintptr_t)x, (uintptr_t)r.p, (uintptr_t)r0, (uintptr_t)poller.hw, (uintptr_t)hist_d, (uintptr_t)dinv.mode, (uintptr_t)dinv.d, 0,
           (uintptr_t)poll, (uintptr_t)fmode, (uintptr_t)fold_at, (uintptr_t)pv.p, (uintptr_t)w.p, (uintptr_t)pv2,
           (uintptr_t)part.p, (uintptr_t)xb, (uintptr_t)pv3, (uintptr_t)pv4, (uintptr_t)pbs.b[4],
           (uintptr_t)pbs.b[5], (uintptr_t)pbs.b[6], (uintptr_t)pbs.b[7]};
    const int *kw = reinterpret_cast<const int *>(&g_knobs);
    for (size_t q = 0; q < sizeof(Knobs) / sizeof(int); ++q) key.push_back((uintptr_t)(uint32_t)kw[q]);
    std::memcpy(&key[7], &dinv.c, sizeof(double));
  }
  bool use_graph = graph && A->cg_graph && A->cg_key == key;
  // A capture records a batch of `poll` iterations without running them. A
  // single-rank communicator captures before its first iteration (so a short
  // first solve -- KSPSetUp, a warmup -- leaves the graph for the next one);
  // a multi-rank one after its first eager batch, which also warms every RCCL
  // connection the batch uses, so the capture holds only steady-state calls.
  // A batch shorter than `poll` (the max_it remainder) runs eagerly: replaying
  // a whole batch would launch iterations that only test the done flag.
  auto capture = [&]() {
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
  };
  if (graph && !use_graph && c->size == 1 && i < p.max_it) capture();
  for (; i < p.max_it;) {
    // knob 67: the solve's first batch is launched eagerly even when a graph
    // is cached -- the first replayed node started ~20 us after the launch
    // (the GPU idle after the state-init kernel) where eager launches keep
    // the queue ahead of these long kernels from the first one
    if (use_graph && p.max_it - i >= poll) {
      HIPCHECK(hipGraphLaunch(A->cg_graph, st));
      i += poll;
    } else {
      for (int k = 0; k < poll && i < p.max_it; ++k, ++i) iteration(i);
    }
    if (poller.batch(i)) break;
    if (graph && !use_graph && i < p.max_it) capture();
  }
  // the pending x steps (neither pass changes what the other reads), then
  // the tail: max_it launched without a stop, the result into the host words
  if (xb > 1) {
    cg_finish_xb_kernel<<<egrid, 256, 0, st>>>(n, s, pbs.b[0], pbs.b[1] - pbs.b[0], xb, x);
    HIPCHECK(hipGetLastError());
  } else if (defer_x) {   // p is in place for mode 2: both buffer slots are pv
    cg_finish_x_kernel<<<egrid, 256, 0, st>>>(n, s, pv.p, fuse_cg ? pv2 : pv.p, x);
    HIPCHECK(hipGetLastError());
  }
  cg_tail_kernel<<<1, 64, 0, st>>>(s, hist_d, poller.hw);
  HIPCHECK(hipGetLastError());
  c->wait_stream(st);
  res.its = poller.word(HW_ITS);
  res.reason = poller.word(HW_REASON);
  std::memcpy(&res.rnorm, (const void *)(poller.hw + HW_DP), sizeof(double));
  // device time: the state-init kernel to the tail kernel, on the device clock
  long long ticks = 0;
  std::memcpy(&ticks, (const void *)(poller.hw + HW_TICKS), sizeof(ticks));
  res.solve_ms = (double)ticks / wall_clock_khz(c->device);
  res.launched_its = i;
  timer.collect(res.spmv_ms, res.spmv_count);
  utimer.collect(res.upd_ms, res.upd_count);
  ptimer.collect(res.pb_ms, res.pb_count);
  wtimer.collect(res.pbw_ms, res.pbw_count);
  res.cg_mode = fmode;
  res.cg_xbatch = xb;
  if (hist_host)
    HIPCHECK(hipMemcpy(hist_host, hist.p, sizeof(double) * ((size_t)res.its + 1), hipMemcpyDeviceToHost));
}

// Grid of every MDot launch of a solve (one partial row stride for the
// finish): knob 36, default one resident generation of the chunk kernel (153
// VGPRs: three workgroups per CU -- 768 on 256 CUs -- instead of 1024 in two
// uneven generations)
static int mdot_grid() {
  if (g_knobs.mdot_grid > 0) return g_knobs.mdot_grid;
  return std::min(RED_BLOCKS, 3 * device_cu_count());
}

template <int NV>
static void launch_mdot(hipStream_t st, int64_t n, const double *w, const double *V, int64_t ldv, int j0, int k,
                        const double *vscale, double *partials, const int *stop_flag, int grid) {
  mdot_kernel<NV><<<grid, 256, 0, st>>>(n, w, V, ldv, j0, k, vscale, partials, stop_flag);
}

// VecMDot of nv vectors: one pass over w (chunk form) up to 32 vectors (every
// GMRES(30) step), groups of 8 vectors per pass beyond (restart > 31).
// Partials rows [j0, j0 + NV) are written (rows >= nv with zeros): the
// buffer holds max_k + 2 rows rounded up to 32
static void mdot(hipStream_t st, int64_t n, const double *w, const double *V, int64_t ldv, int nv,
                 const double *vscale, double *partials, const int *stop_flag, int grid) {
  if (nv <= 32) {
    launch_timed(&mdot_chunk_kernel, grid, st, n, w, V, ldv, nv, vscale, partials, stop_flag);
    HIPCHECK(hipGetLastError());
    return;
  }
  for (int j0 = 0; j0 < nv; j0 += 8) {
    const int k = std::min(8, nv - j0);
    if (k <= 2) launch_mdot<2>(st, n, w, V, ldv, j0, k, vscale, partials, stop_flag, grid);
    else if (k <= 4) launch_mdot<4>(st, n, w, V, ldv, j0, k, vscale, partials, stop_flag, grid);
    else launch_mdot<8>(st, n, w, V, ldv, j0, k, vscale, partials, stop_flag, grid);
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
  // basis stride: n rounded up to 32 rows, plus knob 54's extra rows (the
  // vectors' relative placement in HBM: an A/B lever for the MDot / MAXPY)
  const int64_t ldv = (std::max<int64_t>(n, 1) + 31) / 32 * 32 + std::max(0, g_knobs.gm_pad) / 32 * 32;
  const size_t nV = (size_t)ldv * (max_k + 1), nh = (size_t)ld * (max_k + 1);
  const size_t prow = std::max<size_t>((size_t)max_k + 2, ((size_t)max_k + 1 + 31) / 32 * 32);   // MDot groups of 32
  const size_t npart = (size_t)RED_BLOCKS * prow + (size_t)spmv_blocks(A) + 128;
  const int mgrid = mdot_grid();   // <= RED_BLOCKS
  const size_t nhist = hist_host ? (size_t)p.max_it + 2 : 1;
  const size_t k1 = (size_t)max_k + 1, k2 = (size_t)max_k + 2;
  Carve cv(workspace(A, carve_size({nV, (size_t)ldv, nh, k2, k1, k1, k2, k2, npart, nhist})));
  struct B { double *p; size_t n; };
  B V{cv.take(nV), nV}, tmat{cv.take(ldv), (size_t)ldv}, hh{cv.take(nh), nh}, grs{cv.take(k2), k2},
      cc{cv.take(k1), k1}, ss{cv.take(k1), k1}, red{cv.take(k2), k2}, vsc{cv.take(k2), k2},
      part{cv.take(npart), npart}, hist{cv.take(nhist), nhist};
  vec_set(st, (int64_t)vsc.n, 1.0, vsc.p);
  HIPCHECK(hipMemsetAsync(hh.p, 0, sizeof(double) * hh.n, st));
  if (hist_host) HIPCHECK(hipMemsetAsync(hist.p, 0, sizeof(double) * hist.n, st));   // as in CG
  struct { KspState *p; } sd{state_buf(A)};
  KspState hs;
  init_state(hs, p, MX_NORM_PRECONDITIONED);
  if (p.norm_type != MX_NORM_DEFAULT && p.norm_type != MX_NORM_PRECONDITIONED)
    fail(MX_ERR_UNSUPPORTED, "GMRES with left preconditioning supports the preconditioned norm only");
  hs.max_k = max_k;
  write_state(A, st, sd.p, hs);
  KspState *s = sd.p;
  double *sred = reinterpret_cast<double *>(s);
  const bool fused = c->size == 1;
  double *hist_d = hist_host ? hist.p : nullptr;
  Events ev(A);
  SpmvTimer timer((p.profile & 1) != 0, st, std::min(p.max_it, 4096));
  timer.ext = c->size == 1;
  SpmvTimer dtimer((p.profile & 2) != 0, st, std::min(p.max_it, 4096));   // MDot
  dtimer.ext = c->size == 1;
  SpmvTimer xtimer((p.profile & 4) != 0, st, std::min(p.max_it, 4096));   // MAXPY + norm
  xtimer.ext = c->size == 1;
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
    c->wait_stream(st);
    snorm = std::sqrt(snorm);
  }
  int first = 1, launched = 0;
  int *istop = &s->inner_stop;
  Poller poller(A, st);            // its pinned words: the step count (HW_PROGRESS)
  Fold fnorm;                      // ||w||^2 of the MAXPY pass, folded in-launch into s->red[0]
  // MAXPY + norm grid (knob 77; one partial per workgroup, within part's rows)
  // the MAXPY + norm pass walks the basis in chunks on MDot's grid (maxpy_norm_kernel)
  const int xgrid = g_knobs.maxpy_grid > 0 ? std::min<int>(g_knobs.maxpy_grid, (int)std::min<size_t>(npart, 16384)) : mdot_grid();
  fnorm.cnt = s->fold_upd; fnorm.out = sred; fnorm.ntotal = fnorm.ncount = xgrid;
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
    gm_start_kernel<<<1, 256, 0, st>>>(s, part.p, RED_BLOCKS, fused, grs.p, hist_d, first ? snorm : 0.0, vsc.p);
    HIPCHECK(hipGetLastError());
    first = 0;
    const long long cycle_base = launched;   // the progress word before this cycle's steps
    for (int k = 0; k < max_k; ++k) {
      double *vk = V.p + (int64_t)k * ldv, *vk1 = V.p + (int64_t)(k + 1) * ldv;
      timer.begin();
      matmult_overlap(A, vk, vk1, dinv.mode ? SPMV_JACOBI_S : SPMV_PLAIN_S, dinv, nullptr, istop, nullptr,
                      nullptr, vsc.p + k);
      timer.end();
      dtimer.begin();
      mdot(st, n, vk1, V.p, ldv, k + 1, vsc.p, part.p, istop, mgrid);
      dtimer.end();
      finish_many_kernel<<<k + 1, 256, 0, st>>>(part.p, mgrid, red.p, istop);
      c->allreduce_sum(red.p, k + 1);
      // orthogonalisation coefficients + MAXPY + ||w||^2 folded in-launch
      xtimer.begin();
      launch_timed(&maxpy_norm_kernel, xgrid, st, n, vk1, (const double *)V.p, ldv, k + 1, s,
                   (const double *)red.p, (const double *)vsc.p, hh.p, ld, part.p, fnorm);
      xtimer.end();
      c->allreduce_sum(sred, 1);
      ++launched;
      gm_step_kernel<<<1, 256, 0, st>>>(s, k, part.p, xgrid, 0, hh.p, ld, grs.p, cc.p, ss.p, hist_d, vsc.p,
                                        poller.hw, launched);
      HIPCHECK(hipGetLastError());
    }
    gm_buildsoln_kernel<<<1, 256, 0, st>>>(s, hh.p, ld, grs.p);
    gm_update_x_kernel<<<egrid, 256, 0, st>>>(n, s, V.p, ldv, vsc.p, grs.p, x);
    gm_cycle_end_kernel<<<1, 64, 0, st>>>(s);
    HIPCHECK(hipGetLastError());
    if (g_knobs.gm_stall_us > 0) debug_stall(st, g_knobs.gm_stall_us);   // knob 61: the deadline tests
    // the cycle's state read-back: a wait that observes the step count
    HIPCHECK(hipMemcpyAsync(A->state_pinned, s, sizeof(KspState), hipMemcpyDeviceToHost, st));
    c->wait_until([] { return false; }, st, [&] { return (long long)poller.word(HW_PROGRESS); }, cycle_base);
    std::memcpy(&hs, A->state_pinned, sizeof(KspState));
    if (hs.top.done) break;
  }
  HIPCHECK(hipEventRecord(ev.b, st));
  c->wait_event(ev.b);
  float ms = 0.f;
  HIPCHECK(hipEventElapsedTime(&ms, ev.a, ev.b));
  res.its = hs.its;
  res.reason = hs.reason;
  res.rnorm = hs.ksp_rnorm;
  res.solve_ms = ms;
  res.launched_its = launched;
  timer.collect(res.spmv_ms, res.spmv_count);
  dtimer.collect(res.mdot_ms, res.mdot_count);
  xtimer.collect(res.maxpy_ms, res.maxpy_count);
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

// this translation unit's code object, loaded now rather than at the first
// launch of one of its kernels (load_code_objects)
void load_code_ksp() {
  hipFuncAttributes a;
  (void)hipFuncGetAttributes(&a, reinterpret_cast<const void *>(&jacobi_setup_kernel));
  (void)hipGetLastError();
}

}  // namespace mx
