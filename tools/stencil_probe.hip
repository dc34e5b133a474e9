// Ceiling probe for the 256^3 7-point MatMult (not product code): how fast can
// y = A x with x read and y written once run on this GPU, by access scheme?
//   copy      : y = x, 16 B per lane (the stream ceiling for 268 MB)
//   pairs<U>  : matrix-free 7-point, two rows per lane, U units per wave step,
//               each XCD sweeping one contiguous eighth (the product's order)
//   zmarch    : 2.5D: a workgroup owns a y-tile of lines and marches z,
//               keeping planes in LDS (x read once from HBM per tile)
// hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/stencil_probe tools/stencil_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <algorithm>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
typedef double dbl2 __attribute__((ext_vector_type(2)));

constexpr int N = 256;
constexpr int64_t NN = (int64_t)N * N, M = NN * N;

__global__ void copy_kernel(const dbl2 *__restrict__ x, dbl2 *__restrict__ y, int64_t n2) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n2; i += (int64_t)gridDim.x * blockDim.x)
    y[i] = __builtin_nontemporal_load(x + i);
}

template <bool UP>
__device__ __forceinline__ double wave_shift(double v, double edge) {
  const long long b = __double_as_longlong(v), e = __double_as_longlong(edge);
  constexpr int ctrl = UP ? 0x138 : 0x130;
  const int lo = __builtin_amdgcn_update_dpp((int)e, (int)b, ctrl, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp((int)(e >> 32), (int)(b >> 32), ctrl, 0xf, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

__device__ __forceinline__ double xat(const double *x, int64_t i) { return (i >= 0 && i < M) ? x[i] : 0.0; }
__device__ __forceinline__ dbl2 xpair(const double *x, int64_t i) {
  return (i >= 0 && i + 1 < M) ? *reinterpret_cast<const dbl2 *>(x + i) : dbl2{0.0, 0.0};
}

// one 128-row unit: lane = rows r0, r0 + 1
struct UnitL { dbl2 zm, ym, c, yp, zp; double elo, ehi; };
__device__ __forceinline__ void unit_load(const double *x, int64_t u, int lane, UnitL &t) {
  const int64_t ub = u * 128, r0 = ub + 2 * lane;
  t.zm = xpair(x, r0 - NN); t.ym = xpair(x, r0 - N); t.c = xpair(x, r0);
  t.yp = xpair(x, r0 + N); t.zp = xpair(x, r0 + NN);
  t.elo = xat(x, ub - 1); t.ehi = xat(x, ub + 128);
}
__device__ __forceinline__ void unit_finish(double *y, int64_t u, int lane, const UnitL &t) {
  const int64_t r0 = u * 128 + 2 * lane;
  const double lo = wave_shift<true>(t.c.y, t.elo), hi = wave_shift<false>(t.c.x, t.ehi);
  const double s0 = 6.0 * t.c.x - t.zm.x - t.ym.x - lo - t.c.y - t.yp.x - t.zp.x;
  const double s1 = 6.0 * t.c.y - t.zm.y - t.ym.y - t.c.x - hi - t.yp.y - t.zp.y;
  *reinterpret_cast<dbl2 *>(y + r0) = dbl2{s0, s1};
}

template <int U>
__global__ void __launch_bounds__(256) pairs_kernel(const double *__restrict__ x, double *__restrict__ y, int64_t nunits) {
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int per = gridDim.x >> 3, xcd = blockIdx.x & 7, j = blockIdx.x >> 3;
  const int64_t chunk = (nunits + 7) >> 3;
  const int64_t s0 = xcd * chunk + (int64_t)j * 4 + wid, step = (int64_t)per * 4;
  const int64_t send = min(nunits, (xcd + 1) * chunk);
  int64_t u = s0;
  for (; u + (U - 1) * step < send; u += U * step) {
    UnitL t[U];
#pragma unroll
    for (int k = 0; k < U; ++k) unit_load(x, u + k * step, lane, t[k]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int k = 0; k < U; ++k) unit_finish(y, u + k * step, lane, t[k]);
  }
  for (; u < send; u += step) { UnitL t; unit_load(x, u, lane, t); unit_finish(y, u, lane, t); }
}

// the product's row-pair scheme with its coded values: per unit a 16-B code
// block per lane from a small dictionary (L2), codes -> values through an LDS
// table, absent slots skipped by select; optional p.w dot partial (DOT)
constexpr int ABSENT = 255;
template <int U, bool DOT, bool META>
__global__ void __launch_bounds__(256) pcodes_kernel(const double *__restrict__ x, double *__restrict__ y, int64_t nunits,
                                                     const uint8_t *__restrict__ dict, const int32_t *__restrict__ pblk,
                                                     const double *__restrict__ vtab_g, double *__restrict__ part) {
  __shared__ double vtab[256];
  for (int i = threadIdx.x; i < 256; i += 256) vtab[i] = vtab_g[i];
  __syncthreads();
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int per = gridDim.x >> 3, xcd = blockIdx.x & 7, j = blockIdx.x >> 3;
  const int64_t chunk = (nunits + 7) >> 3;
  const int64_t s0 = xcd * chunk + (int64_t)j * 4 + wid, step = (int64_t)per * 4;
  const int64_t send = min(nunits, (xcd + 1) * chunk);
  double dot = 0.0;
  struct T { UnitL l; u32x4 cw; };
  auto ld = [&](int64_t u, T &t) {
    unit_load(x, u, lane, t.l);
    const int blk = META ? pblk[u] : (int)(u & 1);
    t.cw = *reinterpret_cast<const u32x4 *>(dict + ((int64_t)blk * 64 + lane) * 16);
  };
  auto fin = [&](int64_t u, const T &t) {
    const int64_t r0 = u * 128 + 2 * lane;
    auto code = [&](int i) -> int { return (t.cw[(i >> 2) & 3] >> (8 * (i & 3))) & 0xff; };
    const double lo = wave_shift<true>(t.l.c.y, t.l.elo), hi = wave_shift<false>(t.l.c.x, t.l.ehi);
    const double a0[7] = {t.l.zm.x, t.l.ym.x, lo, t.l.c.x, t.l.c.y, t.l.yp.x, t.l.zp.x};
    const double a1[7] = {t.l.zm.y, t.l.ym.y, t.l.c.x, t.l.c.y, hi, t.l.yp.y, t.l.zp.y};
    double s0 = 0.0, s1 = 0.0;
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      const int c0 = code(k), c1 = code(7 + k);
      const double q0 = s0 + vtab[c0] * a0[k], q1 = s1 + vtab[c1] * a1[k];
      s0 = c0 != ABSENT ? q0 : s0;
      s1 = c1 != ABSENT ? q1 : s1;
    }
    *reinterpret_cast<dbl2 *>(y + r0) = dbl2{s0, s1};
    if (DOT) { dot += t.l.c.x * s0; dot += t.l.c.y * s1; }
  };
  int64_t u = s0;
  for (; u + (U - 1) * step < send; u += U * step) {
    T t[U];
#pragma unroll
    for (int k = 0; k < U; ++k) ld(u + k * step, t[k]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int k = 0; k < U; ++k) fin(u + k * step, t[k]);
  }
  for (; u < send; u += step) { T t; ld(u, t); fin(u, t); }
  if (DOT) {
    for (int o = 32; o > 0; o >>= 1) dot += __shfl_xor(dot, o);
    if (lane == 0) part[blockIdx.x * 4 + wid] = dot;
  }
}

// pcodes with buffer loads (out-of-range reads return 0: no bounds logic) and
// the dictionary block ids of the wave's next 64 steps in one vector load,
// read per step by readlane (no dependent scalar load per unit)
// DREG: the dictionary's two blocks held in VGPRs (loaded once per wave),
// the unit's block selected by its id -- no dependent code load per unit
template <int U, bool DOT, int META = 1, bool BUF = true, bool DREG = false>
__global__ void __launch_bounds__(256) pbuf_kernel(const double *__restrict__ x, double *__restrict__ y, int64_t nunits,
                                                   const uint8_t *__restrict__ dict, const int32_t *__restrict__ pblk,
                                                   const double *__restrict__ vtab_g, double *__restrict__ part) {
  __shared__ double vtab[256];
  for (int i = threadIdx.x; i < 256; i += 256) vtab[i] = vtab_g[i];
  __syncthreads();
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int per = gridDim.x >> 3, xcd = blockIdx.x & 7, j = blockIdx.x >> 3;
  const int64_t chunk = (nunits + 7) >> 3;
  const int64_t s0 = xcd * chunk + (int64_t)j * 4 + wid, step = (int64_t)per * 4;
  const int64_t send = min(nunits, (xcd + 1) * chunk);
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void *)x, 0, (int)(M * 8), 0x00020000);
  double dot = 0.0;
  struct T { dbl2 zm, ym, c, yp, zp; double elo, ehi; u32x4 cw; };
  u32x4 dreg0 = {0, 0, 0, 0}, dreg1 = {0, 0, 0, 0};
  if (DREG) {
    dreg0 = *reinterpret_cast<const u32x4 *>(dict + (int64_t)lane * 16);
    dreg1 = *reinterpret_cast<const u32x4 *>(dict + (int64_t)(64 + lane) * 16);
  }
  auto ldp = [&](int64_t i) -> dbl2 {
    if (!BUF) return xpair(x, i);
    return __builtin_bit_cast(dbl2, __builtin_amdgcn_raw_buffer_load_b128(xr, (int)(i * 8), 0, 0));
  };
  auto lds = [&](int64_t i) -> double {
    if (!BUF) return xat(x, i);
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(xr, (int)(i * 8), 0, 0));
  };
  auto ld = [&](int64_t u, int blk, T &t) {
    const int64_t ub = u * 128, r0 = ub + 2 * lane;
    t.zm = ldp(r0 - NN); t.ym = ldp(r0 - N); t.c = ldp(r0); t.yp = ldp(r0 + N); t.zp = ldp(r0 + NN);
    t.elo = lds(ub - 1); t.ehi = lds(ub + 128);
    if (DREG) t.cw = blk ? dreg1 : dreg0;
    else t.cw = *reinterpret_cast<const u32x4 *>(dict + ((int64_t)blk * 64 + lane) * 16);
  };
  auto fin = [&](int64_t u, const T &t) {
    const int64_t r0 = u * 128 + 2 * lane;
    auto code = [&](int i) -> int { return (t.cw[(i >> 2) & 3] >> (8 * (i & 3))) & 0xff; };
    const double lo = wave_shift<true>(t.c.y, t.elo), hi = wave_shift<false>(t.c.x, t.ehi);
    const double a0[7] = {t.zm.x, t.ym.x, lo, t.c.x, t.c.y, t.yp.x, t.zp.x};
    const double a1[7] = {t.zm.y, t.ym.y, t.c.x, t.c.y, hi, t.yp.y, t.zp.y};
    double s0 = 0.0, s1 = 0.0;
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      const int c0 = code(k), c1 = code(7 + k);
      const double q0 = s0 + vtab[c0] * a0[k], q1 = s1 + vtab[c1] * a1[k];
      s0 = c0 != ABSENT ? q0 : s0;
      s1 = c1 != ABSENT ? q1 : s1;
    }
    *reinterpret_cast<dbl2 *>(y + r0) = dbl2{s0, s1};
    if (DOT) { dot += t.c.x * s0; dot += t.c.y * s1; }
  };
  int64_t u = s0;
  int kstep = 64;
  int bv = 0;
  for (; u + (U - 1) * step < send; u += U * step) {
    if (META && kstep + U > 64) {          // refill: block ids of the next 64 steps
      const int64_t uu = u + lane * step;
      bv = uu < send ? pblk[uu] : 0;
      kstep = 0;
    }
    T t[U];
#pragma unroll
    for (int k = 0; k < U; ++k) ld(u + k * step, META ? __builtin_amdgcn_readlane(bv, kstep + k) : (int)((u + k * step) & 1), t[k]);
    kstep += U;
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int k = 0; k < U; ++k) fin(u + k * step, t[k]);
  }
  for (; u < send; u += step) { T t; ld(u, pblk[u], t); fin(u, t); }
  if (DOT) {
    for (int o = 32; o > 0; o >>= 1) dot += __shfl_xor(dot, o);
    if (lane == 0) part[blockIdx.x * 4 + wid] = dot;
  }
}

// wave-blocked sweep: each wave owns a CONTIGUOUS run of C units (XCD-major
// numbering, so an XCD's waves cover one contiguous eighth and the +-n^2
// neighbours 512 units away are 16 waves over, on the same XCD at the same
// step); the run's dictionary block ids come in with ONE vector load
template <int U, bool DOT, int META>
__global__ void __launch_bounds__(256) pblk_kernel(const double *__restrict__ x, double *__restrict__ y, int64_t nunits,
                                                   const uint8_t *__restrict__ dict, const int32_t *__restrict__ pblk,
                                                   const double *__restrict__ vtab_g, double *__restrict__ part) {
  __shared__ double vtab[256];
  for (int i = threadIdx.x; i < 256; i += 256) vtab[i] = vtab_g[i];
  __syncthreads();
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int per = gridDim.x >> 3, xcd = blockIdx.x & 7, j = blockIdx.x >> 3;
  const int64_t nw = (int64_t)gridDim.x * 4;
  const int64_t C = (nunits + nw - 1) / nw;
  const int64_t w = (int64_t)xcd * per * 4 + j * 4 + wid;    // XCD-major wave number
  const int64_t u0 = w * C, u1 = min(nunits, u0 + C);
  double dot = 0.0;
  int bv = 0;
  if (META == 1) bv = (u0 + lane < u1) ? pblk[u0 + lane] : 0;
  struct T { UnitL l; u32x4 cw; };
  auto ld = [&](int64_t u, int blk, T &t) {
    unit_load(x, u, lane, t.l);
    t.cw = *reinterpret_cast<const u32x4 *>(dict + ((int64_t)blk * 64 + lane) * 16);
  };
  auto fin = [&](int64_t u, const T &t) {
    const int64_t r0 = u * 128 + 2 * lane;
    auto code = [&](int i) -> int { return (t.cw[(i >> 2) & 3] >> (8 * (i & 3))) & 0xff; };
    const double lo = wave_shift<true>(t.l.c.y, t.l.elo), hi = wave_shift<false>(t.l.c.x, t.l.ehi);
    const double a0[7] = {t.l.zm.x, t.l.ym.x, lo, t.l.c.x, t.l.c.y, t.l.yp.x, t.l.zp.x};
    const double a1[7] = {t.l.zm.y, t.l.ym.y, t.l.c.x, t.l.c.y, hi, t.l.yp.y, t.l.zp.y};
    double s0 = 0.0, s1 = 0.0;
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      const int c0 = code(k), c1 = code(7 + k);
      const double q0 = s0 + vtab[c0] * a0[k], q1 = s1 + vtab[c1] * a1[k];
      s0 = c0 != ABSENT ? q0 : s0;
      s1 = c1 != ABSENT ? q1 : s1;
    }
    *reinterpret_cast<dbl2 *>(y + r0) = dbl2{s0, s1};
    if (DOT) { dot += t.l.c.x * s0; dot += t.l.c.y * s1; }
  };
  auto blk_of = [&](int64_t u) -> int {
    if (META == 1) return __builtin_amdgcn_readlane(bv, (int)(u - u0));
    if (META == 2) return pblk[u];
    return (int)(u & 1);
  };
  int64_t u = u0;
  for (; u + U - 1 < u1; u += U) {
    T t[U];
#pragma unroll
    for (int k = 0; k < U; ++k) ld(u + k, blk_of(u + k), t[k]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int k = 0; k < U; ++k) fin(u + k, t[k]);
  }
  for (; u < u1; ++u) { T t; ld(u, blk_of(u), t); fin(u, t); }
  if (DOT) {
    for (int o = 32; o > 0; o >>= 1) dot += __shfl_xor(dot, o);
    if (lane == 0) part[blockIdx.x * 4 + wid] = dot;
  }
}

// pcodes with the prologue overlapped: the value table's global load and the
// first step's x loads are issued before the table is written to LDS and the
// workgroup barrier; block ids by scalar loads one step ahead (META 1) or
// from the unit index (META 0)
template <bool DOT, int META>
__global__ void __launch_bounds__(256) pov_kernel(const double *__restrict__ x, double *__restrict__ y, int64_t nunits,
                                                  const uint8_t *__restrict__ dict, const int32_t *__restrict__ pblk,
                                                  const double *__restrict__ vtab_g, double *__restrict__ part) {
  __shared__ double vtab[256];
  const double vt_reg = vtab_g[threadIdx.x];
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int per = gridDim.x >> 3, xcd = blockIdx.x & 7, j = blockIdx.x >> 3;
  const int64_t chunk = (nunits + 7) >> 3;
  const int64_t s0 = xcd * chunk + (int64_t)j * 4 + wid, step = (int64_t)per * 4;
  const int64_t send = min(nunits, (xcd + 1) * chunk);
  double dot = 0.0;
  struct T { UnitL l; u32x4 cw; };
  auto ldx = [&](int64_t u, T &t) { unit_load(x, u, lane, t.l); };
  auto ldc = [&](int blk, T &t) { t.cw = *reinterpret_cast<const u32x4 *>(dict + ((int64_t)blk * 64 + lane) * 16); };
  auto fin = [&](int64_t u, const T &t) {
    const int64_t r0 = u * 128 + 2 * lane;
    auto code = [&](int i) -> int { return (t.cw[(i >> 2) & 3] >> (8 * (i & 3))) & 0xff; };
    const double lo = wave_shift<true>(t.l.c.y, t.l.elo), hi = wave_shift<false>(t.l.c.x, t.l.ehi);
    const double a0[7] = {t.l.zm.x, t.l.ym.x, lo, t.l.c.x, t.l.c.y, t.l.yp.x, t.l.zp.x};
    const double a1[7] = {t.l.zm.y, t.l.ym.y, t.l.c.x, t.l.c.y, hi, t.l.yp.y, t.l.zp.y};
    double s0 = 0.0, s1 = 0.0;
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      const int c0 = code(k), c1 = code(7 + k);
      const double q0 = s0 + vtab[c0] * a0[k], q1 = s1 + vtab[c1] * a1[k];
      s0 = c0 != ABSENT ? q0 : s0;
      s1 = c1 != ABSENT ? q1 : s1;
    }
    *reinterpret_cast<dbl2 *>(y + r0) = dbl2{s0, s1};
    if (DOT) { dot += t.l.c.x * s0; dot += t.l.c.y * s1; }
  };
  auto mb = [&](int64_t u) -> int { return u < send ? (META ? pblk[u] : (int)(u & 1)) : 0; };
  int64_t u = s0;
  int ba = mb(u), bb = mb(u + step);
  bool first = true;
  while (true) {
    const bool two = u + step < send, one = u < send;
    T ta, tb;
    if (one) ldx(u, ta);
    if (two) ldx(u + step, tb);
    if (one) ldc(ba, ta);
    if (two) ldc(bb, tb);
    const int na = mb(u + 2 * step), nb = mb(u + 3 * step);   // next step's block ids, behind this step's loads
    __builtin_amdgcn_sched_barrier(0);
    if (first) {                         // the table lands while the first loads are in flight
      vtab[threadIdx.x] = vt_reg;
      __syncthreads();
      first = false;
    }
    if (!one) break;
    fin(u, ta);
    if (two) fin(u + step, tb);
    u += 2 * step;
    ba = na; bb = nb;
  }
  if (DOT) {
    for (int o = 32; o > 0; o >>= 1) dot += __shfl_xor(dot, o);
    if (lane == 0) part[blockIdx.x * 4 + wid] = dot;
  }
}

// codes without the LDS table: two distinct values selected per slot from
// kernel-argument scalars (the constant-coefficient stencils have exactly
// two), so no LDS read shares lgkmcnt with the scalar block-id loads;
// META 0: block id from the unit index, 1: scalar loads two steps ahead
template <int META>
__global__ void __launch_bounds__(256) psel_kernel(const double *__restrict__ x, double *__restrict__ y, int64_t nunits,
                                                   const uint8_t *__restrict__ dict, const int32_t *__restrict__ pblk,
                                                   double v0, double v1, double *__restrict__ part) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int per = gridDim.x >> 3, xcd = blockIdx.x & 7, j = blockIdx.x >> 3;
  const int64_t chunk = (nunits + 7) >> 3;
  const int64_t s0 = xcd * chunk + (int64_t)j * 4 + wid, step = (int64_t)per * 4;
  const int64_t send = min(nunits, (xcd + 1) * chunk);
  double dot = 0.0;
  struct T { UnitL l; u32x4 cw; };
  auto ld = [&](int64_t u, int blk, T &t) {
    unit_load(x, u, lane, t.l);
    t.cw = *reinterpret_cast<const u32x4 *>(dict + ((int64_t)blk * 64 + lane) * 16);
  };
  auto fin = [&](int64_t u, const T &t) {
    const int64_t r0 = u * 128 + 2 * lane;
    auto code = [&](int i) -> int { return (t.cw[(i >> 2) & 3] >> (8 * (i & 3))) & 0xff; };
    const double lo = wave_shift<true>(t.l.c.y, t.l.elo), hi = wave_shift<false>(t.l.c.x, t.l.ehi);
    const double a0[7] = {t.l.zm.x, t.l.ym.x, lo, t.l.c.x, t.l.c.y, t.l.yp.x, t.l.zp.x};
    const double a1[7] = {t.l.zm.y, t.l.ym.y, t.l.c.x, t.l.c.y, hi, t.l.yp.y, t.l.zp.y};
    double s0 = 0.0, s1 = 0.0;
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      const int c0 = code(k), c1 = code(7 + k);
      const double q0 = s0 + (c0 == 0 ? v0 : v1) * a0[k], q1 = s1 + (c1 == 0 ? v0 : v1) * a1[k];
      s0 = c0 != ABSENT ? q0 : s0;
      s1 = c1 != ABSENT ? q1 : s1;
    }
    *reinterpret_cast<dbl2 *>(y + r0) = dbl2{s0, s1};
    dot += t.l.c.x * s0; dot += t.l.c.y * s1;
  };
  auto mb = [&](int64_t u) -> int { return u < send ? (META ? pblk[u] : (int)(u & 1)) : 0; };
  int64_t u = s0;
  int ca = mb(u), cb = mb(u + step), na = mb(u + 2 * step), nb = mb(u + 3 * step);
  for (; u + step < send; u += 2 * step) {
    const int fa = mb(u + 4 * step), fb = mb(u + 5 * step);
    T ta, tb;
    ld(u, ca, ta);
    ld(u + step, cb, tb);
    __builtin_amdgcn_sched_barrier(0);
    fin(u, ta);
    fin(u + step, tb);
    ca = na; cb = nb; na = fa; nb = fb;
  }
  for (; u < send; u += step) { T t; ld(u, mb(u), t); fin(u, t); }
  for (int o = 32; o > 0; o >>= 1) dot += __shfl_xor(dot, o);
  if (lane == 0) part[blockIdx.x * 4 + wid] = dot;
}

// narrow codes: 2 bits per slot (0, 1 = table entries, 3 = absent), the 14
// slots of a lane in ONE 4-byte word: the code-block load is 256 B per wave
// instead of 1 KB (TA/L1 work is the bound); values still from the LDS table
template <bool META>
__global__ void __launch_bounds__(256) pnarrow_kernel(const double *__restrict__ x, double *__restrict__ y, int64_t nunits,
                                                      const uint32_t *__restrict__ dict2, const int32_t *__restrict__ pblk,
                                                      const double *__restrict__ vtab_g, double *__restrict__ part) {
  __shared__ double vtab[256];
  for (int i = threadIdx.x; i < 256; i += 256) vtab[i] = vtab_g[i];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int per = gridDim.x >> 3, xcd = blockIdx.x & 7, j = blockIdx.x >> 3;
  const int64_t chunk = (nunits + 7) >> 3;
  const int64_t s0 = xcd * chunk + (int64_t)j * 4 + wid, step = (int64_t)per * 4;
  const int64_t send = min(nunits, (xcd + 1) * chunk);
  double dot = 0.0;
  struct T { UnitL l; uint32_t cw; };
  auto ld = [&](int64_t u, int blk, T &t) {
    unit_load(x, u, lane, t.l);
    t.cw = dict2[(int64_t)blk * 64 + lane];
  };
  auto fin = [&](int64_t u, const T &t) {
    const int64_t r0 = u * 128 + 2 * lane;
    const double lo = wave_shift<true>(t.l.c.y, t.l.elo), hi = wave_shift<false>(t.l.c.x, t.l.ehi);
    const double a0[7] = {t.l.zm.x, t.l.ym.x, lo, t.l.c.x, t.l.c.y, t.l.yp.x, t.l.zp.x};
    const double a1[7] = {t.l.zm.y, t.l.ym.y, t.l.c.x, t.l.c.y, hi, t.l.yp.y, t.l.zp.y};
    double s0 = 0.0, s1 = 0.0;
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      const int c0 = (t.cw >> (2 * k)) & 3, c1 = (t.cw >> (2 * (7 + k))) & 3;
      const double q0 = s0 + vtab[c0] * a0[k], q1 = s1 + vtab[c1] * a1[k];
      s0 = c0 != 3 ? q0 : s0;
      s1 = c1 != 3 ? q1 : s1;
    }
    *reinterpret_cast<dbl2 *>(y + r0) = dbl2{s0, s1};
    dot += t.l.c.x * s0; dot += t.l.c.y * s1;
  };
  auto mb = [&](int64_t u) -> int { return u < send ? (META ? pblk[u] : (int)(u & 1)) : 0; };
  int64_t u = s0;
  int ca = mb(u), cb = mb(u + step), na = mb(u + 2 * step), nb = mb(u + 3 * step);
  for (; u + step < send; u += 2 * step) {
    const int fa = mb(u + 4 * step), fb = mb(u + 5 * step);
    T ta, tb;
    ld(u, ca, ta);
    ld(u + step, cb, tb);
    __builtin_amdgcn_sched_barrier(0);
    fin(u, ta);
    fin(u + step, tb);
    ca = na; cb = nb; na = fa; nb = fb;
  }
  for (; u < send; u += step) { T t; ld(u, mb(u), t); fin(u, t); }
  for (int o = 32; o > 0; o >>= 1) dot += __shfl_xor(dot, o);
  if (lane == 0) part[blockIdx.x * 4 + wid] = dot;
}

// 2.5D z-march: workgroup = (tile of TY lines in y) x (z range of ZR planes),
// 256 threads = one line's columns, PER = TY values per thread per plane plus
// the two y-halo values.  Planes live in a 4-slot register ring (static slot
// indices: the z loop is unrolled by 4), loaded two planes ahead; x+-1 and
// y+-1 neighbours come from the current plane staged in LDS.
template <int TY, int ZR>
__global__ void __launch_bounds__(256) zmarch_kernel(const double *__restrict__ x, double *__restrict__ y) {
  static_assert(ZR % 4 == 0, "ring");
  constexpr int PER = TY + 2;                    // [0] halo y0-1, [1..TY] tile lines, [TY+1] halo y0+TY
  __shared__ double pl[2][(TY + 2) * N + 2];
  const int ntile = N / TY;
  const int tile = blockIdx.x % ntile, zb = blockIdx.x / ntile;
  const int y0 = tile * TY, z0 = zb * ZR;
  const int t = threadIdx.x;
  double ring[4][PER];
  auto load = [&](int z, double *dst) {
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int yy = y0 - 1 + k;
      const bool ok = z >= 0 && z < N && yy >= 0 && yy < N;
      const int64_t g = ok ? (int64_t)z * NN + (int64_t)yy * N + t : 0;
      const double v = (k == 0 || k == PER - 1) ? x[g] : __builtin_nontemporal_load(x + g);
      dst[k] = ok ? v : 0.0;
    }
  };
  load(z0 - 1, ring[3]);
  load(z0, ring[0]);
  load(z0 + 1, ring[1]);
  for (int zz = z0; zz < z0 + ZR; zz += 4) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int z = zz + q;
      double *prev = ring[(q + 3) & 3], *cur = ring[q], *next = ring[(q + 1) & 3];
      load(z + 2, ring[(q + 2) & 3]);            // overwrites plane z - 2's slot
      double *P = pl[q & 1];
#pragma unroll
      for (int k = 0; k < PER; ++k) P[1 + k * N + t] = cur[k];
      if (t == 0) { P[0] = 0.0; P[(TY + 2) * N + 1] = 0.0; }
      __syncthreads();
#pragma unroll
      for (int k = 1; k <= TY; ++k) {
        const int li = 1 + k * N + t;
        const double xm = t > 0 ? P[li - 1] : 0.0, xp = t < N - 1 ? P[li + 1] : 0.0;
        const double s = 6.0 * cur[k] - prev[k] - P[li - N] - xm - xp - P[li + N] - next[k];
        y[(int64_t)z * NN + (int64_t)(y0 + k - 1) * N + t] = s;
      }
    }
  }
}

__global__ void ref_kernel(const double *__restrict__ x, double *__restrict__ y) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= M) return;
  const int c = i % N, r = (i / N) % N, z = i / NN;
  double s = 6.0 * x[i];
  if (z > 0) s -= x[i - NN];
  if (r > 0) s -= x[i - N];
  if (c > 0) s -= x[i - 1];
  if (c < N - 1) s -= x[i + 1];
  if (r < N - 1) s -= x[i + N];
  if (z < N - 1) s -= x[i + NN];
  y[i] = s;
}

// CG-like vector passes around the MatMult (state experiments): the direction
// update p = c r + b pp (r, pp read non-temporally) and the residual update
// r = r - a w (w, r read non-temporally); NTS: non-temporal stores
template <bool NTS>
__global__ void pb_like(const double *__restrict__ r, const double *__restrict__ pp, double *__restrict__ p, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double v = 0.25 * __builtin_nontemporal_load(r + i) + 0.5 * __builtin_nontemporal_load(pp + i);
    if (NTS) __builtin_nontemporal_store(v, p + i); else p[i] = v;
  }
}
template <bool NTS>
__global__ void upd_like(const double *__restrict__ w, double *__restrict__ r, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double v = __builtin_nontemporal_load(r + i) - 1e-3 * __builtin_nontemporal_load(w + i);
    if (NTS) __builtin_nontemporal_store(v, r + i); else r[i] = v;
  }
}

// Uniform-slot dictionary: every present code of a slot-row of a block is
// the same value, so a block is 14 wave-uniform values and 14 lane masks
// (SGPRs by scalar loads); presence is the mask itself as the exec/select
// condition (inverse ballot) -- no code bytes, no LDS table, no compares
struct BMeta { double v[16]; unsigned long long pm[16]; };
// OPT bit 1: a slot-row whose mask is all lanes skips the select (uniform
// branch); bit 2: a slot-row valued exactly -1 or +1 adds/subtracts the
// operand (fl(-1 * a) = -a exactly, so the sum has the same bits)
template <int U, bool DOT, int OPT = 0>
__global__ void __launch_bounds__(256) puni_kernel(const double *__restrict__ x, double *__restrict__ y, int64_t nunits,
                                                   const BMeta *__restrict__ bm, const int32_t *__restrict__ pblk,
                                                   double *__restrict__ part) {
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int per = gridDim.x >> 3, xcd = blockIdx.x & 7, j = blockIdx.x >> 3;
  const int64_t chunk = (nunits + 7) >> 3;
  const int64_t s0 = xcd * chunk + (int64_t)j * 4 + wid, step = (int64_t)per * 4;
  const int64_t send = min(nunits, (xcd + 1) * chunk);
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void *)x, 0, (int)(M * 8), 0x00020000);
  double dot = 0.0;
  struct T { dbl2 zm, ym, c, yp, zp; double elo, ehi; };
  auto ldp = [&](int64_t i) -> dbl2 {
    return __builtin_bit_cast(dbl2, __builtin_amdgcn_raw_buffer_load_b128(xr, (int)(i * 8), 0, 0));
  };
  auto lds = [&](int64_t i) -> double {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(xr, (int)(i * 8), 0, 0));
  };
  auto ld = [&](int64_t u, T &t) {
    const int64_t ub = u * 128, r0 = ub + 2 * lane;
    t.zm = ldp(r0 - NN); t.ym = ldp(r0 - N); t.c = ldp(r0); t.yp = ldp(r0 + N); t.zp = ldp(r0 + NN);
    t.elo = lds(ub - 1); t.ehi = lds(ub + 128);
  };
  auto fin = [&](int64_t u, int blk, const T &t) {
    const int64_t r0 = u * 128 + 2 * lane;
    const BMeta &B = bm[blk];
    const double lo = wave_shift<true>(t.c.y, t.elo), hi = wave_shift<false>(t.c.x, t.ehi);
    const double a0[7] = {t.zm.x, t.ym.x, lo, t.c.x, t.c.y, t.yp.x, t.zp.x};
    const double a1[7] = {t.zm.y, t.ym.y, t.c.x, t.c.y, hi, t.yp.y, t.zp.y};
    double s0 = 0.0, s1 = 0.0;
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      auto term = [&](double s, double v, double a, unsigned long long pm) {
        double q;
        if ((OPT & 2) && v == -1.0) q = s - a;
        else if ((OPT & 2) && v == 1.0) q = s + a;
        else q = s + v * a;
        if ((OPT & 1) && pm == ~0ull) return q;
        return __builtin_amdgcn_inverse_ballot_w64(pm) ? q : s;
      };
      s0 = term(s0, B.v[k], a0[k], B.pm[k]);
      s1 = term(s1, B.v[7 + k], a1[k], B.pm[7 + k]);
    }
    *reinterpret_cast<dbl2 *>(y + r0) = dbl2{s0, s1};
    if (DOT) { dot += t.c.x * s0; dot += t.c.y * s1; }
  };
  int64_t u = s0;
  int kstep = 64;
  int bv = 0;
  for (; u + (U - 1) * step < send; u += U * step) {
    if (kstep + U > 64) {
      const int64_t uu = u + lane * step;
      bv = uu < send ? pblk[uu] : 0;
      kstep = 0;
    }
    T t[U];
    int bk[U];
#pragma unroll
    for (int k = 0; k < U; ++k) { ld(u + k * step, t[k]); bk[k] = __builtin_amdgcn_readlane(bv, kstep + k); }
    kstep += U;
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int k = 0; k < U; ++k) fin(u + k * step, bk[k], t[k]);
  }
  for (; u < send; u += step) { T t; ld(u, t); fin(u, pblk[u], t); }
  if (DOT) {
    for (int o = 32; o > 0; o >>= 1) dot += __shfl_xor(dot, o);
    if (lane == 0) part[blockIdx.x * 4 + wid] = dot;
  }
}

// Select-free uniform-slot body ("clean" dictionaries): every absent slot's
// operand is made exactly 0.0 by an out-of-range buffer read -- whole runs
// whose slot-rows are empty for both rows (y/z boundaries), and the run's
// edge value where lane 0 row 0 lacks -1 / lane 63 row 1 lacks +1 -- so
// sum + v * 0 = sum (a running sum from +0.0 is never -0.0) and no select is
// needed.  Flags per unit in the block-id word: bit 22 + r = run r empty,
// bit 27 = low edge absent, bit 28 = high edge absent.
constexpr int CL_RUN = 22, CL_ELO = 27, CL_EHI = 28, CL_ID = (1 << 22) - 1;
constexpr int OOR = 1 << 28;   // element offset added to an absent read: bytes >= 2^30 > M * 8
template <int U, bool DOT>
__global__ void __launch_bounds__(256) pclean_kernel(const double *__restrict__ x, double *__restrict__ y, int64_t nunits,
                                                     const BMeta *__restrict__ bm, const int32_t *__restrict__ pblk,
                                                     double *__restrict__ part) {
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int per = gridDim.x >> 3, xcd = blockIdx.x & 7, j = blockIdx.x >> 3;
  const int chunk = (int)((nunits + 7) >> 3);
  const int s0 = xcd * chunk + j * 4 + wid, step = per * 4;
  const int send = (int)min(nunits, (int64_t)(xcd + 1) * chunk);
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void *)x, 0, (int)(M * 8), 0x00020000);
  const int anchor[5] = {-(int)NN, -N, 0, N, (int)NN};
  const int eoff = lane == 0 ? -1 : 128;            // lane 0: x[ub - 1], others x[ub + 128]
  double dot = 0.0;
  struct T { dbl2 L[5]; double e; int bw; };
  auto ldp = [&](int i) -> dbl2 { return __builtin_bit_cast(dbl2, __builtin_amdgcn_raw_buffer_load_b128(xr, (int)((unsigned)i * 8u), 0, 0)); };
  auto lds = [&](int i) -> double { return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(xr, (int)((unsigned)i * 8u), 0, 0)); };
  auto ld = [&](int u, int bw, T &t) {
    const int ub = u * 128, r0 = ub + 2 * lane;
#pragma unroll
    for (int r = 0; r < 5; ++r) t.L[r] = ldp(r0 + anchor[r] + (((bw >> (CL_RUN + r)) & 1) ? OOR : 0));
    const int elo = ((bw >> CL_ELO) & 1) ? OOR : 0, ehi = ((bw >> CL_EHI) & 1) ? OOR : 0;
    t.e = lds(ub + eoff + (lane == 0 ? elo : ehi));
    t.bw = bw;
  };
  auto fin = [&](int u, const T &t) {
    const int r0 = u * 128 + 2 * lane;
    const BMeta &B = bm[t.bw & CL_ID];
    const double lo = wave_shift<true>(t.L[2].y, t.e), hi = wave_shift<false>(t.L[2].x, t.e);
    const double a0[7] = {t.L[0].x, t.L[1].x, lo, t.L[2].x, t.L[2].y, t.L[3].x, t.L[4].x};
    const double a1[7] = {t.L[0].y, t.L[1].y, t.L[2].x, t.L[2].y, hi, t.L[3].y, t.L[4].y};
    double s0 = 0.0, s1 = 0.0;
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      s0 = s0 + B.v[k] * a0[k];
      s1 = s1 + B.v[7 + k] * a1[k];
    }
    *reinterpret_cast<dbl2 *>(y + r0) = dbl2{s0, s1};
    if (DOT) { dot += t.L[2].x * s0; dot += t.L[2].y * s1; }
  };
  int u = s0;
  int kstep = 64;
  int bv = 0;
  for (; u + (U - 1) * step < send; u += U * step) {
    if (kstep + U > 64) {
      const int uu = u + lane * step;
      bv = uu < send ? pblk[uu] : 0;
      kstep = 0;
    }
    T t[U];
#pragma unroll
    for (int k = 0; k < U; ++k) ld(u + k * step, __builtin_amdgcn_readlane(bv, kstep + k), t[k]);
    kstep += U;
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int k = 0; k < U; ++k) fin(u + k * step, t[k]);
  }
  for (; u < send; u += step) { T t; ld(u, pblk[u], t); fin(u, t); }
  if (DOT) {
    for (int o = 32; o > 0; o >>= 1) dot += __shfl_xor(dot, o);
    if (lane == 0) part[blockIdx.x * 4 + wid] = dot;
  }
}

// Row-pair z-march: a wave owns a column of 128-row units (one half x-line)
// and marches L planes in z, carrying the centre and -n^2 pairs in registers:
// per unit 4 loads (the +n^2 pair -- the only HBM-first line --, the -n and
// +n pairs, the edge) instead of 6.  XCD k takes the z-slab [32k, 32k + 32);
// its waves take (segment, column) tasks segment-major, so the waves running
// together sit in the same planes and the +-n pairs hit L2.  Z steps per
// iteration: ZU (their loads in flight together).
template <int L, int ZU>
__global__ void __launch_bounds__(256) pzm_kernel(const double *__restrict__ x, double *__restrict__ y,
                                                  double *__restrict__ part) {
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int per = gridDim.x >> 3, xcd = blockIdx.x & 7, j = blockIdx.x >> 3;
  const int W = per * 4, w = j * 4 + wid;
  constexpr int COLS = (int)(NN / 128), SLAB = N / 8, SEGS = SLAB / L;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void *)x, 0, (int)(M * 8), 0x00020000);
  auto ldp = [&](int i) -> dbl2 { return __builtin_bit_cast(dbl2, __builtin_amdgcn_raw_buffer_load_b128(xr, (int)((unsigned)i * 8u), 0, 0)); };
  auto lds = [&](int i) -> double { return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(xr, (int)((unsigned)i * 8u), 0, 0)); };
  const int eoff = lane == 0 ? -1 : 128;
  double dot = 0.0;
  for (int t = w; t < COLS * SEGS; t += W) {
    const int seg = t / COLS, col = t % COLS;
    const int zs = xcd * SLAB + seg * L;
    const int cb = col * 128 + 2 * lane;          // row of lane's pair within a plane
    dbl2 zm = ldp((zs - 1) * (int)NN + cb), c = ldp(zs * (int)NN + cb);
    for (int z = zs; z < zs + L; z += ZU) {
      dbl2 zp[ZU], ym[ZU], yp[ZU];
      double e[ZU];
#pragma unroll
      for (int q = 0; q < ZU; ++q) {
        const int r0 = (z + q) * (int)NN + cb, ub = (z + q) * (int)NN + col * 128;
        zp[q] = ldp(r0 + (int)NN);
        ym[q] = ldp(r0 - N);
        yp[q] = ldp(r0 + N);
        e[q] = lds(ub + eoff);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int q = 0; q < ZU; ++q) {
        const int r0 = (z + q) * (int)NN + cb;
        const double lo = wave_shift<true>(c.y, e[q]), hi = wave_shift<false>(c.x, e[q]);
        const double s0 = 6.0 * c.x - zm.x - ym[q].x - lo - c.y - yp[q].x - zp[q].x;
        const double s1 = 6.0 * c.y - zm.y - ym[q].y - c.x - hi - yp[q].y - zp[q].y;
        *reinterpret_cast<dbl2 *>(y + r0) = dbl2{s0, s1};
        dot += c.x * s0; dot += c.y * s1;
        zm = c; c = zp[q];
      }
    }
  }
  for (int o = 32; o > 0; o >>= 1) dot += __shfl_xor(dot, o);
  if (lane == 0) part[blockIdx.x * 4 + wid] = dot;
}

int main(int argc, char **argv) {
  double *x, *y, *yr, *flush;
  CK(hipMalloc(&x, M * 8)); CK(hipMalloc(&y, M * 8)); CK(hipMalloc(&yr, M * 8)); CK(hipMalloc(&flush, 512ull << 20));
  std::vector<double> h(M);
  for (int64_t i = 0; i < M; ++i) h[i] = (double)((i * 2654435761ull) % 1000) / 1000.0;
  CK(hipMemcpy(x, h.data(), M * 8, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  const double bytes = 2.0 * M * 8;
  const std::string only = argc > 1 ? std::string(";") + argv[1] + ";" : std::string();
  auto timeit = [&](const char *name, auto launch, bool check) {
    if (!only.empty() && only.find(std::string(";") + name + ";") == std::string::npos) {
      // "prefix*" tokens select every name with that prefix
      bool hit = false;
      for (size_t a = 1, b; a < only.size() && (b = only.find(';', a)) != std::string::npos; a = b + 1)
        if (b > a && only[b - 1] == '*' && std::string(name).rfind(only.substr(a, b - a - 1), 0) == 0) hit = true;
      if (!hit) return;
    }
    for (int w = 0; w < 3; ++w) launch();
    CK(hipDeviceSynchronize());
    const int it = 50;
    CK(hipEventRecord(a));
    for (int k = 0; k < it; ++k) launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    const double us = ms * 1e3 / it;
    // cold: flush caches first
    float cold = 0;
    for (int k = 0; k < 3; ++k) {
      CK(hipMemsetAsync(flush, k, 512ull << 20));
      CK(hipEventRecord(a)); launch(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
      float t; CK(hipEventElapsedTime(&t, a, b)); cold += t * 1e3f / 3;
    }
    double err = 0;
    if (check) {
      std::vector<double> g(M), r(M);
      CK(hipMemcpy(g.data(), y, M * 8, hipMemcpyDeviceToHost));
      CK(hipMemcpy(r.data(), yr, M * 8, hipMemcpyDeviceToHost));
      for (int64_t i = 0; i < M; ++i) err = fmax(err, fabs(g[i] - r[i]));
    }
    printf("%-22s %8.1f us  %7.0f GB/s  (%.3f of 8 TB/s)  cold %7.1f us  maxerr %.1e\n", name, us, bytes / us * 1e-3,
           bytes / us * 1e-3 / 8000, cold, err);
  };
  ref_kernel<<<(M + 255) / 256, 256>>>(x, yr);
  CK(hipDeviceSynchronize());
  int cus = 256;
  for (int g : {8192})
    timeit((std::string("copy g") + std::to_string(g)).c_str(), [&] { copy_kernel<<<g, 256>>>((const dbl2 *)x, (dbl2 *)y, M / 2); }, false);
  timeit("ref (naive)", [&] { ref_kernel<<<(M + 255) / 256, 256>>>(x, y); }, true);
  for (int wpc : {2, 3, 4}) {
    const int g = cus * wpc - 8;
    char nm[64];
    snprintf(nm, sizeof nm, "pairs<1> %d/CU", wpc);
    timeit(nm, [&] { pairs_kernel<1><<<g, 256>>>(x, y, M / 128); }, wpc == 4);
    snprintf(nm, sizeof nm, "pairs<2> %d/CU", wpc);
    timeit(nm, [&] { pairs_kernel<2><<<g, 256>>>(x, y, M / 128); }, wpc == 4);
    snprintf(nm, sizeof nm, "pairs<4> %d/CU", wpc);
    timeit(nm, [&] { pairs_kernel<4><<<g, 256>>>(x, y, M / 128); }, wpc == 4);
  }
  // dictionary: block 0 = lane 0 row 0 lacks the -1 entry, block 1 = lane 63 row 1 lacks +1
  std::vector<uint8_t> hd(2 * 64 * 16, 0);
  for (int b = 0; b < 2; ++b)
    for (int l = 0; l < 64; ++l) {
      uint8_t *c = &hd[(b * 64 + l) * 16];
      for (int r = 0; r < 2; ++r)
        for (int k = 0; k < 7; ++k) c[7 * r + k] = k == 3 - r + r * 1 ? 0 : 1;   // centre -> 6.0 (code 0), else -1.0 (code 1)
      // row 0 centre is slot 3, row 1 centre is slot 4 (a1 order)
      for (int k = 0; k < 7; ++k) { c[k] = k == 3 ? 0 : 1; c[7 + k] = k == 3 ? 0 : 1; }
      if (b == 0 && l == 0) c[2] = ABSENT;
      if (b == 1 && l == 63) c[7 + 4] = ABSENT;
      c[14] = c[15] = ABSENT;
    }
  uint8_t *dict; int32_t *pblk; double *vt, *part;
  CK(hipMalloc(&dict, hd.size())); CK(hipMemcpy(dict, hd.data(), hd.size(), hipMemcpyHostToDevice));
  std::vector<int32_t> hb(M / 128); for (size_t u = 0; u < hb.size(); ++u) hb[u] = (int)(u & 1);
  CK(hipMalloc(&pblk, hb.size() * 4)); CK(hipMemcpy(pblk, hb.data(), hb.size() * 4, hipMemcpyHostToDevice));
  std::vector<double> hv(256, 0.0); hv[0] = 6.0; hv[1] = -1.0;
  CK(hipMalloc(&vt, 256 * 8)); CK(hipMemcpy(vt, hv.data(), 256 * 8, hipMemcpyHostToDevice));
  CK(hipMalloc(&part, 1 << 20));
  // the same dictionary in 2-bit codes (code 255 -> 3)
  std::vector<uint32_t> hd2(2 * 64, 0);
  for (int b = 0; b < 2; ++b)
    for (int l = 0; l < 64; ++l) {
      uint32_t w = 0;
      for (int q = 0; q < 14; ++q) {
        const uint8_t c = hd[(b * 64 + l) * 16 + q];
        w |= (uint32_t)(c == ABSENT ? 3 : c) << (2 * q);
      }
      hd2[b * 64 + l] = w;
    }
  // uniform-slot metadata of the same two blocks
  std::vector<BMeta> hbm(2);
  for (int bb = 0; bb < 2; ++bb)
    for (int q = 0; q < 16; ++q) {
      hbm[bb].v[q] = 0.0; hbm[bb].pm[q] = 0;
      for (int l = 0; l < 64; ++l) {
        const uint8_t c = hd[(bb * 64 + l) * 16 + q];
        if (c != ABSENT) { hbm[bb].v[q] = hv[c]; hbm[bb].pm[q] |= 1ull << l; }
      }
    }
  BMeta *dbm;
  CK(hipMalloc(&dbm, 2 * sizeof(BMeta))); CK(hipMemcpy(dbm, hbm.data(), 2 * sizeof(BMeta), hipMemcpyHostToDevice));
  uint32_t *dict2;
  CK(hipMalloc(&dict2, hd2.size() * 4)); CK(hipMemcpy(dict2, hd2.data(), hd2.size() * 4, hipMemcpyHostToDevice));
  // the same two blocks for the select-free body: block ids with edge flags
  std::vector<int32_t> hbc(M / 128);
  for (size_t u = 0; u < hbc.size(); ++u) hbc[u] = (int)(u & 1) | ((u & 1) ? 1 << CL_EHI : 1 << CL_ELO);
  int32_t *pblkc;
  CK(hipMalloc(&pblkc, hbc.size() * 4)); CK(hipMemcpy(pblkc, hbc.data(), hbc.size() * 4, hipMemcpyHostToDevice));
  {
    const int g = cus * 4 - 8;
    puni_kernel<2, true><<<g, 256>>>(x, yr, M / 128, dbm, pblk, part);
    pclean_kernel<2, true><<<g, 256>>>(x, y, M / 128, dbm, pblkc, part);
    CK(hipDeviceSynchronize());
    std::vector<double> g1(M), g2(M);
    CK(hipMemcpy(g1.data(), yr, M * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(g2.data(), y, M * 8, hipMemcpyDeviceToHost));
    int64_t nd = 0;
    for (int64_t i = 0; i < M; ++i) nd += memcmp(&g1[i], &g2[i], 8) != 0;
    printf("pclean vs puni: %lld rows differ bitwise\n", (long long)nd);
  }
  for (int wpc : {2, 3, 4, 5, 6, 8}) {
    for (int gsub : {0, 8}) {
      const int g = cus * wpc - gsub;
      char nm[64];
#define PZM(LL, ZZ)                                                                                          \
      snprintf(nm, sizeof nm, "pzm L%d ZU%d %d/CU-%d", LL, ZZ, wpc, gsub);                                  \
      timeit(nm, [&] { pzm_kernel<LL, ZZ><<<g, 256>>>(x, y, part); }, false);
      PZM(32, 1) PZM(32, 2) PZM(16, 1) PZM(16, 2) PZM(8, 2) PZM(32, 4) PZM(16, 4)
#undef PZM
    }
  }
  for (int wpc : {2, 3, 4, 5}) {
    const int g = cus * wpc - 8;
    char nm[64];
    for (int U3 : {1, 2, 3}) {
      snprintf(nm, sizeof nm, "pclean<%d>+dot %d/CU", U3, wpc);
      if (U3 == 1) timeit(nm, [&] { pclean_kernel<1, true><<<g, 256>>>(x, y, M / 128, dbm, pblkc, part); }, false);
      if (U3 == 2) timeit(nm, [&] { pclean_kernel<2, true><<<g, 256>>>(x, y, M / 128, dbm, pblkc, part); }, false);
      if (U3 == 3) timeit(nm, [&] { pclean_kernel<3, true><<<g, 256>>>(x, y, M / 128, dbm, pblkc, part); }, false);
    }
    snprintf(nm, sizeof nm, "pcodes<1> %d/CU", wpc);
    timeit(nm, [&] { pcodes_kernel<1, false, false><<<g, 256>>>(x, y, M / 128, dict, pblk, vt, part); }, false);
    snprintf(nm, sizeof nm, "pcodes<2> %d/CU", wpc);
    timeit(nm, [&] { pcodes_kernel<2, false, false><<<g, 256>>>(x, y, M / 128, dict, pblk, vt, part); }, false);
    snprintf(nm, sizeof nm, "pcodes<2>+meta %d/CU", wpc);
    timeit(nm, [&] { pcodes_kernel<2, false, true><<<g, 256>>>(x, y, M / 128, dict, pblk, vt, part); }, false);
    snprintf(nm, sizeof nm, "pbuf<1>+dot %d/CU", wpc);
    timeit(nm, [&] { pbuf_kernel<1, true><<<g, 256>>>(x, y, M / 128, dict, pblk, vt, part); }, false);
    snprintf(nm, sizeof nm, "pbuf<2>+dot %d/CU", wpc);
    timeit(nm, [&] { pbuf_kernel<2, true><<<g, 256>>>(x, y, M / 128, dict, pblk, vt, part); }, false);
    snprintf(nm, sizeof nm, "pbuf<3>+dot %d/CU", wpc);
    timeit(nm, [&] { pbuf_kernel<3, true><<<g, 256>>>(x, y, M / 128, dict, pblk, vt, part); }, false);
    snprintf(nm, sizeof nm, "pcodes<2>+dot %d/CU", wpc);
    timeit(nm, [&] { pcodes_kernel<2, true, false><<<g, 256>>>(x, y, M / 128, dict, pblk, vt, part); }, false);
    snprintf(nm, sizeof nm, "glob+batchmeta+dot %d/CU", wpc);
    timeit(nm, [&] { pbuf_kernel<2, true, 1, false><<<g, 256>>>(x, y, M / 128, dict, pblk, vt, part); }, false);
    snprintf(nm, sizeof nm, "buf+nometa+dot %d/CU", wpc);
    timeit(nm, [&] { pbuf_kernel<2, true, 0, true><<<g, 256>>>(x, y, M / 128, dict, pblk, vt, part); }, false);
    snprintf(nm, sizeof nm, "puni<1>+dot %d/CU", wpc);
    timeit(nm, [&] { puni_kernel<1, true><<<g, 256>>>(x, y, M / 128, dbm, pblk, part); }, false);
    snprintf(nm, sizeof nm, "puni<2>+dot %d/CU", wpc);
    timeit(nm, [&] { puni_kernel<2, true><<<g, 256>>>(x, y, M / 128, dbm, pblk, part); }, false);
    snprintf(nm, sizeof nm, "puni<2>+dot opt1 %d/CU", wpc);
    timeit(nm, [&] { puni_kernel<2, true, 1><<<g, 256>>>(x, y, M / 128, dbm, pblk, part); }, false);
    snprintf(nm, sizeof nm, "puni<2>+dot opt2 %d/CU", wpc);
    timeit(nm, [&] { puni_kernel<2, true, 2><<<g, 256>>>(x, y, M / 128, dbm, pblk, part); }, false);
    snprintf(nm, sizeof nm, "puni<2>+dot opt3 %d/CU", wpc);
    timeit(nm, [&] { puni_kernel<2, true, 3><<<g, 256>>>(x, y, M / 128, dbm, pblk, part); }, false);
    snprintf(nm, sizeof nm, "dreg+batchmeta+dot %d/CU", wpc);
    timeit(nm, [&] { pbuf_kernel<2, true, 1, true, true><<<g, 256>>>(x, y, M / 128, dict, pblk, vt, part); }, false);
    snprintf(nm, sizeof nm, "dreg<1>+batchmeta+dot %d/CU", wpc);
    timeit(nm, [&] { pbuf_kernel<1, true, 1, true, true><<<g, 256>>>(x, y, M / 128, dict, pblk, vt, part); }, false);
    snprintf(nm, sizeof nm, "dreg<3>+batchmeta+dot %d/CU", wpc);
    timeit(nm, [&] { pbuf_kernel<3, true, 1, true, true><<<g, 256>>>(x, y, M / 128, dict, pblk, vt, part); }, false);
    snprintf(nm, sizeof nm, "buf+batchmeta+dot %d/CU", wpc);
    timeit(nm, [&] { pbuf_kernel<2, true, 1, true, false><<<g, 256>>>(x, y, M / 128, dict, pblk, vt, part); }, false);
    snprintf(nm, sizeof nm, "glob+nometa+dot %d/CU", wpc);
    timeit(nm, [&] { pbuf_kernel<2, true, 0, false><<<g, 256>>>(x, y, M / 128, dict, pblk, vt, part); }, false);
    for (int U2 : {1, 2, 4}) {
      for (int me : {0, 1, 2}) {
        snprintf(nm, sizeof nm, "blk<%d>+meta%d+dot %d/CU", U2, me, wpc);
        auto go = [&](auto kern) { timeit(nm, [&] { kern<<<g, 256>>>(x, y, M / 128, dict, pblk, vt, part); }, false); };
        if (U2 == 1) { if (me == 0) go(pblk_kernel<1, true, 0>); else if (me == 1) go(pblk_kernel<1, true, 1>); else go(pblk_kernel<1, true, 2>); }
        if (U2 == 2) { if (me == 0) go(pblk_kernel<2, true, 0>); else if (me == 1) go(pblk_kernel<2, true, 1>); else go(pblk_kernel<2, true, 2>); }
        if (U2 == 4) { if (me == 0) go(pblk_kernel<4, true, 0>); else if (me == 1) go(pblk_kernel<4, true, 1>); else go(pblk_kernel<4, true, 2>); }
      }
    }
    snprintf(nm, sizeof nm, "pov+meta0+dot %d/CU", wpc);
    timeit(nm, [&] { pov_kernel<true, 0><<<g, 256>>>(x, y, M / 128, dict, pblk, vt, part); }, false);
    snprintf(nm, sizeof nm, "pov+meta1+dot %d/CU", wpc);
    timeit(nm, [&] { pov_kernel<true, 1><<<g, 256>>>(x, y, M / 128, dict, pblk, vt, part); }, false);
    snprintf(nm, sizeof nm, "psel+meta0 %d/CU", wpc);
    timeit(nm, [&] { psel_kernel<0><<<g, 256>>>(x, y, M / 128, dict, pblk, 6.0, -1.0, part); }, false);
    snprintf(nm, sizeof nm, "psel+meta1 %d/CU", wpc);
    timeit(nm, [&] { psel_kernel<1><<<g, 256>>>(x, y, M / 128, dict, pblk, 6.0, -1.0, part); }, false);
    snprintf(nm, sizeof nm, "pnarrow+meta0 %d/CU", wpc);
    timeit(nm, [&] { pnarrow_kernel<false><<<g, 256>>>(x, y, M / 128, dict2, pblk, vt, part); }, false);
    snprintf(nm, sizeof nm, "pnarrow+meta1 %d/CU", wpc);
    timeit(nm, [&] { pnarrow_kernel<true><<<g, 256>>>(x, y, M / 128, dict2, pblk, vt, part); }, false);
    snprintf(nm, sizeof nm, "pbuf<2> %d/CU", wpc);
    timeit(nm, [&] { pbuf_kernel<2, false><<<g, 256>>>(x, y, M / 128, dict, pblk, vt, part); }, false);
    snprintf(nm, sizeof nm, "pcodes<2>+meta+dot %d/CU", wpc);
    timeit(nm, [&] { pcodes_kernel<2, true, true><<<g, 256>>>(x, y, M / 128, dict, pblk, vt, part); }, false);
  }
  // operand state: the same SpMV (uniform-slot, 4/CU) timed alone by events
  // around each launch, when (a) x was the previous launch's operand too, (b)
  // launches alternate between two operands, (c) a copy kernel has just
  // written x (as CG's direction update writes p_i before the MatMult)
  {
    double *x2, *x3;
    CK(hipMalloc(&x2, M * 8)); CK(hipMalloc(&x3, M * 8));
    CK(hipMemcpy(x2, x, M * 8, hipMemcpyDeviceToDevice)); CK(hipMemcpy(x3, x, M * 8, hipMemcpyDeviceToDevice));
    const int g = cus * 4 - 8;
    auto spmv = [&](const double *xx) { puni_kernel<2, true><<<g, 256>>>(xx, y, M / 128, dbm, pblk, part); };
    auto ev_time = [&](const char *name, auto before, auto op) {
      if (!only.empty() && only.find(std::string(";") + name + ";") == std::string::npos) return;
      std::vector<float> t;
      for (int k = 0; k < 40; ++k) {
        before(k);
        CK(hipEventRecord(a)); op(k); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b)); if (k >= 4) t.push_back(ms * 1e3f);
      }
      std::sort(t.begin(), t.end());
      printf("%-28s median %7.1f us  min %7.1f us\n", name, t[t.size() / 2], t[0]);
    };
    ev_time("state same-x", [&](int) {}, [&](int) { spmv(x); });
    ev_time("state alternate-x", [&](int) {}, [&](int k) { spmv((k & 1) ? x2 : x); });
    ev_time("state x-just-copied", [&](int) { copy_kernel<<<8192, 256>>>((const dbl2 *)x3, (dbl2 *)x2, M / 2); },
            [&](int) { spmv(x2); });
    ev_time("state x-just-copied-nt", [&](int) { copy_kernel<<<8192, 256>>>((const dbl2 *)x3, (dbl2 *)x2, M / 2); CK(hipDeviceSynchronize()); },
            [&](int) { spmv(x2); });
    // the CG iteration's order: pb (r, p_{i-1} -> p_i), MatMult (p_i -> w), update (w, r -> r)
    {
      double *pv[2] = {x2, x3}, *rr, *ww;
      CK(hipMalloc(&rr, M * 8)); CK(hipMalloc(&ww, M * 8));
      CK(hipMemcpy(rr, x, M * 8, hipMemcpyDeviceToDevice));
      auto cg_like = [&](const char *name, bool pnts, bool rnts) {
        ev_time(name, [&](int k) {
                  if (k) { if (rnts) upd_like<true><<<1024, 256>>>(ww, rr, M); else upd_like<false><<<1024, 256>>>(ww, rr, M); }
                  if (pnts) pb_like<true><<<8192, 256>>>(rr, pv[(k + 1) & 1], pv[k & 1], M);
                  else pb_like<false><<<8192, 256>>>(rr, pv[(k + 1) & 1], pv[k & 1], M);
                },
                [&](int k) { puni_kernel<2, true><<<g, 256>>>(pv[k & 1], ww, M / 128, dbm, pblk, part); });
      };
      cg_like("state cg-like", false, false);
      cg_like("state cg-like p-nts", true, false);
      cg_like("state cg-like r-nts", false, true);
      cg_like("state cg-like both-nts", true, true);
    }
    ev_time("state copy-other", [&](int) { copy_kernel<<<8192, 256>>>((const dbl2 *)x3, (dbl2 *)yr, M / 2); },
            [&](int) { spmv(x); });
  }
  timeit("zmarch TY4 ZR16", [&] { zmarch_kernel<4, 16><<<(N / 4) * (N / 16), 256>>>(x, y); }, true);
  timeit("zmarch TY4 ZR32", [&] { zmarch_kernel<4, 32><<<(N / 4) * (N / 32), 256>>>(x, y); }, true);
  timeit("zmarch TY2 ZR32", [&] { zmarch_kernel<2, 32><<<(N / 2) * (N / 32), 256>>>(x, y); }, true);
  timeit("zmarch TY8 ZR16", [&] { zmarch_kernel<8, 16><<<(N / 8) * (N / 16), 256>>>(x, y); }, true);
  timeit("zmarch TY4 ZR64", [&] { zmarch_kernel<4, 64><<<(N / 4) * (N / 64), 256>>>(x, y); }, true);
  return 0;
}
