// mx_spmv.hip -- MatMult_MPIAIJ on gfx950: VecScatter halo + SELL-64 SpMV.
//
// Replaces KSP_MatMult -> MatMult_MPIAIJ, reached from
// ksp.solve at test.py:50.  PETSc's order is kept exactly (oracle/petsc_oracle.c
// block_mult): for each row, sum = 0; sum += a_j * x[c_j] over the diagonal
// block in ascending column order (MatMult_SeqAIJ), then the off-diagonal
// block continues the same running sum in ascending ghost order
// (MatMultAdd_SeqAIJ with sum = y_i).  Every multiply and add rounds
// separately (-ffp-contract=off), as PETSc's -march=nocona C loop does, so the
// GPU product is bitwise equal to the CPU one.
//
// Layout (HBM): SELL-C with C = 64 = one wavefront, sigma = 1 (no row
// reordering, so the halo and the vectors keep PETSc's natural numbering).
// Slice s holds rows [64 s, 64 s + 64); entry j of the 64 rows is stored
// contiguously at sptr[s] + 64 j + lane, so every wave-wide load of values
// (512 B) and column ids (256 B) is fully coalesced, and each lane walks its
// own row sequentially -- which is exactly the order PETSc sums in.  Padding
// slots carry column -1 and are skipped.  A_o gets its own SELL structure;
// slices with no ghost entries have width 0 and cost one scalar load.
// On top of that (mx_assembly.hip): aligned-offset slices with a
// shared offset-pattern table, one-byte value codes into an LDS table when
// the block has <= 255 distinct values, and a row-pair copy of the codes for
// 5/7/27-point patterns (two rows per lane, x read as 16-byte pairs, +-1
// neighbours by DPP wave shifts).  Every variant sums each row in the same
// order, so all give the same bits.
#include <algorithm>
#include <mutex>
#include <unordered_map>

#include <atomic>

#include "mx_cg.hpp"
#include "mx_device.hpp"
#include "mx_internal.hpp"
#include "mx_pair.hpp"
#include "mx_launch.hpp"

namespace mx {

constexpr int SPMV_WAVES = 4;  // 256-thread workgroups, one slice per wave at a time
#ifndef SPMV_PAIR_TWO
#define SPMV_PAIR_TWO 1   // 5/7-point row pairs: two units' loads in flight per wave
#endif
Knobs g_knobs;
thread_local ExtTiming g_ext_timing;
std::atomic<long long> g_dispatch[DSP_COUNT];
void note_dispatch(int kind) { g_dispatch[kind].fetch_add(1, std::memory_order_relaxed); }

typedef int int2v __attribute__((ext_vector_type(2)));

template <bool NT, class T> __device__ __forceinline__ T ld(const T *p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}

// The operand of the product is read through a source functor: a plain
// vector, or (SPMV_CG) the CG direction p_i = z + b p_{i-1}, z = jac(r),
// evaluated from r and p_{i-1} at every index the product touches.  The
// expression is the one VecAYPX applies (one multiply, one add, each rounded),
// so every evaluation of p_i[j] -- here, in the halo pack and in the owner's
// store -- yields the same bits as a separate update pass would.
// at(base, lane) = value at base + lane for a wave-uniform base: the address
// is one SGPR pair plus the lane's fixed byte offset, shared by every gather
template <bool S = false>
struct XPlainT {
  const double *__restrict__ x;
  double s = 1.0;             // S: the operand is fl(s * x[j]) (a lazily normalised vector)
  __device__ __forceinline__ double operator()(int64_t j) const { return S ? s * x[j] : x[j]; }
  __device__ __forceinline__ double at(int64_t base, int lane) const {
    return S ? s * (x + base)[lane] : (x + base)[lane];
  }
  // the operand at i and i + 1 (i even: one 16-byte load)
  __device__ __forceinline__ dbl2 pair(int64_t i) const {
    const dbl2 v = *reinterpret_cast<const dbl2 *>(x + i);
    return S ? dbl2{s * v.x, s * v.y} : v;
  }
};
using XPlain = XPlainT<false>;
// JM = the Jacobi form, compile-time so every load is unconditional (a
// runtime form turns each gather into a branch around the dinv load)
template <int JM>
struct XCg {
  const double *__restrict__ r;
  const double *__restrict__ p;
  const double *__restrict__ d;
  double c, b;
  __device__ __forceinline__ double form(double rj, double pj, double dj) const {
    double z = rj;
    if constexpr (JM == 1) z = rj * dj;             // PCApply_Jacobi, vector
    else if constexpr (JM == 2) z = rj * c;         // uniform diagonal, scalar
    // VecAYPX_Seq.  Its b == 0 copy needs no select: iteration 0 runs with
    // b = +0 against p_{-1} = -0.0, and z + (+0)(-0) = z + (-0) = z for every z
    return z + b * pj;
  }
  __device__ __forceinline__ double operator()(int64_t j) const {
    return form(r[j], p[j], JM == 1 ? d[j] : 0.0);
  }
  __device__ __forceinline__ double at(int64_t base, int lane) const {
    return form((r + base)[lane], (p + base)[lane], JM == 1 ? (d + base)[lane] : 0.0);
  }
  __device__ __forceinline__ dbl2 pair(int64_t i) const {
    const dbl2 rv = *reinterpret_cast<const dbl2 *>(r + i), pv = *reinterpret_cast<const dbl2 *>(p + i);
    const dbl2 dv = JM == 1 ? *reinterpret_cast<const dbl2 *>(d + i) : dbl2{0.0, 0.0};
    return dbl2{form(rv.x, pv.x, dv.x), form(rv.y, pv.y, dv.y)};
  }
};

// Buffer-load forms of the operand sources for the row-pair body
// (vec_rsrc / bload1 / bload2: mx_pair.hpp).
template <class XS> struct XBuf;
template <bool S> struct XBuf<XPlainT<S>> {
  __amdgpu_buffer_rsrc_t x;
  double s;
  __device__ __forceinline__ XBuf(const XPlainT<S> &X, int64_t n) : x(vec_rsrc(X.x, n)), s(X.s) {}
  __device__ __forceinline__ double operator()(int i) const { const double v = bload1(x, i); return S ? s * v : v; }
  __device__ __forceinline__ dbl2 pair(int i) const {
    const dbl2 v = bload2(x, i);
    return S ? dbl2{s * v.x, s * v.y} : v;
  }
};
template <int JM> struct XBuf<XCg<JM>> {
  __amdgpu_buffer_rsrc_t r, p, d;
  XCg<JM> f;
  __device__ __forceinline__ XBuf(const XCg<JM> &X, int64_t n)
      : r(vec_rsrc(X.r, n)), p(vec_rsrc(X.p, n)), d(vec_rsrc(JM == 1 ? X.d : X.r, n)), f(X) {}
  __device__ __forceinline__ double operator()(int i) const {
    return f.form(bload1(r, i), bload1(p, i), JM == 1 ? bload1(d, i) : 0.0);
  }
  __device__ __forceinline__ dbl2 pair(int i) const {
    const dbl2 rv = bload2(r, i), pv = bload2(p, i);
    const dbl2 dv = JM == 1 ? bload2(d, i) : dbl2{0.0, 0.0};
    return dbl2{f.form(rv.x, pv.x, dv.x), f.form(rv.y, pv.y, dv.y)};
  }
};

// Matrix values of one slice: fp64 in the paired layout (slot j of a lane at
// pair j / 2), or one-byte codes into the matrix's value table (copied to LDS
// at kernel start): batch b = entries 8 b .. 8 b + 7 of every lane, one 8-B
// load per lane = one 512-B wave load (SELL-64 code blocks, mx_assembly.hip).
// A table entry is the stored value itself, so both give the same bits.
template <bool NT>
struct VDense {
  const double *__restrict__ b;   // the slice's first slot
  // entries 2 p0 .. 2 p0 + 7 (pairs p0 .. p0 + 3, those below np)
  __device__ __forceinline__ void eight(int p0, int np, int lane, double v[8]) const {
    const dbl2 *__restrict__ vp = reinterpret_cast<const dbl2 *>(b) + lane;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int p = p0 + q;
      const dbl2 t = p < np ? ld<NT>(vp + (int64_t)p * SLICE) : dbl2{0.0, 0.0};
      v[2 * q] = t.x;
      v[2 * q + 1] = t.y;
    }
  }
  // the unpaired last entry 2 np of an odd width
  __device__ __forceinline__ double last(int np, int lane) const { return ld<NT>(b + (int64_t)np * 2 * SLICE + lane); }
  template <int K>
  __device__ __forceinline__ void fixed(int lane, double v[K]) const {
    constexpr int NP = K / 2;
    const dbl2 *__restrict__ vp = reinterpret_cast<const dbl2 *>(b) + lane;
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const dbl2 t = ld<NT>(vp + p * SLICE);
      v[2 * p] = t.x;
      v[2 * p + 1] = t.y;
    }
    if constexpr (K & 1) v[K - 1] = ld<NT>(b + NP * 2 * SLICE + lane);
  }
  // two phases (loads of several slices in flight before the first use)
  static constexpr bool kCodedPresence = false;   // presence comes from the row masks
  template <int K> struct Raw { double v[K]; };
  template <int K> __device__ __forceinline__ void fetch(int lane, Raw<K> &r) const { fixed<K>(lane, r.v); }
  template <int K> __device__ __forceinline__ void decode(const Raw<K> &r, double v[K]) const {
#pragma unroll
    for (int j = 0; j < K; ++j) v[j] = r.v[j];
  }
};

template <bool NT>
struct VCoded {
  const uint8_t *__restrict__ b;  // the slice's code block
  const double *t;                // value table (LDS)
  __device__ __forceinline__ uint64_t batch(int bi, int lane) const {
    return ld<NT>(reinterpret_cast<const uint64_t *>(b + (int64_t)bi * CODE_BATCH) + lane);
  }
  __device__ __forceinline__ void eight(int p0, int, int lane, double v[8]) const {
    const uint64_t c = batch(p0 >> 2, lane);
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = t[(c >> (8 * q)) & 0xff];
  }
  __device__ __forceinline__ double last(int np, int lane) const {
    const int j = 2 * np;
    return t[b[(int64_t)(j >> 3) * CODE_BATCH + lane * 8 + (j & 7)]];
  }
  template <int K>
  __device__ __forceinline__ void fixed(int lane, double v[K]) const {
#pragma unroll
    for (int bi = 0; bi < (K + 7) / 8; ++bi) {
      const uint64_t c = batch(bi, lane);
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (8 * bi + q < K) v[8 * bi + q] = t[(c >> (8 * q)) & 0xff];
    }
  }
  // the aligned-offset code blocks mark absent slots with VCODE_ABSENT, so
  // the fixed-width body needs no presence-mask load
  static constexpr bool kCodedPresence = true;
  template <int K> struct Raw { uint64_t c[(K + 7) / 8]; };
  template <int K> __device__ __forceinline__ bool present(const Raw<K> &r, int j) const {
    return ((r.c[j >> 3] >> (8 * (j & 7))) & 0xff) != VCODE_ABSENT;
  }
  template <int K> __device__ __forceinline__ uint32_t presence(const Raw<K> &r) const {
    uint32_t mk = 0;
#pragma unroll
    for (int j = 0; j < K; ++j) mk |= present<K>(r, j) ? 1u << j : 0u;
    return mk;
  }
  template <int K> __device__ __forceinline__ void fetch(int lane, Raw<K> &r) const {
#pragma unroll
    for (int bi = 0; bi < (K + 7) / 8; ++bi) r.c[bi] = batch(bi, lane);
  }
  template <int K> __device__ __forceinline__ void decode(const Raw<K> &r, double v[K]) const {
#pragma unroll
    for (int bi = 0; bi < (K + 7) / 8; ++bi)
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (8 * bi + q < K) v[8 * bi + q] = t[(r.c[bi] >> (8 * q)) & 0xff];
  }
};

// Every slice body below issues all of its loads before the first use, with
// predicated (never branching) lanes: absent entries gather the always-valid
// x[0] and are then skipped by a select, so the running sum sees exactly the
// present entries in ascending column order -- PETSc's order, bit for bit.

// aligned-offset slice with a compile-time width K (the stencil's point count)
// inb: every gather of the slice lies inside x (wave-uniform), so the
// absent entries can read their in-range neighbour and every gather uses the
// uniform-base form; otherwise absent entries read x[0]
template <int K, class VS, class XS, class MK>
__device__ __forceinline__ double dia_slice_fixed(const VS &vs, const int32_t *__restrict__ off,
                                                  const MK &mkload, int64_t row, const XS &x, int lane, bool inb,
                                                  int64_t srow, double &xc, bool &hc) {
  // values (or codes), then the gathers, then the code lookups: the
  // scheduling barrier keeps the lookups (which wait for the codes) from being
  // hoisted above the gathers, so both HBM trips are in flight together
  // (the presence mask is loaded after the gathers when they do not need it).
  // xc / hc: the operand at the slice's own rows when the middle offset is 0
  // (symmetric stencils), reused by the DOT / CG epilogue instead of a reload
  typename VS::template Raw<K> raw;
  vs.template fetch<K>(lane, raw);
  double v[K], xv[K];
  uint32_t mk = 0;
  if (inb) {
#pragma unroll
    for (int j = 0; j < K; ++j) xv[j] = x.at(srow + off[j], lane);
    if constexpr (!VS::kCodedPresence) mk = mkload();
  } else {
    if constexpr (VS::kCodedPresence) mk = vs.template presence<K>(raw);
    else mk = mkload();
#pragma unroll
    for (int j = 0; j < K; ++j) xv[j] = x(((mk >> j) & 1u) ? row + off[j] : 0);
  }
  __builtin_amdgcn_sched_barrier(0);
  hc = inb && off[K / 2] == 0;
  xc = xv[K / 2];
  vs.template decode<K>(raw, v);
  double sum = 0.0;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const double t = sum + v[j] * xv[j];
    bool p;
    if constexpr (VS::kCodedPresence) p = inb ? vs.template present<K>(raw, j) : ((mk >> j) & 1u);
    else p = (mk >> j) & 1u;
    sum = p ? t : sum;
  }
  return sum;
}

// aligned-offset slice, runtime width: batches of 8 slots
template <class VS, class XS>
__device__ __forceinline__ double dia_slice_any(const VS &vs, const int32_t *__restrict__ off,
                                                int k, uint32_t mk, int64_t row, const XS &x, int lane, bool inb,
                                                int64_t srow) {
  const int np = k >> 1;
  double sum = 0.0;
  for (int p0 = 0; p0 < np; p0 += 4) {
    double v[8], xv[8];
    vs.eight(p0, np, lane, v);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int j = 2 * p0 + q;
      const bool ok = j < 2 * np && ((mk >> j) & 1u);
      const int jj = j < 2 * np ? j : 0;
      xv[q] = inb ? x.at(srow + off[jj], lane) : x(ok ? row + off[jj] : 0);
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int j = 2 * p0 + q;
      const double t = sum + v[q] * xv[q];
      sum = (j < 2 * np && ((mk >> j) & 1u)) ? t : sum;
    }
  }
  if (k & 1) {
    const double v = vs.last(np, lane);
    const bool ok = (mk >> (k - 1)) & 1u;
    const double xv = inb ? x.at(srow + off[k - 1], lane) : x(ok ? row + off[k - 1] : 0);
    const double t = sum + v * xv;
    sum = ok ? t : sum;
  }
  return sum;
}

// general SELL slice (paired layout), continuing `sum`: batches of 8 entries;
// the unpaired last entry of an odd width rides in the batch that holds pair
// np (a 7-wide slice -- a diagonal plus six off-diagonal entries -- is one
// batch: all column, value and x loads in flight together, instead of a
// dependent second round trip for the last entry)
template <bool NT, class VS, class XS>
__device__ __forceinline__ double sell_slice(const int32_t *__restrict__ cbase, const VS &vs,
                                             int w, double sum, const XS &x, int lane) {
  const int np = w >> 1;
  const bool odd = (w & 1) != 0;
  const int nb = np + (odd ? 1 : 0);          // pairs, the tail counted as one
  const int2v *__restrict__ cp = reinterpret_cast<const int2v *>(cbase) + lane;
  for (int p0 = 0; p0 < nb; p0 += 4) {
    int c[8];
    double v[8], xv[8];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int p = p0 + q;
      int2v cc = int2v{-1, -1};
      if (p < np) cc = ld<NT>(cp + (int64_t)p * SLICE);
      else if (odd && p == np) cc.x = ld<NT>(cbase + (int64_t)np * 2 * SLICE + lane);
      c[2 * q] = cc.x; c[2 * q + 1] = cc.y;
    }
    vs.eight(p0, np, lane, v);
    if (odd && np >= p0 && np < p0 + 4) v[2 * (np - p0)] = vs.last(np, lane);
#pragma unroll
    for (int q = 0; q < 8; ++q) xv[q] = x(c[q] >= 0 ? c[q] : 0);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const double t = sum + v[q] * xv[q];
      sum = c[q] >= 0 ? t : sum;
    }
  }
  return sum;
}

// Row-pair body (units of 128 rows, lane = rows 2 l and 2 l + 1; layout in
// mx_assembly.hip pair_fill_kernel).  x is read as 16-byte pairs, one per run
// of the pattern: a singleton offset o gives both rows' operand (x[r0+o],
// x[r0+1+o]); a run c-1, c, c+1 loads the pair at c, and the two values that
// fall outside it -- x[r0+c-1] for row 0, x[r0+c+2] for row 1 -- come from the
// neighbouring lanes by a DPP wave shift (lanes 0 and 63 take the unit's edge
// values, loaded once per unit).  Per unit: one code load, one load per run,
// one 16-byte store, against two code loads, 2 K gathers and two stores for
// two single-row slices.  Every row still sums its entries in ascending
// column order, one rounding per multiply and add.
// PairShape / wave_shift: mx_pair.hpp

// One wave sweeps slices; lane = row.  Grid-stride over a fixed grid whose
// blocks are grouped by XCD (block b runs on XCD b % 8 under the observed
// round-robin dispatch): each XCD walks one contiguous eighth of the slices in
// order, so the +-1 / +-n / +-n^2 re-reads of x stay in that XCD's 4 MB L2.
// Placement only affects speed, never results.  KD > 0 specialises the
// aligned-offset body for the matrix's dominant slice width.
// UNI (5/7-point row pairs with a uniform-slot dictionary, Sell::puni): a
// unit's values and presence are its block's wave-uniform slot-row values and
// lane masks (scalar loads; the mask is the select condition itself), not
// code bytes looked up in the LDS table -- the same products and sums.
template <int MODE, bool NT, int KD, bool SPLIT, int JM = 0, bool VC = false, int PS = 0, bool UNI = false>
__global__ void __launch_bounds__(256) spmv_sell_kernel(
    int64_t m, int64_t ncols, int64_t nslices, const int64_t *__restrict__ sptr_d,
    const int32_t *__restrict__ wid_d, const int32_t *__restrict__ col_d,
    const double *__restrict__ val_d, const int32_t *__restrict__ doff, const int32_t *__restrict__ dpat,
    const uint32_t *__restrict__ dmask, const uint8_t *__restrict__ dmask8, const int64_t *__restrict__ sptr_o,
    const int32_t *__restrict__ wid_o, const int32_t *__restrict__ col_o,
    const double *__restrict__ val_o, const double *__restrict__ x,
    const double *__restrict__ lvec, double *__restrict__ y, const Jac jac,
    double *__restrict__ partials, const int *__restrict__ done, const CgFuse cg, const Fold fold,
    const double *__restrict__ xscale, const uint8_t *__restrict__ vcode, const int64_t *__restrict__ vcptr,
    const double *__restrict__ vtab_g, int ntab, int ynt, const uint8_t *__restrict__ pcode, int pat_star,
    const int32_t *__restrict__ pblk, int pdict, const PairUni *__restrict__ puni,
    const double *__restrict__ dtab_g) {
  static_assert(PS == 0 || VC, "row pairs: coded values");
  static_assert(!UNI || PS == 5 || PS == 7, "uniform-slot blocks: 5/7-point row pairs");
  CgTopIn top;
  if constexpr (MODE == SPMV_CG) top = cg.st->top;   // one batch of scalar loads, done included
  else if (done && *done) return;  // wave-uniform: solver finished, the launch is a no-op
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // work items: slices, or with PS units of two slices
  const int64_t nitems = PS ? (nslices + 1) / 2 : nslices;
  int s0, sstep, send;
  if ((gridDim.x & 7) == 0) {
    const int per = gridDim.x >> 3;                 // blocks per XCD group
    const int xcd = blockIdx.x & 7, j = blockIdx.x >> 3;
    const int chunk = (int)((nitems + 7) >> 3);
    s0 = xcd * chunk + j * SPMV_WAVES + wid;
    sstep = per * SPMV_WAVES;
    send = (int)min(nitems, (int64_t)(xcd + 1) * chunk);
  } else {
    s0 = blockIdx.x * SPMV_WAVES + wid;
    sstep = gridDim.x * SPMV_WAVES;
    send = (int)nitems;
  }
  // operand source
  constexpr bool SC = spmv_scaled(MODE);
  using XS = typename std::conditional<MODE == SPMV_CG, XCg<JM>, XPlainT<SC>>::type;
  const double xs = SC ? *xscale : 1.0;
  XS X;
  double xa = 0.0;
  bool xpend = false;
  if constexpr (MODE == SPMV_CG) {
    // the iteration's scalar top (convergence of i-1, b), committed by block 0
    if (top.done) return;
    const CgTop t = cg_top(top);
    if (blockIdx.x == 0 && threadIdx.x == 0) cg_commit_top(cg.st, t, cg.hist);
    if (t.reason) return;
    X = XCg<JM>{cg.r, cg.pold, cg.jac.d, cg.jac.c, t.b};
    xa = top.xa;
    xpend = top.xpend != 0.0;
  } else {
    X = XPlainT<SC>{x, xs};
  }
  __shared__ double vtab[VC ? VCODE_MAX : 1];
  // row pairs, Jacobi-fused modes (dtab_g set: the operator's own vector
  // Jacobi): dinv per diagonal code, so no dinv vector is read
  constexpr bool DT = spmv_jac(MODE) && PS != 0 && !UNI;
  __shared__ double dtab[DT ? VCODE_MAX : 1];
  if constexpr (VC) {   // every early return above is workgroup-uniform
    for (int i = threadIdx.x; i < VCODE_MAX; i += 256) vtab[i] = vtab_g[i];   // [ntab, 256) zero
    if constexpr (DT) {
      if (dtab_g)
        for (int i = threadIdx.x; i < VCODE_MAX; i += 256) dtab[i] = dtab_g[i];
    }
    __syncthreads();
  }
  double dot = 0.0;
  using VS = typename std::conditional<VC, VCoded<NT>, VDense<NT>>::type;
  auto vsrc = [&](int s) -> VS {
    if constexpr (VC) return VCoded<NT>{vcode + vcptr[s], vtab};
    else return VDense<NT>{val_d + sptr_d[s]};
  };
  // CG: p_{i-1} and x at the owned rows for the deferred VecAXPY, loaded with
  // the slice's first loads so their latency overlaps the gathers
  struct Own { double p = 0.0, x = 0.0; };
  auto own_load = [&](int64_t row) {
    Own o;
    if constexpr (MODE == SPMV_CG) {
      if (xpend) {
        const int64_t rc = row < m ? row : 0;
        o.p = cg.pold[rc];
        o.x = cg.x[rc];
      }
    }
    return o;
  };
  // everything after the diagonal-block sum of slice s; xc = the operand at
  // the slice's own rows when hc (gathered by the body), else reloaded
  auto finish = [&](int s, double sum, const Own &o, double xc, bool hc) {
    const int64_t row = (int64_t)s * SLICE + lane;
    if constexpr (MODE == SPMV_CG) {
      const double xr = hc ? xc : X(row < m ? row : 0);   // the same expression either way
      if (row < m) {
        cg.pnew[row] = xr;
        if (xpend) cg.x[row] = fma(xa, o.p, o.x);   // VecAXPY(X, a, P) of the previous step
      }
      xc = xr;
    }
    if (SPLIT) {
      // slice with ghost entries: store the diagonal-block sum; the boundary
      // kernel continues it with A_o once the halo has arrived
      if (wid_o[s]) {
        if (row < m) y[row] = sum;
        return;
      }
    } else if (lvec) {
      const int wo = wid_o[s];
      if (wo) sum = sell_slice<false>(col_o + sptr_o[s], VDense<false>{val_o + sptr_o[s]}, wo, sum, XPlainT<SC>{lvec, xs}, lane);
    }
    if (row < m) {
      const double out = spmv_jac(MODE) ? papply(jac, sum, row) : sum;   // PCApply_Jacobi fused: w_i * d_i
      if (ynt) __builtin_nontemporal_store(out, y + row);   // keep L2 for the x re-reads
      else y[row] = out;
      if (MODE == SPMV_DOT) dot += (hc ? xc : x[row]) * sum;   // VecDot(p, w) partial, p = x
      if (MODE == SPMV_CG) dot += xc * sum;
    }
  };
  auto one_slice = [&](int s) __attribute__((always_inline)) {
    const int64_t row = (int64_t)s * SLICE + lane;
    const int w = wid_d[s];
    const VS vs = vsrc(s);
    const Own o = own_load(row);
    double sum, xc = 0.0;
    bool hc = false;
    if (w < 0) {
      const int k = -w;
      auto mkload = [&]() -> uint32_t { return dmask8 ? (uint32_t)dmask8[row] : dmask[row]; };
      const int dp = dpat[s];
      const int32_t *__restrict__ off = doff + (int64_t)(dp & DPAT_ID) * DIA_MAX;
      const int64_t srow = (int64_t)s * SLICE;
      const bool inb = (dp & DPAT_INB) != 0;
      if (KD > 0 && k == KD && (PS == 0 || KD <= 8))   // pair kernels: rare fallback slices take the lean runtime-width body
        sum = dia_slice_fixed<(KD > 0 ? KD : 1)>(vs, off, mkload, row, X, lane, inb, srow, xc, hc);
      else sum = dia_slice_any(vs, off, k, mkload(), row, X, lane, inb, srow);
    } else {
      sum = sell_slice<NT>(col_d + sptr_d[s], vs, w, 0.0, X, lane);
    }
    finish(s, sum, o, xc, hc);
  };
  auto item = [&](int i) -> int { return i; };
  if constexpr (PS == 0) {
    for (int s = s0; s < send; s += sstep) one_slice(item(s));
  } else {
    using SH = PairShape<PS>;
    constexpr int K = SH::K, NR = SH::NR;
    constexpr int PB = (2 * K + 15) / 16 * 16;      // code bytes per lane
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    // the dominant pattern's offsets, and each run's anchor (singleton / centre)
    const int32_t *__restrict__ offs = doff + (int64_t)pat_star * DIA_MAX;
    int anchor[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) anchor[r] = offs[SH::first(r) + (SH::tri(r) ? 1 : 0)];
    const XBuf<XS> XB(X, MODE == SPMV_CG ? m : ncols);
    // pdict bits: 1 = code blocks from the dictionary (cached), 2 = read pblk
    // (dictionary ids and/or ghost flags), 4 = every full unit is a pair unit
    const bool use_pblk = (pdict & 3) != 0;
    // one unit's loads: its code block, every x pair and the edge values
    struct Unit { u32x4 cw[PB / 16]; dbl2 L[NR]; double e[NR]; uint32_t fl; int32_t bid; };
    auto unit_load = [&](int u, int32_t blkw, Unit &t) __attribute__((always_inline)) {
      const int ubase = u * 128, r0 = ubase + 2 * lane;
      const uint32_t bw = (uint32_t)blkw;
      t.fl = bw & ~PBLK_ID;
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        t.L[r] = XB.pair(r0 + anchor[r]);        // the operand (scaled / formed as the mode has it)
        // the run's two edge values in one load: lane 0 reads x[r0 + c - 1]
        // (its row 0's left neighbour), every other lane x[ubase + 128 + c]
        // (lane 63's row 1's right neighbour; one line for the wave)
        if (SH::tri(r)) t.e[r] = XB(lane == 0 ? ubase + anchor[r] - 1 : ubase + 128 + anchor[r]);
      }
      // the unit's code block (after the operand loads: its address waits on
      // the block id): its own (streamed non-temporally), or a dictionary
      // block shared with every unit of the same boundary/value class (cached:
      // the dictionary stays in L2)
      const int64_t blk = use_pblk ? (int64_t)(bw & PBLK_ID) : (int64_t)u;
      t.bid = (int32_t)blk;
      if constexpr (UNI) return;                  // values and presence: puni[blk] at the finish
      const u32x4 *__restrict__ cp = reinterpret_cast<const u32x4 *>(pcode + (blk * 64 + lane) * PB);
      if (pdict & 1) {                            // kernel-uniform
#pragma unroll
        for (int q = 0; q < PB / 16; ++q) t.cw[q] = cp[q];
      } else {
#pragma unroll
        for (int q = 0; q < PB / 16; ++q) t.cw[q] = ld<NT>(cp + q);
      }
    };
    // the lookups, the two row sums and everything stored after them
    auto unit_finish = [&](int u, const Unit &t) __attribute__((always_inline)) {
      const int64_t r0 = (int64_t)u * 128 + 2 * lane;
      auto code = [&](int i) -> int {            // code i of the lane (row 0: 0..K-1, row 1: K..2K-1)
        return (t.cw[i >> 4][(i >> 2) & 3] >> (8 * (i & 3))) & 0xff;
      };
      double sum0 = 0.0, sum1 = 0.0;
      double lo_m1 = 0.0, hi_p1 = 0.0;           // the current run's shifted neighbours
#pragma unroll
      for (int j = 0; j < K; ++j) {
        const int r = SH::run(j), p = SH::pos(j);
        if (SH::tri(r) && p < 0) {
          lo_m1 = wave_shift<true>(t.L[r].y, t.e[r]);    // x[r0 + c - 1] = lane - 1's x[r0' + c + 1]
          hi_p1 = wave_shift<false>(t.L[r].x, t.e[r]);   // x[r0 + c + 2] = lane + 1's x[r0' + c]
        }
        double a0, a1;                           // operand for row 0 / row 1
        if (!SH::tri(r)) { a0 = t.L[r].x; a1 = t.L[r].y; }
        else if (p < 0) { a0 = lo_m1; a1 = t.L[r].x; }
        else if (p == 0) { a0 = t.L[r].x; a1 = t.L[r].y; }
        else { a0 = t.L[r].y; a1 = hi_p1; }
        if constexpr (UNI) {
          const PairUni &B = puni[t.bid];        // wave-uniform: scalar loads
          const double t0 = sum0 + B.v[j] * a0, t1 = sum1 + B.v[K + j] * a1;
          sum0 = __builtin_amdgcn_inverse_ballot_w64(B.pm[j]) ? t0 : sum0;
          sum1 = __builtin_amdgcn_inverse_ballot_w64(B.pm[K + j]) ? t1 : sum1;
        } else {
          const int c0 = code(j), c1 = code(K + j);
          const double t0 = sum0 + vtab[c0] * a0, t1 = sum1 + vtab[c1] * a1;
          sum0 = c0 != VCODE_ABSENT ? t0 : sum0;
          sum1 = c1 != VCODE_ABSENT ? t1 : sum1;
        }
      }
      // SPLIT: rows of a slice with A_o entries store the diagonal-block sum;
      // the boundary kernel continues it (and applies the epilogue)
      const bool gh = SPLIT && (t.fl & (lane < 32 ? PBLK_GHOST_LO : PBLK_GHOST_HI)) != 0;
      double o0 = sum0, o1 = sum1;
      if constexpr (spmv_jac(MODE)) {
        if (!gh) {
          if constexpr (DT) {
            if (dtab_g) {                        // the rows' diagonal slot: offset 0 of the centre run
              constexpr int JC = SH::first(SH::CENTER_RUN) + 1;
              o0 = sum0 * dtab[code(JC)];
              o1 = sum1 * dtab[code(K + JC)];
            } else {
              o0 = papply(jac, sum0, r0); o1 = papply(jac, sum1, r0 + 1);
            }
          } else {
            o0 = papply(jac, sum0, r0); o1 = papply(jac, sum1, r0 + 1);
          }
        }
      }
      if (ynt) __builtin_nontemporal_store(dbl2{o0, o1}, reinterpret_cast<dbl2 *>(y + r0));
      else *reinterpret_cast<dbl2 *>(y + r0) = dbl2{o0, o1};
      if constexpr (MODE == SPMV_CG) {
        // p_i at the own rows is the centre run's pair: store it, and the
        // previous step's deferred VecAXPY(X, a, P) on the own rows
        *reinterpret_cast<dbl2 *>(cg.pnew + r0) = t.L[SH::CENTER_RUN];
        if (xpend) {
          const dbl2 po = *reinterpret_cast<const dbl2 *>(cg.pold + r0);
          const dbl2 xo = *reinterpret_cast<const dbl2 *>(cg.x + r0);
          *reinterpret_cast<dbl2 *>(cg.x + r0) = dbl2{fma(xa, po.x, xo.x), fma(xa, po.y, xo.y)};
        }
      }
      if constexpr (MODE == SPMV_DOT || MODE == SPMV_CG) {   // operand at the own rows = the centre pair
        if (!gh) {
          dot += t.L[SH::CENTER_RUN].x * sum0;
          dot += t.L[SH::CENTER_RUN].y * sum1;
        }
      }
    };
    // is unit v stored as row pairs (wave-uniform)
    auto is_pair = [&](int v) -> bool {
      return (pdict & 4) ? (int64_t)v * 128 + 127 < m : (dpat[2 * v] & DPAT_PAIR) != 0;
    };
    auto one_unit = [&](int u) __attribute__((always_inline)) {
      if (!is_pair(u)) {
        one_slice(2 * u);
        if (2 * u + 1 < nslices) one_slice(2 * u + 1);
        return;
      }
      Unit t;
      unit_load(u, use_pblk ? pblk[u] : 0, t);
      __builtin_amdgcn_sched_barrier(0);          // every load issued before the first lookup
      unit_finish(u, t);
    };
    int u = s0;
    // SPMV_PAIR_TWO: a wave takes its next two units together, both units'
    // loads in flight before the first lookup (twice the bytes in flight per
    // wave at the same occupancy); the units still finish in sweep order, so
    // the per-lane dot partial sums in the same order
    // The step's metadata (pair flags, dictionary block ids) is loaded one
    // step ahead, behind the current step's vector loads, so the branch and
    // the code-block address never wait on a scalar round trip of their own.
    if constexpr (SPMV_PAIR_TWO && PS != 27 && MODE != SPMV_CG) {
      struct Meta { int32_t da = 0, db = 0, ba = 0, bb = 0; };
      auto meta = [&](int v) __attribute__((always_inline)) {   // step starting at sweep index v
        Meta q;
        if (v + sstep < send) {
          const int va = item(v), vb = item(v + sstep);
          q.da = is_pair(va) ? DPAT_PAIR : 0;
          q.db = is_pair(vb) ? DPAT_PAIR : 0;
          if (use_pblk) { q.ba = pblk[va]; q.bb = pblk[vb]; }
        }
        return q;
      };
      // block ids two steps ahead: a wave sweeps only ~16 steps, so the
      // first steps' scalar round trips must not sit in front of their loads
      Meta cur = meta(u), nx1 = meta(u + 2 * sstep);
      for (; u + sstep < send; u += 2 * sstep) {
        const int ua = item(u), ub = item(u + sstep);
        const Meta nx2 = meta(u + 4 * sstep);
        if ((cur.da & DPAT_PAIR) && (cur.db & DPAT_PAIR)) {   // wave-uniform
          Unit ta, tb;
          unit_load(ua, cur.ba, ta);
          unit_load(ub, cur.bb, tb);
          __builtin_amdgcn_sched_barrier(0);
          unit_finish(ua, ta);
          unit_finish(ub, tb);
        } else {
          one_unit(ua);
          one_unit(ub);
        }
        cur = nx1;
        nx1 = nx2;
      }
    }
    for (; u < send; u += sstep) one_unit(item(u));
  }
  if (MODE == SPMV_DOT || MODE == SPMV_CG) {
    double v[1] = {dot};
    block_partials<1>(v, partials, gridDim.x, fold);
  }
}

// launch-geometry caches, shared by the host threads of in-process ranks
static std::mutex g_geom_mu;

int device_cu_count() {
  static int cus[64] = {0};
  int dev = 0;
  HIPCHECK(hipGetDevice(&dev));
  if (dev < 0 || dev >= 64) return 256;
  std::lock_guard<std::mutex> lk(g_geom_mu);
  if (!cus[dev]) HIPCHECK(hipDeviceGetAttribute(&cus[dev], hipDeviceAttributeMultiprocessorCount, dev));
  return cus[dev];
}

// Upper bound of the main launch's grid (partial-sum buffers are sized by it)
int spmv_blocks(const Mat *A, int) {
  const int64_t need = cdiv(A->sd.nslices, SPMV_WAVES);
  const int64_t cap = g_knobs.spmv_grid > 0 ? g_knobs.spmv_grid : 8 * (int64_t)device_cu_count();
  return (int)std::max<int64_t>(1, std::min<int64_t>(need, std::max<int64_t>({cap, (int64_t)8192, (int64_t)g_knobs.spmv_fp64_grid})));
}

// Grid of the main SpMV launch (value-coded layouts): exactly the workgroups
// that are resident at once (one generation).  Each XCD then walks its slices in one sweep with a
// window of ~ the resident waves, so the x lines of the +-n^2 neighbours are
// re-read from L2 (tools/pmc_spmv.sh: FETCH_SIZE = the compulsory bytes at
// this grid, ~2x at a 4.6-generation grid) and no second generation leaves a
// tail.  Blocks per CU: the occupancy API, capped at 6 (knob 26): the kernels
// hold 106 SGPRs, which allow 6 waves per SIMD, while the API reports one
// more at that count (MI355X guide, correctness boundaries).  The row-pair
// kernels stream twice the rows per wave and do best at 4 (knob 28; 256^3:
// 82 us at 4, 87 at 5, 93 at 6).  SPMV_CG
// evaluates the iteration's scalar top once per workgroup, so it keeps >= 4
// slices per wave.  Knob 3 > 0 overrides the grid.
int main_grid(const Mat *A, int mode, const void *kf, bool pairs) {
  const int64_t need = cdiv(A->sd.nslices, SPMV_WAVES);
  int64_t g;
  const bool coded = A->sd.ntab > 0 && g_knobs.vcodes;
  if (g_knobs.spmv_grid > 0) {
    g = g_knobs.spmv_grid;
  } else if (!pairs && !coded && g_knobs.spmv_fp64_grid > 0) {
    // fp64 values streamed (more than 255 distinct values): the matrix stream
    // dominates, and several workgroup generations keep more of it in flight
    // than one resident generation (variable-coefficient 7-point 256^3:
    // 214 -> 203 us standalone, CG -4% per iteration at 8192; knob 43)
    g = g_knobs.spmv_fp64_grid;
  } else {
    static std::unordered_map<const void *, int> bpc_of;
    int bpc;
    {
      std::lock_guard<std::mutex> lk(g_geom_mu);
      auto it = bpc_of.find(kf);
      if (it == bpc_of.end()) {
        int b = 0;
        HIPCHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, kf, 256, 0));
        it = bpc_of.emplace(kf, std::max(1, b)).first;
      }
      bpc = it->second;
    }
    const int cap = pairs ? g_knobs.spmv_pair_bpc : g_knobs.spmv_bpc;
    g = (int64_t)std::min(bpc, std::max(1, cap)) * device_cu_count();
    // one workgroup fewer per XCD: a per-XCD wave count that is a multiple of
    // 256 (grids of 1024 / 1536) puts the concurrent x streams on aliasing
    // strides -- measured +35..+80% MatMult time (tools/op_ab.py)
    if (g > 64) g -= 8;
  }
  g = std::min<int64_t>(g, need);
  if (mode == SPMV_CG) g = std::min<int64_t>(g, std::max<int64_t>(512, need / 4));
  if (g >= 64) g &= ~int64_t(7);   // multiple of 8: XCD grouping
  return (int)std::max<int64_t>(1, g);
}

// Second half of an overlapped MatMult: y_i continues from the diagonal-block
// sum with the A_o entries in ghost order (MatMultAdd_SeqAIJ), then the fused
// epilogue.  One wave per listed slice.
template <int MODE>
__global__ void __launch_bounds__(256) spmv_boundary_kernel(
    int64_t m, const int32_t *__restrict__ list, int nlist, const int64_t *__restrict__ sptr_o,
    const int32_t *__restrict__ wid_o, const int32_t *__restrict__ col_o, const double *__restrict__ val_o,
    const double *__restrict__ x, const double *__restrict__ lvec, double *__restrict__ y, const Jac jac,
    double *__restrict__ partials, const int *__restrict__ done, const Fold fold,
    const double *__restrict__ xscale) {
  if (done && *done) return;
  constexpr bool SC = spmv_scaled(MODE);
  const double xs = SC ? *xscale : 1.0;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  double dot = 0.0;
  for (int k = blockIdx.x * SPMV_WAVES + wid; k < nlist; k += gridDim.x * SPMV_WAVES) {
    const int s = list[k];
    const int64_t row = (int64_t)s * SLICE + lane;
    double sum = row < m ? y[row] : 0.0;
    sum = sell_slice<false>(col_o + sptr_o[s], VDense<false>{val_o + sptr_o[s]}, wid_o[s], sum, XPlainT<SC>{lvec, xs}, lane);
    if (row < m) {
      if (spmv_jac(MODE)) y[row] = papply(jac, sum, row);
      else y[row] = sum;
      if (MODE == SPMV_DOT) dot += x[row] * sum;
    }
  }
  if (MODE == SPMV_DOT) {
    double v[1] = {dot};
    block_partials<1>(v, partials, gridDim.x, fold);
  }
}

__global__ void pack_kernel(int64_t n, const int32_t *__restrict__ idx, const double *__restrict__ x,
                            double *__restrict__ buf) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += stride) buf[k] = x[idx[k]];
}

// halo payload of the CG direction p_i, formed from r and p_{i-1}
template <int JM>
__global__ void pack_cg_kernel(int64_t n, const int32_t *__restrict__ idx, const CgFuse cg,
                               const int *__restrict__ done, double *__restrict__ buf) {
  const CgTopIn top = cg.st->top;
  if (top.done) return;
  const CgTop t = cg_top(top);                  // read-only: the MatMult commits it
  if (t.reason) return;
  const XCg<JM> X{cg.r, cg.pold, cg.jac.d, cg.jac.c, t.b};
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += stride) buf[k] = X(idx[k]);
}

// VecScatterBegin/End(x -> lvec): pack (only if some peer's rows are not a
// contiguous range; always for the CG operand, which is formed on the fly),
// then one grouped send/recv with every neighbour, on stream `st`.
static void halo_exchange(Mat *A, const double *x, const CgFuse *cg, const int *done, hipStream_t st) {
  Halo &H = A->halo;
  const bool pack = cg || H.need_pack;
  if (pack && H.nsend) {
    const unsigned g = grid_for(H.nsend, 256, 4096);
    if (cg && cg->jac.mode == 1) pack_cg_kernel<1><<<g, 256, 0, st>>>(H.nsend, H.send_idx.p, *cg, done, H.send_buf.p);
    else if (cg && cg->jac.mode == 2) pack_cg_kernel<2><<<g, 256, 0, st>>>(H.nsend, H.send_idx.p, *cg, done, H.send_buf.p);
    else if (cg) pack_cg_kernel<0><<<g, 256, 0, st>>>(H.nsend, H.send_idx.p, *cg, done, H.send_buf.p);
    else pack_kernel<<<grid_for(H.nsend, 256, 4096), 256, 0, st>>>(H.nsend, H.send_idx.p, x, H.send_buf.p);
    HIPCHECK(hipGetLastError());
  }
  std::vector<Msg> sends, recvs;
  for (size_t i = 0; i < H.send_peer.size(); ++i) {
    void *buf = (!cg && H.send_contig_start[i] >= 0) ? (void *)(x + H.send_contig_start[i])
                                                     : (void *)(H.send_buf.p + H.send_off[i]);
    sends.push_back({H.send_peer[i], buf, sizeof(double) * (size_t)H.send_cnt[i]});
  }
  for (size_t i = 0; i < H.recv_peer.size(); ++i)
    recvs.push_back({H.recv_peer[i], H.lvec.p + H.recv_off[i], sizeof(double) * (size_t)H.recv_cnt[i]});
  A->comm->exchange(sends, recvs, st);
}

void halo_begin(Mat *A, const double *x) {
  if (A->comm->size == 1) return;
  halo_exchange(A, x, nullptr, nullptr, A->comm->stream);
}

// the pair body's pdict argument (see the kernel)
static int pair_flags(const Mat *A) {
  const Sell &S = A->sd;
  return (S.pair_blocks > 0 ? 1 : 0) | (S.pair_blocks > 0 || S.pair_ghosts ? 2 : 0) | (S.pair_all ? 4 : 0);
}

// returns the grid; a fold (cnt set) counts all of its workgroups
static int launch_main(Mat *A, const double *x, double *y, int mode, Jac jac, double *partials,
                       int *done_flag, bool split, hipStream_t st, const CgFuse *cgp, const Fold &fold_in,
                       const double *xscale) {
  // row-pair z-march kernels (mx_spmv_pair.hip; each row's sum has the same
  // bits): constant-coefficient 5/7/27-point blocks, fp64 row pairs, and the
  // coded z-march for non-uniform code dictionaries (every non-CG mode,
  // GMRES's scaled operand included)
  if (!cgp) {
    if (cb_applies(A, mode, split)) return cb_launch(A, mode, split, x, y, jac, partials, done_flag, fold_in, xscale, st);
    const int lg = pair_lean_launch(A, mode, split, x, y, partials, done_flag, fold_in, st, jac, xscale);
    if (lg) return lg;
  }
  const double *lvec = (A->nghost && !split) ? A->halo.lvec.p : nullptr;
  const int kd = A->sd.dia_k;
  const CgFuse cg = cgp ? *cgp : CgFuse{};
  // value codes (when the matrix has them; knob 23 = 0 reads the fp64 values)
  const bool vcode = A->sd.ntab > 0 && g_knobs.vcodes;
  const VCodes vc{A->sd.code.p, A->sd.cptr.p, A->sd.vtab.p, A->sd.ntab};
#define SPMV_ARGS                                                                           \
  A->m, A->n, A->sd.nslices, A->sd.sptr.p, A->sd.width.p, A->sd.col.p, A->sd.val.p, A->sd.doff.p, A->sd.dpat.p, \
      A->sd.mask.p, A->sd.mask8.p, A->so.sptr.p, A->so.width.p, A->so.col.p, A->so.val.p, x, lvec, y, jac, \
      partials, done_flag, cg, fold, xscale, vc.code, vc.cptr, vc.tab, vc.ntab, g_knobs.spmv_ynt, \
      A->sd.pcode.p, A->sd.pat_star, A->sd.pblk.p, pair_flags(A), A->sd.puni.p, dtab
  using KFn = decltype(&spmv_sell_kernel<SPMV_PLAIN, true, 0, false, 0, false>);
  KFn kf = nullptr;
#define SPMV_KDU(MODE, NT, SP, JM, VC, K) kf = &spmv_sell_kernel<MODE, NT, K, SP, JM, VC>
#define SPMV_KD(MODE, NT, SP, JM, VC)                                                                 \
  do {                                                                                                \
    switch (kd) {                                                                                     \
      case 5: SPMV_KDU(MODE, NT, SP, JM, VC, 5); break;                                               \
      case 7: SPMV_KDU(MODE, NT, SP, JM, VC, 7); break;                                               \
      case 27: SPMV_KDU(MODE, NT, SP, JM, VC, 27); break;                                             \
      default: SPMV_KDU(MODE, NT, SP, JM, VC, 0); break;                                              \
    }                                                                                                 \
  } while (0)
#define SPMV_CGKD(JM, SP)                                                                    \
  do {                                                                                       \
    if (ps == 5) { if (uni) kf = &spmv_sell_kernel<SPMV_CG, true, 5, SP, JM, true, 5, true>;   \
                   else kf = &spmv_sell_kernel<SPMV_CG, true, 5, SP, JM, true, 5>; }          \
    else if (ps == 7) { if (uni) kf = &spmv_sell_kernel<SPMV_CG, true, 7, SP, JM, true, 7, true>; \
                        else kf = &spmv_sell_kernel<SPMV_CG, true, 7, SP, JM, true, 7>; }     \
    else if (ps == 27) kf = &spmv_sell_kernel<SPMV_CG, true, 27, SP, JM, true, 27>;          \
    else if (vcode) SPMV_KD(SPMV_CG, true, SP, JM, true);                                    \
    else SPMV_KD(SPMV_CG, true, SP, JM, false);                                              \
  } while (0)
  // code blocks are always read non-temporally; row pairs when the matrix has them
  const int ps = vcode && g_knobs.spmv_pairs ? A->sd.pair_shape : 0;
  // uniform-slot dictionary (knob 35 = 0: the LDS table path)
  const bool uni = ps && A->sd.puni.p && g_knobs.pair_uni && (pair_flags(A) & 1);
  // Jacobi by diagonal code (knob 37): the operator's own vector Jacobi only
  const double *dtab = ps && !uni && spmv_jac(mode) && jac.mode == 1 && jac.d == A->jac_dinv.p && A->sd.dtab.p &&
                               g_knobs.pair_dtab ? A->sd.dtab.p : nullptr;
#define SPMV_PS(MODE, SP)                                                                         \
  do {                                                                                            \
    if (ps == 5) { if (uni) kf = &spmv_sell_kernel<MODE, true, 5, SP, 0, true, 5, true>;           \
                   else kf = &spmv_sell_kernel<MODE, true, 5, SP, 0, true, 5>; }                  \
    else if (ps == 7) { if (uni) kf = &spmv_sell_kernel<MODE, true, 7, SP, 0, true, 7, true>;      \
                        else kf = &spmv_sell_kernel<MODE, true, 7, SP, 0, true, 7>; }             \
    else kf = &spmv_sell_kernel<MODE, true, 27, SP, 0, true, 27>;                                 \
  } while (0)
#define SPMV_GO(MODE)                                                         \
  do {                                                                        \
    if (ps) { if (split) SPMV_PS(MODE, true); else SPMV_PS(MODE, false); }   \
    else if (vcode) { if (split) SPMV_KD(MODE, true, true, 0, true); else SPMV_KD(MODE, true, false, 0, true); } \
    else if (split) { if (g_knobs.spmv_nt) SPMV_KD(MODE, true, true, 0, false); else SPMV_KD(MODE, false, true, 0, false); } \
    else { if (g_knobs.spmv_nt) SPMV_KD(MODE, true, false, 0, false); else SPMV_KD(MODE, false, false, 0, false); }     \
  } while (0)
  switch (mode) {
    case SPMV_PLAIN: SPMV_GO(SPMV_PLAIN); break;
    case SPMV_JACOBI: SPMV_GO(SPMV_JACOBI); break;
    case SPMV_PLAIN_S: SPMV_GO(SPMV_PLAIN_S); break;
    case SPMV_JACOBI_S: SPMV_GO(SPMV_JACOBI_S); break;
    case SPMV_DOT: SPMV_GO(SPMV_DOT); break;
    case SPMV_CG:   // always non-temporal; Jacobi form as a template argument
      if (!cgp) fail(MX_ERR_INTERNAL, "CG-fused SpMV without operands");
      switch (cg.jac.mode) {
        case 1: if (split) SPMV_CGKD(1, true); else SPMV_CGKD(1, false); break;
        case 2: if (split) SPMV_CGKD(2, true); else SPMV_CGKD(2, false); break;
        default: if (split) SPMV_CGKD(0, true); else SPMV_CGKD(0, false); break;
      }
      break;
    default: fail(MX_ERR_INTERNAL, "bad spmv mode");
  }
  const int grid = main_grid(A, mode, reinterpret_cast<const void *>(kf), ps != 0);
  Fold fold = fold_in;
  if (fold.cnt) { fold.ntotal = fold.ncount = grid; fold.base = 0; }
  note_dispatch(mode == SPMV_CG ? DSP_SELL_CG : DSP_SELL);
  launch_timed(kf, grid, st, SPMV_ARGS);
#undef SPMV_GO
#undef SPMV_PS
#undef SPMV_CGKD
#undef SPMV_KD
#undef SPMV_KDU
#undef SPMV_ARGS
  HIPCHECK(hipGetLastError());
  return grid;
}

void spmv_launch(Mat *A, const double *x, double *y, int mode, Jac jac, double *partials,
                 int *done_flag) {
  launch_main(A, x, y, mode, jac, partials, done_flag, false, A->comm->stream, nullptr, Fold{}, nullptr);
}

constexpr int BND_BLOCKS = 2048;   // one boundary slice per wave: the launch runs after the interior, alone on the GPU

// The product splits (diagonal-block launch, then the boundary kernel adds
// A_o) when the halo overlaps the interior, and always when some row-pair
// unit has A_o entries: the pair body has no A_o continuation of its own.
static bool pair_forces_split(const Mat *A) { return A->sd.pair_ghosts && A->sd.ntab > 0 && g_knobs.vcodes && g_knobs.spmv_pairs; }
bool matmult_splits(const Mat *A) {
  return A->comm->size > 1 && A->halo.nbnd > 0 && (g_knobs.overlap || pair_forces_split(A));
}

// CG mode 5 on P > 1 ranks, the iterations between x-step batches (knob 80):
// the direction update fused into the split p.Ap pass.  The halo pack forms
// the ghost planes' p_i = z_i + b p_{i-1} from r_i and p_{i-1} (pack_cg_kernel,
// as CG mode 1 does) and sends it on the comm stream while the fused pass
// (pair_cg5_pbws_launch) forms every operand the same way, stores p_i and the
// ghost units' diagonal-block sums; the boundary kernel then continues those
// rows over the halo from the stored p_i -- the launches, partials and bits of
// cg_pb_kernel + matmult_overlap(SPMV_PW) without the direction update's pass.
int cg5_pbws_matmult(Mat *A, KspState *s, const double *r, double *const pb[8], int xb, int it, double *hist,
                     const Jac &jac, double *y, double *partials, int *done, const Fold *fold) {
  Comm *c = A->comm;
  Halo &H = A->halo;
  hipStream_t st = c->stream;
  CgFuse cg;
  cg.r = r;
  cg.pold = pb[(it + xb - 1) % xb];
  cg.pnew = pb[it % xb];
  cg.st = s;
  cg.hist = hist;
  cg.jac = jac;
  int nmain;
  if (g_knobs.overlap) {
    hipStream_t cs = c->comm_stream;
    if (!H.ev_x) {
      HIPCHECK(hipEventCreateWithFlags(&H.ev_x, hipEventDisableTiming));
      HIPCHECK(hipEventCreateWithFlags(&H.ev_done, hipEventDisableTiming));
    }
    HIPCHECK(hipEventRecord(H.ev_x, st));
    HIPCHECK(hipStreamWaitEvent(cs, H.ev_x, 0));
    halo_exchange(A, nullptr, &cg, done, cs);
    HIPCHECK(hipEventRecord(H.ev_done, cs));
    nmain = pair_cg5_pbws_launch(A, s, r, pb, xb, hist, jac.mode, jac.c, y, partials, st);
    HIPCHECK(hipStreamWaitEvent(st, H.ev_done, 0));
  } else {
    halo_exchange(A, nullptr, &cg, done, st);
    nmain = pair_cg5_pbws_launch(A, s, r, pb, xb, hist, jac.mode, jac.c, y, partials, st);
  }
  const int nb = std::min(g_knobs.bnd_grid > 0 ? g_knobs.bnd_grid : BND_BLOCKS, (H.nbnd + SPMV_WAVES - 1) / SPMV_WAVES);
  Fold f;
  if (fold) { f = *fold; f.ntotal = nmain + nb; f.base = nmain; f.ncount = nb; }
  double *pbn = partials ? (fold ? partials : partials + nmain) : nullptr;
  note_dispatch(DSP_BOUNDARY);
  spmv_boundary_kernel<SPMV_DOT><<<nb, 256, 0, st>>>(A->m, H.bnd_slices.p, H.nbnd, A->so.sptr.p, A->so.width.p,
                                                    A->so.col.p, A->so.val.p, cg.pnew, H.lvec.p, y, Jac{}, pbn, done,
                                                    f, nullptr);
  HIPCHECK(hipGetLastError());
  return nmain + nb;
}

int matmult_overlap(Mat *A, const double *x, double *y, int mode, Jac jac, double *partials,
                    int *done_flag, const CgFuse *cg, const Fold *fold, const double *xscale) {
  Comm *c = A->comm;
  Halo &H = A->halo;
  hipStream_t st = c->stream;
  if (!matmult_splits(A)) {
    if (c->size > 1) halo_exchange(A, x, mode == SPMV_CG ? cg : nullptr, done_flag, st);
    return launch_main(A, x, y, mode, jac, partials, done_flag, false, st, cg, fold ? *fold : Fold{}, xscale);
  }
  int nmain;
  if (g_knobs.overlap) {
    hipStream_t cs = c->comm_stream;
    if (!H.ev_x) {
      HIPCHECK(hipEventCreateWithFlags(&H.ev_x, hipEventDisableTiming));
      HIPCHECK(hipEventCreateWithFlags(&H.ev_done, hipEventDisableTiming));
    }
    // halo on the comm stream, after the operand's inputs are final on the
    // compute stream; the CG operand's inputs (r, p_{i-1}) are only read by both
    HIPCHECK(hipEventRecord(H.ev_x, st));
    HIPCHECK(hipStreamWaitEvent(cs, H.ev_x, 0));
    halo_exchange(A, x, mode == SPMV_CG ? cg : nullptr, done_flag, cs);
    HIPCHECK(hipEventRecord(H.ev_done, cs));
    // interior slices meanwhile; boundary slices after the exchange
    nmain = launch_main(A, x, y, mode, jac, partials, done_flag, true, st, cg, Fold{}, xscale);
    HIPCHECK(hipStreamWaitEvent(st, H.ev_done, 0));
  } else {                      // no overlap: exchange, split product, boundary pass
    halo_exchange(A, x, mode == SPMV_CG ? cg : nullptr, done_flag, st);
    nmain = launch_main(A, x, y, mode, jac, partials, done_flag, true, st, cg, Fold{}, xscale);
  }
  const int nb = std::min(g_knobs.bnd_grid > 0 ? g_knobs.bnd_grid : BND_BLOCKS, (H.nbnd + SPMV_WAVES - 1) / SPMV_WAVES);
  // the boundary launch folds the partials of both launches (fold) or
  // appends its own after the main launch's
  Fold f;
  if (fold) { f = *fold; f.ntotal = nmain + nb; f.base = nmain; f.ncount = nb; }
  double *pb = partials ? (fold ? partials : partials + nmain) : nullptr;
  // the boundary rows' operand values were stored by the main kernel (CG)
  const double *xb = mode == SPMV_CG ? cg->pnew : x;
#define BND(MODE) spmv_boundary_kernel<MODE><<<nb, 256, 0, st>>>(A->m, H.bnd_slices.p, H.nbnd, A->so.sptr.p, \
      A->so.width.p, A->so.col.p, A->so.val.p, xb, H.lvec.p, y, jac, pb, done_flag, f, xscale)
  note_dispatch(DSP_BOUNDARY);
  switch (mode) {
    case SPMV_PLAIN: BND(SPMV_PLAIN); break;
    case SPMV_JACOBI: BND(SPMV_JACOBI); break;
    case SPMV_PLAIN_S: BND(SPMV_PLAIN_S); break;
    case SPMV_JACOBI_S: BND(SPMV_JACOBI_S); break;
    default: BND(SPMV_DOT); break;
  }
#undef BND
  HIPCHECK(hipGetLastError());
  return nmain + nb;
}

void mat_mult(Mat *A, const double *x, double *y) {
  matmult_overlap(A, x, y, SPMV_PLAIN, Jac{}, nullptr, nullptr);
}

// this translation unit's code object, loaded now rather than at the first
// launch of one of its kernels (load_code_objects)
void load_code_spmv() {
  hipFuncAttributes a;
  (void)hipFuncGetAttributes(&a, reinterpret_cast<const void *>(&pack_kernel));
  (void)hipGetLastError();
}

}  // namespace mx
