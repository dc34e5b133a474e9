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
#include <algorithm>

#include "mx_cg.hpp"
#include "mx_device.hpp"
#include "mx_internal.hpp"

namespace mx {

constexpr int SPMV_WAVES = 4;  // 256-thread workgroups, one slice per wave at a time
Knobs g_knobs;

typedef double dbl2 __attribute__((ext_vector_type(2)));
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
};

// Every slice body below issues all of its loads before the first use, with
// predicated (never branching) lanes: absent entries gather the always-valid
// x[0] and are then skipped by a select, so the running sum sees exactly the
// present entries in ascending column order -- PETSc's order, bit for bit.

// aligned-offset slice with a compile-time width K (the stencil's point count)
// inb: every gather of the slice lies inside x (wave-uniform), so the
// absent entries can read their in-range neighbour and every gather uses the
// uniform-base form; otherwise absent entries read x[0]
template <int K, bool NT, class XS>
__device__ __forceinline__ double dia_slice_fixed(const double *__restrict__ vbase, const int32_t *__restrict__ off,
                                                  uint32_t mk, int64_t row, const XS &x, int lane, bool inb,
                                                  int64_t srow) {
  constexpr int NP = K / 2;
  double v[K], xv[K];
  const dbl2 *__restrict__ vp = reinterpret_cast<const dbl2 *>(vbase) + lane;
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const dbl2 t = ld<NT>(vp + p * SLICE);
    v[2 * p] = t.x;
    v[2 * p + 1] = t.y;
  }
  if constexpr (K & 1) v[K - 1] = ld<NT>(vbase + NP * 2 * SLICE + lane);
  if (inb) {
#pragma unroll
    for (int j = 0; j < K; ++j) xv[j] = x.at(srow + off[j], lane);
  } else {
#pragma unroll
    for (int j = 0; j < K; ++j) xv[j] = x(((mk >> j) & 1u) ? row + off[j] : 0);
  }
  double sum = 0.0;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const double t = sum + v[j] * xv[j];
    sum = ((mk >> j) & 1u) ? t : sum;
  }
  return sum;
}

// aligned-offset slice, runtime width: batches of 8 slots
template <bool NT, class XS>
__device__ __forceinline__ double dia_slice_any(const double *__restrict__ vbase, const int32_t *__restrict__ off,
                                                int k, uint32_t mk, int64_t row, const XS &x, int lane, bool inb,
                                                int64_t srow) {
  const int np = k >> 1;
  const dbl2 *__restrict__ vp = reinterpret_cast<const dbl2 *>(vbase) + lane;
  double sum = 0.0;
  for (int p0 = 0; p0 < np; p0 += 4) {
    double v[8], xv[8];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int p = p0 + q;
      const dbl2 t = p < np ? ld<NT>(vp + (int64_t)p * SLICE) : dbl2{0.0, 0.0};
      v[2 * q] = t.x;
      v[2 * q + 1] = t.y;
    }
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
    const double v = ld<NT>(vbase + (int64_t)np * 2 * SLICE + lane);
    const bool ok = (mk >> (k - 1)) & 1u;
    const double xv = inb ? x.at(srow + off[k - 1], lane) : x(ok ? row + off[k - 1] : 0);
    const double t = sum + v * xv;
    sum = ok ? t : sum;
  }
  return sum;
}

// general SELL slice (paired layout), continuing `sum`: batches of 8 entries
template <bool NT, class XS>
__device__ __forceinline__ double sell_slice(const int32_t *__restrict__ cbase, const double *__restrict__ vbase,
                                             int w, double sum, const XS &x, int lane) {
  const int np = w >> 1;
  const int2v *__restrict__ cp = reinterpret_cast<const int2v *>(cbase) + lane;
  const dbl2 *__restrict__ vp = reinterpret_cast<const dbl2 *>(vbase) + lane;
  for (int p0 = 0; p0 < np; p0 += 4) {
    int c[8];
    double v[8], xv[8];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int p = p0 + q;
      const int2v cc = p < np ? ld<NT>(cp + (int64_t)p * SLICE) : int2v{-1, -1};
      const dbl2 t = p < np ? ld<NT>(vp + (int64_t)p * SLICE) : dbl2{0.0, 0.0};
      c[2 * q] = cc.x; c[2 * q + 1] = cc.y;
      v[2 * q] = t.x; v[2 * q + 1] = t.y;
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) xv[q] = x(c[q] >= 0 ? c[q] : 0);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const double t = sum + v[q] * xv[q];
      sum = c[q] >= 0 ? t : sum;
    }
  }
  if (w & 1) {
    const int64_t t = (int64_t)np * 2 * SLICE + lane;
    const int c = ld<NT>(cbase + t);
    const double v = ld<NT>(vbase + t);
    const double xv = x(c >= 0 ? c : 0);
    const double tt = sum + v * xv;
    sum = c >= 0 ? tt : sum;
  }
  return sum;
}

// One wave sweeps slices; lane = row.  Grid-stride over a fixed grid whose
// blocks are grouped by XCD (block b runs on XCD b % 8 under the observed
// round-robin dispatch): each XCD walks one contiguous eighth of the slices in
// order, so the +-1 / +-n / +-n^2 re-reads of x stay in that XCD's 4 MB L2.
// Placement only affects speed, never results.  KD > 0 specialises the
// aligned-offset body for the matrix's dominant slice width.
template <int MODE, bool NT, int KD, bool SPLIT, int JM = 0>
__global__ void __launch_bounds__(256) spmv_sell_kernel(
    int64_t m, int64_t ncols, int64_t nslices, const int64_t *__restrict__ sptr_d,
    const int32_t *__restrict__ wid_d, const int32_t *__restrict__ col_d,
    const double *__restrict__ val_d, const int32_t *__restrict__ doff,
    const uint32_t *__restrict__ dmask, const uint8_t *__restrict__ dmask8, const int64_t *__restrict__ sptr_o,
    const int32_t *__restrict__ wid_o, const int32_t *__restrict__ col_o,
    const double *__restrict__ val_o, const double *__restrict__ x,
    const double *__restrict__ lvec, double *__restrict__ y, const Jac jac,
    double *__restrict__ partials, const int *__restrict__ done, const CgFuse cg, const Fold fold,
    const double *__restrict__ xscale) {
  CgTopIn top;
  if constexpr (MODE == SPMV_CG) top = cg.st->top;   // one batch of scalar loads, done included
  else if (done && *done) return;  // wave-uniform: solver finished, the launch is a no-op
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int s0, sstep, send;
  if ((gridDim.x & 7) == 0) {
    const int per = gridDim.x >> 3;                 // blocks per XCD group
    const int xcd = blockIdx.x & 7, j = blockIdx.x >> 3;
    const int chunk = (int)((nslices + 7) >> 3);
    s0 = xcd * chunk + j * SPMV_WAVES + wid;
    sstep = per * SPMV_WAVES;
    send = (int)min(nslices, (int64_t)(xcd + 1) * chunk);
  } else {
    s0 = blockIdx.x * SPMV_WAVES + wid;
    sstep = gridDim.x * SPMV_WAVES;
    send = (int)nslices;
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
  double dot = 0.0;
  for (int s = s0; s < send; s += sstep) {
    const int64_t row = (int64_t)s * SLICE + lane;
    const int w = wid_d[s];
    const int64_t base = sptr_d[s];
    // CG: the owned row's r, p_{i-1}, x (and dinv) are loaded with the
    // slice's first loads so their latency overlaps the gathers
    double own_r = 0.0, own_p = 0.0, own_x = 0.0, own_d = 0.0;
    if constexpr (MODE == SPMV_CG) {
      const int64_t rc = row < m ? row : 0;
      own_r = cg.r[rc];
      own_p = cg.pold[rc];
      own_x = cg.x[rc];
      if constexpr (JM == 1) own_d = cg.jac.d[rc];
    }
    double sum;
    if (w < 0) {
      const int k = -w;
      const uint32_t mk = dmask8 ? (uint32_t)dmask8[row] : dmask[row];
      const int32_t *__restrict__ off = doff + (int64_t)s * DIA_MAX;
      const int64_t srow = (int64_t)s * SLICE;
      int omin = off[0], omax = off[0];
      for (int j = 1; j < k; ++j) { omin = min(omin, off[j]); omax = max(omax, off[j]); }
      const bool inb = srow + omin >= 0 && srow + (SLICE - 1) + omax < ncols;
      if (KD > 0 && k == KD) sum = dia_slice_fixed<(KD > 0 ? KD : 1), NT>(val_d + base, off, mk, row, X, lane, inb, srow);
      else sum = dia_slice_any<NT>(val_d + base, off, k, mk, row, X, lane, inb, srow);
    } else {
      sum = sell_slice<NT>(col_d + base, val_d + base, w, 0.0, X, lane);
    }
    double xr = 0.0;   // operand at the owned row (DOT / CG)
    if constexpr (MODE == SPMV_CG) {
      double z = own_r;                         // same expression as XCg
      if constexpr (JM == 1) z = own_r * own_d;
      else if constexpr (JM == 2) z = own_r * cg.jac.c;
      xr = z + X.b * own_p;
      if (row < m) {
        cg.pnew[row] = xr;
        if (xpend) cg.x[row] = fma(xa, own_p, own_x);   // VecAXPY(X, a, P) of the previous step
      }
    }
    if (SPLIT) {
      // slice with ghost entries: store the diagonal-block sum; the boundary
      // kernel continues it with A_o once the halo has arrived
      if (wid_o[s]) {
        if (row < m) y[row] = sum;
        continue;
      }
    } else if (lvec) {
      const int wo = wid_o[s];
      if (wo) sum = sell_slice<false>(col_o + sptr_o[s], val_o + sptr_o[s], wo, sum, XPlainT<SC>{lvec, xs}, lane);
    }
    if (row < m) {
      if (spmv_jac(MODE)) y[row] = papply(jac, sum, row);   // PCApply_Jacobi fused: w_i * d_i
      else y[row] = sum;
      if (MODE == SPMV_DOT) dot += x[row] * sum;           // VecDot(p, w) partial, p = x
      if (MODE == SPMV_CG) dot += xr * sum;
    }
  }
  if (MODE == SPMV_DOT || MODE == SPMV_CG) {
    double v[1] = {dot};
    block_partials<1>(v, partials, gridDim.x, fold);
  }
}

// Grid of the main SpMV launch (an upper bound for every mode).  SPMV_CG
// evaluates the iteration's scalar top in every workgroup, a dependent chain
// of scalar loads paid once per workgroup generation, so it keeps >= 4 slices
// per wave (tools/coll_ab.py: -6% per CG iteration at 2M rows per rank).
int spmv_blocks(const Mat *A, int mode) {
  const int64_t need = cdiv(A->sd.nslices, SPMV_WAVES);
  int64_t g = std::min<int64_t>(need, g_knobs.spmv_grid);
  if (mode == SPMV_CG) g = std::min<int64_t>(g, std::max<int64_t>(2048, need / 4));
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
    sum = sell_slice<false>(col_o + sptr_o[s], val_o + sptr_o[s], wid_o[s], sum, XPlainT<SC>{lvec, xs}, lane);
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

static void launch_main(Mat *A, const double *x, double *y, int mode, Jac jac, double *partials,
                        int *done_flag, bool split, hipStream_t st, const CgFuse *cgp, const Fold &fold,
                        const double *xscale) {
  const unsigned grid = (unsigned)spmv_blocks(A, mode);
  const double *lvec = (A->nghost && !split) ? A->halo.lvec.p : nullptr;
  const int kd = A->sd.dia_k;
  const CgFuse cg = cgp ? *cgp : CgFuse{};
#define SPMV_ARGS                                                                           \
  A->m, A->n, A->sd.nslices, A->sd.sptr.p, A->sd.width.p, A->sd.col.p, A->sd.val.p, A->sd.doff.p, \
      A->sd.mask.p, A->sd.mask8.p, A->so.sptr.p, A->so.width.p, A->so.col.p, A->so.val.p, x, lvec, y, jac, \
      partials, done_flag, cg, fold, xscale
#define SPMV_KD(MODE, NT, SP)                                                                    \
  do {                                                                                           \
    switch (kd) {                                                                                \
      case 5: spmv_sell_kernel<MODE, NT, 5, SP><<<grid, 256, 0, st>>>(SPMV_ARGS); break;         \
      case 7: spmv_sell_kernel<MODE, NT, 7, SP><<<grid, 256, 0, st>>>(SPMV_ARGS); break;         \
      case 27: spmv_sell_kernel<MODE, NT, 27, SP><<<grid, 256, 0, st>>>(SPMV_ARGS); break;       \
      default: spmv_sell_kernel<MODE, NT, 0, SP><<<grid, 256, 0, st>>>(SPMV_ARGS); break;        \
    }                                                                                            \
  } while (0)
#define SPMV_CGKD(JM, SP)                                                                                   \
  do {                                                                                                      \
    switch (kd) {                                                                                           \
      case 5: spmv_sell_kernel<SPMV_CG, true, 5, SP, JM><<<grid, 256, 0, st>>>(SPMV_ARGS); break;           \
      case 7: spmv_sell_kernel<SPMV_CG, true, 7, SP, JM><<<grid, 256, 0, st>>>(SPMV_ARGS); break;           \
      case 27: spmv_sell_kernel<SPMV_CG, true, 27, SP, JM><<<grid, 256, 0, st>>>(SPMV_ARGS); break;         \
      default: spmv_sell_kernel<SPMV_CG, true, 0, SP, JM><<<grid, 256, 0, st>>>(SPMV_ARGS); break;          \
    }                                                                                                       \
  } while (0)
#define SPMV_GO(MODE)                                                         \
  do {                                                                        \
    if (split) { if (g_knobs.spmv_nt) SPMV_KD(MODE, true, true); else SPMV_KD(MODE, false, true); } \
    else { if (g_knobs.spmv_nt) SPMV_KD(MODE, true, false); else SPMV_KD(MODE, false, false); }     \
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
#undef SPMV_GO
#undef SPMV_CGKD
#undef SPMV_KD
#undef SPMV_ARGS
  HIPCHECK(hipGetLastError());
}

void spmv_launch(Mat *A, const double *x, double *y, int mode, Jac jac, double *partials,
                 int *done_flag) {
  launch_main(A, x, y, mode, jac, partials, done_flag, false, A->comm->stream, nullptr, Fold{}, nullptr);
}

constexpr int BND_BLOCKS = 2048;   // one boundary slice per wave: the launch runs after the interior, alone on the GPU

bool matmult_splits(const Mat *A) { return A->comm->size > 1 && A->halo.nbnd > 0 && g_knobs.overlap; }

int matmult_overlap(Mat *A, const double *x, double *y, int mode, Jac jac, double *partials,
                    int *done_flag, const CgFuse *cg, const Fold *fold, const double *xscale) {
  Comm *c = A->comm;
  Halo &H = A->halo;
  hipStream_t st = c->stream;
  const int nmain = spmv_blocks(A, mode);
  if (c->size == 1 || H.nbnd == 0 || !g_knobs.overlap) {
    if (c->size > 1) halo_exchange(A, x, mode == SPMV_CG ? cg : nullptr, done_flag, st);
    Fold f;
    if (fold) { f = *fold; f.ntotal = nmain; f.base = 0; f.ncount = nmain; }
    launch_main(A, x, y, mode, jac, partials, done_flag, false, st, cg, f, xscale);
    return nmain;
  }
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
  launch_main(A, x, y, mode, jac, partials, done_flag, true, st, cg, Fold{}, xscale);
  HIPCHECK(hipStreamWaitEvent(st, H.ev_done, 0));
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

}  // namespace mx
