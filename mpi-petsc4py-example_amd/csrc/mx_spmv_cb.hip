// mx_spmv_cb.hip -- the column-block two-pass MatMult for unstructured AIJ
// blocks (test.py:14's scipy.sparse.random family; MatMult_SeqAIJ order).
//
// The one-pass SELL kernel gathers x[c] once per entry.  On a matrix whose
// columns are spread over the whole vector (uniformly random patterns) every
// gather is an L2 miss that fetches a 64-B sector from the memory side, and
// the kernel runs at the rate of those misses: 2^24 rows x 7 take 1.99 ms,
// the gathers alone 1.87 ms (tools/gather_probe.hip).  Gathers that hit L2 run
// about 2.8x faster (x of 2 MB: 150 G gathers/s against 54 G).  So:
//
//   pass 1 (cb_prod_kernel): the entries in (column block, row, column)
//     order -- column blocks of 2^bs doubles of x (2 MB at 2^24 rows) --
//     each XCD walking every 8th block with all its workgroups, so the
//     block's piece of x is in that XCD's L2 while the values and column ids
//     stream in and the products p_k = a_k * x[c_k] stream out in that order;
//   pass 2 (cb_sum_kernel): the SELL-64 walk of the rows, summing each row's
//     products in ascending column order through perm (the slot's pass-1
//     position); a slice's products of one column block are contiguous in
//     pass-1 order, so a wave's reads touch a line or two per block instead
//     of one random sector per entry.  The diagonal entries stay out of pass
//     1: pass 2 forms a_ii * x_i from the diagonal and x, both coalesced.
//
// Every product is rounded once and every row is summed from 0.0 in
// ascending column order, one rounding per add: the bits of MatMult_SeqAIJ
// and of the one-pass kernel (tests/test_gpu_cb.py).  Built at assembly for
// general SELL diagonal blocks whose entries mostly lie far from the
// diagonal (build_cb, a counting placement: no sort); key 84 selects it.
#include "mx_device.hpp"
#include "mx_internal.hpp"

namespace mx {

namespace {
typedef double d2v __attribute__((ext_vector_type(2)));
typedef int i2v __attribute__((ext_vector_type(2)));
constexpr int CB_E = 4;   // pass 1: entries per thread per step (two 16-B value loads in flight)
constexpr int32_t CB_DIAG = -2;   // perm: the row's diagonal entry (its product formed in pass 2)

template <class T> __device__ __forceinline__ T ldnt(const T *p) { return __builtin_nontemporal_load(p); }

// -------------------------------------------------------------- build kernels
// far-entry count: |col - row| >= 2^17 (outside what one slice's L2 reuse
// can serve), summed per block
__global__ void __launch_bounds__(256) cb_far_kernel(int64_t m, const int64_t *__restrict__ ptr,
                                                     const int32_t *__restrict__ col, unsigned long long *far) {
  unsigned long long c = 0;
  for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < m; r += (int64_t)gridDim.x * 256)
    for (int64_t e = ptr[r]; e < ptr[r + 1]; ++e) {
      const int64_t d = (int64_t)col[e] - r;
      c += (d >= (1 << 17) || d <= -(1 << 17)) ? 1 : 0;
    }
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(far, c);
}

// Pass-1 order without a sort: entry e (CSR order) goes to
//   base[bin][R] + (entries of its bin in earlier rows of its 256-row group R)
//                + (its rank among the row's entries of that bin),
// base = the exclusive scan of the per-(bin, group) counts in bin-major
// order.  Columns ascend along a row, so a row's entries of one bin are
// consecutive, and the order within a bin is (row, column).  At most
// CB_MAXBLK bins (the block size grows past 2^18 columns to keep it).
constexpr int CB_MAXBLK = 64;
__global__ void __launch_bounds__(256) cb_count_kernel(int64_t m, const int64_t *__restrict__ ptr,
                                                       const int32_t *__restrict__ col, int64_t doff, int bs, int nblk,
                                                       int64_t ngrp, int64_t *__restrict__ cnt) {
  __shared__ unsigned c[CB_MAXBLK];
  for (int64_t R = blockIdx.x; R < ngrp; R += gridDim.x) {
    if (threadIdx.x < CB_MAXBLK) c[threadIdx.x] = 0;
    __syncthreads();
    const int64_t r = R * 256 + threadIdx.x;
    if (r < m)
      for (int64_t e = ptr[r]; e < ptr[r + 1]; ++e)
        if (col[e] != r + doff) atomicAdd(&c[(uint32_t)col[e] >> bs], 1u);
    __syncthreads();
    if (threadIdx.x < nblk) cnt[(int64_t)threadIdx.x * ngrp + R] = c[threadIdx.x];
    __syncthreads();
  }
}

__global__ void __launch_bounds__(256) cb_place_kernel(int64_t m, int64_t nnz, const int64_t *__restrict__ ptr,
                                                       const int32_t *__restrict__ col, const double *__restrict__ val,
                                                       int64_t doff, int bs, int nblk, int64_t ngrp,
                                                       const int64_t *__restrict__ base,
                                                       int32_t *__restrict__ c1, double *__restrict__ v1,
                                                       int32_t *__restrict__ pinv, int64_t *__restrict__ bstart) {
  __shared__ int pre[CB_MAXBLK][256];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  for (int64_t R = blockIdx.x; R < ngrp; R += gridDim.x) {
    for (int b = 0; b < nblk; ++b) pre[b][t] = 0;
    const int64_t r = R * 256 + t;
    const int64_t e0 = r < m ? ptr[r] : 0, e1 = r < m ? ptr[r + 1] : 0;
    for (int64_t e = e0; e < e1; ++e)
      if (col[e] != r + doff) pre[(uint32_t)col[e] >> bs][t] += 1;
    __syncthreads();
    // per bin, the exclusive prefix over the group's rows: wave wv takes bins
    // wv, wv + 4, ...; lane l the rows 4 l .. 4 l + 3
    for (int b = wv; b < nblk; b += 4) {
      const int a0 = pre[b][4 * lane], a1 = pre[b][4 * lane + 1], a2 = pre[b][4 * lane + 2], a3 = pre[b][4 * lane + 3];
      int incl = a0 + a1 + a2 + a3;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int u = __shfl_up(incl, o, 64);
        if (lane >= o) incl += u;
      }
      const int ex = incl - (a0 + a1 + a2 + a3);
      pre[b][4 * lane] = ex;
      pre[b][4 * lane + 1] = ex + a0;
      pre[b][4 * lane + 2] = ex + a0 + a1;
      pre[b][4 * lane + 3] = ex + a0 + a1 + a2;
    }
    __syncthreads();
    int pb = -1, k = 0;
    for (int64_t e = e0; e < e1; ++e) {
      if (col[e] == r + doff) { pinv[e] = CB_DIAG; continue; }   // the diagonal: pass 2 forms it
      const int b = (int)((uint32_t)col[e] >> bs);
      k = b == pb ? k + 1 : 0;
      pb = b;
      const int64_t pos = base[(int64_t)b * ngrp + R] + pre[b][t] + k;
      c1[pos] = col[e];
      v1[pos] = val[e];
      pinv[e] = (int32_t)pos;
    }
    if (R == 0 && t <= nblk) bstart[t] = t < nblk ? base[(int64_t)t * ngrp] : nnz;   // nnz: the pass-1 entries
    __syncthreads();
  }
}

// perm in the SELL-64 slot layout of A_d (Sell: pair p of lane l at sptr +
// 128 p + 2 l (+0/+1), the odd tail at sptr + 128 (w/2) + l); padding -1
__global__ void cb_perm_kernel(int64_t m, const int64_t *__restrict__ ptr, const int64_t *__restrict__ sptr,
                               const int32_t *__restrict__ wid, const int32_t *__restrict__ pinv,
                               int32_t *__restrict__ perm) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < m; r += (int64_t)gridDim.x * blockDim.x) {
    const int64_t s = r / SLICE;
    const int lane = (int)(r % SLICE);
    const int w = wid[s], np = w >> 1;
    const int64_t base = sptr[s];
    const int64_t e0 = ptr[r], len = ptr[r + 1] - e0;
    for (int j = 0; j < w; ++j) {
      const int64_t pos = j < 2 * np ? base + 128 * (j >> 1) + 2 * lane + (j & 1) : base + 128 * np + lane;
      perm[pos] = j < len ? pinv[e0 + j] : -1;
    }
  }
}

// -------------------------------------------------------------- pass 1
// block b of the grid runs on XCD b % 8 (round-robin dispatch: blocks b and
// b + 8 share an XCD; speed only, never results); that XCD's workgroups
// split each of its column blocks' entry ranges between them
template <bool SC>
__global__ void __launch_bounds__(256) cb_prod_kernel(int nblk, const int64_t *__restrict__ bstart,
                                                      const int32_t *__restrict__ c1, const double *__restrict__ v1,
                                                      const double *__restrict__ x, const double *__restrict__ xscale,
                                                      double *__restrict__ prod, const int *__restrict__ done) {
  if (done && *done) return;
  const double s = SC ? *xscale : 1.0;
  // the operand as the one-pass kernel forms it: x, or fl(s * x) (GMRES's
  // unnormalised basis vector), then one rounding for the product
  auto opnd = [&](int32_t c) { const double v = x[c]; return SC ? s * v : v; };
  const int xg = blockIdx.x & 7, wi = blockIdx.x >> 3, nper = gridDim.x >> 3;
  for (int C = xg; C < nblk; C += 8) {
    const int64_t b0 = bstart[C], b1 = bstart[C + 1], len = b1 - b0;
    const int64_t chunk = ((len + nper - 1) / nper + 1) & ~(int64_t)1;
    const int64_t lo = b0 + chunk * wi, hi = min(b1, lo + chunk);
    int64_t k = lo + 2 * threadIdx.x;
    for (; k + 512 * (CB_E / 2 - 1) + 1 < hi; k += 512 * (CB_E / 2)) {
      d2v v[CB_E / 2];
      i2v c[CB_E / 2];
#pragma unroll
      for (int e = 0; e < CB_E / 2; ++e) {
        v[e] = ldnt(reinterpret_cast<const d2v *>(v1 + k + 512 * e));
        c[e] = ldnt(reinterpret_cast<const i2v *>(c1 + k + 512 * e));
      }
      double xa[CB_E / 2], xb[CB_E / 2];
#pragma unroll
      for (int e = 0; e < CB_E / 2; ++e) { xa[e] = opnd(c[e].x); xb[e] = opnd(c[e].y); }
#pragma unroll
      for (int e = 0; e < CB_E / 2; ++e) {
        d2v p;
        p.x = v[e].x * xa[e];
        p.y = v[e].y * xb[e];
        __builtin_nontemporal_store(p, reinterpret_cast<d2v *>(prod + k + 512 * e));
      }
    }
    for (; k < hi; k += 512) {
      prod[k] = ldnt(v1 + k) * opnd(ldnt(c1 + k));
      if (k + 1 < hi) prod[k + 1] = ldnt(v1 + k + 1) * opnd(ldnt(c1 + k + 1));
    }
  }
}

// -------------------------------------------------------------- pass 2
// one wave per slice; the row's products in ascending column order (batches
// of 8 entries: every perm and product load of a batch in flight together),
// then the mode's epilogue as the one-pass kernel has it (mx_spmv.hip finish)
// SPLIT (P > 1 with ghost entries): a slice with A_o entries (wid_o) stores
// its rows' diagonal-block sums; the halo-boundary kernel continues them over
// A_o once the halo has arrived and applies the epilogue (mx_spmv.hip)
template <int MODE, bool SC, bool SPLIT>
__global__ void __launch_bounds__(256) cb_sum_kernel(int64_t m, int64_t nslices, const int64_t *__restrict__ sptr,
                                                     const int32_t *__restrict__ wid, const int32_t *__restrict__ wid_o,
                                                     const int32_t *__restrict__ perm,
                                                     const double *__restrict__ prod, const double *__restrict__ x,
                                                     const double *__restrict__ diag, int64_t doff,
                                                     const double *__restrict__ xscale, double *__restrict__ y,
                                                     const Jac jac, double *__restrict__ partials,
                                                     const int *__restrict__ done, const Fold fold) {
  if (done && *done) return;
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const double xs = SC ? *xscale : 1.0;
  double dot = 0.0;
  for (int64_t s = (int64_t)blockIdx.x * 4 + wv; s < nslices; s += (int64_t)gridDim.x * 4) {
    // the diagonal entry's product (CB_DIAG in perm): a_ii * x_i from the
    // diagonal and x itself, coalesced, instead of through pass 1 -- the
    // same single rounding (of the scaled operand first, as pass 1 has it)
    const int64_t rd = min(s * SLICE + lane, m - 1);
    const double xd = x[rd + doff];
    const double dprod = diag[rd] * (SC ? xs * xd : xd);
    const int w = wid[s];
    const int np = w >> 1;
    const bool odd = (w & 1) != 0;
    const int nb = np + (odd ? 1 : 0);
    const int32_t *__restrict__ pb = perm + sptr[s];
    const i2v *__restrict__ pp = reinterpret_cast<const i2v *>(pb) + lane;
    double sum = 0.0;
    for (int p0 = 0; p0 < nb; p0 += 4) {
      int c[8];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int p = p0 + q;
        i2v cc = i2v{-1, -1};
        if (p < np) cc = ldnt(pp + (int64_t)p * SLICE);
        else if (odd && p == np) cc.x = ldnt(pb + (int64_t)np * 2 * SLICE + lane);
        c[2 * q] = cc.x;
        c[2 * q + 1] = cc.y;
      }
      double t[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) t[q] = prod[c[q] >= 0 ? c[q] : 0];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const double u = sum + (c[q] == CB_DIAG ? dprod : t[q]);
        sum = (c[q] >= 0 || c[q] == CB_DIAG) ? u : sum;
      }
    }
    const int64_t row = s * SLICE + lane;
    if (SPLIT && wid_o[s]) {
      if (row < m) y[row] = sum;
      continue;
    }
    if (row < m) {
      const double out = spmv_jac(MODE) ? papply(jac, sum, row) : sum;   // PCApply_Jacobi fused: w_i * d_i
      y[row] = out;
      if (MODE == SPMV_DOT) dot += x[row] * sum;                          // VecDot(p, w) partial, p = x (SC: never)
    }
  }
  if constexpr (MODE == SPMV_DOT) {
    double v[1] = {dot};
    block_partials<1>(v, partials, gridDim.x, fold);
  }
}
}  // namespace

// one rank, or P > 1 when the product splits (the boundary kernel finishes
// the rows with ghost entries); the inline A_o continuation stays with the
// one-pass kernel
bool cb_applies(const Mat *A, int mode, bool split) {
  return A->sd.cb_nblk > 0 && g_knobs.cb != 0 && (split || A->nghost == 0) &&
         (mode == SPMV_PLAIN || mode == SPMV_PLAIN_S || mode == SPMV_JACOBI || mode == SPMV_JACOBI_S ||
          mode == SPMV_DOT);
}

int cb_launch(Mat *A, int mode, bool split, const double *x, double *y, const Jac &jac, double *partials,
              const int *done, const Fold &fold_in, const double *xscale, hipStream_t st) {
  Sell &S = A->sd;
  const unsigned g1 = (unsigned)(2 * device_cu_count()) & ~7u;   // two workgroups per CU, a multiple of 8
  const bool sc = spmv_scaled(mode);
  // (plain launches: a dispatch-attached timer, g_ext_timing, would time one
  // of the two passes; callers' events around the MatMult time both)
  if (sc) cb_prod_kernel<true><<<g1, 256, 0, st>>>(S.cb_nblk, S.cb_bstart.p, S.cb_col.p, S.cb_val.p, x, xscale,
                                                   S.cb_prod.p, done);
  else cb_prod_kernel<false><<<g1, 256, 0, st>>>(S.cb_nblk, S.cb_bstart.p, S.cb_col.p, S.cb_val.p, x, xscale,
                                                   S.cb_prod.p, done);
  HIPCHECK(hipGetLastError());
  const int g2 = (int)std::min<int64_t>(8192, std::max<int64_t>(1, cdiv(S.nslices, 4)));
  Fold fold = fold_in;
  if (fold.cnt) { fold.ntotal = fold.ncount = g2; fold.base = 0; }
  note_dispatch(DSP_CB);
  const int64_t doff = A->rstart - A->cstart;   // A_d's column of row r's diagonal: r + doff
#define CBS2(MD, SCL, SPL) cb_sum_kernel<MD, SCL, SPL><<<g2, 256, 0, st>>>(A->m, S.nslices, S.sptr.p, S.width.p, \
      A->so.width.p, S.cb_perm.p, S.cb_prod.p, x, A->diag.p, doff, xscale, y, jac, partials, done, fold)
#define CBS(MD, SCL) do { if (split) CBS2(MD, SCL, true); else CBS2(MD, SCL, false); } while (0)
  switch (mode) {
    case SPMV_PLAIN: CBS(SPMV_PLAIN, false); break;
    case SPMV_PLAIN_S: CBS(SPMV_PLAIN, true); break;
    case SPMV_JACOBI: CBS(SPMV_JACOBI, false); break;
    case SPMV_JACOBI_S: CBS(SPMV_JACOBI, true); break;
    case SPMV_DOT: CBS(SPMV_DOT, false); break;
    default: fail(MX_ERR_INTERNAL, "column-block MatMult: unsupported mode");
  }
#undef CBS
#undef CBS2
  HIPCHECK(hipGetLastError());
  return g2;
}

// Build the pass-1 arrays and perm for A_d when it is a general SELL block
// whose entries mostly lie far from the diagonal (key 84: 1 = that test and
// at least 2^20 rows, 2 = any general block -- tests; 0 = never).
void build_cb(Mat *A, hipStream_t st) {
  Sell &S = A->sd;
  S.cb_nblk = 0;
  const int64_t m = A->m, nnz = A->nnz_d;
  if (!g_knobs.cb || m < 64 || nnz < 1 || S.dia_slices != 0 || S.ntab != 0 || S.pair_shape != 0 ||
      nnz >= ((int64_t)1 << 31))
    return;
  if (g_knobs.cb == 1) {
    if (m < ((int64_t)1 << 20)) return;
    DBuf<unsigned long long> far(1);
    HIPCHECK(hipMemsetAsync(far.p, 0, sizeof(unsigned long long), st));
    cb_far_kernel<<<grid_for(m, 256, 4096), 256, 0, st>>>(m, A->dptr.p, A->dcol.p, far.p);
    HIPCHECK(hipGetLastError());
    unsigned long long h = 0;
    HIPCHECK(hipMemcpyAsync(&h, far.p, sizeof(h), hipMemcpyDeviceToHost, st));
    HIPCHECK(hipStreamSynchronize(st));
    if (h * 2 < (unsigned long long)nnz) return;   // half the entries or more far from the diagonal
  }
  // column blocks: 2 MB of x (2^18 doubles) from 2^22 columns; fewer columns
  // per block below, so that every XCD gets at least two, and more above
  // 2^24 columns (at most CB_MAXBLK blocks)
  int bs = 18;
  while (bs > 6 && (A->n >> bs) < 16) --bs;
  while (((A->n + ((int64_t)1 << bs) - 1) >> bs) > CB_MAXBLK) ++bs;
  const int nblk = (int)((A->n + ((int64_t)1 << bs) - 1) >> bs);
  const int64_t ngrp = cdiv(m, 256);
  DBuf<int64_t> cnt((size_t)nblk * (size_t)ngrp, kScratch);
  DBuf<int32_t> pinv((size_t)nnz, kScratch);
  const int64_t doff = A->rstart - A->cstart;
  cb_count_kernel<<<(unsigned)std::min<int64_t>(ngrp, 16384), 256, 0, st>>>(m, A->dptr.p, A->dcol.p, doff, bs, nblk,
                                                                          ngrp, cnt.p);
  HIPCHECK(hipGetLastError());
  int64_t nnz1 = 0;   // the off-diagonal entries (pass 1)
  exclusive_scan_i64(cnt.p, cnt.p, (int64_t)nblk * ngrp, st, &nnz1);
  S.cb_col.alloc((size_t)nnz);
  S.cb_val.alloc((size_t)nnz);
  S.cb_prod.alloc((size_t)nnz);
  S.cb_bstart.alloc((size_t)nblk + 1);
  S.cb_perm.alloc((size_t)std::max<int64_t>(S.slots, 1));
  cb_place_kernel<<<(unsigned)std::min<int64_t>(ngrp, 16384), 256, 0, st>>>(m, nnz1, A->dptr.p, A->dcol.p, A->dval.p,
                                                                          doff, bs, nblk, ngrp, cnt.p, S.cb_col.p,
                                                                          S.cb_val.p, pinv.p, S.cb_bstart.p);
  HIPCHECK(hipGetLastError());
  HIPCHECK(hipMemsetAsync(S.cb_perm.p, 0xFF, sizeof(int32_t) * (size_t)std::max<int64_t>(S.slots, 1), st));
  cb_perm_kernel<<<grid_for(m, 256, 8192), 256, 0, st>>>(m, A->dptr.p, S.sptr.p, S.width.p, pinv.p, S.cb_perm.p);
  HIPCHECK(hipGetLastError());
  HIPCHECK(hipStreamSynchronize(st));   // the scratch arrays are freed on return
  S.cb_bs = bs;
  S.cb_nblk = nblk;
}

void load_code_spmv_cb() {
  hipFuncAttributes a;
  (void)hipFuncGetAttributes(&a, reinterpret_cast<const void *>(&cb_sum_kernel<SPMV_PLAIN, false, false>));
  (void)hipGetLastError();
}

}  // namespace mx
