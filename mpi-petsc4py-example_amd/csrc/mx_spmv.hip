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

// Every slice body below issues all of its loads before the first use, with
// predicated (never branching) lanes: absent entries gather the always-valid
// x[0] and are then skipped by a select, so the running sum sees exactly the
// present entries in ascending column order -- PETSc's order, bit for bit.

// aligned-offset slice with a compile-time width K (the stencil's point count)
template <int K, bool NT>
__device__ __forceinline__ double dia_slice_fixed(const double *__restrict__ vbase, const int32_t *__restrict__ off,
                                                  uint32_t mk, int64_t row, const double *__restrict__ x, int lane) {
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
#pragma unroll
  for (int j = 0; j < K; ++j) xv[j] = x[((mk >> j) & 1u) ? row + off[j] : 0];
  double sum = 0.0;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const double t = sum + v[j] * xv[j];
    sum = ((mk >> j) & 1u) ? t : sum;
  }
  return sum;
}

// aligned-offset slice, runtime width: batches of 8 slots
template <bool NT>
__device__ __forceinline__ double dia_slice_any(const double *__restrict__ vbase, const int32_t *__restrict__ off,
                                                int k, uint32_t mk, int64_t row, const double *__restrict__ x, int lane) {
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
      xv[q] = x[ok ? row + off[j < 2 * np ? j : 0] : 0];
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
    const double xv = x[ok ? row + off[k - 1] : 0];
    const double t = sum + v * xv;
    sum = ok ? t : sum;
  }
  return sum;
}

// general SELL slice (paired layout), continuing `sum`: batches of 8 entries
template <bool NT>
__device__ __forceinline__ double sell_slice(const int32_t *__restrict__ cbase, const double *__restrict__ vbase,
                                             int w, double sum, const double *__restrict__ x, int lane) {
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
    for (int q = 0; q < 8; ++q) xv[q] = x[c[q] >= 0 ? c[q] : 0];
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
    const double xv = x[c >= 0 ? c : 0];
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
template <int MODE, bool NT, int KD, bool SPLIT>
__global__ void __launch_bounds__(256) spmv_sell_kernel(
    int64_t m, int64_t nslices, const int64_t *__restrict__ sptr_d,
    const int32_t *__restrict__ wid_d, const int32_t *__restrict__ col_d,
    const double *__restrict__ val_d, const int32_t *__restrict__ doff,
    const uint32_t *__restrict__ dmask, const int64_t *__restrict__ sptr_o,
    const int32_t *__restrict__ wid_o, const int32_t *__restrict__ col_o,
    const double *__restrict__ val_o, const double *__restrict__ x,
    const double *__restrict__ lvec, double *__restrict__ y, const Jac jac,
    double *__restrict__ partials, const int *__restrict__ done) {
  if (done && *done) return;  // wave-uniform: solver finished, the launch is a no-op
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
  double dot = 0.0;
  for (int s = s0; s < send; s += sstep) {
    const int64_t row = (int64_t)s * SLICE + lane;
    const int w = wid_d[s];
    const int64_t base = sptr_d[s];
    double sum;
    if (w < 0) {
      const int k = -w;
      const uint32_t mk = dmask[row];
      const int32_t *__restrict__ off = doff + (int64_t)s * DIA_MAX;
      if (KD > 0 && k == KD) sum = dia_slice_fixed<(KD > 0 ? KD : 1), NT>(val_d + base, off, mk, row, x, lane);
      else sum = dia_slice_any<NT>(val_d + base, off, k, mk, row, x, lane);
    } else {
      sum = sell_slice<NT>(col_d + base, val_d + base, w, 0.0, x, lane);
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
      if (wo) sum = sell_slice<false>(col_o + sptr_o[s], val_o + sptr_o[s], wo, sum, lvec, lane);
    }
    if (row < m) {
      if (MODE == SPMV_JACOBI) y[row] = papply(jac, sum, row);   // PCApply_Jacobi fused: w_i * d_i
      else y[row] = sum;
      if (MODE == SPMV_DOT) dot += x[row] * sum;           // VecDot(p, w) partial, p = x
    }
  }
  if (MODE == SPMV_DOT) {
    double v[1] = {dot};
    block_sum_to_partials<1>(v, partials, gridDim.x);
  }
}

int spmv_blocks(const Mat *A) {
  const int64_t need = cdiv(A->sd.nslices, SPMV_WAVES);
  int64_t g = std::min<int64_t>(need, g_knobs.spmv_grid);
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
    double *__restrict__ partials, const int *__restrict__ done) {
  if (done && *done) return;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  double dot = 0.0;
  for (int k = blockIdx.x * SPMV_WAVES + wid; k < nlist; k += gridDim.x * SPMV_WAVES) {
    const int s = list[k];
    const int64_t row = (int64_t)s * SLICE + lane;
    double sum = row < m ? y[row] : 0.0;
    sum = sell_slice<false>(col_o + sptr_o[s], val_o + sptr_o[s], wid_o[s], sum, lvec, lane);
    if (row < m) {
      if (MODE == SPMV_JACOBI) y[row] = papply(jac, sum, row);
      else y[row] = sum;
      if (MODE == SPMV_DOT) dot += x[row] * sum;
    }
  }
  if (MODE == SPMV_DOT) {
    double v[1] = {dot};
    block_sum_to_partials<1>(v, partials, gridDim.x);
  }
}

__global__ void pack_kernel(int64_t n, const int32_t *__restrict__ idx, const double *__restrict__ x,
                            double *__restrict__ buf) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += stride) buf[k] = x[idx[k]];
}

// VecScatterBegin/End(x -> lvec): pack (only if some peer's rows are not a
// contiguous range), then one grouped send/recv with every neighbour.
void halo_begin(Mat *A, const double *x) {
  Halo &H = A->halo;
  if (A->comm->size == 1) return;
  hipStream_t st = A->comm->stream;
  if (H.need_pack && H.nsend) {
    pack_kernel<<<grid_for(H.nsend, 256, 4096), 256, 0, st>>>(H.nsend, H.send_idx.p, x, H.send_buf.p);
    HIPCHECK(hipGetLastError());
  }
  std::vector<Msg> sends, recvs;
  for (size_t i = 0; i < H.send_peer.size(); ++i) {
    void *buf = H.send_contig_start[i] >= 0 ? (void *)(x + H.send_contig_start[i])
                                            : (void *)(H.send_buf.p + H.send_off[i]);
    sends.push_back({H.send_peer[i], buf, sizeof(double) * (size_t)H.send_cnt[i]});
  }
  for (size_t i = 0; i < H.recv_peer.size(); ++i)
    recvs.push_back({H.recv_peer[i], H.lvec.p + H.recv_off[i], sizeof(double) * (size_t)H.recv_cnt[i]});
  A->comm->exchange(sends, recvs);
}

static void launch_main(Mat *A, const double *x, double *y, int mode, Jac jac, double *partials,
                        int *done_flag, bool split, hipStream_t st) {
  const unsigned grid = (unsigned)spmv_blocks(A);
  const double *lvec = (A->nghost && !split) ? A->halo.lvec.p : nullptr;
  const int kd = A->sd.dia_k;
#define SPMV_ARGS                                                                           \
  A->m, A->sd.nslices, A->sd.sptr.p, A->sd.width.p, A->sd.col.p, A->sd.val.p, A->sd.doff.p, \
      A->sd.mask.p, A->so.sptr.p, A->so.width.p, A->so.col.p, A->so.val.p, x, lvec, y, jac,   \
      partials, done_flag
#define SPMV_KD(MODE, NT, SP)                                                                    \
  do {                                                                                           \
    switch (kd) {                                                                                \
      case 5: spmv_sell_kernel<MODE, NT, 5, SP><<<grid, 256, 0, st>>>(SPMV_ARGS); break;         \
      case 7: spmv_sell_kernel<MODE, NT, 7, SP><<<grid, 256, 0, st>>>(SPMV_ARGS); break;         \
      case 27: spmv_sell_kernel<MODE, NT, 27, SP><<<grid, 256, 0, st>>>(SPMV_ARGS); break;       \
      default: spmv_sell_kernel<MODE, NT, 0, SP><<<grid, 256, 0, st>>>(SPMV_ARGS); break;        \
    }                                                                                            \
  } while (0)
#define SPMV_GO(MODE)                                                         \
  do {                                                                        \
    if (split) { if (g_knobs.spmv_nt) SPMV_KD(MODE, true, true); else SPMV_KD(MODE, false, true); } \
    else { if (g_knobs.spmv_nt) SPMV_KD(MODE, true, false); else SPMV_KD(MODE, false, false); }     \
  } while (0)
  switch (mode) {
    case SPMV_PLAIN: SPMV_GO(SPMV_PLAIN); break;
    case SPMV_JACOBI: SPMV_GO(SPMV_JACOBI); break;
    case SPMV_DOT: SPMV_GO(SPMV_DOT); break;
    default: fail(MX_ERR_INTERNAL, "bad spmv mode");
  }
#undef SPMV_GO
#undef SPMV_KD
#undef SPMV_ARGS
  HIPCHECK(hipGetLastError());
}

void spmv_launch(Mat *A, const double *x, double *y, int mode, Jac jac, double *partials,
                 int *done_flag) {
  launch_main(A, x, y, mode, jac, partials, done_flag, false, A->comm->stream);
}

constexpr int BND_BLOCKS = 64;

int matmult_overlap(Mat *A, const double *x, double *y, int mode, Jac jac, double *partials,
                    int *done_flag) {
  Comm *c = A->comm;
  Halo &H = A->halo;
  if (c->size == 1 || H.nbnd == 0 || !g_knobs.overlap) {
    halo_begin(A, x);
    launch_main(A, x, y, mode, jac, partials, done_flag, false, c->stream);
    return spmv_blocks(A);
  }
  hipStream_t st = c->stream, cs = c->comm_stream;
  if (!H.ev_x) {
    HIPCHECK(hipEventCreateWithFlags(&H.ev_x, hipEventDisableTiming));
    HIPCHECK(hipEventCreateWithFlags(&H.ev_done, hipEventDisableTiming));
  }
  // halo on the comm stream, after x is final on the compute stream
  HIPCHECK(hipEventRecord(H.ev_x, st));
  HIPCHECK(hipStreamWaitEvent(cs, H.ev_x, 0));
  if (H.need_pack && H.nsend) {
    pack_kernel<<<grid_for(H.nsend, 256, 4096), 256, 0, cs>>>(H.nsend, H.send_idx.p, x, H.send_buf.p);
    HIPCHECK(hipGetLastError());
  }
  std::vector<Msg> sends, recvs;
  for (size_t i = 0; i < H.send_peer.size(); ++i) {
    void *buf = H.send_contig_start[i] >= 0 ? (void *)(x + H.send_contig_start[i])
                                            : (void *)(H.send_buf.p + H.send_off[i]);
    sends.push_back({H.send_peer[i], buf, sizeof(double) * (size_t)H.send_cnt[i]});
  }
  for (size_t i = 0; i < H.recv_peer.size(); ++i)
    recvs.push_back({H.recv_peer[i], H.lvec.p + H.recv_off[i], sizeof(double) * (size_t)H.recv_cnt[i]});
  c->exchange(sends, recvs, cs);
  HIPCHECK(hipEventRecord(H.ev_done, cs));
  // interior slices meanwhile; boundary slices after the exchange
  const int nmain = spmv_blocks(A);
  launch_main(A, x, y, mode, jac, partials, done_flag, true, st);
  HIPCHECK(hipStreamWaitEvent(st, H.ev_done, 0));
  const int nb = std::min(BND_BLOCKS, (H.nbnd + SPMV_WAVES - 1) / SPMV_WAVES);
  double *pb = partials ? partials + nmain : nullptr;
#define BND(MODE) spmv_boundary_kernel<MODE><<<nb, 256, 0, st>>>(A->m, H.bnd_slices.p, H.nbnd, A->so.sptr.p, \
      A->so.width.p, A->so.col.p, A->so.val.p, x, H.lvec.p, y, jac, pb, done_flag)
  switch (mode) {
    case SPMV_PLAIN: BND(SPMV_PLAIN); break;
    case SPMV_JACOBI: BND(SPMV_JACOBI); break;
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
