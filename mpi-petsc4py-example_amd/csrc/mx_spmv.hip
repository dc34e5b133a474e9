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

// One wave sweeps slices; lane = row.  Grid-stride over a fixed grid whose
// blocks are grouped by XCD (block b runs on XCD b % 8 under the observed
// round-robin dispatch): each XCD walks one contiguous eighth of the slices in
// order, so the +-1 / +-n / +-n^2 re-reads of x stay in that XCD's 4 MB L2.
// Placement only affects speed, never results.
template <int MODE, bool NT, bool PAIRED>
__global__ void __launch_bounds__(256) spmv_sell_kernel(
    int64_t m, int64_t nslices, const int64_t *__restrict__ sptr_d,
    const int32_t *__restrict__ wid_d, const int32_t *__restrict__ col_d,
    const double *__restrict__ val_d, const int64_t *__restrict__ sptr_o,
    const int32_t *__restrict__ wid_o, const int32_t *__restrict__ col_o,
    const double *__restrict__ val_o, const double *__restrict__ x,
    const double *__restrict__ lvec, double *__restrict__ y, const double *__restrict__ dinv,
    double *__restrict__ partials, const int *__restrict__ done) {
  if (done && *done) return;  // wave-uniform: solver finished, the launch is a no-op
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int64_t s0, sstep, send;
  if ((gridDim.x & 7) == 0) {
    const int64_t per = gridDim.x >> 3;                 // blocks per XCD group
    const int64_t xcd = blockIdx.x & 7, j = blockIdx.x >> 3;
    const int64_t chunk = (nslices + 7) >> 3;
    s0 = xcd * chunk + j * SPMV_WAVES + wid;
    sstep = per * SPMV_WAVES;
    send = min(nslices, (xcd + 1) * chunk);
  } else {
    s0 = (int64_t)blockIdx.x * SPMV_WAVES + wid;
    sstep = (int64_t)gridDim.x * SPMV_WAVES;
    send = nslices;
  }
  double dot = 0.0;
  for (int64_t s = s0; s < send; s += sstep) {
    const int64_t row = s * SLICE + lane;
    double sum = 0.0;
    const int w = wid_d[s];
    const int64_t base = sptr_d[s];
    if (PAIRED) {
      const int np = w >> 1;
      const int2v *__restrict__ cp = reinterpret_cast<const int2v *>(col_d + base) + lane;
      const dbl2 *__restrict__ vp = reinterpret_cast<const dbl2 *>(val_d + base) + lane;
#pragma unroll 2
      for (int p = 0; p < np; ++p) {
        const int2v c = ld<NT>(cp + (int64_t)p * SLICE);
        const dbl2 v = ld<NT>(vp + (int64_t)p * SLICE);
        if (c.x >= 0) sum = sum + v.x * x[c.x];
        if (c.y >= 0) sum = sum + v.y * x[c.y];
      }
      if (w & 1) {
        const int64_t t = base + (int64_t)np * 2 * SLICE + lane;
        const int c = ld<NT>(col_d + t);
        const double v = ld<NT>(val_d + t);
        if (c >= 0) sum = sum + v * x[c];
      }
    } else {
      const int32_t *__restrict__ cp = col_d + base + lane;
      const double *__restrict__ vp = val_d + base + lane;
#pragma unroll 4
      for (int j = 0; j < w; ++j) {
        const int c = ld<NT>(cp + (int64_t)j * SLICE);
        const double v = ld<NT>(vp + (int64_t)j * SLICE);
        if (c >= 0) sum = sum + v * x[c];
      }
    }
    if (lvec) {
      const int wo = wid_o[s];
      if (wo) {   // ghost block: rare, plain sequential continuation of the row sum
        const int64_t bo = sptr_o[s];
        for (int j = 0; j < wo; ++j) {
          int64_t t;
          if (PAIRED) t = bo + ((j >> 1) < (wo >> 1) ? (int64_t)(j >> 1) * 2 * SLICE + 2 * lane + (j & 1)
                                                     : (int64_t)(wo >> 1) * 2 * SLICE + lane);
          else t = bo + (int64_t)j * SLICE + lane;
          const int c = col_o[t];
          const double v = val_o[t];
          if (c >= 0) sum = sum + v * lvec[c];
        }
      }
    }
    if (row < m) {
      if (MODE == SPMV_JACOBI) y[row] = sum * dinv[row];   // PCApply_Jacobi fused: w_i * d_i
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

void spmv_launch(Mat *A, const double *x, double *y, int mode, const double *dinv,
                 double *partials, int *done_flag) {
  hipStream_t st = A->comm->stream;
  const unsigned grid = (unsigned)spmv_blocks(A);
  const double *lvec = A->nghost ? A->halo.lvec.p : nullptr;
  const bool plain = g_knobs.spmv_plain && A->sd.col_plain.p;
  const int32_t *cd = plain ? A->sd.col_plain.p : A->sd.col.p;
  const double *vd = plain ? A->sd.val_plain.p : A->sd.val.p;
  const int32_t *co = plain ? A->so.col_plain.p : A->so.col.p;
  const double *vo = plain ? A->so.val_plain.p : A->so.val.p;
  if (plain && A->nghost && !co) fail(MX_ERR_INTERNAL, "plain SELL copy missing");
#define SPMV_ARGS                                                                        \
  A->m, A->sd.nslices, A->sd.sptr.p, A->sd.width.p, cd, vd, A->so.sptr.p, A->so.width.p, \
      co, vo, x, lvec, y, dinv, partials, done_flag
#define SPMV_GO(MODE)                                                                           \
  do {                                                                                          \
    if (plain) {                                                                                \
      if (g_knobs.spmv_nt) spmv_sell_kernel<MODE, true, false><<<grid, 256, 0, st>>>(SPMV_ARGS);  \
      else spmv_sell_kernel<MODE, false, false><<<grid, 256, 0, st>>>(SPMV_ARGS);                 \
    } else {                                                                                    \
      if (g_knobs.spmv_nt) spmv_sell_kernel<MODE, true, true><<<grid, 256, 0, st>>>(SPMV_ARGS);   \
      else spmv_sell_kernel<MODE, false, true><<<grid, 256, 0, st>>>(SPMV_ARGS);                  \
    }                                                                                           \
  } while (0)
  switch (mode) {
    case SPMV_PLAIN: SPMV_GO(SPMV_PLAIN); break;
    case SPMV_JACOBI: SPMV_GO(SPMV_JACOBI); break;
    case SPMV_DOT: SPMV_GO(SPMV_DOT); break;
    default: fail(MX_ERR_INTERNAL, "bad spmv mode");
  }
#undef SPMV_GO
#undef SPMV_ARGS
  HIPCHECK(hipGetLastError());
}

void mat_mult(Mat *A, const double *x, double *y) {
  halo_begin(A, x);
  spmv_launch(A, x, y, SPMV_PLAIN, nullptr, nullptr, nullptr);
}

}  // namespace mx
