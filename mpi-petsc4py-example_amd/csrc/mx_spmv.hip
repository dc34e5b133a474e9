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
#include "mx_device.hpp"
#include "mx_internal.hpp"

namespace mx {

constexpr int SPMV_WAVES = 4;  // 256-thread workgroups, one slice per wave

template <int MODE>
__global__ void __launch_bounds__(256) spmv_sell_kernel(
    int64_t m, int64_t nslices, const int64_t *__restrict__ sptr_d,
    const int32_t *__restrict__ wid_d, const int32_t *__restrict__ col_d,
    const double *__restrict__ val_d, const int64_t *__restrict__ sptr_o,
    const int32_t *__restrict__ wid_o, const int32_t *__restrict__ col_o,
    const double *__restrict__ val_o, const double *__restrict__ x,
    const double *__restrict__ lvec, double *__restrict__ y, const double *__restrict__ dinv,
    double *__restrict__ partials, const int *__restrict__ done) {
  if (done && *done) return;  // wave-uniform: solver finished, the launch is a no-op
  const int lane = threadIdx.x & 63;
  const int64_t s = (int64_t)blockIdx.x * SPMV_WAVES + (threadIdx.x >> 6);
  const int64_t row = s * SLICE + lane;
  double sum = 0.0;
  if (s < nslices) {
    const int w = wid_d[s];
    const int32_t *__restrict__ cp = col_d + sptr_d[s] + lane;
    const double *__restrict__ vp = val_d + sptr_d[s] + lane;
#pragma unroll 4
    for (int j = 0; j < w; ++j) {
      const int c = cp[(int64_t)j * SLICE];
      const double v = vp[(int64_t)j * SLICE];
      if (c >= 0) sum = sum + v * x[c];
    }
    if (lvec) {
      const int wo = wid_o[s];
      if (wo) {
        const int32_t *__restrict__ co = col_o + sptr_o[s] + lane;
        const double *__restrict__ vo = val_o + sptr_o[s] + lane;
        for (int j = 0; j < wo; ++j) {
          const int c = co[(int64_t)j * SLICE];
          const double v = vo[(int64_t)j * SLICE];
          if (c >= 0) sum = sum + v * lvec[c];
        }
      }
    }
  }
  if (MODE == SPMV_JACOBI) {
    if (row < m) y[row] = sum * dinv[row];      // PCApply_Jacobi fused: w_i * d_i
  } else {
    if (row < m) y[row] = sum;
  }
  if (MODE == SPMV_DOT) {                       // VecDot(p, w) partial, p = x
    double v[1] = {row < m ? x[row] * sum : 0.0};
    block_sum_to_partials<1>(v, partials, gridDim.x);
  }
}

int spmv_blocks(const Mat *A) { return (int)std::max<int64_t>(1, cdiv(A->sd.nslices, SPMV_WAVES)); }

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
#define SPMV_ARGS                                                                              \
  A->m, A->sd.nslices, A->sd.sptr.p, A->sd.width.p, A->sd.col.p, A->sd.val.p, A->so.sptr.p,   \
      A->so.width.p, A->so.col.p, A->so.val.p, x, lvec, y, dinv, partials, done_flag
  switch (mode) {
    case SPMV_PLAIN: spmv_sell_kernel<SPMV_PLAIN><<<grid, 256, 0, st>>>(SPMV_ARGS); break;
    case SPMV_JACOBI: spmv_sell_kernel<SPMV_JACOBI><<<grid, 256, 0, st>>>(SPMV_ARGS); break;
    case SPMV_DOT: spmv_sell_kernel<SPMV_DOT><<<grid, 256, 0, st>>>(SPMV_ARGS); break;
    default: fail(MX_ERR_INTERNAL, "bad spmv mode");
  }
#undef SPMV_ARGS
  HIPCHECK(hipGetLastError());
}

void mat_mult(Mat *A, const double *x, double *y) {
  halo_begin(A, x);
  spmv_launch(A, x, y, SPMV_PLAIN, nullptr, nullptr, nullptr);
}

}  // namespace mx
