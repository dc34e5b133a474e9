// mx_spmv_pair.hip -- the lean row-pair MatMult for constant-coefficient
// 5/7-point blocks (uniform-slot dictionaries, Sell::puni).
//
// Replaces the same MatMult_MPIAIJ diagonal-block product as the general SELL
// kernel (mx_spmv.hip spmv_sell_kernel<..., PS, UNI = true>; reached from
// ksp.solve at test.py:50 and from MatMult), for the matrices whose every
// 128-row unit is a row-pair unit with a uniform-slot dictionary block.  The
// general kernel carries the whole SELL argument list and its fallback bodies
// (non-pair slices, A_o continuation, CG-fused operands), and spends SGPRs --
// spilled to VGPR lanes -- and a scalar metadata pipeline on them; this one
// takes one small argument block and does only the pair body:
//   * block ids for the wave's next 64 units in one vector load, read per
//     unit by readlane (no dependent scalar load per step);
//   * per unit: one 16-byte operand load per run, one edge load, the block's
//     2K slot-row values by scalar loads, one 16-byte store;
//   * CLEAN (every block select-free, Sell::pair_clean): each absent slot's
//     operand is made exactly 0.0 by an out-of-range buffer read -- a run
//     empty for both rows (PBLK_RUN0 << r), the tri run's edge value where
//     lane 0 row 0 lacks -1 (PBLK_ELO) or lane 63 row 1 lacks +1 (PBLK_EHI) --
//     and its slot-row value is the uniform value (0 for empty rows).  A row
//     sum that starts at +0.0 is never -0.0, so sum + v * 0.0 == sum bit for
//     bit: the same result as skipping the slot, with no presence select;
//   * !CLEAN: the lane masks as select conditions (the general UNI body).
// Each row still sums its entries in ascending column order, one rounding per
// multiply and add (PETSc's MatMult_SeqAIJ), so the product is bitwise equal
// to the general kernel's and to the oracle's (tests/test_gpu_vcodes.py).
#include "mx_device.hpp"
#include "mx_internal.hpp"
#include "mx_pair.hpp"

namespace mx {

// element offset added to an absent read: with n <= 2^27 rows every
// redirected byte offset lies in [2^30, 2^32) -- past the vector, unwrapped
constexpr int PAIR_OOR = 1 << 28;
constexpr int64_t PAIR_CLEAN_MAX_ROWS = int64_t(1) << 27;
constexpr int LEAN_WAVES = 4;

struct PairLeanArgs {
  int m, n, nunits;            // rows, operand length, 128-row units (m = 128 nunits)
  int anchor[5];               // per run: the singleton offset, or the tri run's centre
  double *partials;            // SPMV_DOT: one p.y partial per workgroup
  const int *done;             // solver stop flag (the launch is then a no-op)
  Fold fold;
};

// The vectors and tables are __restrict__ kernel arguments: the block's slot
// values then compile to scalar loads (a pointer inside the by-value struct
// is not known unclobbered, and the values went through vector loads).
template <int MODE, int PS, bool SPLIT, bool CLEAN>
__global__ void __launch_bounds__(256) spmv_pair_lean_kernel(const PairLeanArgs a, const double *__restrict__ x,
                                                             double *__restrict__ y,
                                                             const int32_t *__restrict__ pblk,
                                                             const PairUni *__restrict__ puni) {
  if (a.done && *a.done) return;   // wave-uniform: solver finished
  using SH = PairShape<PS>;
  constexpr int K = SH::K, NR = SH::NR, C = SH::CENTER_RUN;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // the general kernel's XCD-grouped sweep: each XCD walks one contiguous
  // eighth of the units, its waves interleaved (the +-n / +-n^2 re-reads of x
  // stay in that XCD's L2)
  int s0, sstep, send;
  if ((gridDim.x & 7) == 0) {
    const int per = gridDim.x >> 3, xcd = blockIdx.x & 7, j = blockIdx.x >> 3;
    const int chunk = (a.nunits + 7) >> 3;
    s0 = xcd * chunk + j * LEAN_WAVES + wid;
    sstep = per * LEAN_WAVES;
    send = min(a.nunits, (xcd + 1) * chunk);
  } else {
    s0 = blockIdx.x * LEAN_WAVES + wid;
    sstep = gridDim.x * LEAN_WAVES;
    send = a.nunits;
  }
  const __amdgpu_buffer_rsrc_t xr = vec_rsrc(x, a.n);
  constexpr int TR = PS == 5 ? 1 : 2;                       // the tri run
  // the tri run's edge values in one load: lane 0 reads x[ub + c - 1] (its
  // row 0's left neighbour), the others x[ub + 128 + c] (lane 63's row 1's
  // right neighbour; one line for the wave)
  const int ecst = lane == 0 ? a.anchor[TR] - 1 : 128 + a.anchor[TR];
  double dot = 0.0;
  struct Unit { dbl2 L[NR]; double e; uint32_t bw; };
  auto load = [&](int u, uint32_t bw, Unit &t) __attribute__((always_inline)) {
    const int ub = u * 128, r0 = ub + 2 * lane;
#pragma unroll
    for (int r = 0; r < NR; ++r)
      t.L[r] = bload2(xr, r0 + a.anchor[r] + (CLEAN && (bw & (PBLK_RUN0 << r)) ? PAIR_OOR : 0));
    int eo = ecst;
    if constexpr (CLEAN) eo += lane == 0 ? ((bw & PBLK_ELO) ? PAIR_OOR : 0) : ((bw & PBLK_EHI) ? PAIR_OOR : 0);
    t.e = bload1(xr, ub + eo);
    t.bw = bw;
  };
  auto finish = [&](int u, const Unit &t) __attribute__((always_inline)) {
    const int r0 = u * 128 + 2 * lane;
    const PairUni &B = puni[t.bw & PBLK_ID];              // wave-uniform: scalar loads
    double s0v = 0.0, s1v = 0.0, lo = 0.0, hi = 0.0;
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const int r = SH::run(j), p = SH::pos(j);
      if (SH::tri(r) && p < 0) {
        lo = wave_shift<true>(t.L[r].y, t.e);    // x[r0 + c - 1] = lane - 1's x[r0' + c + 1]
        hi = wave_shift<false>(t.L[r].x, t.e);   // x[r0 + c + 2] = lane + 1's x[r0' + c]
      }
      double a0, a1;
      if (!SH::tri(r)) { a0 = t.L[r].x; a1 = t.L[r].y; }
      else if (p < 0) { a0 = lo; a1 = t.L[r].x; }
      else if (p == 0) { a0 = t.L[r].x; a1 = t.L[r].y; }
      else { a0 = t.L[r].y; a1 = hi; }
      const double q0 = s0v + B.v[j] * a0, q1 = s1v + B.v[K + j] * a1;
      if constexpr (CLEAN) {
        s0v = q0;
        s1v = q1;
      } else {
        s0v = __builtin_amdgcn_inverse_ballot_w64(B.pm[j]) ? q0 : s0v;
        s1v = __builtin_amdgcn_inverse_ballot_w64(B.pm[K + j]) ? q1 : s1v;
      }
    }
    *reinterpret_cast<dbl2 *>(y + r0) = dbl2{s0v, s1v};
    if constexpr (MODE == SPMV_DOT) {
      // SPLIT: rows with A_o entries stored their diagonal-block sum; the
      // boundary kernel continues them and adds their p.y terms
      const bool gh = SPLIT && (t.bw & (lane < 32 ? PBLK_GHOST_LO : PBLK_GHOST_HI)) != 0;
      if (!gh) {
        dot += t.L[C].x * s0v;
        dot += t.L[C].y * s1v;
      }
    }
  };
  // two units per wave step, both units' loads in flight before the first
  // product; block words of the next 64 units in one vector load
  int u = s0, k = 64;
  int bv = 0;
  for (; u + sstep < send; u += 2 * sstep) {
    if (k + 2 > 64) {
      const int uu = u + lane * sstep;
      bv = uu < send ? pblk[uu] : 0;
      k = 0;
    }
    Unit ta, tb;
    load(u, (uint32_t)__builtin_amdgcn_readlane(bv, k), ta);
    load(u + sstep, (uint32_t)__builtin_amdgcn_readlane(bv, k + 1), tb);
    k += 2;
    __builtin_amdgcn_sched_barrier(0);
    finish(u, ta);
    finish(u + sstep, tb);
  }
  if (u < send) {
    Unit t;
    load(u, (uint32_t)pblk[u], t);
    finish(u, t);
  }
  if constexpr (MODE == SPMV_DOT) {
    double v[1] = {dot};
    block_partials<1>(v, a.partials, gridDim.x, a.fold);
  }
}

using LeanFn = void (*)(PairLeanArgs, const double *, double *, const int32_t *, const PairUni *);

// the lean kernel for this product, or null (the general kernel then runs)
// the layout side of the choice (mode and split aside): 0 none, 1 lean, 2 lean select-free
int pair_lean_kind(const Mat *A) {
  const Sell &S = A->sd;
  if (!g_knobs.pair_lean || !g_knobs.vcodes || !g_knobs.spmv_pairs || !g_knobs.pair_uni || g_knobs.spmv_ynt ||
      g_knobs.spmv_rev)
    return 0;
  if (S.ntab <= 0 || (S.pair_shape != 5 && S.pair_shape != 7) || !S.puni.p || S.pair_blocks <= 0 || !S.pair_all)
    return 0;
  if (A->m % 128 != 0 || A->m >= PAIR_MAX_ROWS || A->n >= PAIR_MAX_ROWS || S.nunits * 128 != A->m) return 0;
  return S.pair_clean && A->m <= PAIR_CLEAN_MAX_ROWS && A->n <= PAIR_CLEAN_MAX_ROWS ? 2 : 1;
}

const void *pair_lean_select(const Mat *A, int mode, bool split) {
  const Sell &S = A->sd;
  if (mode != SPMV_PLAIN && mode != SPMV_DOT) return nullptr;
  const int kind = pair_lean_kind(A);
  if (!kind) return nullptr;
  if (!split && (A->nghost > 0 || S.pair_ghosts)) return nullptr;   // A_o continues in the general kernel
  const bool clean = kind == 2;
  LeanFn f = nullptr;
#define LEAN_PICK(MODE, PS)                                                              \
  do {                                                                                   \
    if (split) f = clean ? &spmv_pair_lean_kernel<MODE, PS, true, true> : &spmv_pair_lean_kernel<MODE, PS, true, false>; \
    else f = clean ? &spmv_pair_lean_kernel<MODE, PS, false, true> : &spmv_pair_lean_kernel<MODE, PS, false, false>;      \
  } while (0)
  if (mode == SPMV_PLAIN) { if (S.pair_shape == 5) LEAN_PICK(SPMV_PLAIN, 5); else LEAN_PICK(SPMV_PLAIN, 7); }
  else { if (S.pair_shape == 5) LEAN_PICK(SPMV_DOT, 5); else LEAN_PICK(SPMV_DOT, 7); }
#undef LEAN_PICK
  return reinterpret_cast<const void *>(f);
}

void pair_lean_run(const Mat *A, const void *kf, int grid, const double *x, double *y, double *partials,
                   const int *done, const Fold &fold, hipStream_t st) {
  const Sell &S = A->sd;
  PairLeanArgs a{};
  a.m = (int)A->m;
  a.n = (int)A->n;
  a.nunits = (int)S.nunits;
  const int ps = S.pair_shape;
  for (int r = 0; r < 5; ++r) {
    // run r's anchor: the singleton's offset, or the tri run's centre slot
    const bool tri = ps == 5 ? r == 1 : r == 2;
    const int first = ps == 5 ? (r == 0 ? 0 : r == 1 ? 1 : 4) : (r < 2 ? r : r == 2 ? 2 : r + 2);
    a.anchor[r] = (ps == 5 && r >= 3) ? 0 : S.pat_star_off[(size_t)(first + (tri ? 1 : 0))];
  }
  a.partials = partials;
  a.done = done;
  a.fold = fold;
  reinterpret_cast<LeanFn>(const_cast<void *>(kf))<<<grid, 256, 0, st>>>(a, x, y, S.pblk.p, S.puni.p);
  HIPCHECK(hipGetLastError());
}

}  // namespace mx
