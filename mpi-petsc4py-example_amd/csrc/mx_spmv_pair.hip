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
//   * !CLEAN: the lane masks as select conditions (the general UNI body);
//   * z-march (spmv_pair_zm_kernel, the default where the pattern's outermost
//     runs are +-D with D a multiple of 128 rows -- the 3D planes, the 2D
//     lines): a wave owns a column of units one plane (D rows) apart and
//     marches it, carrying the -D and centre pairs in registers, so a unit
//     loads 3 operand pairs and its edge instead of 5 and its edge; the
//     ceiling probe's matrix-free form of it runs at the copy rate
//     (tools/stencil_probe.hip pzm_kernel).
// Each row still sums its entries in ascending column order, one rounding per
// multiply and add (PETSc's MatMult_SeqAIJ), so the product is bitwise equal
// to the general kernel's and to the oracle's (tests/test_gpu_vcodes.py).
#include "mx_cg.hpp"
#include "mx_device.hpp"
#include "mx_internal.hpp"
#include "mx_pair.hpp"
#include "mx_launch.hpp"

namespace mx {

// element offset added to an absent read: with n <= 2^27 rows every
// redirected byte offset lies in [2^30, 2^32) -- past the vector, unwrapped
constexpr int PAIR_OOR = 1 << 28;
constexpr int PAIR_OOR_EDGE = 1 << 27;   // 27-point form 2's edge redirect (n <= 2^27; may add to PAIR_OOR)
constexpr int64_t PAIR_CLEAN_MAX_ROWS = int64_t(1) << 27;
constexpr int LEAN_WAVES = 4;

struct PairLeanArgs {
  int m, n, nunits;            // rows, operand length, 128-row units (m = 128 nunits)
  int anchor[5];               // per run: the singleton offset, or the tri run's centre
  int P, NZ, L, S;             // z-march: units per plane, planes, planes per segment, segments
  double *partials;            // SPMV_DOT: one p.y partial per workgroup
  const int *done;             // solver stop flag (the launch is then a no-op)
  Fold fold;
};

// One unit's products: L[r] = run r's operand pair, e = the tri run's edge
// value (lane 0: x[r0 + c - 1], lane 63: x[r0 + 127 + c + 1]), bw = the unit's
// block word.  Each row sums its slots in ascending column order.
template <int PS, bool CLEAN>
__device__ __forceinline__ dbl2 pair_sums(const dbl2 (&L)[PairShape<PS>::NR], double e, uint32_t bw,
                                          const PairUni *__restrict__ puni, int lane) {
  using SH = PairShape<PS>;
  constexpr int K = SH::K;
  const PairUni &B = puni[bw & PBLK_ID];                  // wave-uniform: scalar loads
  // !CLEAN: the lane's own presence bits (one vector load; 2K wave-uniform
  // masks beside the 2K values spilled SGPRs)
  const uint32_t pb = CLEAN ? 0u : B.lane[lane];
  double s0v = 0.0, s1v = 0.0, lo = 0.0, hi = 0.0;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const int r = SH::run(j), p = SH::pos(j);
    if (SH::tri(r) && p < 0) {
      lo = wave_shift<true>(L[r].y, e);    // x[r0 + c - 1] = lane - 1's x[r0' + c + 1]
      hi = wave_shift<false>(L[r].x, e);   // x[r0 + c + 2] = lane + 1's x[r0' + c]
    }
    double a0, a1;
    if (!SH::tri(r)) { a0 = L[r].x; a1 = L[r].y; }
    else if (p < 0) { a0 = lo; a1 = L[r].x; }
    else if (p == 0) { a0 = L[r].x; a1 = L[r].y; }
    else { a0 = L[r].y; a1 = hi; }
    const double q0 = s0v + B.v[j] * a0, q1 = s1v + B.v[K + j] * a1;
    if constexpr (CLEAN) {
      s0v = q0;
      s1v = q1;
    } else {
      s0v = ((pb >> j) & 1u) ? q0 : s0v;
      s1v = ((pb >> (K + j)) & 1u) ? q1 : s1v;
    }
  }
  return dbl2{s0v, s1v};
}

// y = the sums (not stored for SPMV_PW); SPMV_DOT / SPMV_PW: + the p.y terms
template <int MODE, int PS, bool SPLIT, bool CLEAN>
__device__ __forceinline__ void pair_unit(const dbl2 (&L)[PairShape<PS>::NR], double e, uint32_t bw,
                                          const PairUni *__restrict__ puni, double *__restrict__ y, int r0,
                                          int lane, double &dot) {
  constexpr int C = PairShape<PS>::CENTER_RUN;
  const dbl2 sv = pair_sums<PS, CLEAN>(L, e, bw, puni, lane);
  // SPLIT: rows with A_o entries store their diagonal-block sum; the boundary
  // kernel continues them and adds their p.y terms.  SPMV_PW stores only those
  const bool gh = SPLIT && (bw & (lane < 32 ? PBLK_GHOST_LO : PBLK_GHOST_HI)) != 0;
  if (MODE != SPMV_PW || gh) *reinterpret_cast<dbl2 *>(y + r0) = sv;
  if constexpr (MODE == SPMV_DOT || MODE == SPMV_PW) {
    if (!gh) {
      dot += L[C].x * sv.x;
      dot += L[C].y * sv.y;
    }
  }
}

// The vectors and tables are __restrict__ kernel arguments: the block's slot
// values then compile to scalar loads (a pointer inside the by-value struct
// is not known unclobbered, and the values went through vector loads).
// Sweep form: the general kernel's XCD-grouped order, two units per step.
template <int MODE, int PS, bool SPLIT, bool CLEAN>
__global__ void __launch_bounds__(256) spmv_pair_lean_kernel(const PairLeanArgs a, const double *__restrict__ x,
                                                             double *__restrict__ y,
                                                             const int32_t *__restrict__ pblk,
                                                             const PairUni *__restrict__ puni) {
  if (a.done && *a.done) return;   // wave-uniform: solver finished
  using SH = PairShape<PS>;
  constexpr int NR = SH::NR;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // each XCD walks one contiguous eighth of the units, its waves interleaved
  // (the +-n / +-n^2 re-reads of x stay in that XCD's L2)
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
    pair_unit<MODE, PS, SPLIT, CLEAN>(ta.L, ta.e, ta.bw, puni, y, u * 128 + 2 * lane, lane, dot);
    pair_unit<MODE, PS, SPLIT, CLEAN>(tb.L, tb.e, tb.bw, puni, y, (u + sstep) * 128 + 2 * lane, lane, dot);
  }
  for (; u < send; u += sstep) {
    Unit t;
    load(u, (uint32_t)pblk[u], t);
    pair_unit<MODE, PS, SPLIT, CLEAN>(t.L, t.e, t.bw, puni, y, u * 128 + 2 * lane, lane, dot);
  }
  if constexpr (MODE == SPMV_DOT) {
    double v[1] = {dot};
    block_partials<1>(v, a.partials, gridDim.x, a.fold);
  }
}

// CG mode 5's p.Ap pass on a symmetric 5/7-point operator (Mat::sym57,
// checked once per operator by sym_check_kernel; knob 59): each row sums only
// its forward slots (+1, and for 7-point +n and +D; 5-point: +1, +D),
// t_i = a_ii p_i + 2 fwd_i, and p.Ap = sum_i p_i t_i -- mode 2's p.w to
// rounding (the same exact terms, another order).  The -n run is not loaded.
template <int PS>
__device__ __forceinline__ dbl2 pair_fwd(const dbl2 (&L)[PairShape<PS>::NR], double e, uint32_t bw,
                                         const PairUni *__restrict__ puni) {
  using SH = PairShape<PS>;
  constexpr int K = SH::K, C = SH::CENTER_RUN, JD = SH::first(C) + 1;   // the diagonal slot
  const PairUni &B = puni[bw & PBLK_ID];                  // wave-uniform: scalar loads
  const double hi = wave_shift<false>(L[C].x, e);         // x[r0 + c + 2]: row 1's +1
  double f0 = B.v[JD + 1] * L[C].y, f1 = B.v[K + JD + 1] * hi;
#pragma unroll
  for (int j = JD + 2; j < K; ++j) {                      // the singleton runs past the centre
    const int r = SH::run(j);
    f0 = f0 + B.v[j] * L[r].x;
    f1 = f1 + B.v[K + j] * L[r].y;
  }
  return dbl2{fma(2.0, f0, B.v[JD] * L[C].x), fma(2.0, f1, B.v[K + JD] * L[C].y)};
}

// Z-march form.  The pattern's first and last runs are -D and +D (D = P
// units: a 3D plane, a 2D line); unit u and unit u + P are one plane apart.
// A task is (segment of L planes, column of units); XCD x takes segments
// [S x / 8, S (x + 1) / 8) -- a contiguous slab of planes -- and its waves take
// the slab's tasks segment-major, so the waves running together sit in the
// same planes and the +-n pairs and edges they load hit L2.  Along a column
// the -D pair of a unit is the previous unit's centre pair and its centre the
// previous +D pair: carried in registers, so a unit loads the +D pair (the
// one line x is read from HBM for), its inner runs and its edge.  CLEAN: a
// carried operand whose run is empty for this unit is zeroed at use (it is
// real x, read for the neighbouring unit); inner runs and the edge take the
// out-of-range read as in the sweep form.
//
// CG mode 5 (one rank; x = p_i, the direction): w = A p is never stored.
//   SPMV_PW: only the p.w partials (the MatMult's 8 B/row of y written and
//   the update pass's 8 B/row of w read disappear);
//   SPMV_RUPD: the update pass -- every workgroup folds p.w from the PW pass's
//   partials and evaluates alpha (cg_alpha, workgroup 0 commits it), then per
//   unit recomputes A p (the same sums, the same bits as the PW pass's) and
//   forms r = r - alpha A p (BLAS daxpy's fma), z = c r and the [z.z, z.r, r.r]
//   partials, folded in-launch into red3.  p is re-read from the memory-side
//   cache the PW pass left it in; r is read non-temporally (the direction
//   update reads the r written here next).
//   SPLIT (P > 1): the PW pass stored the diagonal-block sums of the units
//   with A_o entries and the boundary kernel finished them (w = A p there,
//   plus their p.w terms); the residual update reads those rows' w instead of
//   its own (diagonal-block only) sums.
struct PairRuArgs {
  KspState *s;
  const double *w;             // SPLIT: the finished products of the ghost units' rows
  double *r;                   // r_i in, r_{i+1} out
  const double *r0;            // iteration 0 of a zero-guess solve reads r_0 = b (not copied into r)
  const double *dot_part;      // the PW pass's partials, folded here by every workgroup
  int ndot, xb;
  double c;                    // JM 2: the uniform Jacobi scalar 1 / d
  int *hw;                     // the host's pinned words (Poller)
};

template <int MODE, int PS, bool SPLIT, bool CLEAN, int ZU, int JM = 0, bool SYM = false>
__global__ void __launch_bounds__(256) spmv_pair_zm_kernel(const PairLeanArgs a, const double *__restrict__ x,
                                                           double *__restrict__ y, const int32_t *__restrict__ pblk,
                                                           const PairUni *__restrict__ puni, const PairRuArgs ru) {
  constexpr bool RU = MODE == SPMV_RUPD;
  double alpha = 0.0;
  const double *rin = nullptr;
  if constexpr (RU) {
    KspState *s = ru.s;
    if (s->top.done) {
      if (ru.hw && blockIdx.x == 0 && threadIdx.x == 0) host_store(ru.hw + HW_DONE, 1);
      return;
    }
    const double pw = ru.ndot > 0 ? block_sum_array<16>(ru.dot_part, ru.ndot) : s->red1;
    const CgAlpha al = cg_alpha(s, pw);
    if (blockIdx.x == 0 && threadIdx.x == 0) cg_commit_alpha(s, al, pw, ru.xb, false, ru.hw);
    if (al.reason) return;
    alpha = al.alpha;
    rin = (ru.r0 && al.i == 0) ? ru.r0 : ru.r;
  } else {
    if (a.done && *a.done) return;   // wave-uniform: solver finished
  }
  using SH = PairShape<PS>;
  constexpr int NR = SH::NR, TR = PS == 5 ? 1 : 2, LAST = NR - 1, C = SH::CENTER_RUN;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int sb, se, W, w;
  if ((gridDim.x & 7) == 0) {
    const int xcd = blockIdx.x & 7;
    W = (gridDim.x >> 3) * LEAN_WAVES;
    w = (blockIdx.x >> 3) * LEAN_WAVES + wid;
    sb = a.S * xcd / 8;
    se = a.S * (xcd + 1) / 8;
  } else {
    W = gridDim.x * LEAN_WAVES;
    w = blockIdx.x * LEAN_WAVES + wid;
    sb = 0;
    se = a.S;
  }
  const __amdgpu_buffer_rsrc_t xr = vec_rsrc(x, a.n);
  const int D = a.anchor[LAST];
  const int ecst = lane == 0 ? a.anchor[TR] - 1 : 128 + a.anchor[TR];
  constexpr uint32_t CARRY = PBLK_RUN0 | (PBLK_RUN0 << TR) | (PBLK_RUN0 << LAST);
  double dot = 0.0;
  double nv[3] = {0.0, 0.0, 0.0};            // RU: [z.z, z.r, r.r]
  const int ntask = (se - sb) * a.P;
  for (int t = w; t < ntask; t += W) {
    const int seg = sb + t / a.P, col = t % a.P;
    const int z0 = seg * a.L, z1 = min(z0 + a.L, a.NZ);
    const int cb = col * 128 + 2 * lane;       // the lane's rows within a plane
    dbl2 zm = bload2(xr, z0 * D + cb - D), c = bload2(xr, z0 * D + cb);
    uint32_t bwn = (uint32_t)pblk[z0 * a.P + col];
    // NQ units (planes z .. z + NQ - 1) with all their loads in flight
    auto step = [&](int z, auto nq) __attribute__((always_inline)) {
      constexpr int NQ = decltype(nq)::value;
      dbl2 L[NQ][NR], zp[NQ], rq[NQ];
      double e[NQ];
      uint32_t bw[NQ];
      bw[0] = bwn;
#pragma unroll
      for (int q = 1; q < NQ; ++q) bw[q] = (uint32_t)pblk[(z + q) * a.P + col];
      if (z + NQ < z1) bwn = (uint32_t)pblk[(z + NQ) * a.P + col];   // next step's, ahead
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int r0 = (z + q) * D + cb, ub = (z + q) * D + col * 128;
        zp[q] = bload2(xr, r0 + D);
#pragma unroll
        for (int r = 1; r < LAST; ++r)
          if (r != TR && !(SYM && r < TR))                 // SYM: no backward inner run
            L[q][r] = bload2(xr, r0 + a.anchor[r] + (CLEAN && (bw[q] & (PBLK_RUN0 << r)) ? PAIR_OOR : 0));
        int eo = ecst;
        if constexpr (CLEAN) eo += lane == 0 ? ((bw[q] & PBLK_ELO) ? PAIR_OOR : 0) : ((bw[q] & PBLK_EHI) ? PAIR_OOR : 0);
        e[q] = bload1(xr, ub + eo);
        if constexpr (RU) rq[q] = __builtin_nontemporal_load(reinterpret_cast<const dbl2 *>(rin + r0));
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        L[q][0] = q == 0 ? zm : q == 1 ? c : zp[q - 2];
        L[q][TR] = q == 0 ? c : zp[q - 1];
        L[q][LAST] = zp[q];
        if constexpr (CLEAN) {
          if (bw[q] & CARRY) {                     // wave-uniform, rare: an empty carried run
            if (bw[q] & PBLK_RUN0) L[q][0] = dbl2{0.0, 0.0};
            if (bw[q] & (PBLK_RUN0 << TR)) L[q][TR] = dbl2{0.0, 0.0};
            if (bw[q] & (PBLK_RUN0 << LAST)) L[q][LAST] = dbl2{0.0, 0.0};
          }
        }
        const int r0 = (z + q) * D + cb;
        if constexpr (RU) {
          dbl2 w2 = pair_sums<PS, CLEAN>(L[q], e[q], bw[q], puni, lane);
          if constexpr (SPLIT) {
            if (bw[q] & (PBLK_GHOST_LO | PBLK_GHOST_HI)) {        // wave-uniform, rare
              if (bw[q] & (lane < 32 ? PBLK_GHOST_LO : PBLK_GHOST_HI)) w2 = *reinterpret_cast<const dbl2 *>(ru.w + r0);
            }
          }
          const double ra = fma(-alpha, w2.x, rq[q].x), rb = fma(-alpha, w2.y, rq[q].y);
          const double za = JM == 2 ? ra * ru.c : ra, zb = JM == 2 ? rb * ru.c : rb;
          nv[0] += za * za; nv[1] += za * ra; nv[2] += ra * ra;
          nv[0] += zb * zb; nv[1] += zb * rb; nv[2] += rb * rb;
          *reinterpret_cast<dbl2 *>(ru.r + r0) = dbl2{ra, rb};
        } else if constexpr (SYM) {
          static_assert(MODE == SPMV_PW && CLEAN && !SPLIT, "symmetric p.Ap pass: one rank, select-free");
          const dbl2 t = pair_fwd<PS>(L[q], e[q], bw[q], puni);
          dot += L[q][C].x * t.x;
          dot += L[q][C].y * t.y;
        } else {
          pair_unit<MODE, PS, SPLIT, CLEAN>(L[q], e[q], bw[q], puni, y, r0, lane, dot);
        }
      }
      if constexpr (NQ == 1) zm = c;
      else zm = zp[NQ - 2];
      c = zp[NQ - 1];
    };
    int z = z0;
    for (; z + ZU <= z1; z += ZU) step(z, std::integral_constant<int, ZU>{});
    for (; z < z1; ++z) step(z, std::integral_constant<int, 1>{});
  }
  if constexpr (MODE == SPMV_DOT || MODE == SPMV_PW) {
    double v[1] = {dot};
    block_partials<1>(v, a.partials, gridDim.x, a.fold);
  } else if constexpr (RU) {
    block_partials<3>(nv, a.partials, gridDim.x, a.fold);
  }
}

// CG mode 5's residual update on a clean one-rank 7-point layout, two lines
// per wave (knob 68): a wave marches the columns of lines y and y + 1 (y
// even) together, so line y's +n operand is line y + 1's own centre pair and
// line y + 1's -n operand line y's -- per plane the two units load their +D
// pairs, the outer lines y - 1 and y + 2, their edges and r: 8 vector loads
// for two units instead of 10 (the residual update is vector-memory issue
// bound: profiles/r04g_pmc_c3_iteration.txt).  Each unit sums its rows with
// pair_sums, as spmv_pair_zm_kernel<SPMV_RUPD> does: the same bits.
// WPE: the waves-per-SIMD floor asked of the register allocator (knob 68 = 2:
// 5, i.e. at most 96 VGPRs, against 98 -> 4 waves unconstrained).
template <int JM, int WPE>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) spmv_pair_zm2l_kernel(const PairLeanArgs a, const double *__restrict__ x,
                                                             const int32_t *__restrict__ pblk,
                                                             const PairUni *__restrict__ puni, const PairRuArgs ru) {
  constexpr int PS = 7, NR = 5, TR = 2, LAST = 4;
  KspState *s = ru.s;
  if (s->top.done) {
    if (ru.hw && blockIdx.x == 0 && threadIdx.x == 0) host_store(ru.hw + HW_DONE, 1);
    return;
  }
  const double pw = ru.ndot > 0 ? block_sum_array<16>(ru.dot_part, ru.ndot) : s->red1;
  const CgAlpha al = cg_alpha(s, pw);
  if (blockIdx.x == 0 && threadIdx.x == 0) cg_commit_alpha(s, al, pw, ru.xb, false, ru.hw);
  if (al.reason) return;
  const double alpha = al.alpha;
  const double *rin = (ru.r0 && al.i == 0) ? ru.r0 : ru.r;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int sb, se, W, w;
  if ((gridDim.x & 7) == 0) {
    const int xcd = blockIdx.x & 7;
    W = (gridDim.x >> 3) * LEAN_WAVES;
    w = (blockIdx.x >> 3) * LEAN_WAVES + wid;
    sb = a.S * xcd / 8;
    se = a.S * (xcd + 1) / 8;
  } else {
    W = gridDim.x * LEAN_WAVES;
    w = blockIdx.x * LEAN_WAVES + wid;
    sb = 0;
    se = a.S;
  }
  const __amdgpu_buffer_rsrc_t xr = vec_rsrc(x, a.n);
  const int D = a.anchor[LAST], NL = a.anchor[3];           // plane, line
  const int PL = NL / 128, PH = a.P / 2;                     // columns per line, column pairs per plane
  const int ecst = lane == 0 ? a.anchor[TR] - 1 : 128 + a.anchor[TR];
  constexpr uint32_t CARRY = PBLK_RUN0 | (PBLK_RUN0 << TR) | (PBLK_RUN0 << LAST);
  double nv[3] = {0.0, 0.0, 0.0};
  const int ntask = (se - sb) * PH;
  for (int t = w; t < ntask; t += W) {
    const int seg = sb + t / PH, cp = t % PH;
    const int colA = (cp / PL) * 2 * PL + cp % PL, colB = colA + PL;
    const int z0 = seg * a.L, z1 = min(z0 + a.L, a.NZ);
    const int cbA = colA * 128 + 2 * lane, cbB = colB * 128 + 2 * lane;
    dbl2 zmA = bload2(xr, z0 * D + cbA - D), cA = bload2(xr, z0 * D + cbA);
    dbl2 zmB = bload2(xr, z0 * D + cbB - D), cB = bload2(xr, z0 * D + cbB);
    // block words one plane ahead (their scalar loads off the step's path)
    uint32_t bwAn = (uint32_t)pblk[z0 * a.P + colA], bwBn = (uint32_t)pblk[z0 * a.P + colB];
    for (int z = z0; z < z1; ++z) {
      const uint32_t bwA = bwAn, bwB = bwBn;
      if (z + 1 < z1) { bwAn = (uint32_t)pblk[(z + 1) * a.P + colA]; bwBn = (uint32_t)pblk[(z + 1) * a.P + colB]; }
      const int rA = z * D + cbA, rB = z * D + cbB;
      const dbl2 zpA = bload2(xr, rA + D), zpB = bload2(xr, rB + D);
      const dbl2 nA = bload2(xr, rA + a.anchor[1] + ((bwA & (PBLK_RUN0 << 1)) ? PAIR_OOR : 0));
      const dbl2 nB = bload2(xr, rB + a.anchor[3] + ((bwB & (PBLK_RUN0 << 3)) ? PAIR_OOR : 0));
      int eA = ecst, eB = ecst;
      eA += lane == 0 ? ((bwA & PBLK_ELO) ? PAIR_OOR : 0) : ((bwA & PBLK_EHI) ? PAIR_OOR : 0);
      eB += lane == 0 ? ((bwB & PBLK_ELO) ? PAIR_OOR : 0) : ((bwB & PBLK_EHI) ? PAIR_OOR : 0);
      const double edA = bload1(xr, z * D + colA * 128 + eA), edB = bload1(xr, z * D + colB * 128 + eB);
      const dbl2 rqA = __builtin_nontemporal_load(reinterpret_cast<const dbl2 *>(rin + rA));
      const dbl2 rqB = __builtin_nontemporal_load(reinterpret_cast<const dbl2 *>(rin + rB));
      __builtin_amdgcn_sched_barrier(0);
      // line y's +n run is line y + 1's rows, line y + 1's -n run line y's
      // (an empty run -- a grid edge, rare -- reads as 0.0, as its
      // out-of-range load would)
      const dbl2 Z{0.0, 0.0};
      dbl2 LA[NR] = {zmA, nA, cA, (bwA & (PBLK_RUN0 << 3)) ? Z : cB, zpA};
      dbl2 LB[NR] = {zmB, (bwB & (PBLK_RUN0 << 1)) ? Z : cA, cB, nB, zpB};
      if (bwA & CARRY) {                         // wave-uniform, rare: an empty carried run
        if (bwA & PBLK_RUN0) LA[0] = Z;
        if (bwA & (PBLK_RUN0 << TR)) LA[TR] = Z;
        if (bwA & (PBLK_RUN0 << LAST)) LA[LAST] = Z;
      }
      if (bwB & CARRY) {
        if (bwB & PBLK_RUN0) LB[0] = Z;
        if (bwB & (PBLK_RUN0 << TR)) LB[TR] = Z;
        if (bwB & (PBLK_RUN0 << LAST)) LB[LAST] = Z;
      }
      const dbl2 wA = pair_sums<PS, true>(LA, edA, bwA, puni, lane);
      const dbl2 wB = pair_sums<PS, true>(LB, edB, bwB, puni, lane);
      auto upd = [&](dbl2 w2, dbl2 rq, int r0) __attribute__((always_inline)) {
        const double ra = fma(-alpha, w2.x, rq.x), rb = fma(-alpha, w2.y, rq.y);
        const double za = JM == 2 ? ra * ru.c : ra, zb = JM == 2 ? rb * ru.c : rb;
        nv[0] += za * za; nv[1] += za * ra; nv[2] += ra * ra;
        nv[0] += zb * zb; nv[1] += zb * rb; nv[2] += rb * rb;
        *reinterpret_cast<dbl2 *>(ru.r + r0) = dbl2{ra, rb};
      };
      upd(wA, rqA, rA);
      upd(wB, rqB, rB);
      zmA = cA; cA = zpA;
      zmB = cB; cB = zpB;
    }
  }
  block_partials<3>(nv, a.partials, gridDim.x, a.fold);
}

// CG mode 5's direction update fused into its p.Ap pass (knob 69; one rank,
// a clean symmetric 5/7-point layout, batched x steps): the pass forms
// p_i = z_i + b p_{i-1} (cg_dir, the expression cg_pb_kernel uses) for the
// operands its forward-half rows need -- the centre pair, +n, +D and the
// line's +1 edge -- from r_i and p_{i-1}, stores the centre rows' p_i and sums
// p.Ap as the symmetric PW pass does (pair_fwd, the same units in the same
// order on the same grid: the same partials).  Per row: r and p_{i-1} read,
// p_i written -- against the separate direction update (r, p_{i-1} read, p_i
// written) plus the PW pass (p_i read again).  Operands of neighbouring rows
// are formed by every unit that needs them from the same loads: the same bits
// as the owner's stored p_i.  Launched only for iterations i % B != 0 (the
// host's iteration index is the device's: a captured batch starts on a
// multiple of B): the x-step batch iterations keep cg_pb_kernel + the PW pass
// (their extra streams in one z-march measured 205 us against 162).
struct PairPbArgs {
  KspState *s;
  const double *r;             // r_i
  const double *r0;            // iteration 0 of a zero-guess solve: r_0 = b (not copied into r)
  double *pb;                  // p_j in buffer j % B, at pb + (j % B) ps
  int64_t ps;
  double *hist;
  double c;                    // JM 2: the uniform Jacobi scalar
};

template <int PS, int JM, int B, int ZU>
__global__ void __launch_bounds__(256) spmv_pair_pbw_kernel(const PairLeanArgs a, const int32_t *__restrict__ pblk,
                                                            const PairUni *__restrict__ puni, const PairPbArgs pa) {
  KspState *s = pa.s;
  const CgTopIn top = s->top;
  if (top.done) return;
  const CgTop t = cg_top(top);
  if (blockIdx.x == 0 && threadIdx.x == 0) cg_commit_top(s, t, pa.hist);
  if (t.reason) return;
  const int i = t.i;
  const double b = t.b;
  using SH = PairShape<PS>;
  constexpr int NR = SH::NR, TR = PS == 5 ? 1 : 2, LAST = NR - 1, C = SH::CENTER_RUN;
  auto pick = [&](int k) -> double * { return pa.pb + k * pa.ps; };
  double *pout = pick(i % B);
  const double *pprev = pick((i + B - 1) % B);
  const double *rs = (pa.r0 && i == 0) ? pa.r0 : pa.r;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int sb, se, W, w;
  if ((gridDim.x & 7) == 0) {
    const int xcd = blockIdx.x & 7;
    W = (gridDim.x >> 3) * LEAN_WAVES;
    w = (blockIdx.x >> 3) * LEAN_WAVES + wid;
    sb = a.S * xcd / 8;
    se = a.S * (xcd + 1) / 8;
  } else {
    W = gridDim.x * LEAN_WAVES;
    w = blockIdx.x * LEAN_WAVES + wid;
    sb = 0;
    se = a.S;
  }
  const __amdgpu_buffer_rsrc_t rr = vec_rsrc(rs, a.n), pr = vec_rsrc(pprev, a.n);
  const int D = a.anchor[LAST];
  // the tri run's +1 edge: lane 63's x[ub + 128] (the backward edge is not
  // needed by the forward half); the other lanes load the same line
  const int eoff = 128 + a.anchor[TR];
  constexpr uint32_t CARRY = PBLK_RUN0 | (PBLK_RUN0 << TR) | (PBLK_RUN0 << LAST);
  const int ntask = (se - sb) * a.P;
  double dot = 0.0;
  // NP: b == 0 (iteration 0, a restart), p_{i-1} not read
  auto march = [&](auto npc) __attribute__((always_inline)) {
    constexpr bool NP = decltype(npc)::value;
    auto dir = [&](dbl2 r2, dbl2 p2) __attribute__((always_inline)) {
      return dbl2{cg_dir(jac1<JM>(r2.x, 0.0, pa.c), b, NP ? 0.0 : p2.x),
                  cg_dir(jac1<JM>(r2.y, 0.0, pa.c), b, NP ? 0.0 : p2.y)};
    };
    for (int tk = w; tk < ntask; tk += W) {
      const int seg = sb + tk / a.P, col = tk % a.P;
      const int z0 = seg * a.L, z1 = min(z0 + a.L, a.NZ);
      const int cb = col * 128 + 2 * lane;
      dbl2 pc = dir(bload2(rr, z0 * D + cb), NP ? dbl2{0.0, 0.0} : bload2(pr, z0 * D + cb));   // p_i, centre
      uint32_t bwn = (uint32_t)pblk[z0 * a.P + col];
      auto step = [&](int z, auto nq) __attribute__((always_inline)) {
        constexpr int NQ = decltype(nq)::value;
        dbl2 zr[NQ], zpp[NQ], nr[NQ], npp[NQ];
        double er[NQ], epp[NQ];
        uint32_t bw[NQ];
        bw[0] = bwn;
#pragma unroll
        for (int q = 1; q < NQ; ++q) bw[q] = (uint32_t)pblk[(z + q) * a.P + col];
        if (z + NQ < z1) bwn = (uint32_t)pblk[(z + NQ) * a.P + col];
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          const int r0 = (z + q) * D + cb, ub = (z + q) * D + col * 128;
          zr[q] = bload2(rr, r0 + D);
          zpp[q] = NP ? dbl2{0.0, 0.0} : bload2(pr, r0 + D);
          if constexpr (PS == 7) {
            const int no = r0 + a.anchor[3] + ((bw[q] & (PBLK_RUN0 << 3)) ? PAIR_OOR : 0);
            nr[q] = bload2(rr, no);
            npp[q] = NP ? dbl2{0.0, 0.0} : bload2(pr, no);
          }
          // a line's last unit has no +1 edge (wave-uniform: no loads)
          er[q] = 0.0;
          epp[q] = 0.0;
          if (!(bw[q] & PBLK_EHI)) {
            er[q] = bload1(rr, ub + eoff);
            if constexpr (!NP) epp[q] = bload1(pr, ub + eoff);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          const int r0 = (z + q) * D + cb;
          const dbl2 pz = dir(zr[q], zpp[q]);
          const double pe = cg_dir(jac1<JM>(er[q], 0.0, pa.c), b, NP ? 0.0 : epp[q]);
          *reinterpret_cast<dbl2 *>(pout + r0) = pc;
          dbl2 L[NR];
          L[0] = dbl2{0.0, 0.0};                   // -D: not in the forward half
          if constexpr (PS == 7) { L[1] = dbl2{0.0, 0.0}; L[3] = dir(nr[q], npp[q]); }
          L[TR] = pc;
          L[LAST] = pz;
          if (bw[q] & CARRY) {                     // wave-uniform, rare: an empty carried run
            if (bw[q] & (PBLK_RUN0 << TR)) L[TR] = dbl2{0.0, 0.0};
            if (bw[q] & (PBLK_RUN0 << LAST)) L[LAST] = dbl2{0.0, 0.0};
          }
          const dbl2 tq = pair_fwd<PS>(L, pe, bw[q], puni);
          dot += L[C].x * tq.x;
          dot += L[C].y * tq.y;
          pc = pz;
        }
      };
      int z = z0;
      for (; z + ZU <= z1; z += ZU) step(z, std::integral_constant<int, ZU>{});
      for (; z < z1; ++z) step(z, std::integral_constant<int, 1>{});
    }
  };
  const std::true_type T{};
  const std::false_type F{};
  if (b == 0.0) march(T);
  else march(F);
  double v[1] = {dot};
  block_partials<1>(v, a.partials, gridDim.x, a.fold);
}

// The direction update fused into CG mode 5's p.Ap pass on P > 1 ranks
// (knob 80): the split PW pass of spmv_pair_zm_kernel
// <SPMV_PW, PS, SPLIT = true> -- full rows, the ghost units' diagonal-block
// sums stored for the boundary kernel -- with every operand it gathers formed
// as p_i = z_i + b p_{i-1} from r_i and p_{i-1} (cg_dir, the direction
// update's expression), the centre rows' p_i stored into the direction
// buffer.  The same units in the same order on the same grid with the same
// sums: p_i, the stored diagonal-block sums and the p.Ap partials are the
// separate passes' bits.  The ghost planes' p_i leave through the halo pack,
// which forms them from r and p_{i-1} too (pack_cg_kernel), before this
// launch starts; the boundary kernel then reads the stored p_i.
template <int PS, bool CLEAN, int ZU, int JM>
__global__ void __launch_bounds__(256) spmv_pair_zmpbs_kernel(const PairLeanArgs a, double *__restrict__ y,
                                                              const int32_t *__restrict__ pblk,
                                                              const PairUni *__restrict__ puni, const PairPbArgs pa,
                                                              int xb) {
  KspState *s = pa.s;
  const CgTopIn top = s->top;
  if (top.done) return;
  const CgTop t = cg_top(top);
  if (blockIdx.x == 0 && threadIdx.x == 0) cg_commit_top(s, t, pa.hist);
  if (t.reason) return;
  const int i = t.i;
  const double b = t.b;
  double *pout = pa.pb + (int64_t)(i % xb) * pa.ps;
  const double *pprev = pa.pb + (int64_t)((i + xb - 1) % xb) * pa.ps;
  using SH = PairShape<PS>;
  constexpr int NR = SH::NR, TR = PS == 5 ? 1 : 2, LAST = NR - 1;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int sb, se, W, w;
  if ((gridDim.x & 7) == 0) {
    const int xcd = blockIdx.x & 7;
    W = (gridDim.x >> 3) * LEAN_WAVES;
    w = (blockIdx.x >> 3) * LEAN_WAVES + wid;
    sb = a.S * xcd / 8;
    se = a.S * (xcd + 1) / 8;
  } else {
    W = gridDim.x * LEAN_WAVES;
    w = blockIdx.x * LEAN_WAVES + wid;
    sb = 0;
    se = a.S;
  }
  const __amdgpu_buffer_rsrc_t rr = vec_rsrc(pa.r, a.n), pr = vec_rsrc(pprev, a.n);
  const int D = a.anchor[LAST];
  const int ecst = lane == 0 ? a.anchor[TR] - 1 : 128 + a.anchor[TR];
  constexpr uint32_t CARRY = PBLK_RUN0 | (PBLK_RUN0 << TR) | (PBLK_RUN0 << LAST);
  auto dir1 = [&](double r1, double p1) __attribute__((always_inline)) {
    return cg_dir(jac1<JM>(r1, 0.0, pa.c), b, p1);
  };
  auto dir2 = [&](dbl2 r2, dbl2 p2) __attribute__((always_inline)) { return dbl2{dir1(r2.x, p2.x), dir1(r2.y, p2.y)}; };
  auto ld2 = [&](int off) __attribute__((always_inline)) { return dir2(bload2(rr, off), bload2(pr, off)); };
  double dot = 0.0;
  const int ntask = (se - sb) * a.P;
  for (int tk = w; tk < ntask; tk += W) {
    const int seg = sb + tk / a.P, col = tk % a.P;
    const int z0 = seg * a.L, z1 = min(z0 + a.L, a.NZ);
    const int cb = col * 128 + 2 * lane;
    dbl2 zm = ld2(z0 * D + cb - D), c = ld2(z0 * D + cb);
    uint32_t bwn = (uint32_t)pblk[z0 * a.P + col];
    auto step = [&](int z, auto nq) __attribute__((always_inline)) {
      constexpr int NQ = decltype(nq)::value;
      dbl2 L[NQ][NR], zp[NQ], zr[NQ], zq[NQ], Lr[NQ][NR], Lp[NQ][NR];
      double e[NQ], er[NQ], ep[NQ];
      uint32_t bw[NQ];
      bw[0] = bwn;
#pragma unroll
      for (int q = 1; q < NQ; ++q) bw[q] = (uint32_t)pblk[(z + q) * a.P + col];
      if (z + NQ < z1) bwn = (uint32_t)pblk[(z + NQ) * a.P + col];
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int r0 = (z + q) * D + cb, ub = (z + q) * D + col * 128;
        zr[q] = bload2(rr, r0 + D);
        zq[q] = bload2(pr, r0 + D);
#pragma unroll
        for (int r = 1; r < LAST; ++r)
          if (r != TR) {
            const int off = r0 + a.anchor[r] + (CLEAN && (bw[q] & (PBLK_RUN0 << r)) ? PAIR_OOR : 0);
            Lr[q][r] = bload2(rr, off);
            Lp[q][r] = bload2(pr, off);
          }
        int eo = ecst;
        if constexpr (CLEAN) eo += lane == 0 ? ((bw[q] & PBLK_ELO) ? PAIR_OOR : 0) : ((bw[q] & PBLK_EHI) ? PAIR_OOR : 0);
        er[q] = bload1(rr, ub + eo);
        ep[q] = bload1(pr, ub + eo);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        zp[q] = dir2(zr[q], zq[q]);
#pragma unroll
        for (int r = 1; r < LAST; ++r)
          if (r != TR) L[q][r] = dir2(Lr[q][r], Lp[q][r]);
        e[q] = dir1(er[q], ep[q]);
      }
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        L[q][0] = q == 0 ? zm : q == 1 ? c : zp[q - 2];
        L[q][TR] = q == 0 ? c : zp[q - 1];
        L[q][LAST] = zp[q];
        const int r0 = (z + q) * D + cb;
        *reinterpret_cast<dbl2 *>(pout + r0) = L[q][TR];        // the unit's own p_i
        if constexpr (CLEAN) {
          if (bw[q] & CARRY) {                     // wave-uniform, rare: an empty carried run
            if (bw[q] & PBLK_RUN0) L[q][0] = dbl2{0.0, 0.0};
            if (bw[q] & (PBLK_RUN0 << TR)) L[q][TR] = dbl2{0.0, 0.0};
            if (bw[q] & (PBLK_RUN0 << LAST)) L[q][LAST] = dbl2{0.0, 0.0};
          }
        }
        pair_unit<SPMV_PW, PS, true, CLEAN>(L[q], e[q], bw[q], puni, y, r0, lane, dot);
      }
      if constexpr (NQ == 1) zm = c;
      else zm = zp[NQ - 2];
      c = zp[NQ - 1];
    };
    int z = z0;
    for (; z + ZU <= z1; z += ZU) step(z, std::integral_constant<int, ZU>{});
    for (; z < z1; ++z) step(z, std::integral_constant<int, 1>{});
  }
  double v[1] = {dot};
  block_partials<1>(v, a.partials, gridDim.x, a.fold);
}

// 27-point z-march (Sell::puni27).  The nine runs are (dz, dy) in {-1,0,1}^2
// at anchors -D-n, -D, -D+n, -n, 0, +n, D-n, D, D+n (each a tri run c-1, c,
// c+1); marching a column in z, the runs of planes z-1 and z (six pairs and
// their edge values) are carried and a unit loads only plane z+1's three runs
// and edges: 3 pair loads + 3 edge loads instead of 9 + 9.  (A three-way
// rotation of plane registers instead of the carry copies measured 106-128
// VGPRs against 78: 4 waves per SIMD instead of 6.)
// The two rows of a lane share each slot's value (the dictionary build
// requires v[j] == v[K + j]): 27 wave-uniform values.  Forms:
//   2 (Sell::pcol27, the column words): every unit's empty runs are its
//     plane's z-boundary runs -- read out of range (before plane 0, past the
//     last), so 0.0 -- and its column's y-boundary runs, and its x-line edges
//     are its column's: the column's empty runs and edges are loaded out of
//     range too (PAIR_OOR), for the carried planes as well (the same column),
//     so every absent slot multiplies 0.0 (sum + v * 0.0 = sum, a row sum is
//     never -0.0) and the unit has neither branches nor selects;
//   1 (every block select-free, Sell::pair_clean27): an empty run is skipped
//     by a wave-uniform branch (its operands are real x of the neighbouring
//     line or plane) and the x-edge value is zeroed at use (U27_ELO /
//     U27_EHI: lane 0's / lane 63's edge);
//   0: presence selects from the lane's own 54 mask bits (PairUni27::lane,
//     one vector load per unit).
//   UV (Sell::pair_unit27, knob 53): every slot value but the diagonal's is
//     -1, 0 or +1, so v * a is exact and sum + v * a == fma(v, a, sum) bit for
//     bit (one rounding either way; an exact product cannot overflow or
//     underflow): one VALU op instead of two for 26 of the 27 slots.
template <int FORM, bool UV = false>
__device__ __forceinline__ dbl2 pair_sums27(const dbl2 (&L)[9], const double (&e)[9], uint32_t bw,
                                            const PairUni27 *__restrict__ puni, int lane) {
  constexpr int K = 27;
  const PairUni27 &B = puni[bw & PBLK_ID];                // wave-uniform: scalar loads
  uint32_t fl = 0;
  unsigned long long pb = 0;
  bool zedge = false;
  if constexpr (FORM == 1) {
    fl = B.flags;
    zedge = lane == 0 ? (fl & U27_ELO) != 0 : (fl & U27_EHI) != 0;
  } else if constexpr (FORM == 0) {
    pb = B.lane[lane];
  }
  double s0v = 0.0, s1v = 0.0;
#pragma unroll
  for (int r = 0; r < 9; ++r) {
    if constexpr (FORM == 1) {
      if (fl & (1u << r)) continue;                       // wave-uniform: an empty run
    }
    double er = e[r];
    if constexpr (FORM == 1) er = zedge ? 0.0 : er;
    const double lo = wave_shift<true>(L[r].y, er);       // x[r0 + c - 1]
    const double hi = wave_shift<false>(L[r].x, er);      // x[r0 + c + 2]
    const double a0[3] = {lo, L[r].x, L[r].y}, a1[3] = {L[r].x, L[r].y, hi};
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      const int j = 3 * r + p;
      const double v = B.v[j];
      double q0, q1;
      if (UV && j != 13) {
        q0 = __builtin_fma(v, a0[p], s0v);
        q1 = __builtin_fma(v, a1[p], s1v);
      } else {
        q0 = s0v + v * a0[p];
        q1 = s1v + v * a1[p];
      }
      if constexpr (FORM == 0) {
        s0v = ((pb >> j) & 1ull) ? q0 : s0v;
        s1v = ((pb >> (K + j)) & 1ull) ? q1 : s1v;
      } else {
        s0v = q0;
        s1v = q1;
      }
    }
  }
  return dbl2{s0v, s1v};
}

// CG mode 5's p.Ap pass on a symmetric 27-point operator (Sell::pair_sym27,
// knob 59): p^T A p = sum_i p_i (a_ii p_i + 2 sum_{d > 0} a_{i,i+d} p_{i+d}),
// so a row needs only its 13 forward slots (14..26: the +1 of the centre run,
// the dy = +1 run of its plane and the three runs of the next plane) -- half
// the products of the full row.  Returns the rows' t_i = a_ii p_i + 2 fwd_i:
// p.Ap equals mode 2's p.w to rounding (a different order of the same exact
// terms), not bit for bit.
template <bool UV>
__device__ __forceinline__ dbl2 pair_fwd27(const dbl2 (&L)[9], const double (&e)[9], uint32_t bw,
                                           const PairUni27 *__restrict__ puni) {
  const PairUni27 &B = puni[bw & PBLK_ID];                // wave-uniform: scalar loads
  double f0 = 0.0, f1 = 0.0;
#pragma unroll
  for (int r = 4; r < 9; ++r) {
    const double hi = wave_shift<false>(L[r].x, e[r]);    // x[r0 + c + 2]
    double lo = 0.0;
    if (r > 4) lo = wave_shift<true>(L[r].y, e[r]);       // x[r0 + c - 1]
    const double a0[3] = {lo, L[r].x, L[r].y}, a1[3] = {L[r].x, L[r].y, hi};
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int j = 3 * r + q;
      if (j <= 13) continue;
      const double v = B.v[j];
      if (UV) {
        f0 = __builtin_fma(v, a0[q], f0);
        f1 = __builtin_fma(v, a1[q], f1);
      } else {
        f0 = f0 + v * a0[q];
        f1 = f1 + v * a1[q];
      }
    }
  }
  const double d = B.v[13];
  return dbl2{fma(2.0, f0, d * L[4].x), fma(2.0, f1, d * L[4].y)};
}

struct PairLean27Args {
  int n, P, NZ, L, S;
  int xcol;                    // two-line kernels: XCDs split the line groups (1) instead of the planes (0)
  int anchor[9];
  double *partials;
  const int *done;
  Fold fold;
};

// The column-word form keeps 6 waves per SIMD (<= 80 VGPRs; the VALU-bound
// body measured fastest there, knob 45); the fma form (UV) otherwise
// allocates 86-105 (one plane per step; two would spill at that bound).
// CG mode 5 on the 27-point operator (one rank, no ghost units): SPMV_PW
// (the p.Ap partials, nothing stored) and SPMV_RUPD (alpha from the PW
// partials, A p recomputed, r = r - alpha A p, z = c r and the three norms),
// as spmv_pair_zm_kernel's (the same sums as the MatMult's, bit for bit).
template <int MODE, bool SPLIT, int FORM, int ZU, bool UV = false, int JM = 0, bool SYM = false>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(UV && ZU == 1 ? 6 : 1)))
spmv_pair_zm27_kernel(const PairLean27Args a, const double *__restrict__ x,
                                                             double *__restrict__ y, const int32_t *__restrict__ pblk,
                                                             const PairUni27 *__restrict__ puni,
                                                             const int32_t *__restrict__ pcol, const PairRuArgs ru) {
  constexpr bool RU = MODE == SPMV_RUPD;
  static_assert(!SPLIT || (MODE != SPMV_PW && !RU), "27-point mode 5: one rank");
  double alpha = 0.0;
  const double *rin = nullptr;
  if constexpr (RU) {
    KspState *s = ru.s;
    if (s->top.done) {
      if (ru.hw && blockIdx.x == 0 && threadIdx.x == 0) host_store(ru.hw + HW_DONE, 1);
      return;
    }
    const double pw = ru.ndot > 0 ? block_sum_array<16>(ru.dot_part, ru.ndot) : s->red1;
    const CgAlpha al = cg_alpha(s, pw);
    if (blockIdx.x == 0 && threadIdx.x == 0) cg_commit_alpha(s, al, pw, ru.xb, false, ru.hw);
    if (al.reason) return;
    alpha = al.alpha;
    rin = (ru.r0 && al.i == 0) ? ru.r0 : ru.r;
  } else {
    if (a.done && *a.done) return;   // wave-uniform: solver finished
  }
  double nv[3] = {0.0, 0.0, 0.0};                  // RU: [z.z, z.r, r.r]
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int sb, se, W, w;
  if ((gridDim.x & 7) == 0) {
    const int xcd = blockIdx.x & 7;
    W = (gridDim.x >> 3) * LEAN_WAVES;
    w = (blockIdx.x >> 3) * LEAN_WAVES + wid;
    sb = a.S * xcd / 8;
    se = a.S * (xcd + 1) / 8;
  } else {
    W = gridDim.x * LEAN_WAVES;
    w = blockIdx.x * LEAN_WAVES + wid;
    sb = 0;
    se = a.S;
  }
  const __amdgpu_buffer_rsrc_t xr = vec_rsrc(x, a.n);
  const int D = a.anchor[7];
  const int eb = lane == 0 ? -1 : 128;                   // edge: lane 0 x[ub + c - 1], others x[ub + 128 + c]
  double dot = 0.0;
  const int ntask = (se - sb) * a.P;
  for (int t = w; t < ntask; t += W) {
    const int seg = sb + t / a.P, col = t % a.P;
    const int z0 = seg * a.L, z1 = min(z0 + a.L, a.NZ);
    const int cb = col * 128 + 2 * lane;
    // form 2: the column's empty runs (dy = -1 / +1) and x-line edges read
    // out of range, in every plane it loads (so the carried runs as well)
    // (an edge offset 2^27 and a run offset 2^28 may add up: 3 * 2^27 rows is
    // still past the vector and inside the 32-bit byte offset, n <= 2^27)
    // (an edge offset 2^27 and a run offset 2^28 may add up: 3 * 2^27 rows is
    // still past the vector and inside the 32-bit byte offset, n <= 2^27)
    int oor[3] = {0, 0, 0}, ebe = eb;
    if constexpr (FORM == 2) {
      const uint32_t cw = (uint32_t)pcol[col];
      oor[0] = (cw & U27C_YLO) ? PAIR_OOR : 0;
      oor[2] = (cw & U27C_YHI) ? PAIR_OOR : 0;
      ebe += (lane == 0 ? (cw & U27_ELO) : (cw & U27_EHI)) ? PAIR_OOR_EDGE : 0;
    }
    dbl2 C[6];                                           // runs 0..5 of the current unit (planes z-1, z)
    double Ce[6];
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      C[r] = bload2(xr, z0 * D + cb + a.anchor[r] + oor[r % 3]);
      Ce[r] = bload1(xr, z0 * D + col * 128 + ebe + a.anchor[r] + oor[r % 3]);
    }
    uint32_t bwn = (uint32_t)pblk[z0 * a.P + col];
    auto step = [&](int z, auto nq) __attribute__((always_inline)) {
      constexpr int NQ = decltype(nq)::value;
      dbl2 Nw[NQ][3], rq[NQ];
      double Ne[NQ][3];
      uint32_t bw[NQ];
      bw[0] = bwn;
#pragma unroll
      for (int q = 1; q < NQ; ++q) bw[q] = (uint32_t)pblk[(z + q) * a.P + col];
      if (z + NQ < z1) bwn = (uint32_t)pblk[(z + NQ) * a.P + col];
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int r0 = (z + q) * D + cb, ub = (z + q) * D + col * 128;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          Nw[q][k] = bload2(xr, r0 + a.anchor[6 + k] + oor[k]);
          Ne[q][k] = bload1(xr, ub + ebe + a.anchor[6 + k] + oor[k]);
        }
        if constexpr (RU) rq[q] = __builtin_nontemporal_load(reinterpret_cast<const dbl2 *>(rin + r0));
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        dbl2 L[9];
        double e[9];
#pragma unroll
        for (int r = 0; r < 6; ++r) { L[r] = C[r]; e[r] = Ce[r]; }
#pragma unroll
        for (int k = 0; k < 3; ++k) { L[6 + k] = Nw[q][k]; e[6 + k] = Ne[q][k]; }
        const int r0 = (z + q) * D + cb;
        if constexpr (SYM) {                             // PW on a symmetric operator: forward half
          static_assert(MODE == SPMV_PW && FORM == 2 && !SPLIT, "symmetric p.Ap pass only");
          const dbl2 t = pair_fwd27<UV>(L, e, bw[q], puni);
          dot += L[4].x * t.x;
          dot += L[4].y * t.y;
        } else if constexpr (RU) {
          const dbl2 sv = pair_sums27<FORM, UV>(L, e, bw[q], puni, lane);
          const double ra = fma(-alpha, sv.x, rq[q].x), rb = fma(-alpha, sv.y, rq[q].y);
          const double za = JM == 2 ? ra * ru.c : ra, zb = JM == 2 ? rb * ru.c : rb;
          nv[0] += za * za; nv[1] += za * ra; nv[2] += ra * ra;
          nv[0] += zb * zb; nv[1] += zb * rb; nv[2] += rb * rb;
          *reinterpret_cast<dbl2 *>(ru.r + r0) = dbl2{ra, rb};
        } else {
          const dbl2 sv = pair_sums27<FORM, UV>(L, e, bw[q], puni, lane);
          if constexpr (MODE != SPMV_PW) *reinterpret_cast<dbl2 *>(y + r0) = sv;
          if constexpr (MODE == SPMV_DOT || MODE == SPMV_PW) {
            const bool gh = SPLIT && (bw[q] & (lane < 32 ? PBLK_GHOST_LO : PBLK_GHOST_HI)) != 0;
            if (!gh) {
              dot += L[4].x * sv.x;
              dot += L[4].y * sv.y;
            }
          }
        }
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          C[k] = C[3 + k]; Ce[k] = Ce[3 + k];
          C[3 + k] = Nw[q][k]; Ce[3 + k] = Ne[q][k];
        }
      }
    };
    int z = z0;
    for (; z + ZU <= z1; z += ZU) step(z, std::integral_constant<int, ZU>{});
    for (; z < z1; ++z) step(z, std::integral_constant<int, 1>{});
  }
  if constexpr (MODE == SPMV_DOT || MODE == SPMV_PW) {
    double v[1] = {dot};
    block_partials<1>(v, a.partials, gridDim.x, a.fold);
  } else if constexpr (RU) {
    block_partials<3>(nv, a.partials, gridDim.x, a.fold);
  }
}


// Plane-pipelined 27-point z-march (column-word form, knob 60).  A unit's 27
// slots are three dz groups of nine (plane z-1, z, z+1), summed in slot
// order; so when a wave loads plane q it advances three units at once: it
// finishes unit q-1 (its dz = +1 group), continues unit q (dz = 0) and starts
// unit q+1 (dz = -1), each with its own dictionary block's nine values.  What
// crosses a step is two running row sums and the centre pair (12 VGPRs)
// instead of six operand pairs and their edges (36), and each plane's +-1
// neighbours take one pair of wave shifts per run instead of three.  The
// same operations in the same order as spmv_pair_zm27_kernel: the same bits.
struct Plane27 { dbl2 L[3]; double lo[3], hi[3]; };

template <bool UV>
__device__ __forceinline__ dbl2 plane27_add(dbl2 s, const PairUni27 &B, int g, const Plane27 &P) {
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const double a0[3] = {P.lo[k], P.L[k].x, P.L[k].y}, a1[3] = {P.L[k].x, P.L[k].y, P.hi[k]};
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      const int j = 9 * g + 3 * k + p;
      const double v = B.v[j];
      if (UV && j != 13) {
        s.x = __builtin_fma(v, a0[p], s.x);
        s.y = __builtin_fma(v, a1[p], s.y);
      } else {
        s.x = s.x + v * a0[p];
        s.y = s.y + v * a1[p];
      }
    }
  }
  return s;
}

template <int MODE, bool SPLIT, bool UV, int JM = 0>
__global__ void __launch_bounds__(256) spmv_pair_zm27p_kernel(const PairLean27Args a, const double *__restrict__ x,
                                                              double *__restrict__ y, const int32_t *__restrict__ pblk,
                                                              const PairUni27 *__restrict__ puni,
                                                              const int32_t *__restrict__ pcol, const PairRuArgs ru) {
  constexpr bool RU = MODE == SPMV_RUPD;
  static_assert(!SPLIT || (MODE != SPMV_PW && !RU), "27-point mode 5: one rank");
  double alpha = 0.0;
  const double *rin = nullptr;
  if constexpr (RU) {
    KspState *s = ru.s;
    if (s->top.done) {
      if (ru.hw && blockIdx.x == 0 && threadIdx.x == 0) host_store(ru.hw + HW_DONE, 1);
      return;
    }
    const double pw = ru.ndot > 0 ? block_sum_array<16>(ru.dot_part, ru.ndot) : s->red1;
    const CgAlpha al = cg_alpha(s, pw);
    if (blockIdx.x == 0 && threadIdx.x == 0) cg_commit_alpha(s, al, pw, ru.xb, false, ru.hw);
    if (al.reason) return;
    alpha = al.alpha;
    rin = (ru.r0 && al.i == 0) ? ru.r0 : ru.r;
  } else {
    if (a.done && *a.done) return;   // wave-uniform: solver finished
  }
  double nv[3] = {0.0, 0.0, 0.0};   // RU: [z.z, z.r, r.r]
  double dot = 0.0;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int sb, se, W, w;
  if ((gridDim.x & 7) == 0) {
    const int xcd = blockIdx.x & 7;
    W = (gridDim.x >> 3) * LEAN_WAVES;
    w = (blockIdx.x >> 3) * LEAN_WAVES + wid;
    sb = a.S * xcd / 8;
    se = a.S * (xcd + 1) / 8;
  } else {
    W = gridDim.x * LEAN_WAVES;
    w = blockIdx.x * LEAN_WAVES + wid;
    sb = 0;
    se = a.S;
  }
  const __amdgpu_buffer_rsrc_t xr = vec_rsrc(x, a.n);
  const int D = a.anchor[7];
  const int eb = lane == 0 ? -1 : 128;                   // edge: lane 0 x[ub + c - 1], others x[ub + 128 + c]
  const int ntask = (se - sb) * a.P;
  for (int t = w; t < ntask; t += W) {
    const int seg = sb + t / a.P, col = t % a.P;
    const int z0 = seg * a.L, z1 = min(z0 + a.L, a.NZ);
    const int cb = col * 128 + 2 * lane;
    // the column's empty dy runs and x-line edges read out of range (form 2)
    const uint32_t cw = (uint32_t)pcol[col];
    const int oor[3] = {(cw & U27C_YLO) ? PAIR_OOR : 0, 0, (cw & U27C_YHI) ? PAIR_OOR : 0};
    const int ebe = eb + ((lane == 0 ? (cw & U27_ELO) : (cw & U27_EHI)) ? PAIR_OOR_EDGE : 0);
    // plane q's three dy runs (anchors 3..5: -n, 0, +n within the plane), their edges and shifts
    auto load = [&](int q, Plane27 &P, double (&e)[3]) __attribute__((always_inline)) {
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        P.L[k] = bload2(xr, q * D + cb + a.anchor[3 + k] + oor[k]);
        e[k] = bload1(xr, q * D + col * 128 + ebe + a.anchor[3 + k] + oor[k]);
      }
    };
    auto shift = [&](Plane27 &P, const double (&e)[3]) __attribute__((always_inline)) {
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        P.lo[k] = wave_shift<true>(P.L[k].y, e[k]);      // x[r0 + c - 1]
        P.hi[k] = wave_shift<false>(P.L[k].x, e[k]);     // x[r0 + c + 2]
      }
    };
    auto blk = [&](int z) -> uint32_t { return (uint32_t)pblk[min(z, a.NZ - 1) * a.P + col]; };
    uint32_t bz = blk(z0), bz1 = blk(z0 + 1);
    Plane27 P;
    double e[3];
    // prologue: plane z0 - 1 starts unit z0, plane z0 continues it and starts z0 + 1
    load(z0 - 1, P, e);
    shift(P, e);
    dbl2 m1 = plane27_add<UV>(dbl2{0.0, 0.0}, puni[bz & PBLK_ID], 0, P);
    load(z0, P, e);
    shift(P, e);
    m1 = plane27_add<UV>(m1, puni[bz & PBLK_ID], 1, P);
    dbl2 m0 = plane27_add<UV>(dbl2{0.0, 0.0}, puni[bz1 & PBLK_ID], 0, P);
    dbl2 cz = P.L[1];                                    // unit z0's own rows
    for (int z = z0; z < z1; ++z) {
      const uint32_t bz2 = blk(z + 2);                   // (past the last plane: a stand-in, never emitted)
      const int r0 = z * D + cb;
      dbl2 rq;
      load(z + 1, P, e);
      if constexpr (RU) rq = __builtin_nontemporal_load(reinterpret_cast<const dbl2 *>(rin + r0));
      shift(P, e);
      // one block's nine values live at a time (the barriers keep the three
      // groups' scalar loads from being hoisted together: 54 SGPRs spilled)
      const dbl2 out = plane27_add<UV>(m1, puni[bz & PBLK_ID], 2, P);   // unit z finished
      __builtin_amdgcn_sched_barrier(0);
      m1 = plane27_add<UV>(m0, puni[bz1 & PBLK_ID], 1, P);              // unit z + 1: 18 slots
      __builtin_amdgcn_sched_barrier(0);
      m0 = plane27_add<UV>(dbl2{0.0, 0.0}, puni[bz2 & PBLK_ID], 0, P);  // unit z + 2: 9 slots
      if constexpr (RU) {
        const double ra = fma(-alpha, out.x, rq.x), rb = fma(-alpha, out.y, rq.y);
        const double za = JM == 2 ? ra * ru.c : ra, zb = JM == 2 ? rb * ru.c : rb;
        nv[0] += za * za; nv[1] += za * ra; nv[2] += ra * ra;
        nv[0] += zb * zb; nv[1] += zb * rb; nv[2] += rb * rb;
        *reinterpret_cast<dbl2 *>(ru.r + r0) = dbl2{ra, rb};
      } else {
        if constexpr (MODE != SPMV_PW) *reinterpret_cast<dbl2 *>(y + r0) = out;
        if constexpr (MODE == SPMV_DOT || MODE == SPMV_PW) {
          const bool gh = SPLIT && (bz & (lane < 32 ? PBLK_GHOST_LO : PBLK_GHOST_HI)) != 0;
          if (!gh) {
            dot += cz.x * out.x;
            dot += cz.y * out.y;
          }
        }
      }
      cz = P.L[1];
      bz = bz1;
      bz1 = bz2;
    }
  }
  if constexpr (MODE == SPMV_DOT || MODE == SPMV_PW) {
    double v[1] = {dot};
    block_partials<1>(v, a.partials, gridDim.x, a.fold);
  } else if constexpr (RU) {
    block_partials<3>(nv, a.partials, gridDim.x, a.fold);
  }
}

// The plane-pipelined 27-point z-march with two lines per wave (knob 70,
// Sell::pair_2l27): a task is the columns of lines y and y + 1 (y even) at
// one x, marched together; line y's dy = +1 run is line y + 1's centre run
// and line y + 1's dy = -1 run line y's, so per plane the pair loads four
// lines (y - 1 .. y + 2) and their edges -- 8 loads for two units instead of
// 12 -- and shifts them once.  Each unit sums its rows exactly as
// spmv_pair_zm27p_kernel does (plane27_add, the same groups in the same
// order): the same row sums.  DOT / PW / RUPD partials then group other rows
// per wave (to rounding).
template <int MODE, bool UV, int JM = 0, bool XC = false>
__global__ void __launch_bounds__(256) spmv_pair_zm27p2l_kernel(const PairLean27Args a, const double *__restrict__ x,
                                                                double *__restrict__ y, const int32_t *__restrict__ pblk,
                                                                const PairUni27 *__restrict__ puni,
                                                                const int32_t *__restrict__ pcol, const PairRuArgs ru) {
  constexpr bool RU = MODE == SPMV_RUPD;
  double alpha = 0.0;
  const double *rin = nullptr;
  if constexpr (RU) {
    KspState *s = ru.s;
    if (s->top.done) {
      if (ru.hw && blockIdx.x == 0 && threadIdx.x == 0) host_store(ru.hw + HW_DONE, 1);
      return;
    }
    const double pw = ru.ndot > 0 ? block_sum_array<16>(ru.dot_part, ru.ndot) : s->red1;
    const CgAlpha al = cg_alpha(s, pw);
    if (blockIdx.x == 0 && threadIdx.x == 0) cg_commit_alpha(s, al, pw, ru.xb, false, ru.hw);
    if (al.reason) return;
    alpha = al.alpha;
    rin = (ru.r0 && al.i == 0) ? ru.r0 : ru.r;
  } else {
    if (a.done && *a.done) return;   // wave-uniform: solver finished
  }
  // alpha and the Jacobi scalar held in VGPRs (an empty asm pins them there):
  // the SGPRs they would keep live across the march spilled
  double alv = alpha, cjv = ru.c;
  if constexpr (RU) asm volatile("" : "+v"(alv), "+v"(cjv));
  double nv[3] = {0.0, 0.0, 0.0};   // RU: [z.z, z.r, r.r]
  double dot = 0.0;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int sb, se, W, w;
  const __amdgpu_buffer_rsrc_t xr = vec_rsrc(x, a.n);
  const int D = a.anchor[7], NL = a.anchor[5];           // plane, line
  const int PL = NL / 128;
  const int eb = lane == 0 ? -1 : 128;
  // task t = (segment, line pair lp, x column xx), cp = lp PL + xx: advanced
  // by W without divisions in the loop (their reciprocals spilled SGPRs).
  // XC (knob 74, grid a multiple of 8): the XCD owns line pairs [lpb, lpb +
  // NLP) of every plane (segments of L planes, all of them) instead of a slab
  // of planes; lp then counts from lpb
  int NLP = a.P / 2 / PL, lpb = 0;
  if constexpr (XC) {
    const int xcd = blockIdx.x & 7, nall = NLP;
    W = (gridDim.x >> 3) * LEAN_WAVES;
    w = (blockIdx.x >> 3) * LEAN_WAVES + wid;
    lpb = nall * xcd / 8;
    NLP = nall * (xcd + 1) / 8 - lpb;
    sb = 0;
    se = a.S;
  } else if ((gridDim.x & 7) == 0) {
    const int xcd = blockIdx.x & 7;
    W = (gridDim.x >> 3) * LEAN_WAVES;
    w = (blockIdx.x >> 3) * LEAN_WAVES + wid;
    sb = a.S * xcd / 8;
    se = a.S * (xcd + 1) / 8;
  } else {
    W = gridDim.x * LEAN_WAVES;
    w = blockIdx.x * LEAN_WAVES + wid;
    sb = 0;
    se = a.S;
  }
  const int PH = NLP * PL;
  int lpbv = lpb;
  if constexpr (XC) asm volatile("" : "+v"(lpbv));
  int seg = sb + w / PH, lp = (w % PH) / PL, xx = w % PL;
  const int dseg = W / PH, dlp = (W % PH) / PL, dx = W % PL;
  for (; seg < se;) {
    // XC: lpb lives in a VGPR across the march (one SGPR fewer: the kernel
    // sits at the SGPR bound), the task's column read back to a scalar
    const int colA = XC ? __builtin_amdgcn_readfirstlane((lpbv + lp) * 2 * PL + xx) : lp * 2 * PL + xx;
    const int colB = colA + PL;
    const int z0 = seg * a.L, z1 = min(z0 + a.L, a.NZ);
    const int cbA = colA * 128 + 2 * lane;               // line y's rows; line y + 1's are + NL
    const uint32_t cwA = (uint32_t)pcol[colA], cwB = (uint32_t)pcol[colB];
    // the four lines y - 1 .. y + 2: the outer two read out of range at a y
    // boundary (per lane: the task's rows and edge offsets in VGPRs)
    const int oA = cbA - NL + ((cwA & U27C_YLO) ? PAIR_OOR : 0), oB = cbA + 2 * NL + ((cwB & U27C_YHI) ? PAIR_OOR : 0);
    const int eA = colA * 128 + eb + ((lane == 0 ? (cwA & U27_ELO) : (cwA & U27_EHI)) ? PAIR_OOR_EDGE : 0);
    const int eo[4] = {eA - NL + ((cwA & U27C_YLO) ? PAIR_OOR : 0), eA, eA + NL, eA + 2 * NL + ((cwB & U27C_YHI) ? PAIR_OOR : 0)};
    const int lo4[4] = {oA, cbA, cbA + NL, oB};
    dbl2 Lq[4];
    double lo[4], hi[4];
    auto fetch = [&](int q, dbl2 (&Lr)[4], double (&er)[4]) __attribute__((always_inline)) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        Lr[k] = bload2(xr, q * D + lo4[k]);
        er[k] = bload1(xr, q * D + eo[k]);
      }
    };
    auto shift = [&](const double (&er)[4]) __attribute__((always_inline)) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        lo[k] = wave_shift<true>(Lq[k].y, er[k]);
        hi[k] = wave_shift<false>(Lq[k].x, er[k]);
      }
    };
    auto load = [&](int q) __attribute__((always_inline)) {
      double e[4];
      fetch(q, Lq, e);
      shift(e);
    };
    auto plane = [&](int k0) __attribute__((always_inline)) {   // lines k0 .. k0 + 2 as one unit's plane
      Plane27 P;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        P.L[k] = Lq[k0 + k];
        P.lo[k] = lo[k0 + k];
        P.hi[k] = hi[k0 + k];
      }
      return P;
    };
    auto blkA = [&](int z) -> uint32_t { return (uint32_t)pblk[min(z, a.NZ - 1) * a.P + colA]; };
    auto blkB = [&](int z) -> uint32_t { return (uint32_t)pblk[min(z, a.NZ - 1) * a.P + colB]; };
    uint32_t az = blkA(z0), az1 = blkA(z0 + 1), bz = blkB(z0), bz1 = blkB(z0 + 1);
    load(z0 - 1);
    dbl2 m1A = plane27_add<UV>(dbl2{0.0, 0.0}, puni[az & PBLK_ID], 0, plane(0));
    dbl2 m1B = plane27_add<UV>(dbl2{0.0, 0.0}, puni[bz & PBLK_ID], 0, plane(1));
    load(z0);
    m1A = plane27_add<UV>(m1A, puni[az & PBLK_ID], 1, plane(0));
    m1B = plane27_add<UV>(m1B, puni[bz & PBLK_ID], 1, plane(1));
    dbl2 m0A = plane27_add<UV>(dbl2{0.0, 0.0}, puni[az1 & PBLK_ID], 0, plane(0));
    dbl2 m0B = plane27_add<UV>(dbl2{0.0, 0.0}, puni[bz1 & PBLK_ID], 0, plane(1));
    dbl2 czA = Lq[1], czB = Lq[2];
    for (int z = z0; z < z1; ++z) {
      const uint32_t az2 = blkA(z + 2), bz2 = blkB(z + 2);
      const int rA = z * D + cbA, rB = rA + NL;
      dbl2 rqA{0.0, 0.0}, rqB{0.0, 0.0};   // read only by the residual update
      load(z + 1);
      if constexpr (RU) {
        rqA = __builtin_nontemporal_load(reinterpret_cast<const dbl2 *>(rin + rA));
        rqB = __builtin_nontemporal_load(reinterpret_cast<const dbl2 *>(rin + rB));
      }
      const dbl2 outA = plane27_add<UV>(m1A, puni[az & PBLK_ID], 2, plane(0));
      __builtin_amdgcn_sched_barrier(0);
      const dbl2 outB = plane27_add<UV>(m1B, puni[bz & PBLK_ID], 2, plane(1));
      __builtin_amdgcn_sched_barrier(0);
      m1A = plane27_add<UV>(m0A, puni[az1 & PBLK_ID], 1, plane(0));
      __builtin_amdgcn_sched_barrier(0);
      m1B = plane27_add<UV>(m0B, puni[bz1 & PBLK_ID], 1, plane(1));
      __builtin_amdgcn_sched_barrier(0);
      m0A = plane27_add<UV>(dbl2{0.0, 0.0}, puni[az2 & PBLK_ID], 0, plane(0));
      __builtin_amdgcn_sched_barrier(0);
      m0B = plane27_add<UV>(dbl2{0.0, 0.0}, puni[bz2 & PBLK_ID], 0, plane(1));
      auto emit = [&](dbl2 out, dbl2 cz, dbl2 rq, int r0) __attribute__((always_inline)) {
        if constexpr (RU) {
          const double ra = fma(-alv, out.x, rq.x), rb = fma(-alv, out.y, rq.y);
          const double za = JM == 2 ? ra * cjv : ra, zb = JM == 2 ? rb * cjv : rb;
          nv[0] += za * za; nv[1] += za * ra; nv[2] += ra * ra;
          nv[0] += zb * zb; nv[1] += zb * rb; nv[2] += rb * rb;
          *reinterpret_cast<dbl2 *>(ru.r + r0) = dbl2{ra, rb};
        } else {
          if constexpr (MODE != SPMV_PW) *reinterpret_cast<dbl2 *>(y + r0) = out;
          if constexpr (MODE == SPMV_DOT || MODE == SPMV_PW) {
            dot += cz.x * out.x;
            dot += cz.y * out.y;
          }
        }
      };
      emit(outA, czA, rqA, rA);
      emit(outB, czB, rqB, rB);
      czA = Lq[1];
      czB = Lq[2];
      az = az1; az1 = az2;
      bz = bz1; bz1 = bz2;
    }
    xx += dx;
    if (xx >= PL) { xx -= PL; ++lp; }
    lp += dlp;
    if (lp >= NLP) { lp -= NLP; ++seg; }
    seg += dseg;
  }
  if constexpr (MODE == SPMV_DOT || MODE == SPMV_PW) {
    double v[1] = {dot};
    block_partials<1>(v, a.partials, gridDim.x, a.fold);
  } else if constexpr (RU) {
    block_partials<3>(nv, a.partials, gridDim.x, a.fold);
  }
}

// CG mode 5's p.Ap pass on a symmetric 27-point operator (pair_fwd27, the
// forward half) with two lines per wave (knob 70): a row's forward slots read
// its own plane's lines y and y + 1 and the next plane's y - 1 .. y + 1, so
// for lines y and y + 1 together a plane step loads the next plane's four
// lines y - 1 .. y + 2 and their edges (8 loads for two units instead of 12)
// and carries three.  Each row's t_i is pair_fwd27's, bit for bit; the p.Ap
// partials group other rows per wave (to rounding).
// G lines per wave (knob 70 = 2: G = 4, Sell::pair_4l27): the next plane's
// G + 2 lines per step, G + 1 carried.
template <bool UV, int G = 2, bool XC = false>
__global__ void __launch_bounds__(256) spmv_pair_zm27s2l_kernel(const PairLean27Args a, const double *__restrict__ x,
                                                                const int32_t *__restrict__ pblk,
                                                                const PairUni27 *__restrict__ puni,
                                                                const int32_t *__restrict__ pcol) {
  if (a.done && *a.done) return;   // wave-uniform: solver finished
  double dot = 0.0;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int sb, se, W, w;
  if ((gridDim.x & 7) == 0) {
    const int xcd = blockIdx.x & 7;
    W = (gridDim.x >> 3) * LEAN_WAVES;
    w = (blockIdx.x >> 3) * LEAN_WAVES + wid;
    sb = a.S * xcd / 8;
    se = a.S * (xcd + 1) / 8;
  } else {
    W = gridDim.x * LEAN_WAVES;
    w = blockIdx.x * LEAN_WAVES + wid;
    sb = 0;
    se = a.S;
  }
  const __amdgpu_buffer_rsrc_t xr = vec_rsrc(x, a.n);
  const int D = a.anchor[7], NL = a.anchor[5];
  const int PL = NL / 128;
  int NLP = a.P / G / PL, lpb = 0;
  if (XC) {                                                // the XCD owns line groups, not planes (knob 74)
    const int xcd = blockIdx.x & 7, nall = NLP;
    lpb = nall * xcd / 8;
    NLP = nall * (xcd + 1) / 8 - lpb;
    sb = 0;
    se = a.S;
  }
  const int PH = NLP * PL;
  const int eb = lane == 0 ? -1 : 128;
  int seg = sb + w / PH, lp = (w % PH) / PL, xx = w % PL;
  const int dseg = W / PH, dlp = (W % PH) / PL, dx = W % PL;
  for (; seg < se;) {
    const int colA = (XC ? lpb + lp : lp) * G * PL + xx;   // line y's column; line y + k's is + k PL
    const int z0 = seg * a.L, z1 = min(z0 + a.L, a.NZ);
    const int cbA = colA * 128 + 2 * lane;
    const uint32_t cwA = (uint32_t)pcol[colA], cwZ = (uint32_t)pcol[colA + (G - 1) * PL];
    const int eA = colA * 128 + eb + ((lane == 0 ? (cwA & U27_ELO) : (cwA & U27_EHI)) ? PAIR_OOR_EDGE : 0);
    const int oM = (cwA & U27C_YLO) ? PAIR_OOR : 0, oP = (cwZ & U27C_YHI) ? PAIR_OOR : 0;
    // line y - 1 + k, k = 0 .. G + 1
    auto lof = [&](int k) { return cbA + (k - 1) * NL + (k == 0 ? oM : k == G + 1 ? oP : 0); };
    auto eof = [&](int k) { return eA + (k - 1) * NL + (k == 0 ? oM : k == G + 1 ? oP : 0); };
    // plane z's lines y .. y + G (carried)
    dbl2 C[G + 1];
    double Ce[G + 1];
#pragma unroll
    for (int k = 0; k <= G; ++k) {
      C[k] = bload2(xr, z0 * D + lof(k + 1));
      Ce[k] = bload1(xr, z0 * D + eof(k + 1));
    }
    auto fetch = [&](int q, dbl2 (&Lr)[G + 2], double (&er)[G + 2]) __attribute__((always_inline)) {
#pragma unroll
      for (int k = 0; k < G + 2; ++k) {
        Lr[k] = bload2(xr, q * D + lof(k));
        er[k] = bload1(xr, q * D + eof(k));
      }
    };
    for (int z = z0; z < z1; ++z) {
      uint32_t bw[G];
#pragma unroll
      for (int u = 0; u < G; ++u) bw[u] = (uint32_t)pblk[z * a.P + colA + u * PL];
      dbl2 N[G + 2];
      double Ne[G + 2];
      fetch(z + 1, N, Ne);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < G; ++u) {
        dbl2 L[9];
        double e[9];
        L[4] = C[u]; e[4] = Ce[u]; L[5] = C[u + 1]; e[5] = Ce[u + 1];
        L[6] = N[u]; e[6] = Ne[u]; L[7] = N[u + 1]; e[7] = Ne[u + 1]; L[8] = N[u + 2]; e[8] = Ne[u + 2];
        const dbl2 t = pair_fwd27<UV>(L, e, bw[u], puni);
        dot += L[4].x * t.x;
        dot += L[4].y * t.y;
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int k = 0; k <= G; ++k) { C[k] = N[k + 1]; Ce[k] = Ne[k + 1]; }
    }
    xx += dx;
    if (xx >= PL) { xx -= PL; ++lp; }
    lp += dlp;
    if (lp >= NLP) { lp -= NLP; ++seg; }
    seg += dseg;
  }
  double v[1] = {dot};
  block_partials<1>(v, a.partials, gridDim.x, a.fold);
}

// fp64 row pairs (Sell::pval, uncoded 5/7-point layouts whose every unit is
// select-free): the z-march with the unit's values streamed (K 16-byte pairs
// per lane, non-temporal) instead of a dictionary block's uniform values.
// Absent slots hold 0.0 and read a 0.0 operand (the flags in Sell::pflag:
// inner runs and edges by out-of-range reads, carried runs zeroed at use), so
// sum + 0.0 * 0.0 = sum.  SPLIT: units with A_o entries (PBLK_GHOST_* in
// the flag word) keep their rows' p.y terms for the boundary kernel.
template <int MODE, int PS, int ZU, bool SPLIT>
__global__ void __launch_bounds__(256) spmv_pair_zmf64_kernel(const PairLeanArgs a, const double *__restrict__ x,
                                                              double *__restrict__ y, const int32_t *__restrict__ pflag,
                                                              const double *__restrict__ pval) {
  if (a.done && *a.done) return;   // wave-uniform: solver finished
  using SH = PairShape<PS>;
  constexpr int K = SH::K, NR = SH::NR, C = SH::CENTER_RUN, TR = PS == 5 ? 1 : 2, LAST = NR - 1;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int sb, se, W, w;
  if ((gridDim.x & 7) == 0) {
    const int xcd = blockIdx.x & 7;
    W = (gridDim.x >> 3) * LEAN_WAVES;
    w = (blockIdx.x >> 3) * LEAN_WAVES + wid;
    sb = a.S * xcd / 8;
    se = a.S * (xcd + 1) / 8;
  } else {
    W = gridDim.x * LEAN_WAVES;
    w = blockIdx.x * LEAN_WAVES + wid;
    sb = 0;
    se = a.S;
  }
  const __amdgpu_buffer_rsrc_t xr = vec_rsrc(x, a.n);
  const int D = a.anchor[LAST];
  const int ecst = lane == 0 ? a.anchor[TR] - 1 : 128 + a.anchor[TR];
  constexpr uint32_t CARRY = PBLK_RUN0 | (PBLK_RUN0 << TR) | (PBLK_RUN0 << LAST);
  const dbl2 *__restrict__ pv = reinterpret_cast<const dbl2 *>(pval) + lane;
  double dot = 0.0;
  const int ntask = (se - sb) * a.P;
  for (int t = w; t < ntask; t += W) {
    const int seg = sb + t / a.P, col = t % a.P;
    const int z0 = seg * a.L, z1 = min(z0 + a.L, a.NZ);
    const int cb = col * 128 + 2 * lane;
    dbl2 zm = bload2(xr, z0 * D + cb - D), c = bload2(xr, z0 * D + cb);
    uint32_t fn = (uint32_t)pflag[z0 * a.P + col];
    auto step = [&](int z, auto nq) __attribute__((always_inline)) {
      constexpr int NQ = decltype(nq)::value;
      dbl2 L[NQ][NR], zp[NQ], V[NQ][K];
      double e[NQ];
      uint32_t fl[NQ];
      fl[0] = fn;
#pragma unroll
      for (int q = 1; q < NQ; ++q) fl[q] = (uint32_t)pflag[(z + q) * a.P + col];
      if (z + NQ < z1) fn = (uint32_t)pflag[(z + NQ) * a.P + col];
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int u = (z + q) * a.P + col;
        const int r0 = (z + q) * D + cb, ub = (z + q) * D + col * 128;
        zp[q] = bload2(xr, r0 + D);
#pragma unroll
        for (int r = 1; r < LAST; ++r)
          if (r != TR) L[q][r] = bload2(xr, r0 + a.anchor[r] + ((fl[q] & (PBLK_RUN0 << r)) ? PAIR_OOR : 0));
        const int eo = ecst + (lane == 0 ? ((fl[q] & PBLK_ELO) ? PAIR_OOR : 0) : ((fl[q] & PBLK_EHI) ? PAIR_OOR : 0));
        e[q] = bload1(xr, ub + eo);
#pragma unroll
        for (int j = 0; j < K; ++j) V[q][j] = __builtin_nontemporal_load(pv + ((int64_t)u * K + j) * 64);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        L[q][0] = q == 0 ? zm : q == 1 ? c : zp[q - 2];
        L[q][TR] = q == 0 ? c : zp[q - 1];
        L[q][LAST] = zp[q];
        if (fl[q] & CARRY) {                       // wave-uniform, rare: an empty carried run
          if (fl[q] & PBLK_RUN0) L[q][0] = dbl2{0.0, 0.0};
          if (fl[q] & (PBLK_RUN0 << TR)) L[q][TR] = dbl2{0.0, 0.0};
          if (fl[q] & (PBLK_RUN0 << LAST)) L[q][LAST] = dbl2{0.0, 0.0};
        }
        const int r0 = (z + q) * D + cb;
        double s0v = 0.0, s1v = 0.0, lo = 0.0, hi = 0.0;
#pragma unroll
        for (int j = 0; j < K; ++j) {
          const int r = SH::run(j), p = SH::pos(j);
          if (SH::tri(r) && p < 0) {
            lo = wave_shift<true>(L[q][r].y, e[q]);
            hi = wave_shift<false>(L[q][r].x, e[q]);
          }
          double a0, a1;
          if (!SH::tri(r)) { a0 = L[q][r].x; a1 = L[q][r].y; }
          else if (p < 0) { a0 = lo; a1 = L[q][r].x; }
          else if (p == 0) { a0 = L[q][r].x; a1 = L[q][r].y; }
          else { a0 = L[q][r].y; a1 = hi; }
          s0v = s0v + V[q][j].x * a0;
          s1v = s1v + V[q][j].y * a1;
        }
        *reinterpret_cast<dbl2 *>(y + r0) = dbl2{s0v, s1v};
        if constexpr (MODE == SPMV_DOT) {
          // SPLIT: rows with A_o entries stored their diagonal-block sum; the
          // boundary kernel continues them and adds their p.y terms
          const bool gh = SPLIT && (fl[q] & (lane < 32 ? PBLK_GHOST_LO : PBLK_GHOST_HI)) != 0;
          if (!gh) {
            dot += L[q][C].x * s0v;
            dot += L[q][C].y * s1v;
          }
        }
      }
      if constexpr (NQ == 1) zm = c;
      else zm = zp[NQ - 2];
      c = zp[NQ - 1];
    };
    int z = z0;
    for (; z + ZU <= z1; z += ZU) step(z, std::integral_constant<int, ZU>{});
    for (; z < z1; ++z) step(z, std::integral_constant<int, 1>{});
  }
  if constexpr (MODE == SPMV_DOT) {
    double v[1] = {dot};
    block_partials<1>(v, a.partials, gridDim.x, a.fold);
  }
}

// Coded z-march (Sell::pair_code_clean): spmv_pair_zm_kernel's march for
// 5/7-point layouts whose dictionary blocks are not uniform per slot-row --
// variable coefficients with few distinct values, e.g. BASELINE C4's
// convection-diffusion operator (10 values, period 4 in x: a slot's value
// differs between lanes).  Per unit: one 16-byte code load per lane from the
// L2-resident dictionary (pcode block pblk[u] & PBLK_ID), the values from the
// LDS table (the absent code's entry is 0.0, and the clean flags' out-of-range
// reads make an absent slot's operand 0.0: sum + 0.0 * 0.0 = sum, no presence
// select), and for the Jacobi modes dinv from dtab by the diagonal slot's code
// (the Jacobi setup's division per code: the same bits as the dinv vector).
// Modes: PLAIN, DOT, JACOBI, and GMRES's PLAIN_S / JACOBI_S -- the operand is
// fl(s * x) with s = *xscale (the basis vector kept unnormalised), formed
// once per loaded value and carried formed.  Each row sums its slots in
// ascending column order: the general kernel's bits (tests/test_gpu_vcodes.py).
struct PairCodeArgs {
  const uint8_t *pcode;        // the code dictionary (64 lanes x 16 bytes per block)
  const double *vtab, *dtab;   // [VCODE_MAX]: values (absent / unused: 0.0), 1 / value
  const double *xscale;        // *_S modes
  Jac jac;                     // JACOBI modes without dtab (DT = false)
};

template <int MODE, int PS, bool SPLIT, int ZU, bool DT>
__global__ void __launch_bounds__(256) spmv_pair_zmc_kernel(const PairLeanArgs a, const double *__restrict__ x,
                                                            double *__restrict__ y, const int32_t *__restrict__ pblk,
                                                            const PairCodeArgs ca) {
  if (a.done && *a.done) return;   // wave-uniform: solver finished
  __shared__ double vtab[VCODE_MAX];
  __shared__ double dtab[DT ? VCODE_MAX : 1];
  for (int i = threadIdx.x; i < VCODE_MAX; i += 256) {
    vtab[i] = ca.vtab[i];
    if constexpr (DT) dtab[i] = ca.dtab[i];
  }
  __syncthreads();
  constexpr bool SC = spmv_scaled(MODE), JAC = spmv_jac(MODE);
  const double xs = SC ? *ca.xscale : 1.0;
  using SH = PairShape<PS>;
  constexpr int K = SH::K, NR = SH::NR, C = SH::CENTER_RUN, TR = PS == 5 ? 1 : 2, LAST = NR - 1;
  constexpr int JC = SH::first(SH::CENTER_RUN) + 1;   // the diagonal slot
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int sb, se, W, w;
  if ((gridDim.x & 7) == 0) {
    const int xcd = blockIdx.x & 7;
    W = (gridDim.x >> 3) * LEAN_WAVES;
    w = (blockIdx.x >> 3) * LEAN_WAVES + wid;
    sb = a.S * xcd / 8;
    se = a.S * (xcd + 1) / 8;
  } else {
    W = gridDim.x * LEAN_WAVES;
    w = blockIdx.x * LEAN_WAVES + wid;
    sb = 0;
    se = a.S;
  }
  const __amdgpu_buffer_rsrc_t xr = vec_rsrc(x, a.n);
  const int D = a.anchor[LAST];
  const int ecst = lane == 0 ? a.anchor[TR] - 1 : 128 + a.anchor[TR];
  constexpr uint32_t CARRY = PBLK_RUN0 | (PBLK_RUN0 << TR) | (PBLK_RUN0 << LAST);
  auto scl = [&](dbl2 v) __attribute__((always_inline)) { return SC ? dbl2{xs * v.x, xs * v.y} : v; };
  const u32x4 *__restrict__ cd = reinterpret_cast<const u32x4 *>(ca.pcode) + lane;
  double dot = 0.0;
  const int ntask = (se - sb) * a.P;
  for (int t = w; t < ntask; t += W) {
    const int seg = sb + t / a.P, col = t % a.P;
    const int z0 = seg * a.L, z1 = min(z0 + a.L, a.NZ);
    const int cb = col * 128 + 2 * lane;
    dbl2 zm = scl(bload2(xr, z0 * D + cb - D)), c = scl(bload2(xr, z0 * D + cb));
    uint32_t bwn = (uint32_t)pblk[z0 * a.P + col];
    auto step = [&](int z, auto nq) __attribute__((always_inline)) {
      constexpr int NQ = decltype(nq)::value;
      dbl2 L[NQ][NR], zp[NQ];
      double e[NQ];
      u32x4 cw[NQ];
      uint32_t bw[NQ];
      bw[0] = bwn;
#pragma unroll
      for (int q = 1; q < NQ; ++q) bw[q] = (uint32_t)pblk[(z + q) * a.P + col];
      if (z + NQ < z1) bwn = (uint32_t)pblk[(z + NQ) * a.P + col];   // next step's, ahead
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int r0 = (z + q) * D + cb, ub = (z + q) * D + col * 128;
        zp[q] = bload2(xr, r0 + D);
#pragma unroll
        for (int r = 1; r < LAST; ++r)
          if (r != TR) L[q][r] = bload2(xr, r0 + a.anchor[r] + ((bw[q] & (PBLK_RUN0 << r)) ? PAIR_OOR : 0));
        const int eo = ecst + (lane == 0 ? ((bw[q] & PBLK_ELO) ? PAIR_OOR : 0) : ((bw[q] & PBLK_EHI) ? PAIR_OOR : 0));
        e[q] = bload1(xr, ub + eo);
        cw[q] = cd[(size_t)(bw[q] & PBLK_ID) * 64];
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        zp[q] = scl(zp[q]);
#pragma unroll
        for (int r = 1; r < LAST; ++r)
          if (r != TR) L[q][r] = scl(L[q][r]);
        if constexpr (SC) e[q] = xs * e[q];
      }
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        L[q][0] = q == 0 ? zm : q == 1 ? c : zp[q - 2];
        L[q][TR] = q == 0 ? c : zp[q - 1];
        L[q][LAST] = zp[q];
        if (bw[q] & CARRY) {                       // wave-uniform, rare: an empty carried run
          if (bw[q] & PBLK_RUN0) L[q][0] = dbl2{0.0, 0.0};
          if (bw[q] & (PBLK_RUN0 << TR)) L[q][TR] = dbl2{0.0, 0.0};
          if (bw[q] & (PBLK_RUN0 << LAST)) L[q][LAST] = dbl2{0.0, 0.0};
        }
        auto code = [&](int i) -> int { return (int)((cw[q][i >> 2] >> (8 * (i & 3))) & 0xffu); };
        const int r0 = (z + q) * D + cb;
        double s0v = 0.0, s1v = 0.0, lo = 0.0, hi = 0.0;
#pragma unroll
        for (int j = 0; j < K; ++j) {
          const int r = SH::run(j), p = SH::pos(j);
          if (SH::tri(r) && p < 0) {
            lo = wave_shift<true>(L[q][r].y, e[q]);
            hi = wave_shift<false>(L[q][r].x, e[q]);
          }
          double a0, a1;
          if (!SH::tri(r)) { a0 = L[q][r].x; a1 = L[q][r].y; }
          else if (p < 0) { a0 = lo; a1 = L[q][r].x; }
          else if (p == 0) { a0 = L[q][r].x; a1 = L[q][r].y; }
          else { a0 = L[q][r].y; a1 = hi; }
          s0v = s0v + vtab[code(j)] * a0;
          s1v = s1v + vtab[code(K + j)] * a1;
        }
        // SPLIT: rows with A_o entries store their diagonal-block sum; the
        // boundary kernel continues them and applies the epilogue
        const bool gh = SPLIT && (bw[q] & (lane < 32 ? PBLK_GHOST_LO : PBLK_GHOST_HI)) != 0;
        double o0 = s0v, o1 = s1v;
        if constexpr (JAC) {
          if (!gh) {
            if constexpr (DT) { o0 = s0v * dtab[code(JC)]; o1 = s1v * dtab[code(K + JC)]; }
            else { o0 = papply(ca.jac, s0v, r0); o1 = papply(ca.jac, s1v, r0 + 1); }
          }
        }
        *reinterpret_cast<dbl2 *>(y + r0) = dbl2{o0, o1};
        if constexpr (MODE == SPMV_DOT) {
          if (!gh) {
            dot += L[q][C].x * s0v;
            dot += L[q][C].y * s1v;
          }
        }
      }
      if constexpr (NQ == 1) zm = c;
      else zm = zp[NQ - 2];
      c = zp[NQ - 1];
    };
    int z = z0;
    for (; z + ZU <= z1; z += ZU) step(z, std::integral_constant<int, ZU>{});
    for (; z < z1; ++z) step(z, std::integral_constant<int, 1>{});
  }
  if constexpr (MODE == SPMV_DOT) {
    double v[1] = {dot};
    block_partials<1>(v, a.partials, gridDim.x, a.fold);
  }
}

using LeanFn = void (*)(PairLeanArgs, const double *, double *, const int32_t *, const PairUni *);
using ZmFn = void (*)(PairLeanArgs, const double *, double *, const int32_t *, const PairUni *, PairRuArgs);

// the layout side of the choice (mode and split aside): 0 none, 1 lean, 2 lean select-free
int pair_lean_kind(const Mat *A) {
  const Sell &S = A->sd;
  if (!g_knobs.pair_lean || !g_knobs.vcodes || !g_knobs.spmv_pairs || !g_knobs.pair_uni || g_knobs.spmv_ynt)
    return 0;
  if (S.pair_shape == 27) {    // the 27-point form exists as a z-march only
    if (S.ntab <= 0 || !S.puni27.p || S.pair_blocks <= 0 || !S.pair_all || !g_knobs.pair_zm) return 0;
    if (A->m % 128 != 0 || A->m >= PAIR_MAX_ROWS || A->n >= PAIR_MAX_ROWS || S.nunits * 128 != A->m) return 0;
    int an[9];
    for (int r = 0; r < 9; ++r) an[r] = S.pat_star_off[(size_t)(3 * r + 1)];
    const int D = an[7];
    if (D <= 0 || D % 128 != 0 || A->m % D != 0) return 0;
    for (int r = 0; r < 6; ++r)
      if (an[r + 3] - an[r] != D) return 0;
    return S.pair_clean27 ? 2 : 1;
  }
  if (S.ntab <= 0 || (S.pair_shape != 5 && S.pair_shape != 7) || !S.puni.p || S.pair_blocks <= 0 || !S.pair_all)
    return 0;
  if (A->m % 128 != 0 || A->m >= PAIR_MAX_ROWS || A->n >= PAIR_MAX_ROWS || S.nunits * 128 != A->m) return 0;
  return S.pair_clean && A->m <= PAIR_CLEAN_MAX_ROWS && A->n <= PAIR_CLEAN_MAX_ROWS ? 2 : 1;
}

// run r's anchor: the singleton's offset, or the tri run's centre slot
static void pair_anchors(const Sell &S, int anchor[5]) {
  const int ps = S.pair_shape;
  for (int r = 0; r < 5; ++r) {
    const bool tri = ps == 5 ? r == 1 : r == 2;
    const int first = ps == 5 ? (r == 0 ? 0 : r == 1 ? 1 : 4) : (r < 2 ? r : r == 2 ? 2 : r + 2);
    anchor[r] = (ps == 5 && r >= 3) ? 0 : S.pat_star_off[(size_t)(first + (tri ? 1 : 0))];
  }
}

// z-march: the outermost runs are -D, +D with D a multiple of 128 rows, m a multiple of D
bool pair_zm_applies(const Mat *A) {
  const Sell &S = A->sd;
  if (S.pair_shape == 27) return pair_lean_kind(A) > 0;   // its only form
  if (!g_knobs.pair_zm || (S.pair_shape != 5 && S.pair_shape != 7)) return false;
  int anchor[5];
  pair_anchors(S, anchor);
  const int D = anchor[S.pair_shape == 5 ? 2 : 4];
  return D > 0 && anchor[0] == -D && D % 128 == 0 && A->m % D == 0;
}

// the z-march geometry of a 5/7-point pattern given its run anchors (0: none)
static int zm_plane(const Mat *A, int ps, const int anchor[5]) {
  const int D = anchor[ps == 5 ? 2 : 4];
  return D > 0 && anchor[0] == -D && D % 128 == 0 && A->m % D == 0 ? D : 0;
}

// grid, segment length and segments of a z-march over NZ planes of P columns
static int zm_geom(int P, int NZ, int &L, int &S, int bpc) {
  int grid = std::max(8, bpc * device_cu_count());
  grid &= ~7;
  const int W = grid / 8 * LEAN_WAVES;               // waves per XCD
  const int slab = (NZ + 7) / 8;                      // planes per XCD
  L = std::min(std::max(1, g_knobs.pair_zm_len), slab);
  while (L > 1 && (int64_t)P * ((slab + L - 1) / L) < W) L = (L + 1) / 2;
  S = (NZ + L - 1) / L;
  return grid;
}

// Knob 65: the workgroups per CU (at most the requested, at least 2) whose
// z-march tasks fill the XCD's waves in whole rounds.  A wave takes tasks
// (segment, column) in turn, so T tasks over W waves take ceil(T / W) rounds
// and a partial last round idles the rest: C5's share (2,048 columns x one
// 8-plane segment per XCD) on 5 workgroups per CU gives 640 waves 3.2 tasks
// each -- four rounds, the last one a fifth full.
static int zm_tasks(int P, int NZ, int &L, int &S, int bpc = 0) {
  const int want = bpc > 0 ? bpc : g_knobs.pair_zm_bpc;
  if (!g_knobs.zm_balance) return zm_geom(P, NZ, L, S, want);
  int best = want;
  double best_eff = -1.0;
  for (int b = want; b >= std::min(2, want); --b) {
    int l, sg;
    const int grid = zm_geom(P, NZ, l, sg, b);
    const int64_t W = grid / 8 * LEAN_WAVES, T = (int64_t)P * ((sg + 7) / 8);
    const double eff = (double)T / (double)(W * ((T + W - 1) / W));
    if (eff > best_eff + 0.02) { best_eff = eff; best = b; }
  }
  return zm_geom(P, NZ, L, S, best);
}

// fp64 row-pair z-march (Sell::pval): uncoded 5/7-point layouts
int pair_f64_kind(const Mat *A) {
  const Sell &S = A->sd;
  if (!S.pair_f64 || !S.pval.p || !g_knobs.pair_lean || !g_knobs.pair_zm) return 0;
  int anchor[5] = {0, 0, 0, 0, 0};
  const int ps = S.pair_f64;
  for (int r = 0; r < (ps == 5 ? 3 : 5); ++r) {
    const bool tri = ps == 5 ? r == 1 : r == 2;
    const int first = ps == 5 ? (r == 0 ? 0 : r == 1 ? 1 : 4) : (r < 2 ? r : r == 2 ? 2 : r + 2);
    anchor[r] = S.pat_star_off[(size_t)(first + (tri ? 1 : 0))];
  }
  return zm_plane(A, ps, anchor) ? ps : 0;
}

static int pair_f64_launch(Mat *A, int mode, bool split, const double *x, double *y, double *partials,
                           const int *done, const Fold &fold_in, hipStream_t st) {
  const Sell &S = A->sd;
  const int ps = S.pair_f64;
  PairLeanArgs a{};
  a.m = (int)A->m;
  a.n = (int)A->n;
  a.nunits = (int)(A->m / 128);
  for (int r = 0; r < 5; ++r) {
    const bool tri = ps == 5 ? r == 1 : r == 2;
    const int first = ps == 5 ? (r == 0 ? 0 : r == 1 ? 1 : 4) : (r < 2 ? r : r == 2 ? 2 : r + 2);
    a.anchor[r] = (ps == 5 && r >= 3) ? 0 : S.pat_star_off[(size_t)(first + (tri ? 1 : 0))];
  }
  const int D = zm_plane(A, ps, a.anchor);
  a.P = D / 128;
  a.NZ = (int)(A->m / D);
  const int grid = zm_tasks(a.P, a.NZ, a.L, a.S);
  a.partials = partials;
  a.done = done;
  Fold fold = fold_in;
  if (fold.cnt) { fold.ntotal = fold.ncount = grid; fold.base = 0; }
  a.fold = fold;
  using F = void (*)(PairLeanArgs, const double *, double *, const int32_t *, const double *);
  F f;
  const bool z2 = g_knobs.pair_zm_units == 2;
#define F64K(MODE, PS) do { if (split) f = z2 ? &spmv_pair_zmf64_kernel<MODE, PS, 2, true> : &spmv_pair_zmf64_kernel<MODE, PS, 1, true>; \
                            else f = z2 ? &spmv_pair_zmf64_kernel<MODE, PS, 2, false> : &spmv_pair_zmf64_kernel<MODE, PS, 1, false>; } while (0)
  if (mode == SPMV_PLAIN) { if (ps == 5) F64K(SPMV_PLAIN, 5); else F64K(SPMV_PLAIN, 7); }
  else { if (ps == 5) F64K(SPMV_DOT, 5); else F64K(SPMV_DOT, 7); }
#undef F64K
  note_dispatch(split ? DSP_PAIR_ZMF64_SPLIT : DSP_PAIR_ZMF64);
  launch_timed(f, grid, st, a, x, y, S.pflag.p, S.pval.p);
  HIPCHECK(hipGetLastError());
  return grid;
}

// The 27-point z-march launch: PLAIN / DOT (the MatMult), and CG mode 5's PW
// and RUPD passes (one rank, column-word form; ru / jm for RUPD)
static int zm27_launch(Mat *A, int mode, bool split, bool clean, const double *x, double *y, double *partials,
                       const int *done, const Fold &fold_in, hipStream_t st, const PairRuArgs &ru, int jm) {
  const Sell &S = A->sd;
  PairLean27Args b{};
  b.n = (int)A->n;
  for (int r = 0; r < 9; ++r) b.anchor[r] = S.pat_star_off[(size_t)(3 * r + 1)];
  const int D = b.anchor[7];
  b.P = D / 128;
  b.NZ = (int)(A->m / D);
  // 6 workgroups per CU (knob 45) with one plane per step (knob 49): the
  // VALU-bound 27-point body at 78-80 VGPRs keeps 6 waves per SIMD (C5's
  // share, round 3: CG MatMult 63 us median against 68-74 at 3-4 per CU or
  // two planes per step, profiles/r03_ab.jsonl)
  // CG mode 5's residual update holds 96 VGPRs (5 waves per SIMD): its grid
  // is the 5 workgroups per CU that fit at once (knob 56; 6 left a partial
  // second generation: 99 -> 89 us per launch, -5% per C5 iteration)
  const int bpc = mode == SPMV_RUPD && g_knobs.pair_zm27_ru_bpc > 0 ? g_knobs.pair_zm27_ru_bpc
                  : g_knobs.pair_zm27_bpc > 0 ? g_knobs.pair_zm27_bpc : g_knobs.pair_zm_bpc;
  int L, Sg;
  int grid = zm_tasks(b.P, b.NZ, L, Sg, bpc);
  b.L = L;
  b.S = Sg;
  b.partials = partials;
  b.done = done;
  Fold fold = fold_in;
  if (fold.cnt) { fold.ntotal = fold.ncount = grid; fold.base = 0; }
  b.fold = fold;
  using F27 = void (*)(PairLean27Args, const double *, double *, const int32_t *, const PairUni27 *,
                       const int32_t *, PairRuArgs);
  F27 f = nullptr;
  const int form = !clean ? 0 : S.pcol27.p ? 2 : 1;
  const bool z2 = g_knobs.pair_zm27_units == 2;
  // the fma form: one plane per step, no ghost units (the SPLIT variant
  // spills a VGPR at the 6-wave bound)
  const bool uv = form == 2 && S.pair_unit27 && g_knobs.pair_unitv && !z2 && !split;
  // the plane-pipelined form (knob 60): column words; the symmetric p.Ap pass
  // keeps the carried-operand kernel
  const bool sym = S.pair_sym27 && g_knobs.pw_sym27;
  // knob 74: the two-line kernels' XCDs split the line groups of every plane
  // (segments of L planes) instead of taking a slab of NZ / 8 planes each,
  // when the waves can still all be busy with segments longer than the
  // slab: each segment re-reads its one or two leading planes, so short
  // slabs (C5's share: 8 planes) re-read a quarter of p.  The residual update
  // runs 2 workgroups per CU (knob 75; 4 are resident at its 100 VGPRs), the
  // p.Ap pass 3 (knob 76; 6 resident at 78 VGPRs) -- every count fills whole
  // rounds here, and fewer waves streaming longer segments measured faster:
  // C5's share, residual update 75.0 -> 72.3 us at 4 per CU -> 69.2 at 2,
  // p.Ap pass 26.0 -> 24.4 at 6 -> 23.5 at 3 (round 5, gpurun_out/r5i-r5n).
  auto xcol_geom = [&](int G, int &L, int &Sg) -> int {
    if (!g_knobs.zm27_xcol || b.anchor[5] % 128 != 0 || b.NZ < 16) return 0;
    int g = zm_tasks(b.P / G, b.NZ, L, Sg, bpc);
    const int xb = mode == SPMV_PW ? g_knobs.zm27_xcol_pw : g_knobs.zm27_xcol_ru;   // knobs 76 / 75
    if (xb > 0) g = (xb * device_cu_count()) & ~7;
    if (g < 8 || (g & 7)) return 0;
    const int PL = b.anchor[5] / 128, nlp = b.P / G / PL;
    const int64_t wx = (int64_t)g / 8 * LEAN_WAVES, cx = (int64_t)(nlp / 8) * PL;
    if (cx <= 0) return 0;
    const int segs = (int)std::min<int64_t>(b.NZ, std::max<int64_t>(1, (wx + cx - 1) / cx));
    const int Lx = (b.NZ + segs - 1) / segs, slab = (b.NZ + 7) / 8;
    if (Lx <= slab) return 0;
    L = Lx;
    Sg = (b.NZ + Lx - 1) / Lx;
    return g;
  };
  auto geom2l = [&](int G) -> int {
    int L2, S2;
    const int gx = (mode == SPMV_PW || mode == SPMV_RUPD) ? xcol_geom(G, L2, S2) : 0;
    if (gx) { b.L = L2; b.S = S2; b.xcol = 1; return gx; }
    b.xcol = 0;
    return zm_tasks(b.P / G, b.NZ, b.L, b.S, bpc);
  };
  // knob 70: two lines per wave (the column words pair up by lines, no ghost units)
  if (form == 2 && g_knobs.zm27_2line && S.pair_2l27 && !split && mode == SPMV_PW && sym) {
    const bool uv2 = S.pair_unit27 && g_knobs.pair_unitv;
    const bool g4 = g_knobs.zm27_2line == 2 && S.pair_4l27;
    if (g4) { b.xcol = 0; grid = zm_tasks(b.P / 4, b.NZ, b.L, b.S, bpc); }
    else grid = geom2l(2);
    if (fold.cnt) { fold.ntotal = fold.ncount = grid; b.fold = fold; }
    using FS = void (*)(PairLean27Args, const double *, const int32_t *, const PairUni27 *, const int32_t *);
    FS fs = g4 ? (uv2 ? &spmv_pair_zm27s2l_kernel<true, 4> : &spmv_pair_zm27s2l_kernel<false, 4>)
               : b.xcol ? (uv2 ? &spmv_pair_zm27s2l_kernel<true, 2, true> : &spmv_pair_zm27s2l_kernel<false, 2, true>)
                        : (uv2 ? &spmv_pair_zm27s2l_kernel<true, 2> : &spmv_pair_zm27s2l_kernel<false, 2>);
    note_dispatch(DSP_ZM_PW);
    launch_timed(fs, grid, st, b, x, S.pblk.p, S.puni27.p, S.pcol27.p);
    HIPCHECK(hipGetLastError());
    return grid;
  }
  if (form == 2 && g_knobs.zm27_2line && S.pair_2l27 && !split &&
      (mode == SPMV_RUPD || mode == SPMV_DOT || mode == SPMV_PLAIN)) {
    const bool uvp = S.pair_unit27 && g_knobs.pair_unitv;
    grid = geom2l(2);
    if (fold.cnt) { fold.ntotal = fold.ncount = grid; b.fold = fold; }
#define P2L(MODE, JM) f = uvp ? &spmv_pair_zm27p2l_kernel<MODE, true, JM> : &spmv_pair_zm27p2l_kernel<MODE, false, JM>
    switch (mode) {
      case SPMV_PLAIN: P2L(SPMV_PLAIN, 0); break;
      case SPMV_DOT: P2L(SPMV_DOT, 0); break;
      default:
        if (b.xcol) f = jm == 2 ? (uvp ? &spmv_pair_zm27p2l_kernel<SPMV_RUPD, true, 2, true>
                                        : &spmv_pair_zm27p2l_kernel<SPMV_RUPD, false, 2, true>)
                                : (uvp ? &spmv_pair_zm27p2l_kernel<SPMV_RUPD, true, 0, true>
                                       : &spmv_pair_zm27p2l_kernel<SPMV_RUPD, false, 0, true>);
        else if (jm == 2) P2L(SPMV_RUPD, 2);
        else P2L(SPMV_RUPD, 0);
    }
#undef P2L
    note_dispatch(mode == SPMV_RUPD ? DSP_ZM_RUPD : DSP_PAIR_ZM27);
  } else if (form == 2 && g_knobs.pair_zm27p && !(mode == SPMV_PW && sym)) {
    const bool uvp = S.pair_unit27 && g_knobs.pair_unitv;
    switch (mode) {
      case SPMV_PLAIN:
        if (split) f = uvp ? &spmv_pair_zm27p_kernel<SPMV_PLAIN, true, true> : &spmv_pair_zm27p_kernel<SPMV_PLAIN, true, false>;
        else f = uvp ? &spmv_pair_zm27p_kernel<SPMV_PLAIN, false, true> : &spmv_pair_zm27p_kernel<SPMV_PLAIN, false, false>;
        break;
      case SPMV_DOT:
        if (split) f = uvp ? &spmv_pair_zm27p_kernel<SPMV_DOT, true, true> : &spmv_pair_zm27p_kernel<SPMV_DOT, true, false>;
        else f = uvp ? &spmv_pair_zm27p_kernel<SPMV_DOT, false, true> : &spmv_pair_zm27p_kernel<SPMV_DOT, false, false>;
        break;
      case SPMV_PW:
        if (split) return 0;
        f = uvp ? &spmv_pair_zm27p_kernel<SPMV_PW, false, true> : &spmv_pair_zm27p_kernel<SPMV_PW, false, false>;
        break;
      case SPMV_RUPD:
        if (split) return 0;
        if (jm == 2) f = uvp ? &spmv_pair_zm27p_kernel<SPMV_RUPD, false, true, 2> : &spmv_pair_zm27p_kernel<SPMV_RUPD, false, false, 2>;
        else f = uvp ? &spmv_pair_zm27p_kernel<SPMV_RUPD, false, true, 0> : &spmv_pair_zm27p_kernel<SPMV_RUPD, false, false, 0>;
        break;
      default: return 0;
    }
    note_dispatch(mode == SPMV_PW ? DSP_ZM_PW : mode == SPMV_RUPD ? DSP_ZM_RUPD : split ? DSP_PAIR_ZM27_SPLIT : DSP_PAIR_ZM27);
  } else if (mode == SPMV_PW || mode == SPMV_RUPD) {      // CG mode 5: form 2, one rank, one plane per step
    if (form != 2 || split) return 0;
    // the symmetric operator's p.Ap pass: forward half of every row (knob 59)
    if (mode == SPMV_PW && sym) f = uv ? &spmv_pair_zm27_kernel<SPMV_PW, false, 2, 1, true, 0, true>
                                       : &spmv_pair_zm27_kernel<SPMV_PW, false, 2, 1, false, 0, true>;
    else if (mode == SPMV_PW) f = uv ? &spmv_pair_zm27_kernel<SPMV_PW, false, 2, 1, true> : &spmv_pair_zm27_kernel<SPMV_PW, false, 2, 1, false>;
    // the residual update without the fma form: with it the kernel holds 101
    // VGPRs, spills SGPRs and measured no faster (101 vs 89 us at C5's share)
    else if (jm == 2) f = &spmv_pair_zm27_kernel<SPMV_RUPD, false, 2, 1, false, 2>;
    else f = &spmv_pair_zm27_kernel<SPMV_RUPD, false, 2, 1, false, 0>;
    note_dispatch(mode == SPMV_PW ? DSP_ZM_PW : DSP_ZM_RUPD);
  } else {
#define Z27U(MODE, SP, FM) f = z2 ? &spmv_pair_zm27_kernel<MODE, SP, FM, 2> : &spmv_pair_zm27_kernel<MODE, SP, FM, 1>
#define Z27(MODE, SP) do { if (form == 2) Z27U(MODE, SP, 2); else if (form == 1) Z27U(MODE, SP, 1); \
                           else Z27U(MODE, SP, 0); } while (0)
    if (uv) f = mode == SPMV_PLAIN ? &spmv_pair_zm27_kernel<SPMV_PLAIN, false, 2, 1, true>
                                   : &spmv_pair_zm27_kernel<SPMV_DOT, false, 2, 1, true>;
    else if (mode == SPMV_PLAIN) { if (split) Z27(SPMV_PLAIN, true); else Z27(SPMV_PLAIN, false); }
    else { if (split) Z27(SPMV_DOT, true); else Z27(SPMV_DOT, false); }
#undef Z27
#undef Z27U
    note_dispatch(split ? DSP_PAIR_ZM27_SPLIT : DSP_PAIR_ZM27);
  }
  launch_timed(f, grid, st, b, x, y, S.pblk.p, S.puni27.p, S.pcol27.p, ru);
  HIPCHECK(hipGetLastError());
  return grid;
}

// Symmetry of A_d (one rank): every off-diagonal entry (i, j, v) has its
// mirror (j, i) with the same bits (canonical rows are sorted: a binary
// search of row j).  A vector store of 1 on a mismatch (benign race).
__global__ void sym_check_kernel(int64_t m, const int64_t *__restrict__ ptr, const int32_t *__restrict__ col,
                                 const double *__restrict__ val, int *__restrict__ bad) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += stride) {
    for (int64_t k = ptr[i]; k < ptr[i + 1]; ++k) {
      const int64_t j = col[k];
      if (j == i) continue;
      if (j < 0 || j >= m) { *bad = 1; return; }
      int64_t lo = ptr[j], hi = ptr[j + 1];
      while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (col[mid] < i) lo = mid + 1; else hi = mid;
      }
      if (lo == ptr[j + 1] || col[lo] != i || __double_as_longlong(val[lo]) != __double_as_longlong(val[k])) {
        *bad = 1;
        return;
      }
    }
  }
}

// (the result is cached per operator; knob 59 is read where the pass is
// launched, so turning it on later still gets the check)
void pair_sym_prepare(Mat *A) {
  if (A->sym >= 0 || !g_knobs.pw_sym27) return;
  A->sym = 0;
  if (A->comm->size != 1 || A->nghost != 0 || A->m != A->n || A->m <= 0 ||
      (A->sd.pair_shape != 5 && A->sd.pair_shape != 7) || !A->dptr.p)
    return;
  hipStream_t st = A->comm->stream;
  DBuf<int> bad(1);
  HIPCHECK(hipMemsetAsync(bad.p, 0, sizeof(int), st));
  sym_check_kernel<<<grid_for(A->m, 256, 8192), 256, 0, st>>>(A->m, A->dptr.p, A->dcol.p, A->dval.p, bad.p);
  HIPCHECK(hipGetLastError());
  int h = 1;
  HIPCHECK(hipMemcpyAsync(&h, bad.p, sizeof(int), hipMemcpyDeviceToHost, st));
  HIPCHECK(hipStreamSynchronize(st));
  A->sym = h == 0 ? 1 : 0;
}

// Launch the lean MatMult for this product; returns its grid, or 0 when it
// does not apply (the general kernel then runs).  A fold (fold.cnt set)
// counts this launch's workgroups.
// the coded z-march (spmv_pair_zmc_kernel) applies: 5 / 7-point row pairs
// from a non-uniform, select-free code dictionary, z-march geometry
bool pair_code_applies(const Mat *A) {
  const Sell &S = A->sd;
  if (!g_knobs.pair_zmc || !g_knobs.pair_zm || !g_knobs.vcodes || !g_knobs.spmv_pairs || g_knobs.spmv_ynt ||
      !S.pair_code_clean || S.ntab <= 0 || S.puni.p || S.pair_blocks <= 0 || !S.pair_all ||
      (S.pair_shape != 5 && S.pair_shape != 7) || !S.pcode.p || !S.vtab.p)
    return false;
  if (A->m % 128 != 0 || A->m > PAIR_CLEAN_MAX_ROWS || A->n > PAIR_CLEAN_MAX_ROWS || S.nunits * 128 != A->m) return false;
  int anchor[5];
  pair_anchors(S, anchor);
  return zm_plane(A, S.pair_shape, anchor) > 0;
}

static int pair_code_launch(Mat *A, int mode, bool split, const double *x, double *y, double *partials,
                            const int *done, const Fold &fold_in, const Jac &jac, const double *xscale,
                            hipStream_t st) {
  const Sell &S = A->sd;
  PairLeanArgs a{};
  a.m = (int)A->m;
  a.n = (int)A->n;
  a.nunits = (int)S.nunits;
  pair_anchors(S, a.anchor);
  const int D = zm_plane(A, S.pair_shape, a.anchor);
  a.P = D / 128;
  a.NZ = (int)(A->m / D);
  const int grid = zm_tasks(a.P, a.NZ, a.L, a.S, g_knobs.zmc_bpc);   // knob 79 (0: key 40's)
  a.partials = partials;
  a.done = done;
  Fold fold = fold_in;
  if (fold.cnt) { fold.ntotal = fold.ncount = grid; fold.base = 0; }
  a.fold = fold;
  // Jacobi by diagonal code: the operator's own vector Jacobi (knob 37)
  const bool dt = spmv_jac(mode) && jac.mode == 1 && jac.d == A->jac_dinv.p && S.dtab.p && g_knobs.pair_dtab;
  const PairCodeArgs ca{S.pcode.p, S.vtab.p, S.dtab.p, xscale, jac};
  using F = void (*)(PairLeanArgs, const double *, double *, const int32_t *, PairCodeArgs);
  F f = nullptr;
  // planes per step (knob 78; 0: key 42's): one measured faster than two at
  // C4 (46.1 -> 44.0 us per MatMult, round 5 gpurun_out/r5p)
  const bool z2 = (g_knobs.zmc_units > 0 ? g_knobs.zmc_units : g_knobs.pair_zm_units) == 2;
#define ZMC_U(MODE, PS, SP, DTV) f = z2 ? &spmv_pair_zmc_kernel<MODE, PS, SP, 2, DTV> : &spmv_pair_zmc_kernel<MODE, PS, SP, 1, DTV>
#define ZMC_S(MODE, PS, DTV) do { if (split) ZMC_U(MODE, PS, true, DTV); else ZMC_U(MODE, PS, false, DTV); } while (0)
#define ZMC_P(MODE, DTV) do { if (S.pair_shape == 5) ZMC_S(MODE, 5, DTV); else ZMC_S(MODE, 7, DTV); } while (0)
  switch (mode) {
    case SPMV_PLAIN: ZMC_P(SPMV_PLAIN, false); break;
    case SPMV_DOT: ZMC_P(SPMV_DOT, false); break;
    case SPMV_PLAIN_S: ZMC_P(SPMV_PLAIN_S, false); break;
    case SPMV_JACOBI: if (dt) ZMC_P(SPMV_JACOBI, true); else ZMC_P(SPMV_JACOBI, false); break;
    case SPMV_JACOBI_S: if (dt) ZMC_P(SPMV_JACOBI_S, true); else ZMC_P(SPMV_JACOBI_S, false); break;
    default: return 0;
  }
#undef ZMC_P
#undef ZMC_S
#undef ZMC_U
  note_dispatch(split ? DSP_PAIR_ZMC_SPLIT : DSP_PAIR_ZMC);
  launch_timed(f, grid, st, a, x, y, S.pblk.p, ca);
  HIPCHECK(hipGetLastError());
  return grid;
}

int pair_lean_launch(Mat *A, int mode, bool split, const double *x, double *y, double *partials, const int *done,
                     const Fold &fold_in, hipStream_t st, const Jac &jac, const double *xscale) {
  const Sell &S = A->sd;
  if (pair_code_applies(A) && (split || (A->nghost == 0 && !S.pair_ghosts)))
    return pair_code_launch(A, mode, split, x, y, partials, done, fold_in, jac, xscale, st);
  if (xscale) return 0;
  if (mode != SPMV_PLAIN && mode != SPMV_DOT && mode != SPMV_PW) return 0;
  if (mode == SPMV_PW && !pair_cg5_applies(A, 0)) return 0;   // CG mode 5's p.Ap pass: the 5/7-point z-march
  if (pair_f64_kind(A) && (split || A->nghost == 0))   // without a split, A_o continues in the general kernel
    return pair_f64_launch(A, mode, split, x, y, partials, done, fold_in, st);
  const int kind = pair_lean_kind(A);
  if (!kind) return 0;
  if (!split && (A->nghost > 0 || S.pair_ghosts)) return 0;   // A_o continues in the general kernel
  const bool clean = kind == 2;
  if (S.pair_shape == 27) return zm27_launch(A, mode, split, clean, x, y, partials, done, fold_in, st, PairRuArgs{}, 0);
  PairLeanArgs a{};
  a.m = (int)A->m;
  a.n = (int)A->n;
  a.nunits = (int)S.nunits;
  pair_anchors(S, a.anchor);
  a.partials = partials;
  a.done = done;
  const int NR = S.pair_shape == 5 ? 3 : 5, D = a.anchor[NR - 1];
  const bool zm = pair_zm_applies(A);
  LeanFn f = nullptr;
  ZmFn fz = nullptr;
  int grid;
  if (zm) {
    a.P = D / 128;
    a.NZ = (int)(A->m / D);
    // CG mode 5's p.Ap pass may take its own grid (knob 57); segments of up
    // to 32 planes, shorter when one slab's columns do not give every wave a
    // task (zm_geom)
    grid = zm_tasks(a.P, a.NZ, a.L, a.S, mode == SPMV_PW && g_knobs.pw_bpc > 0 ? g_knobs.pw_bpc : g_knobs.pair_zm_bpc);
#define ZM_PICK(MODE, PS, SP, CL) \
    fz = g_knobs.pair_zm_units == 2 ? &spmv_pair_zm_kernel<MODE, PS, SP, CL, 2> : &spmv_pair_zm_kernel<MODE, PS, SP, CL, 1>
#define ZM_C(MODE, PS) do { if (split) { if (clean) ZM_PICK(MODE, PS, true, true); else ZM_PICK(MODE, PS, true, false); } \
                            else { if (clean) ZM_PICK(MODE, PS, false, true); else ZM_PICK(MODE, PS, false, false); } } while (0)
    if (mode == SPMV_PLAIN) { if (S.pair_shape == 5) ZM_C(SPMV_PLAIN, 5); else ZM_C(SPMV_PLAIN, 7); }
    else if (mode == SPMV_PW && clean && !split && A->sym == 1 && g_knobs.pw_sym27) {   // symmetric: forward half
      if (S.pair_shape == 5) fz = g_knobs.pair_zm_units == 2 ? &spmv_pair_zm_kernel<SPMV_PW, 5, false, true, 2, 0, true>
                                                             : &spmv_pair_zm_kernel<SPMV_PW, 5, false, true, 1, 0, true>;
      else fz = g_knobs.pair_zm_units == 2 ? &spmv_pair_zm_kernel<SPMV_PW, 7, false, true, 2, 0, true>
                                           : &spmv_pair_zm_kernel<SPMV_PW, 7, false, true, 1, 0, true>;
    }
    else if (mode == SPMV_PW) { if (S.pair_shape == 5) ZM_C(SPMV_PW, 5); else ZM_C(SPMV_PW, 7); }
    else { if (S.pair_shape == 5) ZM_C(SPMV_DOT, 5); else ZM_C(SPMV_DOT, 7); }
#undef ZM_C
#undef ZM_PICK
  } else {
#define LEAN_C(MODE, PS) do { if (split) f = clean ? &spmv_pair_lean_kernel<MODE, PS, true, true> : &spmv_pair_lean_kernel<MODE, PS, true, false>; \
                              else f = clean ? &spmv_pair_lean_kernel<MODE, PS, false, true> : &spmv_pair_lean_kernel<MODE, PS, false, false>; } while (0)
    if (mode == SPMV_PLAIN) { if (S.pair_shape == 5) LEAN_C(SPMV_PLAIN, 5); else LEAN_C(SPMV_PLAIN, 7); }
    else { if (S.pair_shape == 5) LEAN_C(SPMV_DOT, 5); else LEAN_C(SPMV_DOT, 7); }
#undef LEAN_C
    grid = main_grid(A, mode, reinterpret_cast<const void *>(f), true);
  }
  Fold fold = fold_in;
  if (fold.cnt) { fold.ntotal = fold.ncount = grid; fold.base = 0; }
  a.fold = fold;
  note_dispatch(mode == SPMV_PW ? DSP_ZM_PW : !zm ? DSP_PAIR_LEAN : split ? DSP_PAIR_ZM_SPLIT : DSP_PAIR_ZM);
  if (zm) launch_timed(fz, grid, st, a, x, y, S.pblk.p, S.puni.p, PairRuArgs{});
  else launch_timed(f, grid, st, a, x, y, S.pblk.p, S.puni.p);
  HIPCHECK(hipGetLastError());
  return grid;
}

// CG mode 5 (knob 9 = 5): a lean 5/7-point z-march layout (the constant-
// coefficient stencils), no or uniform Jacobi; on P > 1 ranks the product
// must split (the ghost units' rows are finished by the boundary kernel)
// 27-point (knob 55): one rank, the clean column-word layout
bool pair_cg5_applies(const Mat *A, int jac_mode) {
  if (jac_mode != 0 && jac_mode != 2) return false;
  if (A->sd.pair_shape == 27)
    return g_knobs.cg5_27 && pair_lean_kind(A) == 2 && A->sd.pcol27.p && A->nghost == 0 && !A->sd.pair_ghosts;
  return pair_lean_kind(A) > 0 && pair_zm_applies(A) && ((A->nghost == 0 && !A->sd.pair_ghosts) || matmult_splits(A));
}

static int cg5_args(const Mat *A, PairLeanArgs &a, int bpc = 0) {
  const Sell &S = A->sd;
  a = PairLeanArgs{};
  a.m = (int)A->m;
  a.n = (int)A->n;
  a.nunits = (int)S.nunits;
  pair_anchors(S, a.anchor);
  const int D = a.anchor[S.pair_shape == 5 ? 2 : 4];
  a.P = D / 128;
  a.NZ = (int)(A->m / D);
  return zm_tasks(a.P, a.NZ, a.L, a.S, bpc);
}

// knob 69: the fused direction update + p.Ap pass applies (one rank, a clean
// symmetric 5/7-point z-march layout with the forward-half PW pass, no or a
// uniform Jacobi, x batches of 2 or 4).  Default (5): by size -- 7-point up
// to 2^23 rows, 5-point up to 2^24.  Per iteration, off -> on (tools/cg_ab.py,
// gpurun_out/r4z, r4aa): 3D 128^3 37.3 -> 29.8 us, 256 x 128 x 128 57.2 ->
// 48.7, 256 x 256 x 128 97.9 -> 90.1, 256 x 256 x 192 130.4 -> 131.9, 256^3
// 173.4 -> 176.9; 2D 2048^2 55.6 -> 47.8, 4096 x 2048 97.4 -> 89.9, 4096^2
// 170.2 -> 167.3, 8192 x 4096 353.3 -> 353.1.  While the vectors fit the
// memory-side cache the saved pass is pure gain; at 256^3 the fused pass
// saves 4.6 us (79.4 against 62.4 + 21.6) but the residual update after it
// loses 5.2 (72.2 against 67.0: less of p_i left in that cache); reading the
// +D streams non-temporally made it worse (176.5 / 181.0, r4y)
bool pair_cg5_pbw_applies(const Mat *A, int jac_mode, int xb) {
  const int on = g_knobs.cg_pbw != 5 ? g_knobs.cg_pbw
                                     : A->m <= (int64_t(1) << (A->sd.pair_shape == 5 ? 24 : 23));
  return on && (xb == 2 || xb == 4 || xb == 8) && (jac_mode == 0 || jac_mode == 2) && pair_cg5_applies(A, jac_mode) &&
         A->sd.pair_shape != 27 && pair_lean_kind(A) == 2 && A->nghost == 0 && !A->sd.pair_ghosts && A->sym == 1 &&
         g_knobs.pw_sym27 && pair_zm_applies(A);
}

int pair_cg5_pbw_launch(Mat *A, KspState *s, const double *r, const double *r0, double *const pb[8], int xb,
                        double *hist, int jac_mode, double jac_c, double *partials, const Fold &fold_in,
                        hipStream_t st) {
  if (!pair_cg5_pbw_applies(A, jac_mode, xb)) return 0;
  const Sell &S = A->sd;
  PairLeanArgs a{};
  a.m = (int)A->m;
  a.n = (int)A->n;
  a.nunits = (int)S.nunits;
  pair_anchors(S, a.anchor);
  a.partials = partials;
  const int NR = S.pair_shape == 5 ? 3 : 5, D = a.anchor[NR - 1];
  a.P = D / 128;
  a.NZ = (int)(A->m / D);
  // the PW pass's grid (the same tasks, so the same p.Ap partials)
  const int grid = zm_tasks(a.P, a.NZ, a.L, a.S, g_knobs.pw_bpc > 0 ? g_knobs.pw_bpc : g_knobs.pair_zm_bpc);
  Fold fold = fold_in;
  if (fold.cnt) { fold.ntotal = fold.ncount = grid; fold.base = 0; }
  a.fold = fold;
  const PairPbArgs pa{s, r, r0, pb[0], pb[1] - pb[0], hist, jac_c};   // (consecutive carves, cg_solve)
  using PbwFn = void (*)(const PairLeanArgs, const int32_t *, const PairUni *, const PairPbArgs);
  PbwFn f;
  const bool z2 = g_knobs.pair_zm_units == 2;
#define PBW(PS, JM, B) f = z2 ? &spmv_pair_pbw_kernel<PS, JM, B, 2> : &spmv_pair_pbw_kernel<PS, JM, B, 1>
#define PBW_B(PS, JM) do { if (xb == 8) PBW(PS, JM, 8); else if (xb == 4) PBW(PS, JM, 4); else PBW(PS, JM, 2); } while (0)
#define PBW_J(PS) do { if (jac_mode == 2) PBW_B(PS, 2); else PBW_B(PS, 0); } while (0)
  if (S.pair_shape == 5) PBW_J(5);
  else PBW_J(7);
#undef PBW_J
#undef PBW_B
#undef PBW
  note_dispatch(DSP_ZM_PBW);
  launch_timed(f, grid, st, a, S.pblk.p, S.puni.p, pa);
  HIPCHECK(hipGetLastError());
  return grid;
}

// knob 80: the P > 1 fused direction update + split p.Ap pass applies (CG
// mode 5 on a rank whose product splits, a lean 5/7-point z-march layout, no
// or a uniform Jacobi, x batches of 2 / 4 / 8): 0 off, 1 on (default)
bool pair_cg5_pbws_applies(const Mat *A, int jac_mode, int xb) {
  return g_knobs.cg_pbws && A->comm->size > 1 && (xb == 2 || xb == 4 || xb == 8) &&
         (jac_mode == 0 || jac_mode == 2) && A->sd.pair_shape != 27 && pair_cg5_applies(A, jac_mode) &&
         matmult_splits(A) && pair_lean_kind(A) > 0 && pair_zm_applies(A);
}

// the main launch of that pass (the halo and the boundary kernel around it:
// mx_spmv.hip cg5_pbws_matmult); the PW split pass's grid and tasks
int pair_cg5_pbws_launch(Mat *A, KspState *s, const double *r, double *const pb[8], int xb, double *hist, int jac_mode,
                         double jac_c, double *y, double *partials, hipStream_t st) {
  const Sell &S = A->sd;
  PairLeanArgs a{};
  a.m = (int)A->m;
  a.n = (int)A->n;
  a.nunits = (int)S.nunits;
  pair_anchors(S, a.anchor);
  a.partials = partials;
  const int NR = S.pair_shape == 5 ? 3 : 5, D = a.anchor[NR - 1];
  a.P = D / 128;
  a.NZ = (int)(A->m / D);
  const int grid = zm_tasks(a.P, a.NZ, a.L, a.S, g_knobs.pw_bpc > 0 ? g_knobs.pw_bpc : g_knobs.pair_zm_bpc);
  a.fold = Fold{};
  const PairPbArgs pa{s, r, nullptr, pb[0], pb[1] - pb[0], hist, jac_c};   // (consecutive carves, cg_solve)
  using Fn = void (*)(const PairLeanArgs, double *, const int32_t *, const PairUni *, const PairPbArgs, int);
  Fn f;
  const bool clean = pair_lean_kind(A) == 2, z2 = g_knobs.pair_zm_units == 2;
#define PBS(PS, CL, JM) f = z2 ? &spmv_pair_zmpbs_kernel<PS, CL, 2, JM> : &spmv_pair_zmpbs_kernel<PS, CL, 1, JM>
#define PBS_J(PS, CL) do { if (jac_mode == 2) PBS(PS, CL, 2); else PBS(PS, CL, 0); } while (0)
#define PBS_C(PS) do { if (clean) PBS_J(PS, true); else PBS_J(PS, false); } while (0)
  if (S.pair_shape == 5) PBS_C(5);
  else PBS_C(7);
#undef PBS_C
#undef PBS_J
#undef PBS
  note_dispatch(DSP_ZM_PBWS);
  launch_timed(f, grid, st, a, y, S.pblk.p, S.puni.p, pa, xb);
  HIPCHECK(hipGetLastError());
  return grid;
}

int pair_cg5_rupd_launch(Mat *A, KspState *s, const double *p, const double *w, double *r, const double *r0,
                         int jac_mode, double jac_c, double *partials, const Fold &fold_in, const double *dot_part,
                         int ndot, int xb, int *hw, hipStream_t st) {
  if (!pair_cg5_applies(A, jac_mode)) return 0;
  if (A->sd.pair_shape == 27) {
    const PairRuArgs ru{s, w, r, r0, dot_part, ndot, xb, jac_c, hw};
    return zm27_launch(A, SPMV_RUPD, false, true, p, nullptr, partials, nullptr, fold_in, st, ru, jac_mode);
  }
  PairLeanArgs a;
  const int grid = cg5_args(A, a, g_knobs.ru_bpc);   // knob 58 (0: key 40's)
  a.partials = partials;
  Fold fold = fold_in;
  if (fold.cnt) { fold.ntotal = fold.ncount = grid; fold.base = 0; }
  a.fold = fold;
  const bool split = A->sd.pair_ghosts;      // the ghost units' rows: w from the PW pass + boundary kernel
  const PairRuArgs ru{s, w, r, r0, dot_part, ndot, xb, jac_c, hw};
  const bool clean = pair_lean_kind(A) == 2, z2 = g_knobs.pair_zm_units == 2;
  ZmFn f;
#define RU(PS, SP, CL, JM) f = z2 ? &spmv_pair_zm_kernel<SPMV_RUPD, PS, SP, CL, 2, JM> \
                                  : &spmv_pair_zm_kernel<SPMV_RUPD, PS, SP, CL, 1, JM>
#define RU_S(PS, CL, JM) do { if (split) RU(PS, true, CL, JM); else RU(PS, false, CL, JM); } while (0)
#define RU_J(PS, CL) do { if (jac_mode == 2) RU_S(PS, CL, 2); else RU_S(PS, CL, 0); } while (0)
  if (A->sd.pair_shape == 5) { if (clean) RU_J(5, true); else RU_J(5, false); }
  else { if (clean) RU_J(7, true); else RU_J(7, false); }
#undef RU_J
#undef RU_S
#undef RU
  // knob 68: two lines per wave (clean, one rank, 7-point, an even number of
  // lines per plane, whole 128-row columns per line); by default (3) the
  // 5-wave form from 2^23 rows -- at 128^3 the one-line kernel measured
  // faster (37.0 against 38.6 us per iteration), from 512 x 256 x 128 up the
  // two-line one (-1.5 to -3%)
  const int two = g_knobs.ru_2line == 3 ? (A->m >= (int64_t(1) << 23) ? 2 : 0) : g_knobs.ru_2line;
  if (two && clean && !split && A->sd.pair_shape == 7 && a.anchor[3] > 0 && a.anchor[3] % 128 == 0 &&
      (a.anchor[4] / a.anchor[3]) % 2 == 0 && a.anchor[4] % a.anchor[3] == 0 && a.anchor[1] == -a.anchor[3]) {
    // tasks: column pairs per plane; the grid's segment length from the pairs
    int L2, S2;
    const int g2 = zm_tasks(a.P / 2, a.NZ, L2, S2, g_knobs.ru_bpc);
    a.L = L2;
    a.S = S2;
    if (fold.cnt) { fold.ntotal = fold.ncount = g2; fold.base = 0; }
    a.fold = fold;
    note_dispatch(DSP_ZM_RUPD);
    const bool w5 = two == 2;
    if (jac_mode == 2) launch_timed(w5 ? &spmv_pair_zm2l_kernel<2, 5> : &spmv_pair_zm2l_kernel<2, 1>, g2, st, a, p,
                                    A->sd.pblk.p, A->sd.puni.p, ru);
    else launch_timed(w5 ? &spmv_pair_zm2l_kernel<0, 5> : &spmv_pair_zm2l_kernel<0, 1>, g2, st, a, p, A->sd.pblk.p,
                      A->sd.puni.p, ru);
    HIPCHECK(hipGetLastError());
    return g2;
  }
  note_dispatch(DSP_ZM_RUPD);
  launch_timed(f, grid, st, a, p, nullptr, A->sd.pblk.p, A->sd.puni.p, ru);
  HIPCHECK(hipGetLastError());
  return grid;
}

// this translation unit's code object, loaded now rather than at the first
// launch of one of its kernels (load_code_objects)
void load_code_spmv_pair() {
  hipFuncAttributes a;
  (void)hipFuncGetAttributes(&a, reinterpret_cast<const void *>(&sym_check_kernel));
  (void)hipGetLastError();
}

}  // namespace mx
