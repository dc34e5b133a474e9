// mx_pair.hpp -- row-pair SpMV building blocks shared by the general SELL
// kernel (mx_spmv.hip) and the lean uniform-slot kernel (mx_spmv_pair.hip).
//
// A row-pair unit is 128 consecutive rows of a 5/7/27-point aligned-offset
// block: lane l holds rows r0 = 128 u + 2 l and r0 + 1, x is read as 16-byte
// pairs (one load per run of the pattern), and the +-1 neighbours of a run
// c-1, c, c+1 come from the adjacent lanes by DPP wave shifts (lanes 0 and 63
// take the unit's two edge values).  Layout: mx_assembly.hip pair_fill_kernel.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace mx {

typedef double dbl2 __attribute__((ext_vector_type(2)));

// Buffer-load forms of the operand: 32-bit element indices, and a read
// outside the vector (an absent slot of a boundary unit: its offset points
// before row 0 or past the last row) returns 0 by the hardware range check
// instead of faulting.  Bound: n * 8 < 2^31 (PAIR_MAX_ROWS); a negative index
// wraps to an offset >= 2^31, outside every vector.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t vec_rsrc(const double *p, int64_t n) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(p), 0, (int)(n * 8), 0x00020000);
}
__device__ __forceinline__ dbl2 bload2(__amdgpu_buffer_rsrc_t r, int i) {
  return __builtin_bit_cast(dbl2, __builtin_amdgcn_raw_buffer_load_b128(r, (int)((unsigned)i * 8u), 0, 0));
}
__device__ __forceinline__ double bload1(__amdgpu_buffer_rsrc_t r, int i) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, (int)((unsigned)i * 8u), 0, 0));
}

// Slots of the dominant pattern grouped into runs: a singleton offset o gives
// both rows' operand (x[r0+o], x[r0+1+o]) from one pair; a run c-1, c, c+1
// ("tri") loads the pair at c and takes x[r0+c-1] (row 0) and x[r0+c+2]
// (row 1) from the neighbouring lanes.
template <int PS> struct PairShape;
template <> struct PairShape<5> {     // a, -1, 0, 1, b
  static constexpr int K = 5, NR = 3, CENTER_RUN = 1;
  static constexpr int run(int j) { return j == 0 ? 0 : j == 4 ? 2 : 1; }
  static constexpr int pos(int j) { return j >= 1 && j <= 3 ? j - 2 : 0; }
  static constexpr bool tri(int r) { return r == 1; }
  static constexpr int first(int r) { return r == 0 ? 0 : r == 1 ? 1 : 4; }
};
template <> struct PairShape<7> {     // a, b, -1, 0, 1, c, d
  static constexpr int K = 7, NR = 5, CENTER_RUN = 2;
  static constexpr int run(int j) { return j < 2 ? j : j <= 4 ? 2 : j - 2; }
  static constexpr int pos(int j) { return j >= 2 && j <= 4 ? j - 3 : 0; }
  static constexpr bool tri(int r) { return r == 2; }
  static constexpr int first(int r) { return r < 2 ? r : r == 2 ? 2 : r + 2; }
};
template <> struct PairShape<27> {    // nine runs c-1, c, c+1
  static constexpr int K = 27, NR = 9, CENTER_RUN = 4;
  static constexpr int run(int j) { return j / 3; }
  static constexpr int pos(int j) { return j % 3 - 1; }
  static constexpr bool tri(int) { return true; }
  static constexpr int first(int r) { return 3 * r; }
};
template <> struct PairShape<0> {
  static constexpr int K = 1, NR = 1, CENTER_RUN = 0;
  static constexpr int run(int) { return 0; }
  static constexpr int pos(int) { return 0; }
  static constexpr bool tri(int) { return false; }
  static constexpr int first(int) { return 0; }
};

// lane i takes lane i - 1's value (UP) or lane i + 1's (!UP); the edge lane takes `edge`
template <bool UP>
__device__ __forceinline__ double wave_shift(double v, double edge) {
  const long long b = __double_as_longlong(v), e = __double_as_longlong(edge);
  constexpr int ctrl = UP ? 0x138 : 0x130;   // wave_shr:1 / wave_shl:1
  const int lo = __builtin_amdgcn_update_dpp((int)e, (int)b, ctrl, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp((int)(e >> 32), (int)(b >> 32), ctrl, 0xf, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

}  // namespace mx
