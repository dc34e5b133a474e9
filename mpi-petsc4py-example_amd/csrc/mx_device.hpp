// mx_device.hpp -- device helpers shared by the kernels (wave64 reductions).
#pragma once
#include <hip/hip_runtime.h>

namespace mx {

// Fixed xor-butterfly over the 64 lanes: every lane gets the same total and
// the summation tree is the same on every launch (deterministic).
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// 256-thread block: fold NV running sums; thread t < NV stores value t's
// block total to partials[t * nblocks + blockIdx.x].
template <int NV>
__device__ __forceinline__ void block_sum_to_partials(double (&v)[NV], double *partials,
                                                      int nblocks) {
  __shared__ double sh[NV][4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const double s = wave_sum(v[k]);
    if (lane == 0) sh[k][wid] = s;
  }
  __syncthreads();
  if (threadIdx.x < NV) {
    const int k = threadIdx.x;
    partials[(size_t)k * nblocks + blockIdx.x] = (sh[k][0] + sh[k][1]) + (sh[k][2] + sh[k][3]);
  }
}

// 256-thread block: sum of p[0..n) in a fixed order, valid in every thread.
__device__ __forceinline__ double block_sum_array(const double *__restrict__ p, int n) {
  __shared__ double sh[4];
  double s = 0.0;
  int i = threadIdx.x;
  // eight loads in flight, summed in the same sequential order as the
  // plain strided loop (the fold order, hence the bits, are unchanged)
  for (; i + 7 * 256 < n; i += 8 * 256) {
    double t[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) t[q] = p[i + q * 256];
#pragma unroll
    for (int q = 0; q < 8; ++q) s += t[q];
  }
  for (; i < n; i += 256) s += p[i];
  s = wave_sum(s);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
  __syncthreads();
  return (sh[0] + sh[1]) + (sh[2] + sh[3]);
}

}  // namespace mx
