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
// Thread t sums p[t], p[t + 256], ... sequentially, then the fixed wave and
// 4-wave trees; LOADS values are loaded before the first add of a batch (the
// order, hence the bits, are those of the plain strided loop).  SC1: loads
// are agent-coherent (`global_load sc1`), for partials published by other
// workgroups of the same launch.
template <int LOADS = 8, bool SC1 = false>
__device__ __forceinline__ double block_sum_array(const double *__restrict__ p, int n) {
  __shared__ double sh[4];
  double s = 0.0;
  int i = threadIdx.x;
  for (; i + (LOADS - 1) * 256 < n; i += LOADS * 256) {
    double t[LOADS];
#pragma unroll
    for (int q = 0; q < LOADS; ++q) {
      if constexpr (SC1) t[q] = __hip_atomic_load(p + i + q * 256, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else t[q] = p[i + q * 256];
    }
#pragma unroll
    for (int q = 0; q < LOADS; ++q) s += t[q];
  }
  for (; i < n; i += 256) {
    if constexpr (SC1) s += __hip_atomic_load(p + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else s += p[i];
  }
  s = wave_sum(s);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
  __syncthreads();
  return (sh[0] + sh[1]) + (sh[2] + sh[3]);
}

// In-launch reduction: the last workgroup to finish folds every workgroup's
// partials, saving the separate fold kernel and its launch boundary.
// Publication (MI355X_MICROARCH.md, inter-workgroup visibility, counter form
// with write-through stores): each workgroup stores its partials `sc1`,
// drains them (`s_waitcnt vmcnt(0)` in the storing wave), then one lane adds
// to an agent-scope counter; the workgroup whose add completes the count
// reads all partials with `sc1` loads.  Arrivals are counted on 8 shards
// (counting block % 8) and then on a top counter, each on a 256-B line of its
// own (adds to one line serialise, ~90 per us), so no line takes more than
// ~ncount/8 adds.  The reducer sums in block_sum_array's fixed order (the bits
// equal a separate fold kernel's) and re-zeroes the counters; the solver also
// zeroes them at every solve, so a launch cut short by a stop cannot leave a
// partial count behind.
constexpr int FOLD_STRIDE = 64;   // counters 256 B apart: atomics to one line serialise
struct Fold {
  unsigned *cnt = nullptr;   // [9 * FOLD_STRIDE]; null: plain partials, no fold in this launch
  double *out = nullptr;     // [NV] folded values
  int ntotal = 0;            // partials per value (row stride), all launches
  int base = 0;              // partial slot of this launch's workgroup 0
  int ncount = 0;            // workgroups of this launch (all arrive)
};

// true in the workgroup that folded (every thread of it)
template <int NV>
__device__ __forceinline__ bool block_fold(double (&v)[NV], double *partials, const Fold &f) {
  __shared__ double sh[NV][4];
  __shared__ int last;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const double s = wave_sum(v[k]);
    if (lane == 0) sh[k][wid] = s;
  }
  __syncthreads();
  if (wid == 0) {
    if (lane < NV) {
      const double t = (sh[lane][0] + sh[lane][1]) + (sh[lane][2] + sh[lane][3]);
      __hip_atomic_store(partials + (size_t)lane * f.ntotal + f.base + blockIdx.x, t, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) {
      int l = 0;
      const unsigned c = blockIdx.x, shard = c & 7u;
      const unsigned nshard = ((unsigned)f.ncount - shard + 7u) >> 3;
      if (__hip_atomic_fetch_add(f.cnt + shard * FOLD_STRIDE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
          nshard - 1u) {
        const unsigned ntop = f.ncount < 8 ? (unsigned)f.ncount : 8u;
        l = __hip_atomic_fetch_add(f.cnt + 8 * FOLD_STRIDE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
            ntop - 1u;
      }
      last = l;
    }
  }
  __syncthreads();
  if (!last) return false;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const double t = block_sum_array<16, true>(partials + (size_t)k * f.ntotal, f.ntotal);
    if (threadIdx.x == 0) f.out[k] = t;
  }
  if (threadIdx.x < 9)
    __hip_atomic_store(f.cnt + threadIdx.x * FOLD_STRIDE, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return true;
}

// partials of this launch's workgroups: plain block partials, or an in-launch fold
template <int NV>
__device__ __forceinline__ void block_partials(double (&v)[NV], double *partials, int nblocks, const Fold &f) {
  if (f.cnt) block_fold<NV>(v, partials, f);
  else block_sum_to_partials<NV>(v, partials, nblocks);
}

}  // namespace mx
