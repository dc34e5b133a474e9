// Ceiling probe for GMRES's VecMDot (not product code): h_j = w . v_j for
// j < nv over n = 2^24 rows, by access scheme, against a plain read stream.
//   read     : one 2 GiB vector, 16 B per lane, non-temporal (the read ceiling)
//   split<Q> : the product's mdot_split_kernel (4 waves of a workgroup on the
//              same rows, wave g on vectors [gQ, gQ + Q), 16 B per lane)
//   split2<Q>: the same with two consecutive pairs per lane (32 B per lane)
//   chunk    : a workgroup holds 2048 rows of w in registers and walks the
//              vectors one after another (16 KB contiguous per vector per
//              step), nv <= 32 accumulators per thread
// hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/mdot_probe tools/mdot_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cmath>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
typedef double dbl2 __attribute__((ext_vector_type(2)));

constexpr int64_t N = int64_t(1) << 24;
constexpr int NVMAX = 32;

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__global__ void initv_kernel(double *p, int64_t ldv, int nv) {   // vector j: 1 + j / 64 + (i % 7) / 1024
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < ldv * nv; i += (int64_t)gridDim.x * blockDim.x)
    p[i] = 1.0 + (double)(i / ldv) / 64.0 + (double)((i % ldv) % 7) / 1024.0;
}

__global__ void init_kernel(double *p, int64_t n, double s) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    p[i] = s * (double)((i * 2654435761u) % 1000) * 1e-3;
}

__global__ void __launch_bounds__(256) read_kernel(const dbl2 *__restrict__ x, int64_t n2, double *out) {
  double s = 0.0;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n2; i += (int64_t)gridDim.x * 256) {
    const dbl2 t = __builtin_nontemporal_load(x + i);
    s += t.x + t.y;
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * 4 + (threadIdx.x >> 6)] = s;
}

template <int NQ, int U2>
__global__ void __launch_bounds__(256) split_kernel(int64_t n, const double *__restrict__ w, const double *__restrict__ V,
                                                    int64_t ldv, int nv, double *__restrict__ partials) {
  const int lane = threadIdx.x & 63;
  const int g = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int j0 = g * NQ, cnt = min(NQ, nv - j0);
  if (cnt <= 0) return;
  double acc[NQ];
  const dbl2 *__restrict__ vk[NQ];
#pragma unroll
  for (int k = 0; k < NQ; ++k) {
    acc[k] = 0.0;
    vk[k] = reinterpret_cast<const dbl2 *>(V + (int64_t)(j0 + (k < cnt ? k : cnt - 1)) * ldv);
  }
  const dbl2 *__restrict__ w2 = reinterpret_cast<const dbl2 *>(w);
  const int64_t n2 = n >> 1, stride = (int64_t)gridDim.x * 64 * U2;
  for (int64_t i = ((int64_t)blockIdx.x * 64 + lane) * U2; i < n2; i += stride) {
    dbl2 wi[U2], v[U2][NQ];
#pragma unroll
    for (int u = 0; u < U2; ++u) {
      wi[u] = w2[i + u];
#pragma unroll
      for (int k = 0; k < NQ; ++k) v[u][k] = __builtin_nontemporal_load(vk[k] + i + u);
    }
#pragma unroll
    for (int u = 0; u < U2; ++u)
#pragma unroll
      for (int k = 0; k < NQ; ++k) {
        acc[k] += wi[u].x * v[u][k].x;
        acc[k] += wi[u].y * v[u][k].y;
      }
  }
#pragma unroll
  for (int k = 0; k < NQ; ++k) {
    const double s = wave_sum(acc[k]);
    if (lane == 0 && k < cnt) partials[(size_t)(j0 + k) * gridDim.x + blockIdx.x] = s;
  }
}

// chunk: 2048 rows of w per workgroup step held as 4 pairs per thread
template <int WP>
__global__ void __launch_bounds__(256) chunk_kernel(int64_t n, const double *__restrict__ w, const double *__restrict__ V,
                                                    int64_t ldv, int nv, double *__restrict__ partials) {
  double acc[NVMAX];
#pragma unroll
  for (int j = 0; j < NVMAX; ++j) acc[j] = 0.0;
  const dbl2 *__restrict__ w2 = reinterpret_cast<const dbl2 *>(w);
  const int64_t n2 = n >> 1, csz = 256 * WP;
  for (int64_t c0 = blockIdx.x * csz; c0 < n2; c0 += (int64_t)gridDim.x * csz) {
    dbl2 wr[WP];
#pragma unroll
    for (int k = 0; k < WP; ++k) wr[k] = w2[c0 + k * 256 + threadIdx.x];
#pragma unroll
    for (int j = 0; j < NVMAX; ++j) {
      if (j < nv) {
        const dbl2 *__restrict__ vj = reinterpret_cast<const dbl2 *>(V + (int64_t)j * ldv) + c0 + threadIdx.x;
        dbl2 t[WP];
#pragma unroll
        for (int k = 0; k < WP; ++k) t[k] = __builtin_nontemporal_load(vj + k * 256);
#pragma unroll
        for (int k = 0; k < WP; ++k) {
          acc[j] += wr[k].x * t[k].x;
          acc[j] += wr[k].y * t[k].y;
        }
      }
    }
  }
  __shared__ double sh[NVMAX][4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < NVMAX; ++j) {
    if (j < nv) {
      const double s = wave_sum(acc[j]);
      if (lane == 0) sh[j][wid] = s;
    }
  }
  __syncthreads();
  if (threadIdx.x < nv) partials[(size_t)threadIdx.x * gridDim.x + blockIdx.x] =
      (sh[threadIdx.x][0] + sh[threadIdx.x][1]) + (sh[threadIdx.x][2] + sh[threadIdx.x][3]);
}


// chunk with the basis scale applied on read (the product's form: acc +=
// w (s_j v)); RED: per-chunk wave sums, vector j's total kept in lane j
// (one accumulator register instead of nv)
template <int WP, bool RED>
__global__ void __launch_bounds__(256) chunks_kernel(int64_t n, const double *__restrict__ w, const double *__restrict__ V,
                                                     int64_t ldv, int nv, const double *__restrict__ vs,
                                                     double *__restrict__ partials) {
  double acc[RED ? 1 : NVMAX];
#pragma unroll
  for (int j = 0; j < (RED ? 1 : NVMAX); ++j) acc[j] = 0.0;
  const int lane = threadIdx.x & 63;
  const dbl2 *__restrict__ w2 = reinterpret_cast<const dbl2 *>(w);
  const int64_t n2 = n >> 1, csz = 256 * WP;
  for (int64_t c0 = blockIdx.x * csz; c0 < n2; c0 += (int64_t)gridDim.x * csz) {
    dbl2 wr[WP];
#pragma unroll
    for (int k = 0; k < WP; ++k) wr[k] = w2[c0 + k * 256 + threadIdx.x];
#pragma unroll
    for (int j = 0; j < NVMAX; ++j) {
      if (j < nv) {
        const double sj = vs[j];
        const dbl2 *__restrict__ vj = reinterpret_cast<const dbl2 *>(V + (int64_t)j * ldv) + c0 + threadIdx.x;
        dbl2 t[WP];
#pragma unroll
        for (int k = 0; k < WP; ++k) t[k] = __builtin_nontemporal_load(vj + k * 256);
        double a = 0.0;
#pragma unroll
        for (int k = 0; k < WP; ++k) {
          a += wr[k].x * (sj * t[k].x);
          a += wr[k].y * (sj * t[k].y);
        }
        if constexpr (RED) {
          a = wave_sum(a);
          if (lane == j) acc[0] += a;
        } else {
          acc[j] += a;
        }
      }
    }
  }
  __shared__ double sh[NVMAX][4];
  const int wid = threadIdx.x >> 6;
  if constexpr (RED) {
    if (lane < nv) sh[lane][wid] = acc[0];
  } else {
#pragma unroll
    for (int j = 0; j < NVMAX; ++j) {
      if (j < nv) {
        const double s = wave_sum(acc[j]);
        if (lane == 0) sh[j][wid] = s;
      }
    }
  }
  __syncthreads();
  if (threadIdx.x < nv) partials[(size_t)threadIdx.x * gridDim.x + blockIdx.x] =
      (sh[threadIdx.x][0] + sh[threadIdx.x][1]) + (sh[threadIdx.x][2] + sh[threadIdx.x][3]);
}

// round 4 variants of the RED form without the fully unrolled guarded walk
// (which kept 32 vector addresses and scales in SGPRs: 126 spills):
//   pair : two vectors per step (the product after round 4's first fix)
//   grp4 : four vectors per step, loads clamped to the last vector (branch-free),
//          the four lane partials reduced together by a transposed butterfly
//          (7 fp64 shuffles instead of 4 x 6); vector 4g + q's total lands in
//          the lanes 16q..16q+15 and is kept in lane 16q + g
__device__ __forceinline__ double red4(double a0, double a1, double a2, double a3, int lane) {
  const bool b5 = lane & 32, b4 = lane & 16;
  const double k0 = b5 ? a2 : a0, s0 = b5 ? a0 : a2;
  const double k1 = b5 ? a3 : a1, s1 = b5 ? a1 : a3;
  const double c0 = k0 + __shfl_xor(s0, 32, 64);
  const double c1 = k1 + __shfl_xor(s1, 32, 64);
  double c = (b4 ? c1 : c0) + __shfl_xor(b4 ? c0 : c1, 16, 64);
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  return c;                                  // lane l: vector 2 (l >> 5 & 1) + (l >> 4 & 1) of the group
}

template <int WP, int MODE>   // MODE 0 pair, 1 grp4
__global__ void __launch_bounds__(256) chunkv_kernel(int64_t n, const double *__restrict__ w, const double *__restrict__ V,
                                                     int64_t ldv, int nv, const double *__restrict__ vs,
                                                     double *__restrict__ partials) {
  double acc = 0.0;
  const int lane = threadIdx.x & 63;
  const dbl2 *__restrict__ w2 = reinterpret_cast<const dbl2 *>(w);
  const int64_t n2 = n >> 1, csz = 256 * WP;
  for (int64_t c0 = blockIdx.x * csz; c0 < n2; c0 += (int64_t)gridDim.x * csz) {
    dbl2 wr[WP];
#pragma unroll
    for (int k = 0; k < WP; ++k) wr[k] = w2[c0 + k * 256 + threadIdx.x];
    if constexpr (MODE == 0) {
      for (int j = 0; j < nv; j += 2) {
        const bool two = j + 1 < nv;
        const double s0 = vs[j], s1 = two ? vs[j + 1] : 0.0;
        const dbl2 *__restrict__ v0 = reinterpret_cast<const dbl2 *>(V + (int64_t)j * ldv) + c0 + threadIdx.x;
        const dbl2 *__restrict__ v1 = reinterpret_cast<const dbl2 *>(V + (int64_t)(two ? j + 1 : j) * ldv) + c0 + threadIdx.x;
        dbl2 t0[WP], t1[WP];
#pragma unroll
        for (int k = 0; k < WP; ++k) t0[k] = __builtin_nontemporal_load(v0 + k * 256);
        if (two) {
#pragma unroll
          for (int k = 0; k < WP; ++k) t1[k] = __builtin_nontemporal_load(v1 + k * 256);
        }
        double a0 = 0.0, a1 = 0.0;
#pragma unroll
        for (int k = 0; k < WP; ++k) { a0 += wr[k].x * (s0 * t0[k].x); a0 += wr[k].y * (s0 * t0[k].y); }
        a0 = wave_sum(a0);
        if (lane == j) acc += a0;
        if (two) {
#pragma unroll
          for (int k = 0; k < WP; ++k) { a1 += wr[k].x * (s1 * t1[k].x); a1 += wr[k].y * (s1 * t1[k].y); }
          a1 = wave_sum(a1);
          if (lane == j + 1) acc += a1;
        }
      }
    } else {
      for (int j = 0; j < nv; j += 4) {
        dbl2 t[4][WP];
        double sq[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int jq = min(j + q, nv - 1);
          sq[q] = j + q < nv ? vs[jq] : 0.0;
          const dbl2 *__restrict__ vq = reinterpret_cast<const dbl2 *>(V + (int64_t)jq * ldv) + c0 + threadIdx.x;
#pragma unroll
          for (int k = 0; k < WP; ++k) t[q][k] = __builtin_nontemporal_load(vq + k * 256);
        }
        double a[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          a[q] = 0.0;
#pragma unroll
          for (int k = 0; k < WP; ++k) { a[q] += wr[k].x * (sq[q] * t[q][k].x); a[q] += wr[k].y * (sq[q] * t[q][k].y); }
        }
        const double r = red4(a[0], a[1], a[2], a[3], lane);
        if ((lane & 15) == (j >> 2)) acc += r;
      }
    }
  }
  __shared__ double sh[NVMAX][4];
  const int wid = threadIdx.x >> 6;
  if constexpr (MODE == 0) {
    if (lane < nv) sh[lane][wid] = acc;
  } else {
    const int vj = 4 * (lane & 15) + 2 * ((lane >> 5) & 1) + ((lane >> 4) & 1);
    if ((lane & 15) < 8 && vj < nv) sh[vj][wid] = acc;
  }
  __syncthreads();
  if (threadIdx.x < nv) partials[(size_t)threadIdx.x * gridDim.x + blockIdx.x] =
      (sh[threadIdx.x][0] + sh[threadIdx.x][1]) + (sh[threadIdx.x][2] + sh[threadIdx.x][3]);
}

// VecMAXPY + ||w||^2 (GMRES's maxpy_norm_kernel body): w -= sum_j a_j v_j in
// VecMAXPY_Seq's grouping (first nv % 4 vectors, then groups of four)
__global__ void __launch_bounds__(256) maxpy_row_kernel(int64_t n, double *__restrict__ w, const double *__restrict__ V,
                                                        int64_t ldv, int nv, const double *__restrict__ al,
                                                        double *__restrict__ partials) {
  __shared__ double a[NVMAX];
  if (threadIdx.x < NVMAX) a[threadIdx.x] = al[threadIdx.x];
  __syncthreads();
  const int rem = nv & 3;
  double v = 0.0;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    double u = w[i];
    int j = 0;
    auto vj = [&](int j) { return __builtin_nontemporal_load(V + (int64_t)j * ldv + i); };
    if (rem == 1) { u = a[0] * vj(0) + u; j = 1; }
    else if (rem == 2) { u = u + (a[0] * vj(0) + a[1] * vj(1)); j = 2; }
    else if (rem == 3) { u = u + ((a[0] * vj(0) + a[1] * vj(1)) + a[2] * vj(2)); j = 3; }
    for (; j < nv; j += 4)
      u = u + (((a[j] * vj(j) + a[j + 1] * vj(j + 1)) + a[j + 2] * vj(j + 2)) + a[j + 3] * vj(j + 3));
    w[i] = u;
    v += u * u;
  }
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) partials[blockIdx.x * 4 + (threadIdx.x >> 6)] = v;
}

template <int WP>
__global__ void __launch_bounds__(256) maxpy_chunk_kernel(int64_t n, double *__restrict__ w, const double *__restrict__ V,
                                                          int64_t ldv, int nv, const double *__restrict__ al,
                                                          double *__restrict__ partials) {
  __shared__ double a[NVMAX];
  if (threadIdx.x < NVMAX) a[threadIdx.x] = al[threadIdx.x];
  __syncthreads();
  const int rem = nv & 3;
  double v = 0.0;
  dbl2 *__restrict__ w2 = reinterpret_cast<dbl2 *>(w);
  const int64_t n2 = n >> 1, csz = 256 * WP;
  for (int64_t c0 = blockIdx.x * csz; c0 < n2; c0 += (int64_t)gridDim.x * csz) {
    dbl2 u[WP];
#pragma unroll
    for (int k = 0; k < WP; ++k) u[k] = w2[c0 + k * 256 + threadIdx.x];
    auto ld = [&](int j, int k) { return __builtin_nontemporal_load(reinterpret_cast<const dbl2 *>(V + (int64_t)j * ldv) + c0 + k * 256 + threadIdx.x); };
    int j = 0;
    if (rem) {
      dbl2 t[3][WP];
#pragma unroll
      for (int q = 0; q < 3; ++q)
#pragma unroll
        for (int k = 0; k < WP; ++k) t[q][k] = q < rem ? ld(q, k) : dbl2{0.0, 0.0};
#pragma unroll
      for (int k = 0; k < WP; ++k) {
        if (rem == 1) u[k] = dbl2{a[0] * t[0][k].x + u[k].x, a[0] * t[0][k].y + u[k].y};
        else if (rem == 2) u[k] = u[k] + dbl2{a[0] * t[0][k].x + a[1] * t[1][k].x, a[0] * t[0][k].y + a[1] * t[1][k].y};
        else u[k] = u[k] + dbl2{(a[0] * t[0][k].x + a[1] * t[1][k].x) + a[2] * t[2][k].x,
                                (a[0] * t[0][k].y + a[1] * t[1][k].y) + a[2] * t[2][k].y};
      }
      j = rem;
    }
    for (; j < nv; j += 4) {
      dbl2 t[4][WP];
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int k = 0; k < WP; ++k) t[q][k] = ld(j + q, k);
#pragma unroll
      for (int k = 0; k < WP; ++k)
        u[k] = u[k] + dbl2{((a[j] * t[0][k].x + a[j + 1] * t[1][k].x) + a[j + 2] * t[2][k].x) + a[j + 3] * t[3][k].x,
                           ((a[j] * t[0][k].y + a[j + 1] * t[1][k].y) + a[j + 2] * t[2][k].y) + a[j + 3] * t[3][k].y};
    }
#pragma unroll
    for (int k = 0; k < WP; ++k) {
      w2[c0 + k * 256 + threadIdx.x] = u[k];
      v += u[k].x * u[k].x;
      v += u[k].y * u[k].y;
    }
  }
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) partials[blockIdx.x * 4 + (threadIdx.x >> 6)] = v;
}

template <class F>
static float time_it(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main(int argc, char **argv) {
  const int grid = argc > 1 ? atoi(argv[1]) : 1024;
  double *V, *w, *part, *big;
  const int64_t ldv = N;
  CK(hipMalloc(&V, sizeof(double) * ldv * NVMAX));
  CK(hipMalloc(&w, sizeof(double) * N));
  CK(hipMalloc(&part, sizeof(double) * NVMAX * 8192));
  CK(hipMalloc(&big, sizeof(double) * N * 16));
  double *al;
  CK(hipMalloc(&al, sizeof(double) * NVMAX));
  init_kernel<<<1, 64>>>(al, NVMAX, 1e-3);
  initv_kernel<<<4096, 256>>>(V, ldv, NVMAX);
  init_kernel<<<4096, 256>>>(w, N, 0.5);
  init_kernel<<<4096, 256>>>(big, N * 16, 0.25);
  CK(hipDeviceSynchronize());
  const int reps = 10;
  {
    const float ms = time_it([&] { read_kernel<<<2048, 256>>>(reinterpret_cast<const dbl2 *>(big), N * 8, part); }, reps);
    printf("{\"variant\": \"read 2GiB\", \"us\": %.1f, \"TBps\": %.3f}\n", ms * 1e3, 16.0 * N * 8 / ms / 1e9);
  }
  for (int nv : {8, 16, 24, 30}) {
    const double bytes = 8.0 * N * (nv + 1);
    auto rep = [&](const char *name, float ms) {
      printf("{\"variant\": \"%s\", \"nv\": %d, \"grid\": %d, \"us\": %.1f, \"TBps\": %.3f}\n", name, nv, grid, ms * 1e3,
             bytes / ms / 1e9);
    };
    const int q = (nv + 3) / 4;
#define SPLIT(U2)                                                                                        \
    [&] {                                                                                                \
      switch (q) {                                                                                       \
        case 2: split_kernel<2, U2><<<grid, 256>>>(N, w, V, ldv, nv, part); break;                        \
        case 4: split_kernel<4, U2><<<grid, 256>>>(N, w, V, ldv, nv, part); break;                        \
        case 6: split_kernel<6, U2><<<grid, 256>>>(N, w, V, ldv, nv, part); break;                        \
        default: split_kernel<8, U2><<<grid, 256>>>(N, w, V, ldv, nv, part); break;                       \
      }                                                                                                  \
    }
    if (argc > 2) {
      rep("split", time_it(SPLIT(1), reps));
      rep("split2", time_it(SPLIT(2), reps));
    }
    rep("chunk4", time_it([&] { chunk_kernel<4><<<grid, 256>>>(N, w, V, ldv, nv, part); }, reps));
    rep("chunk2", time_it([&] { chunk_kernel<2><<<grid, 256>>>(N, w, V, ldv, nv, part); }, reps));
    rep("chunk4s", time_it([&] { chunks_kernel<4, false><<<grid, 256>>>(N, w, V, ldv, nv, al, part); }, reps));
    rep("chunk4r", time_it([&] { chunks_kernel<4, true><<<grid, 256>>>(N, w, V, ldv, nv, al, part); }, reps));
    rep("chunk8r", time_it([&] { chunks_kernel<8, true><<<grid, 256>>>(N, w, V, ldv, nv, al, part); }, reps));
    rep("chunk4pair", time_it([&] { chunkv_kernel<4, 0><<<grid, 256>>>(N, w, V, ldv, nv, al, part); }, reps));
    rep("chunk4grp4", time_it([&] { chunkv_kernel<4, 1><<<grid, 256>>>(N, w, V, ldv, nv, al, part); }, reps));
    rep("chunk2grp4", time_it([&] { chunkv_kernel<2, 1><<<grid, 256>>>(N, w, V, ldv, nv, al, part); }, reps));
    {   // the variants' totals agree (different sum orders: to rounding)
      auto totals = [&](auto launch) {
        launch();
        CK(hipDeviceSynchronize());
        std::vector<double> h((size_t)nv * grid), t(nv, 0.0);
        CK(hipMemcpy(h.data(), part, sizeof(double) * h.size(), hipMemcpyDeviceToHost));
        for (int j = 0; j < nv; ++j) for (int b = 0; b < grid; ++b) t[j] += h[(size_t)j * grid + b];
        return t;
      };
      auto r0 = totals([&] { chunks_kernel<4, true><<<grid, 256>>>(N, w, V, ldv, nv, al, part); });
      auto r1 = totals([&] { chunkv_kernel<4, 0><<<grid, 256>>>(N, w, V, ldv, nv, al, part); });
      auto r2 = totals([&] { chunkv_kernel<4, 1><<<grid, 256>>>(N, w, V, ldv, nv, al, part); });
      double e = 0.0;
      for (int j = 0; j < nv; ++j) e = fmax(e, fmax(fabs(r1[j] - r0[j]), fabs(r2[j] - r0[j])) / fabs(r0[j]));
      printf("{\"check\": \"variant totals\", \"nv\": %d, \"max_rel_diff\": %.3e}\n", nv, e);
    }
    const double mbytes = 8.0 * N * (nv + 2);
    auto repm = [&](const char *name, float ms) {
      printf("{\"variant\": \"%s\", \"nv\": %d, \"grid\": %d, \"us\": %.1f, \"TBps\": %.3f}\n", name, nv, grid, ms * 1e3,
             mbytes / ms / 1e9);
    };
    repm("maxpy_row", time_it([&] { maxpy_row_kernel<<<grid, 256>>>(N, w, V, ldv, nv, al, part); }, reps));
    repm("maxpy_chunk2", time_it([&] { maxpy_chunk_kernel<2><<<grid, 256>>>(N, w, V, ldv, nv, al, part); }, reps));
    repm("maxpy_chunk4", time_it([&] { maxpy_chunk_kernel<4><<<grid, 256>>>(N, w, V, ldv, nv, al, part); }, reps));
  }
  return 0;
}
