// contig_alias.hip -- is a physically contiguous allocation
// (hipExtMallocWithFlags(hipDeviceMallocContiguous), the library's knob 18)
// disjoint from the other live allocations of the process, and does its
// content stay put?  T host threads each keep a ring of live buffers, some
// contiguous and some plain hipMalloc, filled on the thread's own stream with
// a per-buffer pattern; after every allocation the thread checks (host) that
// no two live address ranges of the process overlap and (device) that every
// buffer it owns still holds its pattern.  Prints the first violations.
//   hipcc --offload-arch=gfx950 -O2 tools/contig_alias.hip -o tools/contig_alias
//   tools/contig_alias [threads] [rounds] [contig 0/1] [min_kib] [max_kib] [nt 0/1]
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <random>
#include <thread>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); std::exit(2); } } while (0)

// nt: non-temporal stores, as the library's vector kernels write
__global__ void fill_kernel(unsigned long long *p, size_t n, unsigned long long tag, int nt) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const unsigned long long v = tag ^ (i * 0x9E3779B97F4A7C15ULL);
    if (nt) __builtin_nontemporal_store(v, p + i);
    else p[i] = v;
  }
}
// the check walks the buffer with the blocks rotated by `shift` against the
// fill (blocks go round-robin to the 8 XCDs: another XCD's translation of
// each address than the one that wrote it)
__global__ void check_kernel(const unsigned long long *p, size_t n, unsigned long long tag, unsigned long long *bad,
                             int shift) {
  const size_t b = (blockIdx.x + (unsigned)shift) % gridDim.x;
  for (size_t i = b * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    if (p[i] != (tag ^ (i * 0x9E3779B97F4A7C15ULL))) { atomicAdd(bad, 1ull); atomicMin(bad + 1, (unsigned long long)i); }
}

struct Buf { unsigned long long *p; size_t bytes; bool contig; unsigned long long tag; };
std::mutex mu;
std::map<uintptr_t, std::pair<size_t, int>> live;   // start -> (bytes, owner thread)
std::atomic<long> overlaps{0}, corrupt{0}, contig_ok{0}, contig_fail{0};

static void add_range(void *p, size_t b, int t) {
  std::lock_guard<std::mutex> g(mu);
  const uintptr_t s = (uintptr_t)p, e = s + b;
  auto it = live.upper_bound(s);
  if (it != live.end() && it->first < e) {
    if (overlaps++ < 8) std::printf("OVERLAP: new [%#lx, +%zu) thread %d with [%#lx, +%zu) thread %d\n", (unsigned long)s, b, t,
                                    (unsigned long)it->first, it->second.first, it->second.second);
  }
  if (it != live.begin()) {
    auto pv = std::prev(it);
    if (pv->first + pv->second.first > s && overlaps++ < 8)
      std::printf("OVERLAP: new [%#lx, +%zu) thread %d with [%#lx, +%zu) thread %d\n", (unsigned long)s, b, t,
                  (unsigned long)pv->first, pv->second.first, pv->second.second);
  }
  live[s] = {b, t};
}
static void del_range(void *p) { std::lock_guard<std::mutex> g(mu); live.erase((uintptr_t)p); }

int main(int argc, char **argv) {
  const int T = argc > 1 ? std::atoi(argv[1]) : 8;
  const int R = argc > 2 ? std::atoi(argv[2]) : 200;
  const int use_contig = argc > 3 ? std::atoi(argv[3]) : 1;
  const size_t lo = (size_t)(argc > 4 ? std::atoi(argv[4]) : 1024) << 10;
  const size_t hi = (size_t)(argc > 5 ? std::atoi(argv[5]) : 80 * 1024) << 10;
  const int nt = argc > 6 ? std::atoi(argv[6]) : 0;
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t)
    th.emplace_back([=] {
      CK(hipSetDevice(0));
      hipStream_t s;
      CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
      unsigned long long *bad;
      CK(hipMalloc(&bad, 16));
      std::mt19937_64 rng(1234 + t);
      std::vector<Buf> ring;
      std::vector<unsigned long long> host;
      for (int r = 0; r < R; ++r) {
        const size_t bytes = (lo + rng() % (hi - lo + 1)) / 4096 * 4096;
        Buf b{nullptr, bytes, use_contig && (rng() & 1), rng()};
        if (b.contig) {
          if (hipExtMallocWithFlags(reinterpret_cast<void **>(&b.p), bytes, hipDeviceMallocContiguous) == hipSuccess) contig_ok++;
          else { (void)hipGetLastError(); contig_fail++; b.contig = false; }
        }
        if (!b.p) CK(hipMalloc(&b.p, bytes));
        add_range(b.p, bytes, t);
        fill_kernel<<<1024, 256, 0, s>>>(b.p, bytes / 8, b.tag, nt);
        ring.push_back(b);
        // every live buffer of this thread still holds its pattern
        for (const Buf &q : ring) {
          const unsigned long long init[2] = {0ull, ~0ull};
          CK(hipMemcpyAsync(bad, init, 16, hipMemcpyHostToDevice, s));
          check_kernel<<<1024, 256, 0, s>>>(q.p, q.bytes / 8, q.tag, bad, 3);
          unsigned long long h[2];
          CK(hipMemcpyAsync(h, bad, 16, hipMemcpyDeviceToHost, s));
          CK(hipStreamSynchronize(s));
          if (h[0] && corrupt++ < 8)
            std::printf("CORRUPT (kernel): thread %d round %d buffer [%#lx, +%zu) contig %d: %llu words differ, first at byte %llu\n",
                        t, r, (unsigned long)q.p, q.bytes, (int)q.contig, h[0], h[1] * 8);
          // and through the copy engine, compared on the host
          host.resize(q.bytes / 8);
          CK(hipMemcpyAsync(host.data(), q.p, q.bytes, hipMemcpyDeviceToHost, s));
          CK(hipStreamSynchronize(s));
          size_t nb = 0, first = 0;
          for (size_t i = 0; i < host.size(); ++i)
            if (host[i] != (q.tag ^ (i * 0x9E3779B97F4A7C15ULL))) { if (!nb++) first = i; }
          if (nb && corrupt++ < 8)
            std::printf("CORRUPT (copy): thread %d round %d buffer [%#lx, +%zu) contig %d: %zu words differ, first at byte %zu\n",
                        t, r, (unsigned long)q.p, q.bytes, (int)q.contig, nb, first * 8);
        }
        if (ring.size() > 4) {   // free a random one
          const size_t k = rng() % ring.size();
          CK(hipStreamSynchronize(s));
          del_range(ring[k].p);
          CK(hipFree(ring[k].p));
          ring.erase(ring.begin() + k);
        }
      }
      for (const Buf &q : ring) { del_range(q.p); CK(hipFree(q.p)); }
      CK(hipFree(bad));
      CK(hipStreamDestroy(s));
    });
  for (auto &x : th) x.join();
  std::printf("threads %d rounds %d contig %d sizes [%zu, %zu] KiB: contiguous allocations %ld (refused %ld), "
              "overlaps %ld, corrupt buffers %ld\n", T, R, use_contig, lo >> 10, hi >> 10, contig_ok.load(),
              contig_fail.load(), overlaps.load(), corrupt.load());
  return (overlaps || corrupt) ? 1 : 0;
}
