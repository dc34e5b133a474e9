// h2d_pin_probe.hip -- host-to-device copy of the host-CSR payload (1.47 GB at
// 256^3, createAIJ(csr=...) from numpy arrays) three ways:
//   pageable   hipMemcpyAsync from the caller's pages (the runtime stages it);
//   registered hipHostRegister of the whole payload, one copy, unregister;
//   pipelined  chunks registered on the host while the previous chunk's copy
//              runs (register + copy overlapped), each unregistered after.
// Times are host wall clock around the whole operation, median of reps.
//   hipcc --offload-arch=gfx950 -O2 tools/h2d_pin_probe.hip -o tools/h2d_pin_probe
//   tools/h2d_pin_probe [MB] [chunk_MB] [reps] [fresh 0/1] [copy streams]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); std::exit(2); } } while (0)
static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main(int argc, char **argv) {
  const size_t mb = argc > 1 ? std::atol(argv[1]) : 1404;
  const size_t chunk = (size_t)(argc > 2 ? std::atol(argv[2]) : 64) << 20;
  const int reps = argc > 3 ? std::atoi(argv[3]) : 5;
  const size_t bytes = mb << 20;
  char *h = static_cast<char *>(std::aligned_alloc(4096, bytes));
  std::memset(h, 1, bytes);   // the caller's arrays exist (touched) before createAIJ
  void *d;
  CK(hipMalloc(&d, bytes));
  hipStream_t s, s2[4];
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const int ns = argc > 5 ? std::max(1, std::min(4, std::atoi(argv[5]))) : 1;   // pipelined copies round-robin over ns streams
  for (auto &q : s2) CK(hipStreamCreateWithFlags(&q, hipStreamNonBlocking));
  auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
  std::vector<double> tp, tr, treg, tcp, tun, tpipe;
  const bool fresh = argc > 4 && std::atoi(argv[4]) != 0;   // a new (touched) host buffer every rep
  for (int r = 0; r < reps; ++r) {
    if (fresh && r) {
      std::free(h);
      h = static_cast<char *>(std::malloc(bytes));
      std::memset(h, r, bytes);
    }
    double t0 = now();
    CK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s));
    CK(hipStreamSynchronize(s));
    tp.push_back(now() - t0);

    t0 = now();
    CK(hipHostRegister(h, bytes, hipHostRegisterDefault));
    const double t1 = now();
    CK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s));
    CK(hipStreamSynchronize(s));
    const double t2 = now();
    CK(hipHostUnregister(h));
    const double t3 = now();
    treg.push_back(t1 - t0); tcp.push_back(t2 - t1); tun.push_back(t3 - t2); tr.push_back(t3 - t0);

    // pipelined: register chunk i + 1 while chunk i copies; unregister after its copy
    t0 = now();
    const size_t nch = (bytes + chunk - 1) / chunk;
    std::vector<hipEvent_t> ev(nch);
    for (auto &e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (size_t i = 0; i < nch; ++i) {
      const size_t off = i * chunk, len = std::min(chunk, bytes - off);
      CK(hipHostRegister(h + off, len, hipHostRegisterDefault));
      hipStream_t q = ns == 1 ? s : s2[i % ns];
      CK(hipMemcpyAsync(static_cast<char *>(d) + off, h + off, len, hipMemcpyHostToDevice, q));
      CK(hipEventRecord(ev[i], q));
      if (i >= 2) {   // keep two chunks in flight; release the one before
        CK(hipEventSynchronize(ev[i - 2]));
        CK(hipHostUnregister(h + (i - 2) * chunk));
      }
    }
    CK(hipStreamSynchronize(s));
    for (auto &q : s2) CK(hipStreamSynchronize(q));
    for (size_t i = nch >= 2 ? nch - 2 : 0; i < nch; ++i) CK(hipHostUnregister(h + i * chunk));
    tpipe.push_back(now() - t0);
    std::printf("rep %d: pageable %.1f ms, register+copy %.1f ms, pipelined %.1f ms\n", r, tp.back() * 1e3,
                tr.back() * 1e3, tpipe.back() * 1e3);
    for (auto &e : ev) CK(hipEventDestroy(e));
  }
  const double gb = bytes / 1e9;
  std::printf("payload %.2f GB, chunk %zu MB, %d copy stream(s)\n", gb, chunk >> 20, ns);
  std::printf("pageable copy           %7.1f ms  %5.1f GB/s\n", med(tp) * 1e3, gb / med(tp));
  std::printf("register + copy + unreg %7.1f ms  %5.1f GB/s  (register %.1f, copy %.1f = %.1f GB/s, unregister %.1f ms)\n",
              med(tr) * 1e3, gb / med(tr), med(treg) * 1e3, med(tcp) * 1e3, gb / med(tcp), med(tun) * 1e3);
  std::printf("pipelined chunks        %7.1f ms  %5.1f GB/s\n", med(tpipe) * 1e3, gb / med(tpipe));
  return 0;
}
