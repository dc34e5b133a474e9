// Stress test of the shared-memory communicator's barrier protocol
// (mpi-petsc4py-example_amd/csrc/mx_shm_barrier.hpp) on host threads, built
// under ThreadSanitizer and AddressSanitizer/UBSan by tests/test_cpu_sanitizers.py.
//   1. P ranks run checked barriers of varying collectives, each followed at
//      once by the next (barrier -> all-reduce -> exchange ...), with random
//      skew; every rank must see `ok` and the shared payload must be exact.
//   2. ranks entering different collectives must fail (mismatch / peer
//      failed) on every rank, never hang.
#include <cstdio>
#include <random>
#include <thread>
#include <vector>

#include "mx_shm_barrier.hpp"

using namespace mx;

static int run_agreeing(int P, int iters) {
  ShmBarrierWords w;
  shm_barrier_init(&w);
  std::vector<long long> slots(P, 0);       // a payload each collective writes then reads
  std::vector<int> bad(P, 0);
  std::vector<std::thread> ts;
  for (int r = 0; r < P; ++r)
    ts.emplace_back([&, r] {
      std::mt19937 rng(1234 + r);
      for (int it = 0; it < iters; ++it) {
        if (rng() % 4 == 0) std::this_thread::sleep_for(std::chrono::microseconds(rng() % 50));
        const int tag = 1000 + (it % 7);    // the collective of this step
        slots[r] = (long long)it * P + r;   // write my slot, then the checked barrier
        if (shm_barrier_wait(&w, r, P, tag, true, std::chrono::seconds(20)) != BarrierResult::ok) { bad[r] = 1; return; }
        long long sum = 0;
        for (int q = 0; q < P; ++q) sum += slots[q];
        if (sum != (long long)it * P * P + (long long)P * (P - 1) / 2) { bad[r] = 2; return; }
        // everyone has read every slot before any is rewritten
        if (shm_barrier_wait(&w, r, P, 0, false, std::chrono::seconds(20)) != BarrierResult::ok) { bad[r] = 3; return; }
        if (it % 5 == 0 && shm_barrier_wait(&w, r, P, 5, true, std::chrono::seconds(20)) != BarrierResult::ok) { bad[r] = 4; return; }
      }
    });
  for (auto &t : ts) t.join();
  for (int r = 0; r < P; ++r)
    if (bad[r]) { std::printf("agreeing P=%d: rank %d failed (%d)\n", P, r, bad[r]); return 1; }
  return 0;
}

static int run_mismatch(int P) {
  ShmBarrierWords w;
  shm_barrier_init(&w);
  std::vector<BarrierResult> res(P, BarrierResult::ok);
  std::vector<std::thread> ts;
  for (int r = 0; r < P; ++r)
    ts.emplace_back([&, r] {
      BarrierResult a = shm_barrier_wait(&w, r, P, 7, true, std::chrono::seconds(20));
      if (a != BarrierResult::ok) { res[r] = a; return; }
      // rank 0 enters another collective than the others
      res[r] = shm_barrier_wait(&w, r, P, r == 0 ? 8 : 9, true, std::chrono::milliseconds(2000));
    });
  for (auto &t : ts) t.join();
  for (int r = 0; r < P; ++r)
    if (res[r] == BarrierResult::ok) { std::printf("mismatch P=%d: rank %d saw ok\n", P, r); return 1; }
  return 0;
}

int main() {
  int fails = 0;
  for (int P : {2, 3, 4, 8}) fails += run_agreeing(P, 3000);
  for (int P : {2, 4}) fails += run_mismatch(P);
  std::printf(fails ? "FAIL\n" : "OK\n");
  return fails ? 1 : 0;
}
