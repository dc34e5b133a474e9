// mx_shm_barrier.hpp -- the generation barrier of the shared-memory
// communicator (ShmComm, mx_comm.hip), host-only so it can be built and
// stress-tested under ThreadSanitizer / AddressSanitizer on the CPU
// (tests/native/shm_barrier_test.cpp).
//
// Ranks are processes (or threads) that share one ShmBarrierWords.  The last
// rank to arrive resets the arrival count and bumps the generation; the others
// spin (yielding) until the generation moves.  Every arrival records the
// collective it is in (a tag; 0 = unchecked) in the row of its generation's
// parity: a rank released from generation g may already write its tag for
// g + 1 while a slower rank still checks g's row, and g + 2 cannot start
// before every rank has left g.  A checked barrier whose row holds another tag
// fails as a mismatch (different collectives) instead of racing.
#pragma once

#include <sched.h>

#include <atomic>
#include <chrono>
#include <cstdint>

namespace mx {

constexpr int SHM_MAX = 64;

struct ShmBarrierWords {
  std::atomic<int64_t> arrived, gen;
  std::atomic<int> abort;
  int tags[2][SHM_MAX];
};

enum class BarrierResult { ok, peer_failed, timeout, mismatch };

inline void shm_barrier_init(ShmBarrierWords *h) {
  h->arrived.store(0);
  h->gen.store(0);
  h->abort.store(0);
  for (auto &row : h->tags)
    for (int &t : row) t = 0;
}

inline BarrierResult shm_barrier_wait(ShmBarrierWords *h, int rank, int size, int tag, bool check,
                                      std::chrono::milliseconds timeout) {
  if (h->abort.load()) return BarrierResult::peer_failed;
  // the generation cannot move between this load and this rank's arrival
  const int64_t g = h->gen.load(std::memory_order_acquire);
  int *tg = h->tags[g & 1];
  tg[rank] = check ? tag : 0;
  if (h->arrived.fetch_add(1, std::memory_order_acq_rel) == size - 1) {
    h->arrived.store(0, std::memory_order_relaxed);
    h->gen.fetch_add(1, std::memory_order_acq_rel);
  } else {
    const auto t0 = std::chrono::steady_clock::now();
    int spins = 0;
    while (h->gen.load(std::memory_order_acquire) == g) {
      if (h->abort.load()) return BarrierResult::peer_failed;
      if (++spins > 1000) {
        sched_yield();
        if ((spins & 1023) == 0 && std::chrono::steady_clock::now() - t0 > timeout) {
          h->abort.store(1);
          return BarrierResult::timeout;
        }
      }
    }
  }
  if (check)
    for (int q = 0; q < size; ++q)
      if (tg[q] != tag) {
        h->abort.store(1);
        return BarrierResult::mismatch;
      }
  return BarrierResult::ok;
}

}  // namespace mx
