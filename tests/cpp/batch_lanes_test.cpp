// batch_lanes_test.cpp — the batcher's lane table (csrc/batch_lanes.hpp) on
// the CPU, under ThreadSanitizer: leader threads take idle lanes for batches,
// every batch's K "packs" report its end from their own threads in random
// order and at random delays, and a lane must never be taken while one of the
// batches it ran is still unfinished.  Checked: the lane in use count never
// exceeds one per lane, every batch is freed exactly once, a stale report
// (a pack of the lane's previous batch) never frees the lane's current batch.
// usage: batch_lanes_test SEED
#include <stdio.h>
#include <stdlib.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <random>
#include <thread>
#include <vector>

#include "batch_lanes.hpp"

int main(int argc, char **argv) {
  const unsigned seed = argc > 1 ? (unsigned)atoi(argv[1]) : 1;
  constexpr int L = 4, kBatches = 400, kPacks = 5;
  ngpu::LaneTable<L> t;
  std::mutex m;
  std::condition_variable cv;
  std::atomic<int> in_use[L] = {};   // batches the lane is running (must stay <= 1)
  std::atomic<int> freed{0}, stale{0}, bad{0};
  std::vector<std::thread> packs;
  std::mutex pm;
  // stale reports: (lane, seq) of batches already freed, replayed later
  std::vector<std::pair<int, uint64_t>> done_batches;
  std::mt19937 rng(seed);
  for (int b = 0; b < kBatches; ++b) {
    int k;
    uint64_t s;
    {
      std::unique_lock<std::mutex> g(m);
      cv.wait(g, [&] { return t.idle() >= 0; });
      k = t.idle();
      s = t.take(k);
    }
    if (in_use[k].fetch_add(1) != 0) bad.fetch_add(1);  // lane reused under a running batch
    const unsigned d0 = rng() % 200;
    std::lock_guard<std::mutex> g(pm);
    for (int p = 0; p < kPacks; ++p) {
      const unsigned d = d0 + rng() % 300;  // the batch "runs" ~d0 us, its packs come back spread
      packs.emplace_back([&, k, s, d] {
        std::this_thread::sleep_for(std::chrono::microseconds(d));
        std::lock_guard<std::mutex> g2(m);
        // the batch has ended once any pack is back: the lane's run ends here
        if (t.end(k, s)) {
          in_use[k].fetch_sub(1);
          freed.fetch_add(1);
          done_batches.emplace_back(k, s);
          cv.notify_all();
        }
      });
    }
  }
  {
    std::lock_guard<std::mutex> g(pm);
    for (auto &th : packs) th.join();
  }
  // late reports of finished batches, after their lanes were retaken
  {
    std::unique_lock<std::mutex> g(m);
    for (int k = 0; k < L; ++k)
      if (t.idle() >= 0) {
        const int i = t.idle();
        t.take(i);
      }
    for (auto &d : done_batches)
      if (t.end(d.first, d.second)) stale.fetch_add(1);
  }
  if (bad.load() || freed.load() != kBatches || stale.load()) {
    printf("FAIL bad=%d freed=%d stale=%d\n", bad.load(), freed.load(), stale.load());
    return 1;
  }
  printf("ok %d batches on %d lanes\n", kBatches, L);
  return 0;
}
