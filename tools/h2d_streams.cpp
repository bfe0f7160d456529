// h2d_streams.cpp — host-side cost of concurrent small H2D copies on many
// streams (the Pack API's eager staging copies, csrc/pack.hip eager_copy):
// T threads, each with its own non-blocking stream (or all on one shared
// stream) and its own pinned buffer, enqueue `pieces` 1 MiB hipMemcpyAsync
// H2D copies, then synchronize.  Prints one JSON line per config: wall ms per
// round, GB/s, and the longest / median host time inside hipMemcpyAsync.
// usage: h2d_streams T ROUNDS [S [PIECE_MIB]]   (S < T: S submitting threads, each with
// one stream, enqueue the T buffers' copies between them -- buffer i on
// thread i % S; default S = T)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <atomic>
#include <chrono>
#include <thread>
#include <vector>

#define CK(x)                                                  \
  do {                                                         \
    if ((x) != hipSuccess) {                                   \
      fprintf(stderr, "%s failed at %d\n", #x, __LINE__);     \
      exit(1);                                                 \
    }                                                          \
  } while (0)

int main(int argc, char **argv) {
  if (argc < 3) return 2;
  const int T = atoi(argv[1]), rounds = atoi(argv[2]);
  const int NS = argc > 3 ? std::max(1, std::min(T, atoi(argv[3]))) : T;
  const size_t piece_mib = argc > 4 ? (size_t)std::max(1, atoi(argv[4])) : 1;
  const size_t bytes = 12ull << 20, piece = piece_mib << 20, pieces = (bytes + piece - 1) / piece;
  std::vector<hipStream_t> st(T);
  std::vector<uint8_t *> h(T), d(T);
  for (int i = 0; i < T; ++i) {
    if (i < NS) CK(hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking));
    CK(hipHostMalloc((void **)&h[i], bytes, hipHostMallocDefault));
    memset(h[i], i, bytes);
    CK(hipMalloc((void **)&d[i], bytes));
  }
  using clk = std::chrono::steady_clock;
  std::vector<double> call_us;
  std::mutex m;
  double best = 1e30, sum = 0;
  std::vector<double> per_round;
  for (int r = 0; r < rounds + 1; ++r) {
    std::atomic<int> go{0};
    std::vector<std::thread> th;
    std::vector<double> mine_all;
    for (int w = 0; w < NS; ++w)
      th.emplace_back([&, w] {
        while (!go.load()) {
        }
        std::vector<double> mine;
        for (size_t p = 0; p < pieces; ++p)
          for (int i = w; i < T; i += NS) {
            const auto a = clk::now();
            const size_t len = std::min(piece, bytes - p * piece);
            CK(hipMemcpyAsync(d[i] + p * piece, h[i] + p * piece, len, hipMemcpyHostToDevice, st[w]));
            mine.push_back(std::chrono::duration<double, std::micro>(clk::now() - a).count());
          }
        CK(hipStreamSynchronize(st[w]));
        std::lock_guard<std::mutex> g(m);
        if (r) call_us.insert(call_us.end(), mine.begin(), mine.end());
      });
    const auto t0 = clk::now();
    go = 1;
    for (auto &t : th) t.join();
    const double ms = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
    if (r) {
      best = std::min(best, ms);
      sum += ms;
      per_round.push_back(ms);
    }
  }
  std::sort(call_us.begin(), call_us.end());
  const double mean = sum / rounds;
  std::sort(per_round.begin(), per_round.end());
  const double med = per_round[per_round.size() / 2];
  printf("{\"piece_mib\": %zu, \"threads\": %d, \"streams\": %d, \"rounds\": %d, \"ms_per_round\": %.3f, \"median_ms\": %.3f, \"best_ms\": %.3f, "
         "\"gbs\": %.2f, \"gbs_median\": %.2f, \"memcpy_call_us_median\": %.1f, \"memcpy_call_us_p99\": %.1f, \"memcpy_call_us_max\": %.1f, "
         "\"sdma\": \"%s\"}\n",
         piece_mib, T, NS, rounds, mean, med, best, (double)bytes * T / (mean * 1e-3) / 1e9,
         (double)bytes * T / (med * 1e-3) / 1e9,
         call_us[call_us.size() / 2], call_us[(size_t)(call_us.size() * 0.99)], call_us.back(),
         getenv("HSA_ENABLE_SDMA") ? getenv("HSA_ENABLE_SDMA") : "default");
  return 0;
}
