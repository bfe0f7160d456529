// c1_concurrent.cpp — small layers converted concurrently through ONE engine,
// driven from C++ the way a cgo caller would (no Python on the submit path).
// K caller streams; each step enqueues, per stream, ngpu_process_device over
// one copy of the layer plus the D2H of its result table, with T host threads
// submitting (T = 1: one thread round-robins the streams).  Prints one JSON
// line: GB/s of file data, us per layer, host enqueue us per layer.
//
// Mode "pack": T threads each loop the converter.Pack drop-in over the layer
// (ngpu_pack_open, ngpu_pack_write in 1 MiB pieces from pageable memory,
// ngpu_pack_close) on the same engine -- PCIe included; the line splits each
// layer's time into its writes and its close.  Mode "memcpy": T threads each
// copy the layer in 1 MiB pieces from pageable memory into a pinned buffer
// of their own, nothing else -- the host-side ceiling of the pack's writes.
//
// usage: c1_concurrent TAR K T STEPS WARMUP [CHUNK_SIZE] [device|pack|memcpy]
// build: hipcc --offload-arch=gfx950 -O2 -std=c++17 -I../include tools/c1_concurrent.cpp \
//          -o tools/c1_concurrent -L nydus-snapshotter_amd -lnydusgpu -Wl,-rpath,<lib dir>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <thread>
#include <vector>

#include "nydus_gpu.h"

#define CK(x)                                                              \
  do {                                                                     \
    if ((x) != hipSuccess) {                                               \
      fprintf(stderr, "%s failed at %d\n", #x, __LINE__);                 \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

struct Lane {
  hipStream_t s;
  void *d_data;
  ngpu_chunk *d_ch;
  ngpu_result *d_out, *h_out;
};

int main(int argc, char **argv) {
  if (argc < 6) return 2;
  FILE *f = fopen(argv[1], "rb");
  if (!f) return 2;
  std::vector<char> tar;
  char buf[1 << 16];
  size_t r;
  while ((r = fread(buf, 1, sizeof buf, f)) > 0) tar.insert(tar.end(), buf, buf + r);
  fclose(f);
  const int K = atoi(argv[2]), T = atoi(argv[3]), steps = atoi(argv[4]), warm = atoi(argv[5]);
  const uint32_t S = argc > 6 ? (uint32_t)strtoul(argv[6], nullptr, 0) : 0x100000;
  const bool pack = argc > 7 && strcmp(argv[7], "pack") == 0;
  const bool mcpy = argc > 7 && strcmp(argv[7], "memcpy") == 0;
  uint64_t n = 0, nf = 0;
  ngpu_tar_chunks(tar.data(), tar.size(), S, nullptr, 0, &n, &nf);
  std::vector<ngpu_chunk> ch(n);
  if (ngpu_tar_chunks(tar.data(), tar.size(), S, ch.data(), n, &n, &nf)) return 1;
  uint64_t bytes = 0;
  for (auto &c : ch) bytes += c.length;
  ngpu_config cfg;
  memset(&cfg, 0, sizeof cfg);
  cfg.chunk_size = S;
  ngpu_engine *eng = nullptr;
  if (ngpu_create(&cfg, &eng)) return 1;
  using clk = std::chrono::steady_clock;
  if (mcpy) {
    std::vector<uint8_t *> pin(T);
    for (auto &b : pin) CK(hipHostMalloc((void **)&b, tar.size(), hipHostMallocDefault));
    std::atomic<int> ready{0};
    std::atomic<bool> go{false};
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
      th.emplace_back([&, t] {
        ready++;
        while (!go.load()) {
        }
        for (int i = 0; i < steps; ++i)
          for (size_t a = 0; a < tar.size(); a += 1 << 20)
            memcpy(pin[t] + a, tar.data() + a, tar.size() - a < (1u << 20) ? tar.size() - a : (1u << 20));
      });
    while (ready.load() < T) {
    }
    const auto t0 = clk::now();
    go = true;
    for (auto &x : th) x.join();
    const double el = std::chrono::duration<double>(clk::now() - t0).count();
    const double layers = (double)T * steps;
    printf("{\"tool\": \"c1_concurrent\", \"mode\": \"memcpy\", \"threads\": %d, \"steps\": %d, "
           "\"file_bytes_per_layer\": %llu, \"tar_gbs\": %.2f, \"us_per_layer\": %.2f}\n",
           T, steps, (unsigned long long)tar.size(), tar.size() * layers / el / 1e9, el / layers * 1e6);
    for (auto &b : pin) (void)hipHostFree(b);
    ngpu_destroy(eng);
    return 0;
  }
  if (pack) {
    std::vector<double> wr_s(T, 0.0), cl_s(T, 0.0);
    auto layer = [&](std::vector<ngpu_result> &keep, int t) {
      const auto a0 = clk::now();
      ngpu_pack *p = nullptr;
      if (ngpu_pack_open(eng, &p)) exit(1);
      for (size_t a = 0; a < tar.size(); a += 1 << 20) {
        const size_t take = tar.size() - a < (1u << 20) ? tar.size() - a : (1u << 20);
        if (ngpu_pack_write(p, tar.data() + a, take)) {
          fprintf(stderr, "write: %s\n", ngpu_last_error(eng));
          exit(1);
        }
      }
      ngpu_chunk *c = nullptr;
      ngpu_result *res = nullptr;
      uint64_t m = 0;
      const auto a1 = clk::now();
      if (ngpu_pack_close(p, &c, &res, &m, nullptr)) {
        fprintf(stderr, "close: %s\n", ngpu_last_error(eng));
        exit(1);
      }
      const auto a2 = clk::now();
      wr_s[t] += std::chrono::duration<double>(a1 - a0).count();
      cl_s[t] += std::chrono::duration<double>(a2 - a1).count();
      keep.assign(res, res + m);
      ngpu_free_host(c);
      ngpu_free_host(res);
    };
    std::vector<std::vector<ngpu_result>> last(T);
    // every thread warms up its own packs (the engine's pools then hold
    // each thread's pinned staging slots, 64 MiB each and ~40 ms to pin)
    std::atomic<int> ready{0};
    std::atomic<bool> go{false};
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
      th.emplace_back([&, t] {
        for (int i = 0; i < warm; ++i) layer(last[t], t);
        wr_s[t] = cl_s[t] = 0;
        ready++;
        while (!go.load()) {
        }
        for (int i = 0; i < steps; ++i) layer(last[t], t);
      });
    while (ready.load() < T) {
    }
    const auto t0 = clk::now();
    go = true;
    for (auto &x : th) x.join();
    const double el = std::chrono::duration<double>(clk::now() - t0).count();
    int same = 1;
    for (auto &v : last)
      same &= v.size() == last[0].size() &&
              memcmp(v.data(), last[0].data(), v.size() * sizeof(ngpu_result)) == 0;
    const double layers = (double)T * steps;
    double wr = 0, cl = 0;
    for (int t = 0; t < T; ++t) wr += wr_s[t], cl += cl_s[t];
    printf("{\"tool\": \"c1_concurrent\", \"mode\": \"pack\", \"threads\": %d, \"steps\": %d, "
           "\"chunks\": %llu, \"file_bytes_per_layer\": %llu, \"gbs\": %.2f, "
           "\"us_per_layer\": %.2f, \"thread_write_us\": %.1f, \"thread_close_us\": %.1f, "
           "\"results_equal\": %s}\n",
           T, steps, (unsigned long long)n, (unsigned long long)bytes, bytes * layers / el / 1e9,
           el / layers * 1e6, wr / layers * 1e6, cl / layers * 1e6, same ? "true" : "false");
    ngpu_destroy(eng);
    return same ? 0 : 1;
  }
  std::vector<Lane> lanes(K);
  for (auto &l : lanes) {
    CK(hipStreamCreateWithFlags(&l.s, hipStreamNonBlocking));
    CK(hipMalloc(&l.d_data, tar.size()));
    CK(hipMalloc((void **)&l.d_ch, n * sizeof(ngpu_chunk)));
    CK(hipMalloc((void **)&l.d_out, n * sizeof(ngpu_result)));
    CK(hipHostMalloc((void **)&l.h_out, n * sizeof(ngpu_result), hipHostMallocDefault));
    CK(hipMemcpy(l.d_data, tar.data(), tar.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(l.d_ch, ch.data(), n * sizeof(ngpu_chunk), hipMemcpyHostToDevice));
  }
  auto one = [&](Lane &l) {
    if (ngpu_process_device(eng, l.d_data, tar.size(), l.d_ch, n, l.d_out, l.s, nullptr)) {
      fprintf(stderr, "process: %s\n", ngpu_last_error(eng));
      exit(1);
    }
    CK(hipMemcpyAsync(l.h_out, l.d_out, n * sizeof(ngpu_result), hipMemcpyDeviceToHost, l.s));
  };
  auto round = [&](int t) {  // thread t submits its share of the streams
    for (int k = t; k < K; k += T) one(lanes[k]);
  };
  for (int i = 0; i < warm; ++i)
    for (int t = 0; t < T; ++t) round(t);
  CK(hipDeviceSynchronize());
  std::atomic<int> ready{0};
  std::atomic<bool> go{false};
  std::vector<double> enq(T, 0.0);
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t)
    th.emplace_back([&, t] {
      ready++;
      while (!go.load()) {
      }
      const auto a = clk::now();
      for (int i = 0; i < steps; ++i) round(t);
      enq[t] = std::chrono::duration<double>(clk::now() - a).count();
    });
  while (ready.load() < T) {
  }
  const auto t0 = clk::now();
  go = true;
  for (auto &x : th) x.join();
  CK(hipDeviceSynchronize());
  const double el = std::chrono::duration<double>(clk::now() - t0).count();
  double enq_max = 0;
  for (double x : enq) enq_max = x > enq_max ? x : enq_max;
  // every stream's last result table equals stream 0's
  int same = 1;
  for (auto &l : lanes) same &= memcmp(l.h_out, lanes[0].h_out, n * sizeof(ngpu_result)) == 0;
  uint64_t nw = 0;
  for (uint64_t i = 0; i < n; ++i) nw += lanes[0].h_out[i].kind == NGPU_NEW;
  const double layers = (double)K * steps;
  printf("{\"tool\": \"c1_concurrent\", \"mode\": \"device\", \"streams\": %d, \"threads\": %d, \"steps\": %d, "
         "\"chunks\": %llu, \"file_bytes_per_layer\": %llu, \"gbs\": %.2f, \"us_per_layer\": %.2f, "
         "\"host_enqueue_us_per_layer\": %.2f, \"results_equal\": %s, \"new_chunks\": %llu}\n",
         K, T, steps, (unsigned long long)n, (unsigned long long)bytes, bytes * layers / el / 1e9,
         el / layers * 1e6, enq_max / (layers / T) * 1e6, same ? "true" : "false",
         (unsigned long long)nw);
  for (auto &l : lanes) {
    (void)hipFree(l.d_data);
    (void)hipFree(l.d_ch);
    (void)hipFree(l.d_out);
    (void)hipHostFree(l.h_out);
    (void)hipStreamDestroy(l.s);
  }
  ngpu_destroy(eng);
  return same ? 0 : 1;
}
