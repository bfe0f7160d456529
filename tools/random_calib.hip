// Read-request calibration for random accesses (the chunk-dict probe's
// pattern).  Does the L2 -> fabric request count (TCC_EA0_RDREQ_*) of a
// kernel that makes ONE random 8-B read per thread equal one 128-B line per
// read, at table sizes from L2-resident to far past the Infinity Cache?  If
// it does, the dict probe's ~0.4 line per probe above its line model
// (dict probe) is the probe's own; if not, it is what a random
// read costs on this chip.  Run under rocprofv3 --pmc; launches go in the
// order printed (size-major, then mode, REPS each).
//   mode 0: one 8-B read at a random slot
//   mode 1: an 8-B read at a random slot and one at the next slot (a linear
//           probe of two; same 128-B line 15 times in 16)
//   mode 2: one 64-B record at a random 64-B aligned offset (two 16-B loads)
//   mode 3: mode 0, then a dependent 64-B record read (a probe that hits)
// No stores reach memory (the XOR of what was read is compared with a value
// it cannot take on a zeroed table).
// usage: random_calib [reads_M=16] [sizes_MiB=16,256,4096,12800]
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull;
  return x ^ (x >> 33);
}

template <int MODE>
__global__ __launch_bounds__(256) void random_reads(const uint64_t *__restrict__ table,
                                                    uint64_t slots, uint64_t n, uint64_t seed,
                                                    uint64_t *__restrict__ sink) {
  const uint64_t t = blockIdx.x * 256ull + threadIdx.x;
  if (t >= n) return;
  const uint64_t h = mix64(t ^ seed);
  uint64_t acc = 0;
  if (MODE == 0 || MODE == 3) {
    const uint64_t p = h % slots;
    const uint64_t s = table[p];
    acc ^= s;
    if (MODE == 3) {
      const uint64_t r = (mix64(h) + s) % (slots / 8);  // 64-B records over the same table
      const uint4 *rec = reinterpret_cast<const uint4 *>(table + 8 * r);
      const uint4 a = rec[0], b = rec[1];
      acc ^= (uint64_t)(a.x ^ a.y ^ a.z ^ a.w) ^ ((uint64_t)(b.x ^ b.y ^ b.z ^ b.w) << 32);
    }
  } else if (MODE == 1) {
    const uint64_t p = h % slots;
    acc ^= table[p];
    acc ^= table[(p + 1) % slots] + 1;
  } else {
    const uint64_t r = h % (slots / 8);
    const uint4 *rec = reinterpret_cast<const uint4 *>(table + 8 * r);
    const uint4 a = rec[0], b = rec[1];
    acc ^= (uint64_t)(a.x ^ a.y ^ a.z ^ a.w) ^ ((uint64_t)(b.x ^ b.y ^ b.z ^ b.w) << 32);
  }
  if (acc == 0x0123456789abcdefull) sink[0] = acc;
}

int main(int argc, char **argv) {
  const uint64_t n = (argc > 1 ? strtoull(argv[1], nullptr, 0) : 16ull) << 20;
  std::vector<uint64_t> sizes;
  {
    char buf[256];
    snprintf(buf, sizeof buf, "%s", argc > 2 ? argv[2] : "16,256,4096,12800");
    for (char *tok = strtok(buf, ","); tok; tok = strtok(nullptr, ","))
      sizes.push_back(strtoull(tok, nullptr, 0) << 20);
  }
  const int reps = 3;
  uint64_t *sink;
  CK(hipMalloc(&sink, 64));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const unsigned blocks = (unsigned)((n + 255) / 256);
  for (uint64_t bytes : sizes) {
    uint64_t *table;
    CK(hipMalloc(&table, bytes));
    CK(hipMemset(table, 0, bytes));
    CK(hipDeviceSynchronize());
    const uint64_t slots = bytes / 8;
    for (int mode = 0; mode < 4; ++mode) {
      float best = 1e30f;
      for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(e0, nullptr));
        const uint64_t seed = 0x9E3779B97F4A7C15ull * (uint64_t)(r + 1);
        switch (mode) {
          case 0: hipLaunchKernelGGL(random_reads<0>, dim3(blocks), dim3(256), 0, nullptr, table, slots, n, seed, sink); break;
          case 1: hipLaunchKernelGGL(random_reads<1>, dim3(blocks), dim3(256), 0, nullptr, table, slots, n, seed, sink); break;
          case 2: hipLaunchKernelGGL(random_reads<2>, dim3(blocks), dim3(256), 0, nullptr, table, slots, n, seed, sink); break;
          default: hipLaunchKernelGGL(random_reads<3>, dim3(blocks), dim3(256), 0, nullptr, table, slots, n, seed, sink); break;
        }
        CK(hipGetLastError());
        CK(hipEventRecord(e1, nullptr));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
      }
      printf("{\"table_bytes\": %llu, \"mode\": %d, \"reads\": %llu, \"launches\": %d, \"best_ms\": %.4f}\n",
             (unsigned long long)bytes, mode, (unsigned long long)n, reps, best);
      fflush(stdout);
    }
    CK(hipFree(table));
  }
  CK(hipFree(sink));
  return 0;
}
