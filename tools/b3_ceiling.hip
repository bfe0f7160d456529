// b3_ceiling.hip — the issue ceiling of b3_groups' own compression stream.
//
// Runs csrc/b3_compress.hpp's compress() (the exact asm-ordered VALU stream
// of the product kernel) back to back on register-resident data: no loads, no
// tree, no control flow but the loop.  What the chip sustains here, at the
// clock it holds under this stream, is the ceiling b3_groups can reach; the
// bench's frac_mix (against the linear 2-/4-cycle model at 2.4 GHz) is read
// against it in DESIGN.md §3.  One JSON line per occupancy: lane-ops/s with
// 680 algorithmic ops per compression.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/b3_ceiling.hip -o tools/b3_ceiling
// usage: b3_ceiling [WAVES_PER_SIMD ...]   (default 1 2 4 6 8)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

namespace ngpu {
namespace {
#include "../nydus-snapshotter_amd/csrc/b3_compress.hpp"
}  // namespace
}  // namespace ngpu

__global__ __launch_bounds__(256) void b3_ceiling(uint32_t *out, uint32_t iters) {
  using namespace ngpu;
  const uint32_t t = blockIdx.x * 256u + threadIdx.x;
  uint32_t m[16], cv[8];
#pragma unroll
  for (int i = 0; i < 16; ++i) m[i] = t * 0x9E3779B9u + (uint32_t)i * 0x85EBCA6Bu;
  set_iv(cv);
  for (uint32_t it = 0; it < iters; ++it) {
    compress(cv, m, it, 64, CHUNK_START);
    m[0] ^= cv[7];  // keeps the message live across trips (1 op per 680)
  }
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) r ^= cv[i];
  if (r == 0x12345678u) out[t] = r;
}

int main(int argc, char **argv) {
  int wps[16] = {1, 2, 4, 6, 8};
  int nw = 5;
  if (argc > 1) {
    nw = 0;
    for (int i = 1; i < argc && nw < 16; ++i) wps[nw++] = atoi(argv[i]);
  }
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  const int simds = prop.multiProcessorCount * 4;
  uint32_t *d;
  if (hipMalloc(&d, 64u << 20) != hipSuccess) return 1;
  for (int k = 0; k < nw; ++k) {
    const int w = wps[k];
    // waves of 64 lanes: w per SIMD over every SIMD, 4 waves per 256-thread block
    const int blocks = simds * w / 4;
    const uint32_t iters = 2048;
    hipLaunchKernelGGL(b3_ceiling, dim3(blocks), dim3(256), 0, 0, d, iters);  // warm
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int reps = 20;
    (void)hipEventRecord(e0);
    for (int r = 0; r < reps; ++r)
      hipLaunchKernelGGL(b3_ceiling, dim3(blocks), dim3(256), 0, 0, d, iters);
    (void)hipEventRecord(e1);
    if (hipEventSynchronize(e1) != hipSuccess) return 2;
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double ops = (double)reps * blocks * 256.0 * iters * 680.0;
    printf("{\"waves_per_simd\": %d, \"blocks\": %d, \"iters\": %u, \"ms_per_launch\": %.4f, "
           "\"Tops\": %.3f}\n", w, blocks, iters, ms / reps, ops / (ms / 1e3) / 1e12);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
  }
  (void)hipFree(d);
  return 0;
}
