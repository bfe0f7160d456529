// valu_peak.hip — microbenchmark for the gfx950 integer VALU roofline used in
// DESIGN.md §3 (SURVEY.md §8(d) asks to validate P_int on the box).
// Each lane runs NCH independent chains of BLAKE3-style ops
// (v_add3_u32 + v_xor_b32 + v_alignbit_b32); waves per SIMD are set by the
// grid.  Prints lane-ops/s for each (chains, waves/SIMD) point.
// Build: hipcc --offload-arch=gfx950 -O3 tools/valu_peak.hip -o valu_peak
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int NCH>
__global__ __launch_bounds__(256) void chains(uint32_t *out, uint32_t iters, uint32_t seed) {
  uint32_t a[NCH], b[NCH];
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    a[i] = seed + threadIdx.x * 7 + i;
    b[i] = seed ^ (blockIdx.x * 13 + i);
  }
  for (uint32_t it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
#pragma unroll
      for (int i = 0; i < NCH; ++i)  // exactly 3 VALU ops per chain step
        asm volatile("v_add3_u32 %0, %0, %1, %2\n\tv_xor_b32 %1, %1, %0\n\t"
                     "v_alignbit_b32 %1, %1, %1, 16"
                     : "+v"(a[i]), "+v"(b[i]) : "v"(it));
    }
  }
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < NCH; ++i) r ^= a[i] ^ b[i];
  if (r == 0x12345678u) out[0] = r;  // keep live
}

template <int NCH>
double run(int blocks, uint32_t iters) {
  uint32_t *d;
  (void)hipMalloc(&d, 4);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(chains<NCH>, dim3(blocks), dim3(256), 0, 0, d, iters, 1u);
  (void)hipEventRecord(e0);
  for (int r = 0; r < 5; ++r)
    hipLaunchKernelGGL(chains<NCH>, dim3(blocks), dim3(256), 0, 0, d, iters, 1u);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double ops = 5.0 * blocks * 256.0 * iters * 4 * NCH * 3;  // add3 + xor + alignbit
  (void)hipFree(d);
  return ops / (ms / 1e3);
}

int main() {
  const uint32_t iters = 20000;
  // 256 CUs; 256-thread blocks = 4 waves = 1 wave per SIMD per block/CU
  for (int wps : {1, 2, 4, 8}) {
    const int blocks = 256 * wps;
    printf("{\"waves_per_simd\": %d, \"chains\": 1, \"Tops\": %.2f}\n", wps, run<1>(blocks, iters) / 1e12);
    printf("{\"waves_per_simd\": %d, \"chains\": 2, \"Tops\": %.2f}\n", wps, run<2>(blocks, iters) / 1e12);
    printf("{\"waves_per_simd\": %d, \"chains\": 4, \"Tops\": %.2f}\n", wps, run<4>(blocks, iters) / 1e12);
    printf("{\"waves_per_simd\": %d, \"chains\": 8, \"Tops\": %.2f}\n", wps, run<8>(blocks, iters) / 1e12);
  }
  return 0;
}
