// valu_exec.hip — does a wave with a partial EXEC mask issue VALU ops faster
// than a full wave64 on gfx950, and what is the dependent-chain latency?
// Decides how SHA-256 (one serial chain per nydus chunk) should lay chunks
// onto lanes.  One wave per SIMD (256-thread blocks, one block per CU) unless
// stated; s_memtime (shader clock) read by lane 0 of block 0.
// Build: hipcc --offload-arch=gfx950 -O3 tools/valu_exec.hip -o tools/valu_exec
#include <hip/hip_runtime.h>
#include <stdio.h>

#define IND8(INSN)                                              \
  asm volatile(INSN "\n" : "+v"(a[0]) : "v"(b[0]));             \
  asm volatile(INSN "\n" : "+v"(a[1]) : "v"(b[1]));             \
  asm volatile(INSN "\n" : "+v"(a[2]) : "v"(b[2]));             \
  asm volatile(INSN "\n" : "+v"(a[3]) : "v"(b[3]));             \
  asm volatile(INSN "\n" : "+v"(a[4]) : "v"(b[4]));             \
  asm volatile(INSN "\n" : "+v"(a[5]) : "v"(b[5]));             \
  asm volatile(INSN "\n" : "+v"(a[6]) : "v"(b[6]));             \
  asm volatile(INSN "\n" : "+v"(a[7]) : "v"(b[7]));
#define DEP8(INSN)                                              \
  asm volatile(INSN "\n" : "+v"(a[0]) : "v"(b[0]));             \
  asm volatile(INSN "\n" : "+v"(a[0]) : "v"(b[1]));             \
  asm volatile(INSN "\n" : "+v"(a[0]) : "v"(b[2]));             \
  asm volatile(INSN "\n" : "+v"(a[0]) : "v"(b[3]));             \
  asm volatile(INSN "\n" : "+v"(a[0]) : "v"(b[4]));             \
  asm volatile(INSN "\n" : "+v"(a[0]) : "v"(b[5]));             \
  asm volatile(INSN "\n" : "+v"(a[0]) : "v"(b[6]));             \
  asm volatile(INSN "\n" : "+v"(a[0]) : "v"(b[7]));

// OP: 0 xor, 1 alignbit.  DEP: one dependent chain instead of 8 independent.
template <int OP, bool DEP>
__global__ __launch_bounds__(256) void ops(uint32_t *out, uint64_t *clk, uint32_t iters,
                                           uint32_t active) {
  uint32_t a[8], b[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    a[i] = threadIdx.x * 7 + i + 1;
    b[i] = blockIdx.x * 13 + i + 3;
  }
  const bool timer = blockIdx.x == 0 && threadIdx.x == 0;
  uint64_t t0 = 0;
  if (timer) t0 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) < active) {
    for (uint32_t it = 0; it < iters; ++it) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (OP == 0 && !DEP) { IND8("v_xor_b32 %0, %0, %1") }
        if (OP == 1 && !DEP) { IND8("v_alignbit_b32 %0, %0, %1, 7") }
        if (OP == 0 && DEP) { DEP8("v_xor_b32 %0, %0, %1") }
        if (OP == 1 && DEP) { DEP8("v_alignbit_b32 %0, %0, %1, 7") }
      }
    }
  }
  if (timer) clk[0] = __builtin_amdgcn_s_memtime() - t0;
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) r ^= a[i] ^ b[i];
  if (r == 0x12345678u) out[0] = r;
}

template <int OP, bool DEP>
void run(uint32_t *d, uint64_t *dc, int wps, uint32_t active) {
  const uint32_t iters = 20000;
  const int blocks = 256 * wps;
  hipLaunchKernelGGL((ops<OP, DEP>), dim3(blocks), dim3(256), 0, 0, d, dc, iters, active);
  (void)hipDeviceSynchronize();
  hipLaunchKernelGGL((ops<OP, DEP>), dim3(blocks), dim3(256), 0, 0, d, dc, iters, active);
  (void)hipDeviceSynchronize();
  uint64_t cyc = 0;
  (void)hipMemcpy(&cyc, dc, 8, hipMemcpyDeviceToHost);
  const double per_wave = (double)iters * 4 * 8;  // instructions one wave issues
  printf("{\"op\": \"%s\", \"chain\": \"%s\", \"waves_per_simd\": %d, \"active_lanes\": %u, "
         "\"cyc_per_instr_per_wave\": %.3f}\n",
         OP ? "v_alignbit_b32" : "v_xor_b32", DEP ? "dependent" : "8 independent", wps, active,
         cyc / per_wave);
}

int main() {
  uint32_t *d;
  uint64_t *dc;
  (void)hipMalloc(&d, 4);
  (void)hipMalloc(&dc, 8);
  for (uint32_t act : {64u, 32u, 16u, 1u}) {
    run<0, false>(d, dc, 1, act);
    run<1, false>(d, dc, 1, act);
  }
  for (int wps : {1, 2, 4}) {
    run<0, true>(d, dc, wps, 64);
    run<1, true>(d, dc, wps, 64);
  }
  run<1, true>(d, dc, 1, 16);
  return 0;
}
