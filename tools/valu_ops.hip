// valu_ops.hip — per-instruction VALU throughput on gfx950 (which integer ops
// issue at 4 cycles per wave64 instruction and which faster), to pin the
// integer roofline used in DESIGN.md §3.  Each lane runs 8 independent
// chains of ONE instruction kind; 8 waves per SIMD.  The shader clock is read
// with s_memtime in the kernel (one lane), so cycles per wave-instruction per
// SIMD are reported directly, independent of DVFS.
// Build: hipcc --offload-arch=gfx950 -O3 tools/valu_ops.hip -o tools/valu_ops
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CHAIN8(INSN)                                                                     \
  asm volatile(INSN "\n" : "+v"(a[0]), "+v"(b[0]));                                      \
  asm volatile(INSN "\n" : "+v"(a[1]), "+v"(b[1]));                                      \
  asm volatile(INSN "\n" : "+v"(a[2]), "+v"(b[2]));                                      \
  asm volatile(INSN "\n" : "+v"(a[3]), "+v"(b[3]));                                      \
  asm volatile(INSN "\n" : "+v"(a[4]), "+v"(b[4]));                                      \
  asm volatile(INSN "\n" : "+v"(a[5]), "+v"(b[5]));                                      \
  asm volatile(INSN "\n" : "+v"(a[6]), "+v"(b[6]));                                      \
  asm volatile(INSN "\n" : "+v"(a[7]), "+v"(b[7]));

template <int OP>
__global__ __launch_bounds__(256) void ops(uint32_t *out, uint64_t *clk, uint32_t iters) {
  uint32_t a[8], b[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    a[i] = threadIdx.x * 7 + i + 1;
    b[i] = blockIdx.x * 13 + i + 3;
  }
  uint64_t t0 = 0;
  if (blockIdx.x == 0 && threadIdx.x == 0) t0 = __builtin_amdgcn_s_memtime();
  for (uint32_t it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (OP == 0) { CHAIN8("v_xor_b32 %0, %0, %1") }
      if (OP == 1) { CHAIN8("v_add_u32 %0, %0, %1") }
      if (OP == 2) { CHAIN8("v_alignbit_b32 %0, %0, %1, 7") }
      if (OP == 3) { CHAIN8("v_add3_u32 %0, %0, %1, %1") }
      if (OP == 4) { CHAIN8("v_bitop3_b32 %0, %0, %1, %1 bitop3:0x96") }
      if (OP == 5) { CHAIN8("v_perm_b32 %0, %0, %1, %1") }
      if (OP == 6) { CHAIN8("v_fma_f32 %0, %0, %1, %1") }
      if (OP == 7) { CHAIN8("v_pk_add_u16 %0, %0, %1") }
      if (OP == 8) { CHAIN8("v_xad_u32 %0, %0, %1, %1") }
      if (OP == 9) { CHAIN8("v_lshl_add_u32 %0, %0, 3, %1") }
      if (OP == 10) { CHAIN8("v_mul_lo_u32 %0, %0, %1") }
      if (OP == 11) { CHAIN8("v_bfi_b32 %0, %0, %1, %1") }
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) clk[0] = __builtin_amdgcn_s_memtime() - t0;
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) r ^= a[i] ^ b[i];
  if (r == 0x12345678u) out[0] = r;
}

static const char *kNames[] = {"v_xor_b32", "v_add_u32", "v_alignbit_b32", "v_add3_u32",
                               "v_bitop3_b32", "v_perm_b32", "v_fma_f32", "v_pk_add_u16",
                               "v_xad_u32", "v_lshl_add_u32", "v_mul_lo_u32", "v_bfi_b32"};

template <int OP>
void run(uint32_t *d, uint64_t *dc, int wps) {
  const uint32_t iters = 20000;
  const int blocks = 256 * wps;  // 256-thread blocks: one wave per SIMD per block
  hipLaunchKernelGGL(ops<OP>, dim3(blocks), dim3(256), 0, 0, d, dc, iters);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(ops<OP>, dim3(blocks), dim3(256), 0, 0, d, dc, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  uint64_t cyc = 0;
  (void)hipMemcpy(&cyc, dc, 8, hipMemcpyDeviceToHost);
  // wave-instructions per SIMD over the kernel: waves/SIMD x per-wave count
  const double per_simd = (double)wps * iters * 4 * 8;
  // s_memtime runs at a constant 100 MHz reference on some parts; report both
  const double lane_ops = (double)blocks * 256 * iters * 4 * 8;
  printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f, \"Tops\": %.2f, "
         "\"memtime_ticks\": %llu, \"clock_ghz\": %.3f, \"cyc_per_wave_instr_per_simd\": %.3f}\n",
         kNames[OP], wps, ms, lane_ops / (ms / 1e3) / 1e12, (unsigned long long)cyc,
         cyc / (ms * 1e6), cyc / per_simd);
}

int main() {
  uint32_t *d;
  uint64_t *dc;
  (void)hipMalloc(&d, 4);
  (void)hipMalloc(&dc, 8);
  for (int wps : {1, 8}) {
    run<0>(d, dc, wps); run<1>(d, dc, wps); run<2>(d, dc, wps); run<3>(d, dc, wps);
    run<4>(d, dc, wps); run<5>(d, dc, wps); run<6>(d, dc, wps); run<7>(d, dc, wps);
    run<8>(d, dc, wps); run<9>(d, dc, wps); run<10>(d, dc, wps); run<11>(d, dc, wps);
  }
  return 0;
}
