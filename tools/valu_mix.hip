// valu_mix.hip — when does gfx950 issue a wave64 VALU op faster than 4
// cycles per SIMD?  tools/valu_ops.hip shows v_xor_b32 / v_add_u32 /
// v_bitop3_b32 / v_fma_f32 reaching ~1.6-1.8x the 4-cycle rate at 8 waves per
// SIMD while v_alignbit / v_add3 / v_perm / v_bfi stay at 4 cycles.  This
// probes mixes: fast and slow ops interleaved, grouped, encodings, and the
// number of waves needed.  One JSON line per case: lane-ops/s.
// Build: hipcc --offload-arch=gfx950 -O3 tools/valu_mix.hip -o tools/valu_mix
#include <hip/hip_runtime.h>
#include <stdio.h>

#define R8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

template <int CASE>
__global__ __launch_bounds__(256) void mix(uint32_t *out, uint32_t iters) {
  uint32_t a[8], b[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    a[i] = threadIdx.x * 7 + i + 1;
    b[i] = blockIdx.x * 13 + i + 3;
  }
  const bool hi = (threadIdx.x >> 6) & 1;  // odd waves of the block
  for (uint32_t it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
#define XOR(i) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[i]), "+v"(b[i]));
#define XOR64(i) asm volatile("v_xor_b32_e64 %0, %0, %1" : "+v"(a[i]), "+v"(b[i]));
#define ALB(i) asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(a[i]), "+v"(b[i]));
#define ADD(i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]), "+v"(b[i]));
#define ADD3(i) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(a[i]), "+v"(b[i]));
#define OR(i) asm volatile("v_or_b32 %0, %0, %1" : "+v"(a[i]), "+v"(b[i]));
#define SHL(i) asm volatile("v_lshlrev_b32 %0, 7, %0" : "+v"(a[i]), "+v"(b[i]));
#define SHR(i) asm volatile("v_lshrrev_b32 %0, 7, %0" : "+v"(a[i]), "+v"(b[i]));
#define LSHLOR(i) asm volatile("v_lshl_or_b32 %0, %0, 7, %1" : "+v"(a[i]), "+v"(b[i]));
#define XA(i) asm volatile("v_xor_b32 %0, %0, %1\n\tv_alignbit_b32 %0, %0, %0, 7" : "+v"(a[i]), "+v"(b[i]));
#define XAXA(i) asm volatile("v_xor_b32 %0, %0, %1\n\tv_alignbit_b32 %0, %0, %0, 7\n\tv_add_u32 %1, %1, %0\n\tv_alignbit_b32 %1, %1, %1, 12" : "+v"(a[i]), "+v"(b[i]));
#define ROTSH(i) asm volatile("v_lshlrev_b32 %1, 7, %0\n\tv_lshrrev_b32 %0, 25, %0\n\tv_or_b32 %0, %0, %1" : "+v"(a[i]), "+v"(b[i]));
#define BOP3(i) asm volatile("v_bitop3_b32 %0, %0, %1, %1 bitop3:0x96" : "+v"(a[i]), "+v"(b[i]));
#define SUB(i) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(a[i]), "+v"(b[i]));
      if (CASE == 0) { R8(XOR) }                       // fast only (reference)
      if (CASE == 1) { R8(ALB) }                       // slow only (reference)
      if (CASE == 2) { R8(XA) }                        // xor, alignbit interleaved per chain
      if (CASE == 3) { R8(XOR) R8(ALB) }               // 8 xor then 8 alignbit
      if (CASE == 4) { if (hi) { R8(XOR) R8(XOR) } else { R8(ALB) R8(ALB) } }  // per-wave split
      if (CASE == 5) { R8(XOR64) }                     // VOP3 encoding of xor
      if (CASE == 6) { R8(ADD) }
      if (CASE == 7) { R8(OR) }
      if (CASE == 8) { R8(SHL) }
      if (CASE == 9) { R8(SHR) }
      if (CASE == 10) { R8(LSHLOR) }
      if (CASE == 11) { R8(XAXA) }                     // BLAKE3-like 1:1 fast/slow
      if (CASE == 12) { R8(ROTSH) }                    // rotate as shl/shr/or
      if (CASE == 13) { R8(ADD3) }
      if (CASE == 14) { R8(SUB) }
      if (CASE == 15) { R8(BOP3) R8(ALB) }
    }
  }
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) r ^= a[i] ^ b[i];
  if (r == 0x12345678u) out[0] = r;
}

// instructions per chain step for each case (lane-ops counted = instructions)
static const int kOps[] = {1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1, 4, 3, 1, 1, 2};
static const char *kName[] = {"xor", "alignbit", "xor,alignbit interleaved", "8xor then 8alignbit",
                              "odd waves xor / even waves alignbit", "xor_e64", "add_u32", "or",
                              "lshlrev", "lshrrev", "lshl_or", "xor,alb,add,alb (G-like)",
                              "rot as shl,shr,or", "add3", "sub_u32", "8bitop3 then 8alignbit"};

template <int C>
void run(uint32_t *d, int wps) {
  const uint32_t iters = 10000;
  const int blocks = 256 * wps;
  hipLaunchKernelGGL(mix<C>, dim3(blocks), dim3(256), 0, 0, d, iters);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(mix<C>, dim3(blocks), dim3(256), 0, 0, d, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double ops = 3.0 * blocks * 256 * iters * 4 * 8 * kOps[C];
  printf("{\"case\": \"%s\", \"waves_per_simd\": %d, \"Tops\": %.2f}\n", kName[C], wps,
         ops / (ms / 1e3) / 1e12);
}

int main() {
  uint32_t *d;
  (void)hipMalloc(&d, 4);
  for (int w : {2, 4, 8}) run<0>(d, w);
  run<1>(d, 8); run<2>(d, 8); run<3>(d, 8); run<4>(d, 8); run<5>(d, 8); run<6>(d, 8);
  run<7>(d, 8); run<8>(d, 8); run<9>(d, 8); run<10>(d, 8); run<11>(d, 8); run<12>(d, 8);
  run<13>(d, 8); run<14>(d, 8); run<15>(d, 8);
  run<11>(d, 4); run<2>(d, 4);
  return 0;
}
