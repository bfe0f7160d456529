// valu_ops2.hip — second probe of gfx950 VALU issue rates (see valu_mix.hip):
// 64-bit shifts as rotations, more encodings, and mixes of FAST ops only.
// Build: hipcc --offload-arch=gfx950 -O3 tools/valu_ops2.hip -o tools/valu_ops2
#include <hip/hip_runtime.h>
#include <stdio.h>

#define R8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

template <int CASE>
__global__ __launch_bounds__(256) void k(uint32_t *out, uint32_t iters) {
  uint64_t p[8];
  uint32_t a[8], b[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    a[i] = threadIdx.x * 7 + i + 1;
    b[i] = blockIdx.x * 13 + i + 3;
    p[i] = ((uint64_t)a[i] << 32) | b[i];
  }
  for (uint32_t it = 0; it < iters; ++it) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#define SHR64(i) asm volatile("v_lshrrev_b64 %0, 7, %0" : "+v"(p[i]));
#define SHL64(i) asm volatile("v_lshlrev_b64 %0, 7, %0" : "+v"(p[i]));
#define ALBY(i) asm volatile("v_alignbyte_b32 %0, %0, %0, 2" : "+v"(a[i]), "+v"(b[i]));
#define OR3(i) asm volatile("v_or3_b32 %0, %0, %1, %1" : "+v"(a[i]), "+v"(b[i]));
#define ANDOR(i) asm volatile("v_and_or_b32 %0, %0, %1, %1" : "+v"(a[i]), "+v"(b[i]));
#define ADDCO(i) asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(a[i]), "+v"(b[i]) : : "vcc");
#define MOV(i) asm volatile("v_mov_b32 %0, %1" : "+v"(a[i]), "+v"(b[i]));
#define BFE(i) asm volatile("v_bfe_u32 %0, %0, 3, 7" : "+v"(a[i]), "+v"(b[i]));
#define MAD24(i) asm volatile("v_mad_u32_u24 %0, %0, %1, %1" : "+v"(a[i]), "+v"(b[i]));
#define ADDF(i) asm volatile("v_add_f32 %0, %0, %1" : "+v"(a[i]), "+v"(b[i]));
#define PKMOV(i) asm volatile("v_pk_mov_b32 %0, %0, %0 op_sel:[1,0]" : "+v"(p[i]));
#define FASTMIX(i) asm volatile("v_xor_b32 %0, %0, %1\n\tv_add_u32 %1, %1, %0\n\tv_bitop3_b32 %0, %0, %1, %1 bitop3:0x96\n\tv_lshrrev_b32 %1, 7, %1" : "+v"(a[i]), "+v"(b[i]));
#define XORADD(i) asm volatile("v_xor_b32 %0, %0, %1\n\tv_add_u32 %1, %1, %0" : "+v"(a[i]), "+v"(b[i]));
#define SUBREV(i) asm volatile("v_subrev_u32 %0, %0, %1" : "+v"(a[i]), "+v"(b[i]));
#define ASHR(i) asm volatile("v_ashrrev_i32 %0, 7, %0" : "+v"(a[i]), "+v"(b[i]));
#define AND(i) asm volatile("v_and_b32 %0, %0, %1" : "+v"(a[i]), "+v"(b[i]));
#define CNDM(i) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[i]), "+v"(b[i]));
#define LSHL2(i) asm volatile("v_lshlrev_b32 %0, %1, %0" : "+v"(a[i]), "+v"(b[i]));
#define LSHLADD64(i) asm volatile("v_lshl_add_u64 %0, %0, 3, %0" : "+v"(p[i]));
#define ADD64(i) asm volatile("v_lshl_add_u64 %0, %0, 0, %0" : "+v"(p[i]));
      if (CASE == 0) { R8(SHR64) }
      if (CASE == 1) { R8(SHL64) }
      if (CASE == 2) { R8(ALBY) }
      if (CASE == 3) { R8(OR3) }
      if (CASE == 4) { R8(ANDOR) }
      if (CASE == 5) { R8(ADDCO) }
      if (CASE == 6) { R8(MOV) }
      if (CASE == 7) { R8(BFE) }
      if (CASE == 8) { R8(MAD24) }
      if (CASE == 9) { R8(ADDF) }
      if (CASE == 10) { R8(PKMOV) }
      if (CASE == 11) { R8(FASTMIX) }
      if (CASE == 12) { R8(XORADD) }
      if (CASE == 13) { R8(SUBREV) }
      if (CASE == 14) { R8(ASHR) }
      if (CASE == 15) { R8(AND) }
      if (CASE == 16) { R8(CNDM) }
      if (CASE == 17) { R8(LSHL2) }
      if (CASE == 18) { R8(LSHLADD64) }
    }
  }
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) r ^= a[i] ^ b[i] ^ (uint32_t)p[i] ^ (uint32_t)(p[i] >> 32);
  if (r == 0x12345678u) out[0] = r;
}

static const int kOps[] = {1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 4, 2, 1, 1, 1, 1, 1, 1};
static const char *kName[] = {"lshrrev_b64", "lshlrev_b64", "alignbyte", "or3", "and_or",
                              "add_co_u32", "mov_b32", "bfe_u32", "mad_u32_u24", "add_f32",
                              "pk_mov_b32", "xor,add,bitop3,lshrrev (fast mix)", "xor,add",
                              "subrev_u32", "ashrrev_i32", "and_b32", "cndmask_b32",
                              "lshlrev_b32 vgpr amount", "lshl_add_u64"};

template <int C>
void run(uint32_t *d, int wps) {
  const uint32_t iters = 10000;
  const int blocks = 256 * wps;
  hipLaunchKernelGGL(k<C>, dim3(blocks), dim3(256), 0, 0, d, iters);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(k<C>, dim3(blocks), dim3(256), 0, 0, d, iters);
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
  run<0>(d, 8); run<1>(d, 8); run<2>(d, 8); run<3>(d, 8); run<4>(d, 8); run<5>(d, 8);
  run<6>(d, 8); run<7>(d, 8); run<8>(d, 8); run<9>(d, 8); run<10>(d, 8); run<11>(d, 8);
  run<12>(d, 8); run<13>(d, 8); run<14>(d, 8); run<15>(d, 8); run<16>(d, 8); run<17>(d, 8);
  run<18>(d, 8);
  run<11>(d, 4); run<12>(d, 4); run<11>(d, 6);
  return 0;
}
