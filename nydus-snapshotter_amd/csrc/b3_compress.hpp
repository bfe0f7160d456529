// b3_compress.hpp — the BLAKE3 compression function in the VALU issue order
// the gfx950 kernels use (blake3.hip) and the ceiling microbenchmark
// (tools/b3_ceiling.hip) measures.  Included INSIDE a namespace block (it
// has no includes of its own); needs <stdint.h> and the HIP device runtime.
#pragma once

constexpr uint32_t IV0 = 0x6A09E667u, IV1 = 0xBB67AE85u, IV2 = 0x3C6EF372u,
                   IV3 = 0xA54FF53Au, IV4 = 0x510E527Fu, IV5 = 0x9B05688Cu,
                   IV6 = 0x1F83D9ABu, IV7 = 0x5BE0CD19u;
enum : uint32_t { CHUNK_START = 1, CHUNK_END = 2, PARENT = 4, ROOT = 8 };

// Message word schedule: round r uses the permutation applied r times.
struct Sched { uint8_t s[7][16]; };
constexpr Sched make_sched() {
  Sched t{};
  const uint8_t perm[16] = {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8};
  uint8_t cur[16] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15};
  for (int r = 0; r < 7; ++r) {
    for (int i = 0; i < 16; ++i) t.s[r][i] = cur[i];
    uint8_t nxt[16] = {};
    for (int i = 0; i < 16; ++i) nxt[i] = cur[perm[i]];
    for (int i = 0; i < 16; ++i) cur[i] = nxt[i];
  }
  return t;
}
constexpr Sched kSched = make_sched();

// In-place compression: cv <- first 8 output words.
//
// The VALU issue order is fixed by hand (inline asm, one op per statement;
// volatile statements keep their order): the 4 independent G of a column /
// diagonal step advance in lockstep, so the 2-cycle ops (v_xor, v_add) issue
// in runs of 4 and 8 between runs of 4-cycle ops (v_add3, v_alignbit).  The
// compiler's own schedule of the same G macro alternates them one by one and
// is 6 % slower on the box (5.89 -> 5.52 ms per 16 GiB C2 launch,
// profiles/r1/ab_issue_order.jsonl); SDWA rotr16 and split v_add3 were
// measured there too and lose, and two leaves per lane in lockstep (runs of
// 8, 108 VGPRs) gain nothing over runs of 4.  Round 2 (same-box A/B): the
// same order in plain C++ behind sched_barriers -- no conservative s_nop
// hazard pads around the asm, 1006 -> 66 s_nops -- is 2.5 % SLOWER
// (profiles/r2/ab_g4_noasm_r2nop.json); all-8-byte encodings with every
// step 8-byte aligned change nothing (ab_g4_e64_r2e64.json).
#define B3_OP3(op, a, b, x) asm volatile(op " %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(x))
#define B3_OP2(op, a, b) asm volatile(op " %0, %0, %1" : "+v"(a) : "v"(b))
#define B3_ROT(a, n) asm volatile("v_alignbit_b32 %0, %0, %0, " #n : "+v"(a))
// One column or diagonal step (4 G in lockstep).
#define B3_G4(a0, b0, c0, d0, a1, b1, c1, d1, a2, b2, c2, d2, a3, b3, c3, d3, x0, x1, x2, x3, \
              y0, y1, y2, y3)                                                               \
  do {                                                                                      \
    B3_OP3("v_add3_u32", a0, b0, x0); B3_OP3("v_add3_u32", a1, b1, x1);                    \
    B3_OP3("v_add3_u32", a2, b2, x2); B3_OP3("v_add3_u32", a3, b3, x3);                    \
    B3_OP2("v_xor_b32", d0, a0); B3_OP2("v_xor_b32", d1, a1);                              \
    B3_OP2("v_xor_b32", d2, a2); B3_OP2("v_xor_b32", d3, a3);                              \
    B3_ROT(d0, 16); B3_ROT(d1, 16); B3_ROT(d2, 16); B3_ROT(d3, 16);                         \
    B3_OP2("v_add_u32", c0, d0); B3_OP2("v_add_u32", c1, d1);                              \
    B3_OP2("v_add_u32", c2, d2); B3_OP2("v_add_u32", c3, d3);                              \
    B3_OP2("v_xor_b32", b0, c0); B3_OP2("v_xor_b32", b1, c1);                              \
    B3_OP2("v_xor_b32", b2, c2); B3_OP2("v_xor_b32", b3, c3);                              \
    B3_ROT(b0, 12); B3_ROT(b1, 12); B3_ROT(b2, 12); B3_ROT(b3, 12);                         \
    B3_OP3("v_add3_u32", a0, b0, y0); B3_OP3("v_add3_u32", a1, b1, y1);                    \
    B3_OP3("v_add3_u32", a2, b2, y2); B3_OP3("v_add3_u32", a3, b3, y3);                    \
    B3_OP2("v_xor_b32", d0, a0); B3_OP2("v_xor_b32", d1, a1);                              \
    B3_OP2("v_xor_b32", d2, a2); B3_OP2("v_xor_b32", d3, a3);                              \
    B3_ROT(d0, 8); B3_ROT(d1, 8); B3_ROT(d2, 8); B3_ROT(d3, 8);                             \
    B3_OP2("v_add_u32", c0, d0); B3_OP2("v_add_u32", c1, d1);                              \
    B3_OP2("v_add_u32", c2, d2); B3_OP2("v_add_u32", c3, d3);                              \
    B3_OP2("v_xor_b32", b0, c0); B3_OP2("v_xor_b32", b1, c1);                              \
    B3_OP2("v_xor_b32", b2, c2); B3_OP2("v_xor_b32", b3, c3);                              \
    B3_ROT(b0, 7); B3_ROT(b1, 7); B3_ROT(b2, 7); B3_ROT(b3, 7);                             \
  } while (0)

// The first column step with the constant row folded in: v8..v11 = IV0..IV3
// enter as VOP2 literals of the c += d adds, v12 / v14 / v15 (counter, block
// length, flags) as sources of 3-operand xors, and v13 = 0 drops its xor.
// Saves the 8 register copies and 1 xor per compression that initialising
// v8..v15 in place costs.
#define B3_XORTO(o, x, y) asm volatile("v_xor_b32 %0, %1, %2" : "=v"(o) : "v"(x), "v"(y))
#define B3_ADDLIT(o, k, y) asm volatile("v_add_u32 %0, %1, %2" : "=v"(o) : "i"(k), "v"(y))
#define B3_G4_FIRST(x0, x1, x2, x3, y0, y1, y2, y3)                                      \
  do {                                                                                  \
    B3_OP3("v_add3_u32", v0, v4, x0); B3_OP3("v_add3_u32", v1, v5, x1);                \
    B3_OP3("v_add3_u32", v2, v6, x2); B3_OP3("v_add3_u32", v3, v7, x3);                \
    B3_XORTO(v12, counter, v0); B3_XORTO(v14, blen, v2); B3_XORTO(v15, flags, v3);     \
    B3_ROT(v12, 16);                                                                    \
    asm volatile("v_alignbit_b32 %0, %1, %1, 16" : "=v"(v13) : "v"(v1));                \
    B3_ROT(v14, 16); B3_ROT(v15, 16);                                                   \
    B3_ADDLIT(v8, IV0, v12); B3_ADDLIT(v9, IV1, v13);                                   \
    B3_ADDLIT(v10, IV2, v14); B3_ADDLIT(v11, IV3, v15);                                 \
    B3_OP2("v_xor_b32", v4, v8); B3_OP2("v_xor_b32", v5, v9);                           \
    B3_OP2("v_xor_b32", v6, v10); B3_OP2("v_xor_b32", v7, v11);                         \
    B3_ROT(v4, 12); B3_ROT(v5, 12); B3_ROT(v6, 12); B3_ROT(v7, 12);                     \
    B3_OP3("v_add3_u32", v0, v4, y0); B3_OP3("v_add3_u32", v1, v5, y1);                \
    B3_OP3("v_add3_u32", v2, v6, y2); B3_OP3("v_add3_u32", v3, v7, y3);                \
    B3_OP2("v_xor_b32", v12, v0); B3_OP2("v_xor_b32", v13, v1);                         \
    B3_OP2("v_xor_b32", v14, v2); B3_OP2("v_xor_b32", v15, v3);                         \
    B3_ROT(v12, 8); B3_ROT(v13, 8); B3_ROT(v14, 8); B3_ROT(v15, 8);                     \
    B3_OP2("v_add_u32", v8, v12); B3_OP2("v_add_u32", v9, v13);                         \
    B3_OP2("v_add_u32", v10, v14); B3_OP2("v_add_u32", v11, v15);                       \
    B3_OP2("v_xor_b32", v4, v8); B3_OP2("v_xor_b32", v5, v9);                           \
    B3_OP2("v_xor_b32", v6, v10); B3_OP2("v_xor_b32", v7, v11);                         \
    B3_ROT(v4, 7); B3_ROT(v5, 7); B3_ROT(v6, 7); B3_ROT(v7, 7);                         \
  } while (0)

#ifndef B3_FOLD
#define B3_FOLD 1
#endif
#ifndef B3_FAST_NT
#define B3_FAST_NT 0
#endif
#ifndef B3_LOAD128
#define B3_LOAD128 1
#endif

__device__ __forceinline__ void compress(uint32_t cv[8], const uint32_t m[16],
                                         uint32_t counter, uint32_t blen, uint32_t flags) {
  uint32_t v0 = cv[0], v1 = cv[1], v2 = cv[2], v3 = cv[3];
  uint32_t v4 = cv[4], v5 = cv[5], v6 = cv[6], v7 = cv[7];
#if B3_FOLD
  uint32_t v8, v9, v10, v11, v12, v13, v14, v15;
  {
    const uint8_t *s = kSched.s[0];
    B3_G4_FIRST(m[s[0]], m[s[2]], m[s[4]], m[s[6]], m[s[1]], m[s[3]], m[s[5]], m[s[7]]);
    B3_G4(v0, v5, v10, v15, v1, v6, v11, v12, v2, v7, v8, v13, v3, v4, v9, v14,
          m[s[8]], m[s[10]], m[s[12]], m[s[14]], m[s[9]], m[s[11]], m[s[13]], m[s[15]]);
  }
#pragma unroll
  for (int r = 1; r < 7; ++r) {
#else
  uint32_t v8 = IV0, v9 = IV1, v10 = IV2, v11 = IV3;
  uint32_t v12 = counter, v13 = 0, v14 = blen, v15 = flags;
#pragma unroll
  for (int r = 0; r < 7; ++r) {
#endif
    const uint8_t *s = kSched.s[r];
    B3_G4(v0, v4, v8, v12, v1, v5, v9, v13, v2, v6, v10, v14, v3, v7, v11, v15,
          m[s[0]], m[s[2]], m[s[4]], m[s[6]], m[s[1]], m[s[3]], m[s[5]], m[s[7]]);
    B3_G4(v0, v5, v10, v15, v1, v6, v11, v12, v2, v7, v8, v13, v3, v4, v9, v14,
          m[s[8]], m[s[10]], m[s[12]], m[s[14]], m[s[9]], m[s[11]], m[s[13]], m[s[15]]);
  }
  cv[0] = v0 ^ v8;  cv[1] = v1 ^ v9;  cv[2] = v2 ^ v10; cv[3] = v3 ^ v11;
  cv[4] = v4 ^ v12; cv[5] = v5 ^ v13; cv[6] = v6 ^ v14; cv[7] = v7 ^ v15;
}

__device__ __forceinline__ void set_iv(uint32_t cv[8]) {
  cv[0] = IV0; cv[1] = IV1; cv[2] = IV2; cv[3] = IV3;
  cv[4] = IV4; cv[5] = IV5; cv[6] = IV6; cv[7] = IV7;
}
