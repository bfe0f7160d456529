// sha256.hip — per-chunk SHA-256 on gfx950.
//
// Replaces RafsDigest::from_buf(buf, Sha256) inside nydus-image
// ([nydus v2.3.0] utils/src/digest.rs) for PackOption.Digester == "sha256"
// (the `--digester sha256` builder path).
//
// SHA-256 has no intra-message parallelism: one lane owns one chunk and walks
// its 64-B blocks (16-B loads, byte-swapped with v_perm).  The message
// schedule is a rolling 16-word window in registers; all 64 rounds are
// unrolled so the round constants fold into immediates.  At 1 MiB chunks a
// 16 GiB layer has only 16384 lanes of work: occupancy, not VALU issue,
// bounds this kernel.
#include "common.hpp"

namespace ngpu {
namespace {

constexpr uint32_t kK[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1,
    0x923f82a4, 0xab1c5ed5, 0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3,
    0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174, 0xe49b69c1, 0xefbe4786,
    0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147,
    0x06ca6351, 0x14292967, 0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13,
    0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85, 0xa2bfe8a1, 0xa81a664b,
    0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a,
    0x5b9cca4f, 0x682e6ff3, 0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208,
    0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

__device__ __forceinline__ uint32_t bswap(uint32_t x) {
  return __builtin_amdgcn_perm(x, x, 0x00010203u);
}

__device__ __forceinline__ uint32_t bswap_words(u32x4 v, int i) {
  return bswap(i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w);
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);  // symmetric truth table
}

// One 64-B block.  Per round: Sigma1/Sigma0 = 3 v_alignbit + 1 v_bitop3 (xor3),
// Ch = v_bfi, Maj = v_bitop3, h+K+W and T1 as two v_add3 -> ~13 VALU ops;
// schedule: sigma0/sigma1 = 2 v_alignbit + v_lshr + v_bitop3, W = v_add3 + v_add.
__device__ __forceinline__ void sha_block(uint32_t h[8], uint32_t w[16]) {
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3];
  uint32_t e = h[4], f = h[5], g = h[6], hh = h[7];
#pragma unroll
  for (int t = 0; t < 64; ++t) {
    uint32_t wt;
    if (t < 16) {
      wt = w[t];
    } else {
      const uint32_t w15 = w[(t - 15) & 15], w2 = w[(t - 2) & 15];
      const uint32_t s0 = xor3(rotr32(w15, 7), rotr32(w15, 18), w15 >> 3);
      const uint32_t s1 = xor3(rotr32(w2, 17), rotr32(w2, 19), w2 >> 10);
      wt = w[t & 15] + s0 + w[(t - 7) & 15] + s1;
      w[t & 15] = wt;
    }
    const uint32_t hkw = hh + kK[t] + wt;
    const uint32_t S1 = xor3(rotr32(e, 6), rotr32(e, 11), rotr32(e, 25));
    const uint32_t ch = (e & f) ^ (~e & g);
    const uint32_t t1 = hkw + S1 + ch;
    const uint32_t S0 = xor3(rotr32(a, 2), rotr32(a, 13), rotr32(a, 22));
    const uint32_t mj = (a & b) | (c & (a | b));
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + S0 + mj;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d;
  h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

// Message block `b` of a chunk (b < full: data; else the padding tail),
// big-endian words.
__device__ __forceinline__ void sha_load_block(const uint8_t *p, uint32_t len, uint32_t b,
                                               uint32_t w[16]) {
  const uint32_t full = len >> 6;
  if (b < full) {
    const uint8_t *q = p + 64ull * b;
    if ((reinterpret_cast<uintptr_t>(q) & 15) == 0) {
      const u32x4 x0 = load_nt16(q), x1 = load_nt16(q + 16);
      const u32x4 x2 = load_nt16(q + 32), x3 = load_nt16(q + 48);
      w[0] = bswap(x0.x); w[1] = bswap(x0.y); w[2] = bswap(x0.z); w[3] = bswap(x0.w);
      w[4] = bswap(x1.x); w[5] = bswap(x1.y); w[6] = bswap(x1.z); w[7] = bswap(x1.w);
      w[8] = bswap(x2.x); w[9] = bswap(x2.y); w[10] = bswap(x2.z); w[11] = bswap(x2.w);
      w[12] = bswap(x3.x); w[13] = bswap(x3.y); w[14] = bswap(x3.z); w[15] = bswap(x3.w);
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i)
        w[i] = ((uint32_t)q[4 * i] << 24) | ((uint32_t)q[4 * i + 1] << 16) |
               ((uint32_t)q[4 * i + 2] << 8) | (uint32_t)q[4 * i + 3];
    }
    return;
  }
  // Tail: remaining bytes, 0x80, zero pad, 64-bit big-endian bit length.
  const uint32_t rem = len & 63;
  const uint32_t tb = b - full;  // 0 or 1
  const uint32_t tail_blocks = rem + 9 <= 64 ? 1 : 2;
  const uint8_t *tp = p + 64ull * full;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t pos = 64 * tb + 4 * i + k;
      uint32_t byte = 0;
      if (pos < rem) byte = tp[pos];
      else if (pos == rem) byte = 0x80;
      x = (x << 8) | byte;
    }
    w[i] = x;
  }
  if (tb + 1 == tail_blocks) {
    const uint64_t bits = (uint64_t)len * 8;
    w[14] = (uint32_t)(bits >> 32);
    w[15] = (uint32_t)bits;
  }
}

// Two waves per 64 chunks (SURVEY.md §7 hard part (c): SHA-256 has one
// independent stream per chunk, so at 1 MiB chunks a 16 GiB layer fills one
// wave per CU).  Wave 1 ("schedule") loads block k+1 and expands its message
// schedule into K[t]+W[t] in LDS while wave 0 ("rounds") runs the 64 rounds
// of block k from LDS: the per-chunk instruction stream on the critical wave
// drops from ~1440 to ~900 VALU ops per block, and the two waves run on two
// SIMDs.  One workgroup barrier per block; LDS ping-pong [2][64 t][64 lanes].
__global__ __launch_bounds__(128) void sha256_split(
    const uint8_t *__restrict__ data, uint64_t data_len,
    const ngpu_chunk *__restrict__ chunks, uint64_t n,
    ngpu_result *__restrict__ out, uint64_t *__restrict__ err) {
  // K+W per lane, lane-major with a 68-word stride: 16-B LDS accesses, and a
  // whole block's 64 values are read into registers before its rounds start.
  __shared__ u32x4 kw[2][64][17];
  const uint32_t lane = threadIdx.x & 63;
  const bool rounds = threadIdx.x < 64;
  // the round wave is the critical path: win issue arbitration on a shared SIMD
  if (rounds) __builtin_amdgcn_s_setprio(3);
  const uint64_t c = blockIdx.x * 64ull + lane;
  bool valid = c < n;
  uint32_t len = 0;
  const uint8_t *p = data;
  if (valid) {
    const ngpu_chunk ch = chunks[c];
    if (ch.offset > data_len || ch.length > data_len - ch.offset) {
      if (rounds) note_bad_desc(err, 1);
      valid = false;
    } else {
      len = ch.length;
      p = data + ch.offset;
    }
  }
  const uint32_t nb = valid ? (len + 8) / 64 + 1 : 0;
  uint32_t nbmax = nb;
#pragma unroll
  for (int o = 32; o; o >>= 1) nbmax = max(nbmax, (uint32_t)__shfl_xor((int)nbmax, o, 64));

  auto produce = [&](uint32_t b, int buf) {
    uint32_t w[16];
    sha_load_block(p, len, b, w);
    u32x4 q;
#pragma unroll
    for (int t = 0; t < 64; ++t) {
      uint32_t wt;
      if (t < 16) {
        wt = w[t];
      } else {
        const uint32_t w15 = w[(t - 15) & 15], w2 = w[(t - 2) & 15];
        const uint32_t s0 = xor3(rotr32(w15, 7), rotr32(w15, 18), w15 >> 3);
        const uint32_t s1 = xor3(rotr32(w2, 17), rotr32(w2, 19), w2 >> 10);
        wt = w[t & 15] + s0 + w[(t - 7) & 15] + s1;
        w[t & 15] = wt;
      }
      q[t & 3] = wt + kK[t];
      if ((t & 3) == 3) kw[buf][lane][t >> 2] = q;
    }
  };

  if (!rounds && nb > 0) produce(0, 0);
  __syncthreads();
  uint32_t h[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                   0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
  for (uint32_t k = 0; k < nbmax; ++k) {
    if (rounds) {
      if (k < nb) {
        const int buf = k & 1;
        u32x4 kv[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) kv[j] = kw[buf][lane][j];
        uint32_t a = h[0], b = h[1], cc = h[2], d = h[3];
        uint32_t e = h[4], f = h[5], g = h[6], hh = h[7];
#pragma unroll
        for (int t = 0; t < 64; ++t) {
          const uint32_t S1 = xor3(rotr32(e, 6), rotr32(e, 11), rotr32(e, 25));
          const uint32_t ch = (e & f) ^ (~e & g);
          const uint32_t t1 = hh + kv[t >> 2][t & 3] + S1 + ch;
          const uint32_t S0 = xor3(rotr32(a, 2), rotr32(a, 13), rotr32(a, 22));
          const uint32_t mj = (a & b) | (cc & (a | b));
          hh = g; g = f; f = e; e = d + t1; d = cc; cc = b; b = a; a = t1 + S0 + mj;
        }
        h[0] += a; h[1] += b; h[2] += cc; h[3] += d;
        h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
      }
    } else if (k + 1 < nb) {
      produce(k + 1, (k + 1) & 1);
    }
    __syncthreads();
  }
  if (rounds && valid) {
    uint4 *dd = reinterpret_cast<uint4 *>(out[c].digest);
    dd[0] = make_uint4(bswap(h[0]), bswap(h[1]), bswap(h[2]), bswap(h[3]));
    dd[1] = make_uint4(bswap(h[4]), bswap(h[5]), bswap(h[6]), bswap(h[7]));
    out[c].kind = NGPU_DIGESTED;  // the dedup stage takes only marked records
  }
}

// One lane per chunk and no wave specialisation: each lane expands its own
// message schedule and runs the rounds (sha_block), with the next block
// prefetched into registers.  No LDS and no barrier, so occupancy is set by
// registers alone (8 waves per SIMD), and with >= 4 chunk waves per SIMD
// (many-chunk layers, e.g. 64 KiB chunks) the SIMD issues at its full rate
// instead of leaving a schedule wave's SIMD half idle.
__global__ __launch_bounds__(256) void sha256_lane(
    const uint8_t *__restrict__ data, uint64_t data_len,
    const ngpu_chunk *__restrict__ chunks, uint64_t n,
    ngpu_result *__restrict__ out, uint64_t *__restrict__ err) {
  const uint64_t c = blockIdx.x * 256ull + threadIdx.x;
  if (c >= n) return;
  const ngpu_chunk ch = chunks[c];
  if (ch.offset > data_len || ch.length > data_len - ch.offset) {
    note_bad_desc(err, 1);
    return;
  }
  const uint32_t len = ch.length;
  const uint8_t *p = data + ch.offset;
  const uint32_t nb = (len + 8) / 64 + 1, full = len >> 6;
  const bool aligned = (reinterpret_cast<uintptr_t>(p) & 15) == 0;
  uint32_t h[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                   0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
  u32x4 pf0 = {}, pf1 = {}, pf2 = {}, pf3 = {};
  bool have_pf = false;
  auto prefetch = [&](uint32_t b) {
    have_pf = aligned && b < full;
    if (have_pf) {
      const u32x4 *q = reinterpret_cast<const u32x4 *>(p + 64ull * b);
      pf0 = q[0]; pf1 = q[1]; pf2 = q[2]; pf3 = q[3];
    }
  };
  prefetch(0);
  for (uint32_t b = 0; b < nb; ++b) {
    uint32_t w[16];
    if (have_pf) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        w[i] = bswap_words(pf0, i); w[4 + i] = bswap_words(pf1, i);
        w[8 + i] = bswap_words(pf2, i); w[12 + i] = bswap_words(pf3, i);
      }
    } else {
      sha_load_block(p, len, b, w);
    }
    prefetch(b + 1);
    sha_block(h, w);
  }
  uint4 *dd = reinterpret_cast<uint4 *>(out[c].digest);
  dd[0] = make_uint4(bswap(h[0]), bswap(h[1]), bswap(h[2]), bswap(h[3]));
  dd[1] = make_uint4(bswap(h[4]), bswap(h[5]), bswap(h[6]), bswap(h[7]));
  out[c].kind = NGPU_DIGESTED;
}

// Two lanes per chunk for the rounds (few, long chunks: the per-chunk round
// chain is the whole critical path, so shortening it is the only lever once
// every chunk has a lane).
//
// With A_t / E_t the new a / e of round t (d = A_{t-4}, h = E_{t-4}):
//   E_t = Sigma1(E_{t-1}) + Ch(E_{t-1}, E_{t-2}, E_{t-3}) + E_{t-4} + K_t + W_t + A_{t-4}
//   A_t = Sigma0(A_{t-1}) + Maj(A_{t-1}, A_{t-2}, A_{t-3}) + E_t - A_{t-4}
// The "E lane" of a chunk walks the E recurrence, the "A lane" the A one, TWO
// ROUNDS BEHIND: in iteration i the E lane makes E_i and the A lane A_{i-2}.
// Both hold their last four values in P0..P3 (newest first), so the values
// each needs from its partner -- A_{i-4} for the E lane, E_{i-2} for the A
// lane -- are both the partner's P1: ONE row_ror:8 DPP add (partner 8 lanes
// away in the 16-lane row) serves both sides, off the critical path:
//   Z   = ((P3 ^ M) + KW) + dpp(P1)  E: E_{i-4} + K+W + A_{i-4}   A: -A_{i-6} + E_{i-2}
//   S   = rotr(P0,r1) ^ rotr(P0,r2) ^ rotr(P0,r3)        (per-lane rotate amounts)
//   sel = P0 ^ (P2 & M)              E: e                  A: a ^ c
//   cm  = bfi(sel, P1, P2)           E: Ch(e,f,g)          A: Maj(a,b,c) = bfi(a^c, b, c)
//   X   = S + cm + Z                 E: E_i                A: A_{i-2}
// 9 VALU ops per round (14 with one lane per chunk) and a 3-deep dependency
// chain.  66 iterations per block: in 0-1 the A lane computes values that are
// discarded (its P0/P1 hold H2/H3 = A_{-3}/A_{-4} for the E lane to read, and
// its registers are reset to H0..H3 at iteration 2); in 64-65 the E lane does.
//
// Waves: wave 0 rounds (32 chunks), wave 1 message schedule for the same 32
// chunks, two blocks per phase (lanes 0-31 the even block, 32-63 the odd one),
// with the next pair of blocks prefetched into registers.  KW[set][half][chunk][t]
// in LDS; chunk row 32 holds the constant 1 the A lanes add (~x + 1 = -x).
constexpr uint32_t kDppRowRor8 = 0x128;

// R round waves + R schedule waves per workgroup (R groups of 32 chunks), so
// one workgroup per CU puts every wave on its own SIMD.  U: the round waves
// run wave-uniform (see the round loop) -- for calls of mixed chunk lengths,
// whose long chains share their waves with finished chunks; a call of
// equal chunks keeps every lane busy and runs 3 % faster masked (C3:
// 21.4 vs 22.1 ms, same box, alternated twice; profiles/r5/c3_sha_uniform_ab_r5p2.log).
template <int R, bool U>
__global__ __launch_bounds__(128 * R) void sha256_pair(
    const uint8_t *__restrict__ data, uint64_t data_len,
    const ngpu_chunk *__restrict__ chunks, uint64_t n,
    ngpu_result *__restrict__ out, uint64_t *__restrict__ err) {
  __shared__ u32x4 kws[R][2][2][33][17];  // [group][set][half][chunk | 32 = ones][t/4]
  __shared__ uint32_t s_nbmax;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = threadIdx.x >> 6;
  const bool rounds = wave < R;
  const uint32_t grp = rounds ? wave : wave - R;
  auto &kw = kws[grp];
  // the round wave is the critical path: win issue arbitration on a shared SIMD
  if (rounds) __builtin_amdgcn_s_setprio(3);
  const uint32_t side = rounds ? (lane >> 3) & 1 : 0;  // 1 = A lane
  const uint32_t ci = rounds ? (lane >> 4) * 8 + (lane & 7) : lane & 31;
  const uint32_t half = rounds ? 0 : lane >> 5;
  const uint64_t c = (blockIdx.x * (uint64_t)R + grp) * 32ull + ci;
  bool valid = c < n;
  uint32_t len = 0;
  const uint8_t *p = data;
  if (threadIdx.x == 0) s_nbmax = 0;
  if (valid) {
    const ngpu_chunk ch = chunks[c];
    if (ch.offset > data_len || ch.length > data_len - ch.offset) {
      if (rounds && side == 0) note_bad_desc(err, 1);
      valid = false;
    } else {
      len = ch.length;
      p = data + ch.offset;
    }
  }
  const uint32_t nb = valid ? (len + 8) / 64 + 1 : 0;
  uint32_t nbmax = nb;
#pragma unroll
  for (int o = 32; o; o >>= 1) nbmax = max(nbmax, (uint32_t)__shfl_xor((int)nbmax, o, 64));
  if (R > 1) {  // every wave of the workgroup runs the same number of phases
    __syncthreads();
    if (lane == 0) atomicMax(&s_nbmax, nbmax);
    __syncthreads();
    nbmax = s_nbmax;
  }
  const uint32_t phases = (nbmax + 1) / 2;

  // Schedule wave state: its next block (b + 2) prefetched into registers.
  const uint32_t full = len >> 6;
  const bool aligned = (reinterpret_cast<uintptr_t>(p) & 15) == 0;
  u32x4 pf0 = {}, pf1 = {}, pf2 = {}, pf3 = {};
  bool have_pf = false;
  auto prefetch = [&](uint32_t b) {
    have_pf = aligned && b < full;
    if (have_pf) {
      const u32x4 *q = reinterpret_cast<const u32x4 *>(p + 64ull * b);
      pf0 = q[0]; pf1 = q[1]; pf2 = q[2]; pf3 = q[3];
    }
  };
  auto produce = [&](uint32_t b, int set) {
    if (b >= nb) return;
    uint32_t w[16];
    if (have_pf) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        w[i] = bswap_words(pf0, i); w[4 + i] = bswap_words(pf1, i);
        w[8 + i] = bswap_words(pf2, i); w[12 + i] = bswap_words(pf3, i);
      }
    } else {
      sha_load_block(p, len, b, w);
    }
    prefetch(b + 2);
    u32x4 *dst = kw[set][half][ci];
    u32x4 q;
#pragma unroll
    for (int t = 0; t < 64; ++t) {
      uint32_t wt;
      if (t < 16) {
        wt = w[t];
      } else {
        const uint32_t w15 = w[(t - 15) & 15], w2 = w[(t - 2) & 15];
        const uint32_t s0 = xor3(rotr32(w15, 7), rotr32(w15, 18), w15 >> 3);
        const uint32_t s1 = xor3(rotr32(w2, 17), rotr32(w2, 19), w2 >> 10);
        wt = w[t & 15] + s0 + w[(t - 7) & 15] + s1;
        w[t & 15] = wt;
      }
      q[t & 3] = wt + kK[t];
      if ((t & 3) == 3) dst[t >> 2] = q;
    }
  };

  if (!rounds) {
    for (uint32_t i = lane; i < 2 * 2 * 17; i += 64)
      kw[i / 34][(i / 17) & 1][32][i % 17] = u32x4{1u, 1u, 1u, 1u};
    if (nb > half) {
      prefetch(half);
      produce(half, 0);
    }
  }
  __syncthreads();

  const uint32_t M = side ? 0xFFFFFFFFu : 0u;
  const uint32_t r1 = side ? 2 : 6, r2 = side ? 13 : 11, r3 = side ? 22 : 25;
  uint32_t H0 = side ? 0x6a09e667u : 0x510e527fu, H1 = side ? 0xbb67ae85u : 0x9b05688cu;
  uint32_t H2 = side ? 0x3c6ef372u : 0x1f83d9abu, H3 = side ? 0xa54ff53au : 0x5be0cd19u;
  const uint32_t kcol = side ? 32 : ci;
  for (uint32_t ph = 0; ph < phases; ++ph) {
    const int set = ph & 1;
    if (rounds) {
#pragma unroll 1
      for (uint32_t hb = 0; hb < 2; ++hb) {
        // every lane runs the rounds while any lane of the wave has a block
        // (a lane past its chunk's end computes on stale words and keeps its
        // H): a lone long chain among finished lanes ran ~25 % slower with
        // them masked off (tools/sha_mix.py, profiles/r5/sha_mix_r5j3.jsonl)
        const bool mine = 2 * ph + hb < nb;
        if (U ? __any(mine) : mine) {
          u32x4 kv[16];
#pragma unroll
          for (int j = 0; j < 16; ++j) kv[j] = kw[set][hb][kcol][j];
          uint32_t P0 = side ? H2 : H0, P1 = side ? H3 : H1, P2 = H2, P3 = H3;
          uint32_t F0 = 0, F1 = 0, F2 = 0, F3 = 0;
#pragma unroll
          for (int it = 0; it < 66; ++it) {
            if (it == 2) {  // the A lane starts its rounds: a,b,c,d = H0..H3
              P0 = side ? H0 : P0; P1 = side ? H1 : P1;
              P2 = side ? H2 : P2; P3 = side ? H3 : P3;
            }
            const uint32_t kwv = it < 64 ? kv[it >> 2][it & 3] : side;
            uint32_t Y = (P3 ^ M) + kwv;
            asm("" : "+v"(Y));  // keep the DPP add a separate VOP2 op
            uint32_t Z =
                Y + (uint32_t)__builtin_amdgcn_update_dpp(0, (int)P1, kDppRowRor8, 0xf, 0xf, false);
            asm("" : "+v"(Z));
            const uint32_t S = xor3(rotr32(P0, r1), rotr32(P0, r2), rotr32(P0, r3));
            // bitop3 truth-table index is S0<<2 | S1<<1 | S2: 0x78 = a ^ (b & c)
            const uint32_t sel = __builtin_amdgcn_bitop3_b32(P0, P2, M, 0x78);
            const uint32_t cm = (sel & P1) | (~sel & P2);
            const uint32_t X = S + cm + Z;
            P3 = P2; P2 = P1; P1 = P0; P0 = X;
            if (it == 63) { F0 = P0; F1 = P1; F2 = P2; F3 = P3; }  // E lane final e,f,g,h
          }
          if (mine) {
            H0 += side ? P0 : F0; H1 += side ? P1 : F1;
            H2 += side ? P2 : F2; H3 += side ? P3 : F3;
          }
        }
      }
    } else {
      produce(2 * ph + 2 + half, set ^ 1);
    }
    __syncthreads();
  }
  if (rounds && valid) {
    uint4 *dd = reinterpret_cast<uint4 *>(out[c].digest) + (side ? 0 : 1);
    *dd = make_uint4(bswap(H0), bswap(H1), bswap(H2), bswap(H3));
    if (side) out[c].kind = NGPU_DIGESTED;
  }
}

}  // namespace

void launch_sha256(const uint8_t *data, uint64_t data_len,
                   const ngpu_chunk *chunks, uint64_t n, ngpu_result *out,
                   uint64_t *err, int variant, bool mixed, hipStream_t s) {
  if (n == 0) return;
  // Auto (same-box sweep, profiles/r2/sha_variants_lane_r2sl.jsonl, GB/s):
  //  * <= 16384 chunks (one 64-chunk workgroup per CU): two lanes per chunk,
  //    each round wave alone on its SIMD; 16384 x 1 MiB: pair 786, lane 385.
  //  * <= 32768 chunks: two lanes per chunk, four groups per workgroup (one
  //    workgroup per CU, a round and a schedule wave on each SIMD); 32768 x
  //    512 KiB: 1343, against 950 for two 2-group workgroups per CU.
  //  * more: one lane per chunk, every wave doing its own schedule;
  //    65536 x 256 KiB lane 1512 / pair-4 1342, 262144 x 64 KiB 1657 / split 1190.
  if (variant < 0) variant = n <= 256ull * 64 ? 1 : n <= 256ull * 128 ? 5 : 2;
  if (variant == 2) {
    hipLaunchKernelGGL(sha256_lane, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, data,
                       data_len, chunks, n, out, err);
    return;
  }
  if (variant >= 1) {
    const dim3 g2((unsigned)((n + 63) / 64)), g1((unsigned)((n + 31) / 32));
    // wave-uniform round waves unless the chunks are (nearly) all full-size:
    // a long chain among short neighbours ran 25-45 % slower masked
    const bool few = mixed;
    switch (variant) {
      case 4:  // one group per workgroup
        if (few)
          hipLaunchKernelGGL((sha256_pair<1, true>), g1, dim3(128), 0, s, data, data_len, chunks, n, out, err);
        else
          hipLaunchKernelGGL((sha256_pair<1, false>), g1, dim3(128), 0, s, data, data_len, chunks, n, out, err);
        break;
      case 5:  // four groups per workgroup: a round and a schedule wave share each SIMD
        hipLaunchKernelGGL((sha256_pair<4, false>), dim3((unsigned)((n + 127) / 128)), dim3(512), 0, s,
                           data, data_len, chunks, n, out, err);
        break;
      default:
        if (few)
          hipLaunchKernelGGL((sha256_pair<2, true>), g2, dim3(256), 0, s, data, data_len, chunks, n, out, err);
        else
          hipLaunchKernelGGL((sha256_pair<2, false>), g2, dim3(256), 0, s, data, data_len, chunks, n, out, err);
    }
    return;
  }
  const uint64_t blocks = (n + 63) / 64;
  hipLaunchKernelGGL(sha256_split, dim3((unsigned)blocks), dim3(128), 0, s, data,
                     data_len, chunks, n, out, err);
}

}  // namespace ngpu
