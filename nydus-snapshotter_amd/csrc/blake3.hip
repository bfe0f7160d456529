// blake3.hip — per-chunk BLAKE3-256 on gfx950.
//
// Replaces RafsDigest::from_buf(buf, Blake3) inside nydus-image
// ([nydus v2.3.0] utils/src/digest.rs), the dominant cost of the reference's
// conversion path.  Each nydus chunk of S bytes is an
// independent BLAKE3 input of ceil(S/1024) 1 KiB BLAKE3 chunks, called
// "leaves" here.
//
// Work decomposition (integer-VALU bound):
//   * b3_groups<D>: one lane per aligned group of 2^D consecutive leaves of
//     one nydus chunk.  The lane hashes its leaves (16 compressions each,
//     64-B message blocks loaded straight into VGPRs with 16-B loads) and
//     merges complete subtrees eagerly through a D-deep CV stack held in
//     named registers, so the 2^D-1 parent compressions of its group are
//     done at full lane occupancy.  Aligned groups are nodes of BLAKE3's
//     left-complete tree, so their CVs are exact subtree CVs.  A chunk that
//     fits one group (<= 2^D KiB) is finished in the lane (ROOT flag).
//   * b3_tree: one workgroup per chunk with >1 group reduces the group CVs
//     level by level in LDS (pairwise with the odd tail promoted == BLAKE3's
//     left-complete tree), 1024 CVs per LDS tile; the last compression gets
//     ROOT.  This carries 1/2^D of the parent work only.
#include <hip/hip_ext.h>

#include "common.hpp"

namespace ngpu {
namespace {

#include "b3_compress.hpp"  // IV, flags, schedule, compress(), set_iv()

// Load one message block of `nbytes` (<= 64) little-endian, zero padded.
// NT: non-temporal (read-once streaming) loads.  A partial block (a chunk's
// tail) still takes the 16-B vector path when the 64 bytes lie inside the
// caller's buffer (`end`): the bytes past the chunk are loaded and masked off,
// so lanes at their tail do not diverge into 64 byte loads.
template <bool NT>
__device__ __forceinline__ void load_block(const uint8_t *p, uint32_t nbytes, const uint8_t *end,
                                           uint32_t m[16]) {
  if (((reinterpret_cast<uintptr_t>(p) & 15) == 0) && (nbytes == 64 || p + 64 <= end)) {
    u32x4 a, b, c, d;
    if (NT) {
      a = load_nt16(p); b = load_nt16(p + 16); c = load_nt16(p + 32); d = load_nt16(p + 48);
    } else {
      const u32x4 *q = reinterpret_cast<const u32x4 *>(p);
      a = q[0]; b = q[1]; c = q[2]; d = q[3];
    }
    m[0] = a.x; m[1] = a.y; m[2] = a.z; m[3] = a.w;
    m[4] = b.x; m[5] = b.y; m[6] = b.z; m[7] = b.w;
    m[8] = c.x; m[9] = c.y; m[10] = c.z; m[11] = c.w;
    m[12] = d.x; m[13] = d.y; m[14] = d.z; m[15] = d.w;
    if (nbytes < 64) {
#pragma unroll
      for (int w = 0; w < 16; ++w) {
        const int v = (int)nbytes - 4 * w;  // valid bytes of word w
        m[w] = v >= 4 ? m[w] : v <= 0 ? 0u : m[w] & ((1u << (8 * v)) - 1u);
      }
    }
    return;
  }
  // Unaligned, or the last bytes of the buffer: byte loads of the valid bytes
  // only (never reads past the chunk, so never past the caller's buffer).
#pragma unroll
  for (int w = 0; w < 16; ++w) {
    uint32_t x = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      uint32_t i = 4 * w + b;
      if (i < nbytes) x |= (uint32_t)p[i] << (8 * b);
    }
    m[w] = x;
  }
}

// A chunk with several leaf groups whose groups all fall in one 256-group
// window (one b3_groups workgroup) is finished inside that workgroup.
__device__ __forceinline__ bool tree_in_workgroup(uint64_t base, uint64_t ng) {
  return ng > 1 && (base >> 8) == ((base + ng - 1) >> 8);
}

// Single-group chunks (<= 2^D leaves: the whole chunk is one lane's work) are
// taken out of the chunk-ordered group space and processed after the
// multi-group chunks' groups, sorted by their 64-B block count, largest
// first: lanes of a wave then carry near-equal work (a 4-KiB file next to a
// full 8-KiB group would leave most of the wave idle).  Counting sort over
// block counts 1 .. 16 * 2^D (kMaxKey for D <= 4).
constexpr int kMaxKey = 16 << 4;

// 0: a multi-group chunk; else the chunk's 64-B block count (its work).
__device__ __forceinline__ uint32_t small_key(const ngpu_chunk &ch, int D) {
  const uint32_t len = ch.length;
  const uint32_t leaves = len == 0 ? 1 : (len + kLeaf - 1) / kLeaf;
  if (leaves > (1u << D)) return 0;
  return len == 0 ? 1 : (len + 63) / 64;
}

// Leaf groups per chunk -> exclusive scan (groups[0..n], single pass with
// decoupled look-back; multi-group chunks only, single-group chunks count 0)
// and the histogram of single-group block counts.  4 consecutive chunks per
// thread, so a workgroup issues its histogram atomics for 1024 chunks.
constexpr int kPlanItems = 4;
constexpr int kPlanTile = kTileThreads * kPlanItems;

__global__ __launch_bounds__(kTileThreads) void b3_plan(const ngpu_chunk *__restrict__ chunks,
                                                        uint64_t n, int D,
                                                        uint64_t *__restrict__ groups,
                                                        uint32_t *__restrict__ hist,
                                                        uint64_t *__restrict__ ts) {
  __shared__ uint32_t h[kMaxKey + 1];
  __shared__ uint64_t sh_tile, sh_pre;
  for (int i = threadIdx.x; i <= kMaxKey; i += blockDim.x) h[i] = 0;
  if (threadIdx.x == 0)
    sh_tile = __hip_atomic_fetch_add(ts, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const uint64_t tile = sh_tile;
  const uint64_t c0 = tile * kPlanTile + threadIdx.x * kPlanItems;
  uint64_t g[kPlanItems], sum = 0;
#pragma unroll
  for (int i = 0; i < kPlanItems; ++i) {
    g[i] = 0;
    const uint64_t c = c0 + i;
    if (c < n) {
      const uint32_t key = small_key(chunks[c], D);
      if (key) {
        atomicAdd(&h[key], 1u);
      } else {
        const uint32_t len = chunks[c].length;
        g[i] = (((len + kLeaf - 1) / kLeaf) + (1u << D) - 1) >> D;
      }
    }
    sum += g[i];
  }
  uint64_t tot;
  uint64_t run = block_exclusive_scan(sum, &tot);  // (its barriers also publish h)
  if (threadIdx.x < 64) {
    const uint64_t pre = wave_lookback(ts + 1, tile, tot);
    if (threadIdx.x == 0) sh_pre = pre;
  }
  for (int i = threadIdx.x; i <= kMaxKey; i += blockDim.x)
    if (h[i]) atomicAdd(&hist[i], h[i]);
  __syncthreads();
  run += sh_pre;
#pragma unroll
  for (int i = 0; i < kPlanItems; ++i) {
    const uint64_t c = c0 + i;
    if (c < n) groups[c] = run;
    run += g[i];
    if (c + 1 == n) groups[n] = run;
  }
}

// small[] = single-group chunk ids sorted by block count (descending; order
// inside a bucket is arbitrary, results do not depend on it).  Every
// workgroup derives the bucket starts from the finished histogram (256 keys,
// one per thread); *nsmall = number of single-group chunks.
__global__ __launch_bounds__(kTileThreads) void b3_small_scatter(
    const ngpu_chunk *__restrict__ chunks, uint64_t n, int D, const uint32_t *__restrict__ hist,
    uint32_t *__restrict__ cursor, uint32_t *__restrict__ small, uint64_t *__restrict__ nsmall) {
  static_assert(kMaxKey == kTileThreads, "one bucket per thread");
  __shared__ uint32_t h[kMaxKey + 1], base[kMaxKey + 1];
  const int t = threadIdx.x;
  const uint32_t bkey = kMaxKey - t;  // 256 .. 1: largest block count first
  uint64_t tot;
  const uint64_t start = block_exclusive_scan(hist[bkey], &tot);
  if (blockIdx.x == 0 && t == 0) *nsmall = tot;
  for (int i = t; i <= kMaxKey; i += blockDim.x) h[i] = 0;
  __syncthreads();
  uint32_t key[kPlanItems], rank[kPlanItems];
#pragma unroll
  for (int i = 0; i < kPlanItems; ++i) {
    const uint64_t c = blockIdx.x * (uint64_t)kPlanTile + i * kTileThreads + t;
    key[i] = c < n ? small_key(chunks[c], D) : 0;
    rank[i] = key[i] ? atomicAdd(&h[key[i]], 1u) : 0;
  }
  __syncthreads();
  if (h[bkey]) base[bkey] = (uint32_t)start + atomicAdd(&cursor[bkey], h[bkey]);
  __syncthreads();
#pragma unroll
  for (int i = 0; i < kPlanItems; ++i) {
    const uint64_t c = blockIdx.x * (uint64_t)kPlanTile + i * kTileThreads + t;
    if (key[i]) small[base[key[i]] + rank[i]] = (uint32_t)c;
  }
}

// group -> chunk map: W lanes per chunk (W = 64 / chunks per wave, a power
// of two sized to the layer's groups per chunk), lanes stride over its groups.
__global__ void b3_fill_group_chunk(const uint64_t *__restrict__ gbase,
                                    uint64_t n, uint32_t *__restrict__ gchunk,
                                    uint64_t cap_g, uint32_t W) {
  const uint32_t per_wave = 64 / W;
  const uint64_t slots = ((gridDim.x * (uint64_t)blockDim.x) >> 6) * per_wave;
  const uint32_t lane = threadIdx.x & 63, sub = lane / W, sl = lane % W;
  for (uint64_t c = ((blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) >> 6) * per_wave + sub;
       c < n; c += slots) {
    const uint64_t b = gbase[c], e = gbase[c + 1];
    for (uint64_t g = b + sl; g < e && g < cap_g; g += W) gchunk[g] = (uint32_t)c;
  }
}

// Small calls (<= kSmallPlanChunks chunks): the stats reset, the tile memset,
// b3_plan, b3_small_scatter and b3_fill_group_chunk in ONE workgroup -- the
// scan, the histogram, the bucket starts and the group -> chunk map all live
// in LDS, so five dispatches (~5 us each, mostly empty) become one.  Same
// outputs as the grid path: groups[0..n], small[] (bucket order), *nsmall,
// gchunk[0..min(groups[n], cap_g)).
constexpr int kSmallPlanThreads = 1024;
static_assert(kSmallPlanChunks == (uint64_t)kSmallPlanThreads * kPlanItems, "one item set");

__device__ __forceinline__ uint64_t block1024_exclusive_scan(uint64_t v, uint64_t *wsum,
                                                             uint64_t *total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint64_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[wid] = x;
  __syncthreads();
  uint64_t pre = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kSmallPlanThreads / 64; ++w) {
    if (w < wid) pre += wsum[w];
    tot += wsum[w];
  }
  __syncthreads();
  *total = tot;
  return pre + x - v;
}

__global__ __launch_bounds__(kSmallPlanThreads) void b3_plan_small(
    const ngpu_chunk *__restrict__ chunks, uint64_t n, int D, uint64_t *__restrict__ groups,
    uint32_t *__restrict__ small, uint32_t *__restrict__ gchunk, uint64_t cap_g,
    uint64_t *__restrict__ stats) {
  __shared__ uint32_t h[kMaxKey + 1], cur[kMaxKey + 1], base[kMaxKey + 1];
  __shared__ uint64_t gpre[kSmallPlanChunks + 1], wsum[kSmallPlanThreads / 64];
  const int t = threadIdx.x;
  if (t < 16) stats[t] = 0;  // the call's device counters (nsmall rewritten below)
  for (int i = t; i <= kMaxKey; i += kSmallPlanThreads) h[i] = cur[i] = 0;
  __syncthreads();
  const uint64_t c0 = (uint64_t)t * kPlanItems;
  uint64_t g[kPlanItems], sum = 0;
  uint32_t key[kPlanItems];
#pragma unroll
  for (int i = 0; i < kPlanItems; ++i) {
    const uint64_t c = c0 + i;
    g[i] = 0;
    key[i] = 0;
    if (c < n) {
      const uint32_t len = chunks[c].length;
      key[i] = small_key(chunks[c], D);
      if (key[i]) atomicAdd(&h[key[i]], 1u);
      else g[i] = (((len + kLeaf - 1) / kLeaf) + (1u << D) - 1) >> D;
    }
    sum += g[i];
  }
  uint64_t tot;
  uint64_t run = block1024_exclusive_scan(sum, wsum, &tot);  // its barriers publish h
#pragma unroll
  for (int i = 0; i < kPlanItems; ++i) {
    const uint64_t c = c0 + i;
    if (c < n) groups[c] = gpre[c] = run;
    run += g[i];
    if (c + 1 == n) groups[n] = gpre[n] = run;
  }
  // bucket starts, largest block count first (keys kMaxKey .. 1 on threads 0 ..)
  const uint32_t bkey = kMaxKey - t;
  const uint64_t start = block1024_exclusive_scan(t < kMaxKey ? h[bkey] : 0, wsum, &tot);
  if (t < kMaxKey) base[bkey] = (uint32_t)start;
  if (t == 0) stats[10] = tot;  // nsmall
  __syncthreads();
#pragma unroll
  for (int i = 0; i < kPlanItems; ++i)
    if (key[i]) small[base[key[i]] + atomicAdd(&cur[key[i]], 1u)] = (uint32_t)(c0 + i);
  // group -> chunk: one wave per chunk writes its contiguous group range
  // (a dependent binary search per group cost ~3 us for a 10K-group layer)
  const uint32_t lane = t & 63, wave = t >> 6;
  for (uint64_t c = wave; c < n; c += kSmallPlanThreads / 64) {
    const uint64_t a = gpre[c], e = gpre[c + 1] < cap_g ? gpre[c + 1] : cap_g;
    for (uint64_t gg = a + lane; gg < e; gg += 64) gchunk[gg] = (uint32_t)c;
  }
}

// LM (load mode): bit0 = non-temporal loads, bit1 = prefetch the next 64-B
// block of the lane's byte stream while the current one is compressed,
// 5 = plain loads without the whole-leaf fast path (A/B reference).
// 4 = diagnostic: no global loads at all (wrong digests; VALU ceiling only).
// It exists only in a diagnostic build (-DNGPU_DIAG_NOLOAD=1, never the
// library the ABI ships): no ngpu_config value reaches it (ngpu_create
// rejects the load-mode values that would).
//
// Hashes leaf group j of chunk c (ng groups).  Returns 0 (no work), 1 (cur =
// root digest: the chunk fits this group) or 2 (cur = the group's subtree CV).
template <int D, int LM>
__device__ __forceinline__ int group_cv(const uint8_t *__restrict__ data, uint64_t data_len,
                                        const ngpu_chunk *__restrict__ chunks, uint32_t c,
                                        uint64_t ng, uint32_t j, uint64_t *__restrict__ err,
                                        uint32_t cur[8]) {
  constexpr int SD = D > 0 ? D : 1;
  const ngpu_chunk ch = chunks[c];
  const uint32_t len = ch.length;
  if (ch.offset > data_len || len > data_len - ch.offset) {  // bad descriptor
    if (j == 0) note_bad_desc(err, 1);
    return 0;
  }
  const uint32_t nleaves = len == 0 ? 1 : (len + kLeaf - 1) / kLeaf;
  const uint32_t first = j << D;
  const uint32_t cnt = min(1u << D, nleaves - first);
  const bool root_group = (ng == 1);
  const uint8_t *src = data + ch.offset;
  constexpr bool NT = LM < 4 && (LM & 1) != 0, PF = LM < 4 && (LM & 2) != 0;
  constexpr bool NOLOAD = LM == 4, FAST = LM == 0;
  // The lane's bytes [pos, gend) are one contiguous stream of 64-B blocks.
  const uint32_t gend = min(len, (first + cnt) * kLeaf);
  uint32_t pos = first * kLeaf;
  uint32_t m[16];
  const uint8_t *end = data + data_len;
  if (PF) load_block<NT>(src + pos, min(64u, gend - pos), end, m);

  uint32_t stk[SD][8];
  uint32_t depth = 0;
  // Leaf k's CV is in cur: merge the complete subtrees it closes (eagerly,
  // through the D-deep stack), then push it unless it is the group's last.
  auto finish = [&](uint32_t k) {
    const bool last = (k + 1 == cnt);
    const uint32_t nm = last ? depth : (uint32_t)__builtin_ctz(k + 1);
    for (uint32_t q = 0; q < nm; ++q) {
      uint32_t pm[16];
#pragma unroll
      for (int i = 0; i < 8; ++i) { pm[i] = stk[0][i]; pm[8 + i] = cur[i]; }
      const uint32_t flags = PARENT | ((last && root_group && q + 1 == nm) ? ROOT : 0);
      set_iv(cur);
      compress(cur, pm, 0, 64, flags);
#pragma unroll
      for (int l = 0; l + 1 < SD; ++l)
#pragma unroll
        for (int i = 0; i < 8; ++i) stk[l][i] = stk[l + 1][i];
      --depth;
    }
    if (!last) {
#pragma unroll
      for (int l = SD - 1; l > 0; --l)
#pragma unroll
        for (int i = 0; i < 8; ++i) stk[l][i] = stk[l - 1][i];
#pragma unroll
      for (int i = 0; i < 8; ++i) stk[0][i] = cur[i];
      ++depth;
    }
  };
  for (uint32_t k = 0; k < cnt; ++k) {
    const uint32_t leaf = first + k;
    const uint32_t off = leaf * kLeaf;
    const uint32_t llen = min(kLeaf, len - off);
    const uint32_t nb = llen == 0 ? 1 : (llen + 63) >> 6;
    set_iv(cur);
    if (FAST && __all(llen == kLeaf && (reinterpret_cast<uintptr_t>(src + off) & 15) == 0)) {
      // Every active lane of the wave has a whole, aligned leaf: 16 blocks of
      // plain 16-B loads, no per-block length / alignment / bounds checks.
      // (Wave-uniform: a wave mixing whole and partial leaves would run both
      // loops, each with its compression, one after the other.)
      const u32x4 *q = reinterpret_cast<const u32x4 *>(src + off);
      const uint32_t fl_end = CHUNK_END | ((root_group && nleaves == 1) ? ROOT : 0);
#if B3_LOAD128
      // Both 64-B blocks of a 128-B line are loaded together (8 x 16-B loads
      // per pair of compressions): a lane's line is requested from the fabric
      // once.  Loading each block just before its compression left ~one
      // compression between the two halves of the line, long enough for the
      // L2 to evict it: 14 % of the lines were fetched twice (TCC_EA0_RDREQ_128B,
      // profiles/r1/pmc_req_c2.json).
      for (uint32_t b = 0; b < 16; b += 2, q += 8) {
#if B3_FAST_NT  // A/B only (default 0): the same line pair with non-temporal loads
        const uint8_t *qb = reinterpret_cast<const uint8_t *>(q);
        const u32x4 x0 = load_nt16(qb), x1 = load_nt16(qb + 16), x2 = load_nt16(qb + 32),
                    x3 = load_nt16(qb + 48);
        const u32x4 x4 = load_nt16(qb + 64), x5 = load_nt16(qb + 80), x6 = load_nt16(qb + 96),
                    x7 = load_nt16(qb + 112);
#else
        const u32x4 x0 = q[0], x1 = q[1], x2 = q[2], x3 = q[3];
        const u32x4 x4 = q[4], x5 = q[5], x6 = q[6], x7 = q[7];
#endif
        m[0] = x0.x; m[1] = x0.y; m[2] = x0.z; m[3] = x0.w;
        m[4] = x1.x; m[5] = x1.y; m[6] = x1.z; m[7] = x1.w;
        m[8] = x2.x; m[9] = x2.y; m[10] = x2.z; m[11] = x2.w;
        m[12] = x3.x; m[13] = x3.y; m[14] = x3.z; m[15] = x3.w;
        compress(cur, m, leaf, 64, b == 0 ? CHUNK_START : 0u);
        m[0] = x4.x; m[1] = x4.y; m[2] = x4.z; m[3] = x4.w;
        m[4] = x5.x; m[5] = x5.y; m[6] = x5.z; m[7] = x5.w;
        m[8] = x6.x; m[9] = x6.y; m[10] = x6.z; m[11] = x6.w;
        m[12] = x7.x; m[13] = x7.y; m[14] = x7.z; m[15] = x7.w;
        compress(cur, m, leaf, 64, b == 14 ? fl_end : 0u);
      }
#else
      // unrolled by 2: keeps this loop's compressions a separate copy (the
      // compiler otherwise merges them with the general loop's)
#pragma unroll 2
      for (uint32_t b = 0; b < 16; ++b, q += 4) {
        const u32x4 x0 = q[0], x1 = q[1], x2 = q[2], x3 = q[3];
        m[0] = x0.x; m[1] = x0.y; m[2] = x0.z; m[3] = x0.w;
        m[4] = x1.x; m[5] = x1.y; m[6] = x1.z; m[7] = x1.w;
        m[8] = x2.x; m[9] = x2.y; m[10] = x2.z; m[11] = x2.w;
        m[12] = x3.x; m[13] = x3.y; m[14] = x3.z; m[15] = x3.w;
        compress(cur, m, leaf, 64, b == 0 ? CHUNK_START : b == 15 ? fl_end : 0u);
      }
#endif
      if (D > 0) finish(k);
      continue;
    }
    for (uint32_t b = 0; b < nb; ++b) {
      const uint32_t bl = min(64u, llen - (b << 6));
      uint32_t flags = (b == 0 ? CHUNK_START : 0) | (b + 1 == nb ? CHUNK_END : 0);
      if (b + 1 == nb && root_group && nleaves == 1) flags |= ROOT;
      if (NOLOAD) {
#pragma unroll
        for (int i = 0; i < 16; ++i) m[i] = pos * 0x9E3779B9u + i;
        compress(cur, m, leaf, bl, flags);
        pos += 64;
      } else if (PF) {
        uint32_t nx[16];
        const uint32_t np = pos + 64;
        if (np < gend) load_block<NT>(src + np, min(64u, gend - np), end, nx);
        compress(cur, m, leaf, bl, flags);
#pragma unroll
        for (int i = 0; i < 16; ++i) m[i] = nx[i];
        pos = np;
      } else {
        load_block<NT>(src + off + (b << 6), bl, end, m);
        compress(cur, m, leaf, bl, flags);
      }
    }
    if (D > 0) finish(k);
  }
  return root_group ? 1 : 2;
}

#ifndef B3_BALANCE
#define B3_BALANCE 1
#endif

// Compressions of leaf group j of a chunk of len bytes (its 64-B blocks plus
// the in-group parent merges): the lane's work.
template <int D>
__device__ __forceinline__ uint32_t group_work(uint32_t len, uint32_t j) {
  const uint32_t nleaves = len == 0 ? 1 : (len + kLeaf - 1) / kLeaf;
  const uint32_t first = j << D;
  if (first >= nleaves) return 0;
  const uint32_t cnt = min(1u << D, nleaves - first);
  const uint32_t start = first * kLeaf, gend = min(len, (first + cnt) * kLeaf);
  const uint32_t blocks = gend > start ? (gend - start + 63) / 64 : 1;
  return blocks + cnt - 1;
}

#ifndef B3_WAVES_PER_EU
#define B3_WAVES_PER_EU 0
#endif

// In-window tree levels by lane quads (defined with compress_quad below).
#ifndef B3_WG_QUAD
#define B3_WG_QUAD 1
#endif
#if B3_WG_QUAD
__device__ __forceinline__ void wg_tree_quad(uint32_t *b0, uint32_t *b1, uint32_t *nit, bool inwg,
                                             uint32_t k, uint32_t j, uint32_t o, uint32_t c,
                                             const uint32_t cur[8], uint32_t slot,
                                             ngpu_result *__restrict__ out);
#endif
#if B3_WAVES_PER_EU
#define B3_OCC __attribute__((amdgpu_waves_per_eu(B3_WAVES_PER_EU)))
#else
#define B3_OCC
#endif

template <int D, int LM>
__global__ __launch_bounds__(256) B3_OCC void b3_groups(
    const uint8_t *__restrict__ data, uint64_t data_len,
    const ngpu_chunk *__restrict__ chunks, uint64_t n,
    const uint64_t *__restrict__ gbase, const uint32_t *__restrict__ gchunk,
    uint64_t cap_g, uint32_t *__restrict__ cv_out,
    ngpu_result *__restrict__ out, uint64_t *__restrict__ err,
    const uint32_t *__restrict__ small, const uint64_t *__restrict__ nsmall,
    uint32_t *__restrict__ tree_list) {
  __shared__ uint32_t lcv[256 * 8];
#if B3_WG_QUAD
  __shared__ uint32_t lcv2[256 * 8];  // ping-pong partner of lcv
#endif
  // groups [0, gm): multi-group chunks in chunk order; [gm, gm + ns): the
  // single-group chunks, largest first
  const uint64_t gm = gbase[n];
  const uint64_t total = gm + *nsmall;
  const uint64_t g0 = blockIdx.x * 256ull;
  // err[1] (stats[8]): more groups than the launch covers (overlapping
  // descriptors); the call fails instead of leaving groups unhashed
  if (blockIdx.x == 0 && threadIdx.x == 0 && (total > gridDim.x * 256ull || total > cap_g))
    note_overlap(err, total);
  uint32_t slot = threadIdx.x;  // the group of this workgroup window this lane hashes
#if B3_BALANCE
  // Lane balance inside the window: a wave runs as long as its longest lane,
  // and the last group of a multi-group chunk is usually partial (real layers:
  // 10 % of the lanes idle).  When the window's groups differ in work, lanes
  // take them in descending work order (counting sort over 64 buckets), so
  // each wave holds groups of near-equal work.  The window's tree reduction
  // is slot-based, so it is unaffected; uniform windows (C2) skip the sort.
  {
    __shared__ uint32_t hb[64], perm[256], key0;
    constexpr int KS = D > 1 ? D - 1 : 0;  // <= 34 buckets for D <= 4
    const uint64_t gs = g0 + threadIdx.x;
    uint32_t key = 0;
    if (gs < total && gs < cap_g) {
      uint32_t cc, jj;
      if (gs < gm) {
        cc = gchunk[gs];
        jj = (uint32_t)(gs - gbase[cc]);
      } else {
        cc = small[gs - gm];
        jj = 0;
      }
      key = group_work<D>(chunks[cc].length, jj);
    }
    if (threadIdx.x == 0) key0 = key;
    if (threadIdx.x < 64) hb[threadIdx.x] = 0;
    __syncthreads();
    if (!__syncthreads_and(key == key0)) {
      const uint32_t b = 63 - min(63u, key >> KS);  // descending work
      const uint32_t r = atomicAdd(&hb[b], 1u);
      __syncthreads();
      if (threadIdx.x < 64) {  // exclusive scan of the 64 bucket counts (wave 0)
        const uint32_t v = hb[threadIdx.x];
        uint32_t x = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const uint32_t y = __shfl_up(x, o, 64);
          if ((int)threadIdx.x >= o) x += y;
        }
        hb[threadIdx.x] = x - v;
      }
      __syncthreads();
      perm[hb[b] + r] = threadIdx.x;
      __syncthreads();
      slot = perm[threadIdx.x];
    }
  }
#endif
  const uint64_t g = g0 + slot;
  uint32_t cur[8], c = 0, j = 0;
  uint64_t base = 0, ng = 0;
  int st = 0;
  if (g < total && g < cap_g) {
    if (g < gm) {
      c = gchunk[g];
      base = gbase[c];
      ng = gbase[c + 1] - base;
      j = (uint32_t)(g - base);
    } else {
      c = small[g - gm];
      base = g;
      ng = 1;
    }
    st = group_cv<D, LM>(data, data_len, chunks, c, ng, j, err, cur);
  }
  if (st == 1) {
    uint4 *d = reinterpret_cast<uint4 *>(out[c].digest);
    d[0] = make_uint4(cur[0], cur[1], cur[2], cur[3]);
    d[1] = make_uint4(cur[4], cur[5], cur[6], cur[7]);
    out[c].kind = NGPU_DIGESTED;  // the dedup stage takes only marked records
  }
  // Chunks whose groups all sit in this workgroup finish here: the upper
  // levels of their tree are reduced in LDS (pairwise, odd tail promoted).
  // Others publish their group CV for b3_tree.
  const bool inwg = st == 2 && tree_in_workgroup(base, ng);
  if (st == 2 && !inwg) {
    if (j == 0) {  // err + 2 == stats[9]: chunks queued for b3_tree
      const uint64_t q = atomicAdd(reinterpret_cast<unsigned long long *>(err + 2), 1ull);
      tree_list[q] = c;
    }
    uint4 *d = reinterpret_cast<uint4 *>(cv_out + g * 8);
    d[0] = make_uint4(cur[0], cur[1], cur[2], cur[3]);
    d[1] = make_uint4(cur[4], cur[5], cur[6], cur[7]);
  }
#if B3_WG_QUAD
  __shared__ uint32_t nit[2];
  if (threadIdx.x == 0) nit[0] = nit[1] = 0;
#endif
  if (!__syncthreads_or(inwg)) return;
  const uint32_t o = (uint32_t)(base - g0);  // chunk's first slot in lcv
  uint32_t k = inwg ? (uint32_t)ng : 1;
#if B3_WG_QUAD
  wg_tree_quad(lcv, lcv2, nit, inwg, k, j, o, c, cur, slot, out);
#else
  if (inwg) {
#pragma unroll
    for (int i = 0; i < 8; ++i) lcv[8 * slot + i] = cur[i];
  }
  for (;;) {
    const bool active = k > 1;
    if (!__syncthreads_or(active)) break;
    uint32_t r[8];
    const uint32_t p = k >> 1;
    const bool comp = active && j < p;
    const bool odd = active && (k & 1) && j == p;
    if (comp) {
      uint32_t m[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) m[i] = lcv[8 * (o + 2 * j) + i];
      set_iv(r);
      compress(r, m, 0, 64, PARENT | (k == 2 ? ROOT : 0));
    }
    if (odd) {
#pragma unroll
      for (int i = 0; i < 8; ++i) r[i] = lcv[8 * (o + k - 1) + i];
    }
    __syncthreads();
    if (comp || odd) {
#pragma unroll
      for (int i = 0; i < 8; ++i) lcv[8 * (o + j) + i] = r[i];
    }
    if (comp && k == 2) {
      uint4 *d = reinterpret_cast<uint4 *>(out[c].digest);
      d[0] = make_uint4(r[0], r[1], r[2], r[3]);
      d[1] = make_uint4(r[4], r[5], r[6], r[7]);
      out[c].kind = NGPU_DIGESTED;
    }
    k = active ? p + (k & 1) : 1;
  }
#endif
}

// Upper levels: one workgroup per chunk with more than one leaf group.
// ---- small layers: one compression per lane QUAD (latency path) ---------------
// A small layer has far fewer 1-KiB leaves than the chip has lanes (C1: ~10K
// leaves, 157 waves for 1,024 SIMDs), so b3_groups runs one wave per SIMD and
// each lane's 16 chained compressions (680 VALU ops each, one op per ~5
// cycles for a lone wave) ARE the kernel time.  Here four lanes share each
// compression, one column of the 4 x 4 state per lane: a G step is the
// lane's own G, and the row rotation between column and diagonal steps rides
// on the first use of b, c and d as DPP quad_perm operands of v_add / v_xor
// (gfx950 has no DPP on VOP3, so b costs one v_mov_dpp): ~190 VALU ops per
// lane per compression instead of 680.  The message block is staged in LDS
// (each lane stores its 16 B, then reads its 28 schedule words at per-lane
// offsets fixed for the kernel) -- the "message words staged in LDS" of the
// north star.  Chunk trees above the leaves go to b3_tree.
constexpr int kQuadThreads = 256;           // 64 quads = 64 leaves per workgroup
// Up to 40K leaves (<= 2.5 quad waves per SIMD).  Measured crossover with the
// lane-per-leaf path (profiles/r2/quad_threshold_r2qt.json, digest ms, lane vs
// quad): 8 MiB 0.030 / 0.018, 16 MiB 0.030 / 0.020, 32 MiB 0.033 / 0.026,
// 48 MiB 0.033 / 0.032, 64 MiB equal.  Round 3 (profiles/r3/ab_quad_max/,
// builds alternated on one box): a 32 MiB layer (32,768 leaves + its chunks)
// missed the old 32K limit by its chunk count: 467-486 GB/s on b3_groups<0>,
// 577 on the quad path; 48 MiB ties (0.032 ms both ways).
#ifndef B3_QUAD_PF
#define B3_QUAD_PF 1
#endif
#ifndef B3_QUAD_MAX_LEAVES
#define B3_QUAD_MAX_LEAVES 40960
#endif
constexpr uint64_t kQuadMaxLeaves = B3_QUAD_MAX_LEAVES;
constexpr int kQP1 = 0x39, kQP2 = 0x4E, kQP3 = 0x93;  // quad_perm: lane i reads lane i+1/+2/+3

template <int P>
__device__ __forceinline__ uint32_t qperm(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, P, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t rotr32(uint32_t x, int n) {
  return __builtin_amdgcn_alignbit(x, x, n);
}
// G on the lane's column, registers aligned.
__device__ __forceinline__ void gq(uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d,
                                   uint32_t mx, uint32_t my) {
  a = a + b + mx; d = rotr32(d ^ a, 16); c = c + d; b = rotr32(b ^ c, 12);
  a = a + b + my; d = rotr32(d ^ a, 8);  c = c + d; b = rotr32(b ^ c, 7);
}
// G whose b, c, d are first read from quad lanes +PB, +PC, +PD (the row
// rotation folded into each word's first use); leaves them rotated.
template <int PB, int PC, int PD>
__device__ __forceinline__ void gq_rot(uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d,
                                       uint32_t mx, uint32_t my) {
  const uint32_t br = qperm<PB>(b);
  a = a + br + mx; d = rotr32(qperm<PD>(d) ^ a, 16); c = qperm<PC>(c) + d;
  b = rotr32(br ^ c, 12);
  a = a + b + my; d = rotr32(d ^ a, 8); c = c + d; b = rotr32(b ^ c, 7);
}
// Lane q of a quad holds cv[q], cv[4 + q] in (x, y); m: the lane's schedule
// words, round r = {column x, column y, diagonal x, diagonal y}; dq = v[12 + q]
// (counter lo, counter hi, block length, flags).
__device__ __forceinline__ void compress_quad(uint32_t &x, uint32_t &y, const uint32_t m[28],
                                              uint32_t ivq, uint32_t dq) {
  uint32_t a = x, b = y, c = ivq, d = dq;
  gq(a, b, c, d, m[0], m[1]);
  gq_rot<kQP1, kQP2, kQP3>(a, b, c, d, m[2], m[3]);  // column -> diagonal
#pragma unroll
  for (int r = 1; r < 7; ++r) {
    gq_rot<kQP3, kQP2, kQP1>(a, b, c, d, m[4 * r], m[4 * r + 1]);      // diagonal -> column
    gq_rot<kQP1, kQP2, kQP3>(a, b, c, d, m[4 * r + 2], m[4 * r + 3]);  // column -> diagonal
  }
  // diagonal alignment: v[8 + q] is on lane q + 2, v[4 + q] on q - 1, v[12 + q] on q + 1
  x = a ^ qperm<kQP2>(c);
  y = qperm<kQP3>(b) ^ qperm<kQP1>(d);
}

// The schedule word of round r, slot s (column x/y, diagonal x/y) for the 4
// lanes of a quad, one nibble per lane.
struct QuadSched { uint16_t w[7][4]; };
constexpr QuadSched make_quad_sched() {
  QuadSched t{};
  for (int r = 0; r < 7; ++r)
    for (int sl = 0; sl < 4; ++sl) {
      uint16_t v = 0;
      for (int q = 0; q < 4; ++q) {
        const int pos = (sl < 2 ? 0 : 8) + 2 * q + (sl & 1);
        v |= (uint16_t)(kSched.s[r][pos] << (4 * q));
      }
      t.w[r][sl] = v;
    }
  return t;
}
constexpr QuadSched kQuadSched = make_quad_sched();

#if B3_WG_QUAD
// The upper levels of the chunks whose groups all sit in one b3_groups
// workgroup.  Each level lists its parents in LDS (source pair, destination
// slot, ROOT, chunk) and the workgroup's 64 quads take them one per quad
// (compress_quad: ~190 VALU per lane), reading one CV buffer and writing the
// other, so a level costs one barrier after its list and one after its
// compressions.  One compression per lane instead ran a 680-op compression in
// every wave holding a parent, however few: on C2 (two 1 MiB chunks of 128
// groups per workgroup) 14 wave-compressions for 3.97 of parent work, about
// 2.7 % of the kernel's issued VALU.  The chunk's own lanes (slot o + j,
// group j of k) list the level's parents and promote an odd tail.
__device__ __forceinline__ void wg_tree_quad(uint32_t *b0, uint32_t *b1, uint32_t *nit, bool inwg,
                                             uint32_t k, uint32_t j, uint32_t o, uint32_t c,
                                             const uint32_t cur[8], uint32_t slot,
                                             ngpu_result *__restrict__ out) {
  __shared__ uint32_t item[128], item_c[128];  // <= 128 parents per level (256 slots)
  const uint32_t q = threadIdx.x & 3, quad = threadIdx.x >> 2;
  if (inwg) {
#pragma unroll
    for (int i = 0; i < 8; ++i) b0[8 * slot + i] = cur[i];
  }
  uint32_t *src = b0, *dst = b1;
  for (uint32_t lv = 0;; ++lv) {
    const bool active = k > 1;
    const uint32_t p = k >> 1;
    if (active && j < p) {
      const uint32_t at = atomicAdd(&nit[lv & 1], 1u);
      item[at] = (o + 2 * j) | ((o + j) << 8) | (k == 2 ? 1u << 16 : 0u);
      item_c[at] = c;
    }
    if (active && (k & 1) && j == p) {  // odd tail promoted
#pragma unroll
      for (int i = 0; i < 8; ++i) dst[8 * (o + p) + i] = src[8 * (o + k - 1) + i];
    }
    if (!__syncthreads_or(active)) break;
    const uint32_t ni = nit[lv & 1];
    // the other counter was last read before the previous level's final barrier
    if (threadIdx.x == 0) nit[(lv & 1) ^ 1] = 0;
    for (uint32_t it = quad; it < ni; it += 64) {
      uint32_t wo[28];
#pragma unroll
      for (int r = 0; r < 7; ++r)
#pragma unroll
        for (int sl = 0; sl < 4; ++sl) wo[4 * r + sl] = (kQuadSched.w[r][sl] >> (4 * q)) & 15u;
      const uint32_t w = item[it];
      const uint32_t *t = src + 8 * (w & 255u);
      uint32_t m[28];
#pragma unroll
      for (int k2 = 0; k2 < 28; ++k2) m[k2] = t[wo[k2]];
      const bool root = (w >> 16) & 1u;
      const uint32_t ivq = q == 0 ? IV0 : q == 1 ? IV1 : q == 2 ? IV2 : IV3;
      const uint32_t ivh = q == 0 ? IV4 : q == 1 ? IV5 : q == 2 ? IV6 : IV7;
      const uint32_t dq = q == 2 ? 64u : q == 3 ? (PARENT | (root ? ROOT : 0u)) : 0u;
      uint32_t x = ivq, y = ivh;
      compress_quad(x, y, m, ivq, dq);
      const uint32_t d = (w >> 8) & 255u;
      dst[8 * d + q] = x;
      dst[8 * d + 4 + q] = y;
      if (root) {
        const uint32_t cc = item_c[it];
        uint32_t *dg = reinterpret_cast<uint32_t *>(out[cc].digest);
        dg[q] = x;
        dg[4 + q] = y;
        if (q == 0) out[cc].kind = NGPU_DIGESTED;
      }
    }
    __syncthreads();
    uint32_t *tmp = src;
    src = dst;
    dst = tmp;
    k = active ? p + (k & 1) : 1;
  }
}
#endif

// The lane's 16 bytes of a block: valid (0..16) bytes, zero padded; byte
// loads when partial or unaligned (never past the chunk).
__device__ __forceinline__ u32x4 load16(const uint8_t *p, int valid) {
  if (valid >= 16 && (reinterpret_cast<uintptr_t>(p) & 15) == 0)
    return *reinterpret_cast<const u32x4 *>(p);
  uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < 16; ++i)
    if (i < valid) w[i >> 2] |= (uint32_t)p[i] << (8 * (i & 3));
  return u32x4{w[0], w[1], w[2], w[3]};
}

// Leaf j of chunk c (a whole 1 KiB BLAKE3 chunk-leaf, or less at the end) by
// one quad: lane q holds state column q.  root_group: the chunk is this one
// leaf (digest straight to out[c], ROOT on the last block); else the leaf's
// CV goes to cv_out[g].  blk: the quad's 16 message words in LDS.
__device__ __forceinline__ void quad_leaf(const uint8_t *__restrict__ data, const ngpu_chunk &ch,
                                          uint32_t c, uint32_t j, bool root_group, uint64_t g,
                                          uint32_t q, uint32_t *blk, uint32_t *__restrict__ cv_out,
                                          ngpu_result *__restrict__ out, uint32_t *lds_row = nullptr) {
  const uint32_t len = ch.length;
  uint32_t wo[28];  // this lane's schedule words: LDS word offsets in the quad's block
#pragma unroll
  for (int r = 0; r < 7; ++r)
#pragma unroll
    for (int sl = 0; sl < 4; ++sl) wo[4 * r + sl] = (kQuadSched.w[r][sl] >> (4 * q)) & 15u;
  const uint32_t off = j * kLeaf;
  const uint32_t llen = min(kLeaf, len - off);
  const uint32_t nb = llen == 0 ? 1 : (llen + 63) >> 6;
  const uint8_t *src = data + ch.offset + off + 16 * q;
  const uint32_t iv_lo[4] = {IV0, IV1, IV2, IV3}, iv_hi[4] = {IV4, IV5, IV6, IV7};
  const uint32_t ivq = q == 0 ? iv_lo[0] : q == 1 ? iv_lo[1] : q == 2 ? iv_lo[2] : iv_lo[3];
  uint32_t x = ivq, y = q == 0 ? iv_hi[0] : q == 1 ? iv_hi[1] : q == 2 ? iv_hi[2] : iv_hi[3];
  auto valid = [&](uint32_t b) { return (int)min(16u, (uint32_t)max(0, (int)llen - (int)(64 * b + 16 * q))); };
#if B3_QUAD_PF
  // the whole leaf in flight at once (16 x 16 B per lane): one memory latency
  // per leaf instead of one per block behind a one-block prefetch
  u32x4 wb[16];
  if (llen == kLeaf && (reinterpret_cast<uintptr_t>(src) & 15) == 0) {
#pragma unroll
    for (int b = 0; b < 16; ++b) wb[b] = *reinterpret_cast<const u32x4 *>(src + 64 * b);
  } else {
#pragma unroll
    for (int b = 0; b < 16; ++b) wb[b] = (uint32_t)b < nb ? load16(src + 64 * b, valid(b)) : u32x4{};
  }
#pragma unroll
  for (uint32_t b = 0; b < 16; ++b) {
    if (b >= nb) continue;  // (not break: keeps the loop unrolled, wb in registers)
    const u32x4 w = wb[b];
#else
  u32x4 w = load16(src, valid(0));
  for (uint32_t b = 0; b < nb; ++b) {
    u32x4 nx = w;
    if (b + 1 < nb) nx = load16(src + 64 * (b + 1), valid(b + 1));  // next block in flight
#endif
    *reinterpret_cast<u32x4 *>(blk + 4 * q) = w;
    // the quad's four stores are in this wave's LDS queue ahead of its loads
    asm volatile("" ::: "memory");
    uint32_t m[28];
#pragma unroll
    for (int k = 0; k < 28; ++k) m[k] = blk[wo[k]];
    asm volatile("" ::: "memory");
    const uint32_t bl = min(64u, llen - 64 * b);
    const uint32_t flags = (b == 0 ? CHUNK_START : 0u) |
                           (b + 1 == nb ? (CHUNK_END | (root_group ? ROOT : 0u)) : 0u);
    const uint32_t dq = q == 0 ? j : q == 1 ? 0u : q == 2 ? bl : flags;
    compress_quad(x, y, m, ivq, dq);
#if !B3_QUAD_PF
    w = nx;
#endif
  }
  if (root_group) {
    uint32_t *d = reinterpret_cast<uint32_t *>(out[c].digest);
    d[q] = x;
    d[4 + q] = y;
    if (q == 0) out[c].kind = NGPU_DIGESTED;
  } else if (lds_row) {  // b3_quad_planned: the CV stays in LDS for the in-wave levels
    lds_row[q] = x;
    lds_row[4 + q] = y;
  } else {
    cv_out[g * 8 + q] = x;
    cv_out[g * 8 + 4 + q] = y;
  }
}

// One leaf per quad: leaves [0, gm) of multi-leaf chunks (CV to cv_out, the
// chunk queued for b3_tree by its leaf 0), then the single-leaf chunks
// (digest, ROOT).  Group == leaf (D = 0).  Planned by the grid kernels.
__global__ __launch_bounds__(kQuadThreads) void b3_quad_leaves(
    const uint8_t *__restrict__ data, uint64_t data_len, const ngpu_chunk *__restrict__ chunks,
    uint64_t n, const uint64_t *__restrict__ gbase, const uint32_t *__restrict__ gchunk,
    uint64_t cap_g, uint32_t *__restrict__ cv_out, ngpu_result *__restrict__ out,
    uint64_t *__restrict__ err, const uint32_t *__restrict__ small,
    const uint64_t *__restrict__ nsmall, uint32_t *__restrict__ tree_list) {
  __shared__ __attribute__((aligned(16))) uint32_t qmsg[kQuadThreads / 4 * 16];
  const uint32_t q = threadIdx.x & 3, quad = threadIdx.x >> 2;
  const uint64_t gm = gbase[n], total = gm + *nsmall;
  const uint64_t g = blockIdx.x * (uint64_t)(kQuadThreads / 4) + quad;
  if (blockIdx.x == 0 && threadIdx.x == 0 &&
      (total > gridDim.x * (uint64_t)(kQuadThreads / 4) || total > cap_g))
    note_overlap(err, total);  // stats[8]: overlapping descriptors (b3_groups)
  if (g >= total || g >= cap_g) return;  // per quad: its four lanes leave together
  uint32_t c, j;
  bool root_group;
  if (g < gm) {
    c = gchunk[g];
    j = (uint32_t)(g - gbase[c]);
    root_group = false;
  } else {
    c = small[g - gm];
    j = 0;
    root_group = true;
  }
  const ngpu_chunk ch = chunks[c];
  if (ch.offset > data_len || ch.length > data_len - ch.offset) {  // bad descriptor
    if (j == 0 && q == 0) note_bad_desc(err, 1);
    return;
  }
  quad_leaf(data, ch, c, j, root_group, g, q, qmsg + quad * 16, cv_out, out);
  if (!root_group && j == 0 && q == 0) {  // err + 2 == stats[9]: chunks queued for b3_tree
    const uint64_t t = atomicAdd(reinterpret_cast<unsigned long long *>(err + 2), 1ull);
    tree_list[t] = c;
  }
}

#ifndef B3_QUAD_GROUPS
#define B3_QUAD_GROUPS 1
#endif
#if B3_QUAD_GROUPS
// Small calls (<= kSmallPlanChunks chunks, quad path): the planning is done
// by every workgroup for itself in LDS, so the call has no planning kernel,
// and the two lowest tree levels of every multi-leaf chunk run inside the
// wave that hashed their leaves.
//   * Slots: the multi-leaf chunks first, in chunk order, each taking its leaf
//     count rounded up to 4 slots (so its leaves 4i..4i+3 are 4 adjacent
//     quads of one wave), then one slot per single-leaf chunk.  mpre / spre:
//     exclusive prefixes of the two (a chunk has width in one of them only).
//   * A leaf's CV stays in LDS (qcv, 8 words per quad, rows of adjacent quads
//     adjacent).  Level 1: the quad of leaf 4i (4i+2) compresses the parent of
//     rows 4i, 4i+1 (4i+2, 4i+3) -- two adjacent rows ARE the parent's
//     16-word message -- and level 2 the parent of rows 4i and 4i+2; the odd
//     tail is promoted.  Aligned groups of 4 leaves are complete BLAKE3
//     subtrees, the last (ragged) group the tree's right edge, so b3_tree
//     continues over ceil(leaves / 4) group CVs exactly as over the leaves;
//     a chunk of <= 4 leaves ends here (ROOT on its last parent) and is not
//     queued.  Group CVs sit at cv[mpre[c] / 4 + i] (groups[c] = mpre[c] / 4).
// The in-wave levels need no barrier: one wave's LDS operations complete in
// order.  Workgroup 0 writes what b3_tree reads: groups[0..n], the queue of
// chunks with more than 4 leaves in chunk order, and the call's counters
// (stats[7] = bad descriptors, stats[9] = queued chunks, the rest zero) --
// deterministic, no atomics.  Round 6: the C1 tree stage dropped its two
// widest levels.
constexpr int kFusedItems = (int)(kSmallPlanChunks / kQuadThreads);
static_assert(kFusedItems * kQuadThreads == (int)kSmallPlanChunks, "one item set");

__global__ __launch_bounds__(kQuadThreads) void b3_quad_planned(
    const uint8_t *__restrict__ data, uint64_t data_len, const ngpu_chunk *__restrict__ chunks,
    uint64_t n, uint64_t cap_g, uint32_t *__restrict__ cv_out, ngpu_result *__restrict__ out,
    uint64_t *__restrict__ groups, uint64_t *__restrict__ stats, uint32_t *__restrict__ tree_list) {
  __shared__ __attribute__((aligned(16))) uint32_t qmsg[kQuadThreads / 4 * 16];
  __shared__ __attribute__((aligned(16))) uint32_t qcv[kQuadThreads / 4 * 8];
  __shared__ uint32_t mpre[kSmallPlanChunks + 1], spre[kSmallPlanChunks + 1];
  __shared__ uint32_t wsum[4][kQuadThreads / 64];
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  // this thread's chunks: c0 .. c0 + kFusedItems - 1 (contiguous)
  const uint32_t c0 = (uint32_t)t * kFusedItems;
  uint32_t lv[kFusedItems], sm = 0, ss = 0, sq = 0, bad = 0, mb = 0;
#pragma unroll
  for (int i = 0; i < kFusedItems; ++i) {
    const uint32_t c = c0 + i;
    lv[i] = 0;
    if (c < n) {
      const ngpu_chunk ch = chunks[c];
      const uint32_t len = ch.length;
      const bool bd = ch.offset > data_len || len > data_len - ch.offset;
      lv[i] = len == 0 ? 1 : (len + kLeaf - 1) / kLeaf;
      if (bd) mb |= 1u << i;  // a bad chunk keeps its slots but is never hashed
      if (lv[i] > 1) sm += (lv[i] + 3) & ~3u;
      else ss += 1;
      sq += lv[i] > 4 && !bd;
      bad += bd;
    }
  }
  // four block scans in one pass (multi slots; single slots; queued chunks; bad)
  uint32_t xm = sm, xs = ss, xq = sq, xb = bad;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t ym = __shfl_up(xm, o, 64), ys = __shfl_up(xs, o, 64);
    const uint32_t yq = __shfl_up(xq, o, 64), yb = __shfl_up(xb, o, 64);
    if (lane >= o) xm += ym, xs += ys, xq += yq, xb += yb;
  }
  if (lane == 63) wsum[0][wid] = xm, wsum[1][wid] = xs, wsum[2][wid] = xq, wsum[3][wid] = xb;
  __syncthreads();
  uint32_t pm = 0, ps = 0, pq = 0, tm = 0, ts = 0, tq = 0, tb = 0;
#pragma unroll
  for (int w = 0; w < kQuadThreads / 64; ++w) {
    if (w < wid) pm += wsum[0][w], ps += wsum[1][w], pq += wsum[2][w];
    tm += wsum[0][w];
    ts += wsum[1][w];
    tq += wsum[2][w];
    tb += wsum[3][w];
  }
  uint32_t rm = pm + xm - sm, rs = ps + xs - ss, rq = pq + xq - sq;
  const bool writer = blockIdx.x == 0;
#pragma unroll
  for (int i = 0; i < kFusedItems; ++i) {
    const uint32_t c = c0 + i;
    if (c < n) {
      mpre[c] = rm;
      spre[c] = rs;
      if (writer) {
        groups[c] = rm / 4;
        if (lv[i] > 4 && !((mb >> i) & 1)) tree_list[rq++] = c;
      }
      if (lv[i] > 1) rm += (lv[i] + 3) & ~3u;
      else rs += 1;
    }
  }
  if (t == 0) {
    mpre[n] = tm;
    spre[n] = ts;
    if (writer) groups[n] = tm / 4;
  }
  // stats[8]: more slots than the launch covers, or more group CVs than the
  // workspace holds -- descriptors that overlap (a tar's file extents never
  // do); the call then fails instead of leaving leaves unhashed
  const uint64_t span = (uint64_t)gridDim.x * (kQuadThreads / 4);
  const uint64_t total = (uint64_t)tm + ts;
  const uint64_t over = total > span || tm / 4 > cap_g ? total : 0;
  if (writer && t < 16)
    stats[t] = t == kStBadDesc ? tb : t == kStTreeQueued ? tq : t == kStOverlap ? over : 0;
  if (writer && t == 0 && tb)
    atomicAdd((unsigned long long *)(stats + kStSticky), (unsigned long long)tb);
  if (writer && t == 0 && over)
    atomicMax((unsigned long long *)(stats + kStSticky + 1), (unsigned long long)over);
  __syncthreads();
  const uint32_t q = t & 3, quad = t >> 2;
  const uint64_t g = blockIdx.x * (uint64_t)(kQuadThreads / 4) + quad;
  if (g >= total || over) return;  // per quad: its four lanes leave together
  // the chunk holding slot g: the last c whose prefix is <= g (a chunk of
  // zero width in that prefix is never the last such c below the total)
  const bool multi = g < tm;
  const uint32_t *pre = multi ? mpre : spre;
  const uint32_t key = multi ? (uint32_t)g : (uint32_t)(g - tm);
  uint32_t lo = 0, hi = (uint32_t)n;  // pre[lo] <= key < pre[hi]
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (pre[mid] <= key) lo = mid;
    else hi = mid;
  }
  const uint32_t c = lo, j = key - pre[c];
  const ngpu_chunk ch = chunks[c];
  if (ch.offset > data_len || ch.length > data_len - ch.offset) return;  // counted above
  const uint32_t nl = ch.length == 0 ? 1 : (ch.length + kLeaf - 1) / kLeaf;
  if (j >= nl) return;  // a padding slot
  uint32_t *row = qcv + quad * 8;
  quad_leaf(data, ch, c, j, !multi, g, q, qmsg + quad * 16, cv_out, out, row);
  if (!multi) return;
  // schedule word offsets in a parent's message (two adjacent rows), from an
  // opaque copy of q: sharing the leaf loop's kept 28 more VGPRs live through
  // it (175 -> 134 VGPRs, 2 -> 3 waves per SIMD)
  uint32_t ql = q;
  asm volatile("" : "+v"(ql));
  uint32_t wo[28];
#pragma unroll
  for (int r = 0; r < 7; ++r)
#pragma unroll
    for (int sl = 0; sl < 4; ++sl) wo[4 * r + sl] = (kQuadSched.w[r][sl] >> (4 * ql)) & 15u;
  const uint32_t ivq = q == 0 ? IV0 : q == 1 ? IV1 : q == 2 ? IV2 : IV3;
  const uint32_t ivh = q == 0 ? IV4 : q == 1 ? IV5 : q == 2 ? IV6 : IV7;
  const uint32_t jr = j & 3, rem = nl - (j - jr);  // leaves of this group of 4
  asm volatile("" ::: "memory");
  if ((jr & 1) == 0 && j + 1 < nl) {  // level 1: rows j, j + 1
    uint32_t m[28];
#pragma unroll
    for (int k = 0; k < 28; ++k) m[k] = row[wo[k]];
    const uint32_t pf = PARENT | (nl == 2 ? ROOT : 0u);
    uint32_t x = ivq, y = ivh;
    compress_quad(x, y, m, ivq, q == 2 ? 64u : q == 3 ? pf : 0u);
    row[q] = x;
    row[4 + q] = y;
  }
  asm volatile("" ::: "memory");
  if (jr == 0 && rem >= 3) {  // level 2: rows j, j + 2
    uint32_t m[28];
#pragma unroll
    for (int k = 0; k < 28; ++k) m[k] = row[wo[k] + (wo[k] & 8u)];  // words 8.. from row j + 2
    const uint32_t pf = PARENT | (nl <= 4 ? ROOT : 0u);
    uint32_t x = ivq, y = ivh;
    compress_quad(x, y, m, ivq, q == 2 ? 64u : q == 3 ? pf : 0u);
    row[q] = x;
    row[4 + q] = y;
  }
  asm volatile("" ::: "memory");
  if (jr != 0) return;
  const uint32_t x = row[q], y = row[4 + q];
  if (nl <= 4) {  // the chunk's root: its digest
    uint32_t *d = reinterpret_cast<uint32_t *>(out[c].digest);
    d[q] = x;
    d[4 + q] = y;
    if (q == 0) out[c].kind = NGPU_DIGESTED;
  } else {  // group j / 4 of the chunk, for b3_tree
    const uint64_t gc = mpre[c] / 4 + j / 4;
    cv_out[gc * 8 + q] = x;
    cv_out[gc * 8 + 4 + q] = y;
  }
}

// Slots b3_quad_planned may need: every multi-leaf chunk rounded up to 4.
uint64_t quad_planned_slots(uint64_t n, uint64_t data_len) { return data_len / kLeaf + 4 * n + 1; }
#else
// Small calls (<= kSmallPlanChunks chunks, quad path): the planning is done
// by every workgroup for itself in LDS, so the call has no planning kernel
// (one launch less: ~4 us of host enqueue and ~5 us of a small layer's GPU
// time).  Leaves are numbered in chunk order (gpre = exclusive scan of each
// chunk's leaf count, a zero-length chunk counting one), quad g takes leaf
// g - gpre[c] of the chunk c with gpre[c] <= g < gpre[c + 1].  Workgroup 0
// also writes what the later kernels and the host read: groups[0..n] = gpre,
// the multi-leaf chunks in chunk order as b3_tree's queue, and the call's
// counters (stats[7] = bad descriptors, stats[9] = queued chunks, the rest
// zero) -- all deterministic, no atomics.
constexpr int kFusedItems = (int)(kSmallPlanChunks / kQuadThreads);
static_assert(kFusedItems * kQuadThreads == (int)kSmallPlanChunks, "one item set");

__global__ __launch_bounds__(kQuadThreads) void b3_quad_planned(
    const uint8_t *__restrict__ data, uint64_t data_len, const ngpu_chunk *__restrict__ chunks,
    uint64_t n, uint64_t cap_g, uint32_t *__restrict__ cv_out, ngpu_result *__restrict__ out,
    uint64_t *__restrict__ groups, uint64_t *__restrict__ stats, uint32_t *__restrict__ tree_list) {
  __shared__ __attribute__((aligned(16))) uint32_t qmsg[kQuadThreads / 4 * 16];
  __shared__ uint32_t gpre[kSmallPlanChunks + 1];
  __shared__ uint32_t wsum[3][kQuadThreads / 64];
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  // this thread's chunks: c0 .. c0 + kFusedItems - 1 (contiguous)
  const uint32_t c0 = (uint32_t)t * kFusedItems;
  uint32_t lv[kFusedItems], sum = 0, multi = 0, bad = 0, mb = 0;
#pragma unroll
  for (int i = 0; i < kFusedItems; ++i) {
    const uint32_t c = c0 + i;
    lv[i] = 0;
    if (c < n) {
      const ngpu_chunk ch = chunks[c];
      const uint32_t len = ch.length;
      const bool bd = ch.offset > data_len || len > data_len - ch.offset;
      lv[i] = len == 0 ? 1 : (len + kLeaf - 1) / kLeaf;
      if (bd) mb |= 1u << i;  // a bad chunk keeps its leaf numbers but is never hashed
      multi += lv[i] > 1 && !bd;
      bad += bd;
    }
    sum += lv[i];
  }
  // three block scans in one pass (leaves; multi-leaf chunks; bad descriptors)
  uint32_t xs = sum, xm = multi, xb = bad;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t ys = __shfl_up(xs, o, 64), ym = __shfl_up(xm, o, 64), yb = __shfl_up(xb, o, 64);
    if (lane >= o) xs += ys, xm += ym, xb += yb;
  }
  if (lane == 63) wsum[0][wid] = xs, wsum[1][wid] = xm, wsum[2][wid] = xb;
  __syncthreads();
  uint32_t ps = 0, pm = 0, ts = 0, tm = 0, tb = 0;
#pragma unroll
  for (int w = 0; w < kQuadThreads / 64; ++w) {
    if (w < wid) ps += wsum[0][w], pm += wsum[1][w];
    ts += wsum[0][w];
    tm += wsum[1][w];
    tb += wsum[2][w];
  }
  uint32_t run = ps + xs - sum, mrun = pm + xm - multi;
  const bool writer = blockIdx.x == 0;
#pragma unroll
  for (int i = 0; i < kFusedItems; ++i) {
    const uint32_t c = c0 + i;
    if (c < n) {
      gpre[c] = run;
      if (writer) {
        groups[c] = run;
        if (lv[i] > 1 && !((mb >> i) & 1)) tree_list[mrun++] = c;
      }
    }
    run += lv[i];
  }
  if (t == 0) {
    gpre[n] = ts;
    if (writer) groups[n] = ts;
  }
  // stats[8]: more leaves than the launch covers -- descriptors that overlap
  // (a tar's file extents never do); the call then fails instead of leaving
  // leaves unhashed
  const uint64_t span = (uint64_t)gridDim.x * (kQuadThreads / 4);
  const uint64_t over = ts > span || ts > cap_g ? ts : 0;
  if (writer && t < 16)
    stats[t] = t == kStBadDesc ? tb : t == kStTreeQueued ? tm : t == kStOverlap ? over : 0;
  if (writer && t == 0 && tb)
    atomicAdd((unsigned long long *)(stats + kStSticky), (unsigned long long)tb);
  if (writer && t == 0 && over)
    atomicMax((unsigned long long *)(stats + kStSticky + 1), (unsigned long long)over);
  __syncthreads();
  const uint32_t q = t & 3, quad = t >> 2;
  const uint64_t g = blockIdx.x * (uint64_t)(kQuadThreads / 4) + quad;
  if (g >= ts || g >= cap_g) return;  // per quad: its four lanes leave together
  // the chunk holding leaf g: the last c with gpre[c] <= g
  uint32_t lo = 0, hi = (uint32_t)n;  // gpre[lo] <= g < gpre[hi]
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (gpre[mid] <= g) lo = mid;
    else hi = mid;
  }
  const uint32_t c = lo, j = (uint32_t)(g - gpre[c]);
  const ngpu_chunk ch = chunks[c];
  if (ch.offset > data_len || ch.length > data_len - ch.offset) return;  // counted above
  quad_leaf(data, ch, c, j, gpre[c + 1] - gpre[c] == 1, g, q, qmsg + quad * 16, cv_out, out);
}

// Slots b3_quad_planned may need.
uint64_t quad_planned_slots(uint64_t n, uint64_t data_len) { return data_len / kLeaf + 2 * n + 1; }
#endif

// 1024 threads = 256 quads: every level of a 1024-CV tile (<= 512 parents)
// runs as compress_quad in at most two passes.  A chain of ~10 levels is the
// kernel's whole time on small layers (a 1 MiB chunk = 1024 leaves): with 256
// threads the two widest levels ran one 680-op compression per lane (2 and 1
// per lane), ~6.8 K issued ops against 2 x 190 here (C1 tree 18.8 -> see
// DESIGN.md §b3_quad_leaves).
//
// Round 6: b3_quad_planned leaves b3_tree at most 512 group CVs per chunk
// (chunk_size <= 2 MiB), most chunks only a few.  For a layer of many chunks
// a 256-thread workgroup with a 512-CV tile (32 KiB of LDS) does: four of
// them fit a CU where one 1024-thread workgroup did, so its many small trees
// run four times as wide (a 30 MB layer of log-normal files: tree 21 -> 11
// us), for one more pass on the widest level of a 1 MiB chunk.
constexpr int kTreeThreads = 1024;
constexpr int kTile = 1024;  // CVs per LDS tile (32 KiB)
#ifndef B3_TREE_NARROW
#define B3_TREE_NARROW 1
#endif
constexpr int kTreeThreadsNarrow = 256;
constexpr uint64_t kTreeNarrowMinChunks = 512;
constexpr int kTileNarrow = 512;

// all_queued: every multi-group chunk was queued (b3_quad_leaves), none was
// finished inside a b3_groups workgroup.
template <int TT, int TILE>
__global__ __launch_bounds__(TT) void b3_tree(
    const uint64_t *__restrict__ gbase, const uint32_t *__restrict__ tree_list,
    const uint64_t *__restrict__ queued, uint64_t cap_g,
    uint32_t *__restrict__ cv, ngpu_result *__restrict__ out, bool all_queued) {
  // two tiles, ping-pong: a level reads one and writes the other, so it needs
  // one barrier (the chain of ~10 narrow levels is the kernel's time on a
  // small layer; with one tile each level read, barriered, wrote, barriered)
  constexpr uint32_t kQ = TT / 4;                         // quads
  constexpr int kPasses = (int)((TILE / 2 + kQ - 1) / kQ);  // quad passes per level
  __shared__ uint32_t tt[2][TILE * 8];
  const int tid = threadIdx.x;
  // a quad of lanes per parent: this lane's column and schedule word offsets
  // in a parent's 16-word message (the two child CVs, adjacent in t)
  const uint32_t qlane = tid & 3, qid = tid >> 2;
  uint32_t wo[28];
#pragma unroll
  for (int r = 0; r < 7; ++r)
#pragma unroll
    for (int sl = 0; sl < 4; ++sl) wo[4 * r + sl] = (kQuadSched.w[r][sl] >> (4 * qlane)) & 15u;
  const uint32_t ivq = qlane == 0 ? IV0 : qlane == 1 ? IV1 : qlane == 2 ? IV2 : IV3;
  const uint32_t ivh = qlane == 0 ? IV4 : qlane == 1 ? IV5 : qlane == 2 ? IV6 : IV7;
  const uint64_t nq = *queued;  // 0: every chunk was finished inside b3_groups
  for (uint64_t qi = blockIdx.x; qi < nq; qi += gridDim.x) {
    const uint32_t c = tree_list[qi];
    const uint64_t base = gbase[c];
    uint64_t k = gbase[c + 1] - base;
    if (k <= 1 || base + k > cap_g || (!all_queued && tree_in_workgroup(base, k))) continue;
    uint32_t *a = cv + base * 8;
    for (;;) {
      const bool final_pass = k <= TILE;
      const uint64_t ntiles = (k + TILE - 1) / TILE;
      for (uint64_t tile = 0; tile < ntiles; ++tile) {
        uint32_t cnt = (uint32_t)min<uint64_t>(TILE, k - tile * TILE);
        const uint32_t *src = a + tile * TILE * 8;
        for (uint32_t w = tid; w < cnt * 8; w += TT) tt[0][w] = src[w];
        __syncthreads();
        int cur = 0;
        while (cnt > 1) {
          const uint32_t *t = tt[cur];
          uint32_t *o = tt[cur ^ 1];
          const uint32_t p = cnt >> 1;
          const uint32_t pflags = PARENT | ((final_pass && cnt == 2) ? ROOT : 0);
          const uint32_t dq = qlane == 2 ? 64u : qlane == 3 ? pflags : 0u;
#pragma unroll
          for (int s = 0; s < kPasses; ++s) {
            const uint32_t pi = qid + s * kQ;
            if (pi < p) {
              uint32_t m[28];
#pragma unroll
              for (int k2 = 0; k2 < 28; ++k2) m[k2] = t[16 * pi + wo[k2]];
              uint32_t rx = ivq, ry = ivh;
              compress_quad(rx, ry, m, ivq, dq);
              o[8 * pi + qlane] = rx;
              o[8 * pi + 4 + qlane] = ry;
            }
          }
          if ((cnt & 1) && tid < 8) o[8 * p + tid] = t[8 * (cnt - 1) + tid];  // odd tail promoted
          __syncthreads();
          cur ^= 1;
          cnt = p + (cnt & 1);
        }
        if (tid < 8) {
          if (final_pass)
            reinterpret_cast<uint32_t *>(out[c].digest)[tid] = tt[cur][tid];
          else
            a[tile * 8 + tid] = tt[cur][tid];
        } else if (tid == 8 && final_pass) {
          out[c].kind = NGPU_DIGESTED;  // (tt is read-only here: same wave as the digest)
        }
        __syncthreads();
      }
      if (final_pass) break;
      k = ntiles;
      __threadfence_block();
    }
  }
}

}  // namespace

// Groups this call can have: its own bound, not the workspace's capacity (a
// workspace sized for a 64 MiB staging slot would otherwise launch ~6x the
// workgroups a 10 MB layer needs -- and every b3_quad_planned workgroup scans
// all descriptors before it finds it has no leaf: 22 -> 67 us per C1 Pack).
static uint64_t call_groups(uint64_t n, uint64_t data_len, int D, const Workspace &ws) {
  const uint64_t g = blake3_max_groups(n, data_len, D);
  return g < ws.cap_g ? g : ws.cap_g;
}

template <int D, int LM>
static void launch_groups_lm(const uint8_t *data, uint64_t data_len,
                             const ngpu_chunk *chunks, uint64_t n, Workspace &ws,
                             ngpu_result *out, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
  const uint64_t blocks = (call_groups(n, data_len, D, ws) + 255) / 256;
  hipExtLaunchKernelGGL((b3_groups<D, LM>), dim3((unsigned)blocks), dim3(256), 0, s, e0, e1, 0,
                        data, data_len, chunks, n, (const uint64_t *)ws.groups,
                        (const uint32_t *)ws.group_chunk, ws.cap_g, ws.cv, out, ws.stats + 7,
                        (const uint32_t *)ws.small, (const uint64_t *)(ws.stats + 10),
                        ws.tree_list);
}

#ifndef NGPU_DIAG_NOLOAD
#define NGPU_DIAG_NOLOAD 0
#endif

// false: a load mode this build has no kernel for (nothing launched).
template <int D>
static bool launch_groups(const uint8_t *data, uint64_t data_len,
                          const ngpu_chunk *chunks, uint64_t n, Workspace &ws,
                          ngpu_result *out, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
  switch (ws.load_mode) {
    case 0: launch_groups_lm<D, 0>(data, data_len, chunks, n, ws, out, s, e0, e1); return true;
    case 1: launch_groups_lm<D, 1>(data, data_len, chunks, n, ws, out, s, e0, e1); return true;
    case 2: launch_groups_lm<D, 2>(data, data_len, chunks, n, ws, out, s, e0, e1); return true;
    case 3: launch_groups_lm<D, 3>(data, data_len, chunks, n, ws, out, s, e0, e1); return true;
    case 5: launch_groups_lm<D, 5>(data, data_len, chunks, n, ws, out, s, e0, e1); return true;
#if NGPU_DIAG_NOLOAD
    case 4: launch_groups_lm<D, 4>(data, data_len, chunks, n, ws, out, s, e0, e1); return true;
#endif
    default: return false;
  }
}

bool blake3_load_mode_ok(int lm) {
  return lm == 0 || lm == 1 || lm == 2 || lm == 3 || lm == 5 || (NGPU_DIAG_NOLOAD && lm == 4);
}

uint64_t blake3_quad_max_leaves() { return kQuadMaxLeaves; }

bool blake3_planned_in_leaves(uint64_t n, uint64_t data_len, int D, const Workspace &ws) {
  return D == 0 && !ws.grid_stages && n <= kSmallPlanChunks &&
         data_len / kLeaf + n <= kQuadMaxLeaves;
}

// Upper bound on leaf groups for n chunks inside a buffer of data_len bytes.
uint64_t blake3_max_groups(uint64_t n, uint64_t data_len, int D) {
  return n + ((data_len / kLeaf + n) >> D) + 1;
}

bool launch_blake3(const uint8_t *data, const ngpu_chunk *chunks, uint64_t n,
                   uint64_t data_len, int D, Workspace &ws, ngpu_result *out,
                   hipStream_t s, hipEvent_t ev_first, hipEvent_t ev_start, hipEvent_t ev_end_groups,
                   hipEvent_t ev_end, uint64_t chunk_size) {
  if (n == 0) {
    (void)hipMemsetAsync(ws.stats, 0, 16 * sizeof(uint64_t), s);
    return false;
  }
  // small layers at one leaf per lane: a quad of lanes per compression instead
  const bool quad = D == 0 && !ws.grid_stages && data_len / kLeaf + n <= kQuadMaxLeaves;
  if (blake3_planned_in_leaves(n, data_len, D, ws)) {
    // planning inside the leaf kernel (b3_quad_planned): the digest starts
    // with the call's first kernel (ev_first; ev_start is left unrecorded,
    // ngpu_timing_at reads ev_first instead)
    (void)ev_start;
    const uint64_t blocks = (quad_planned_slots(n, data_len) + kQuadThreads / 4 - 1) / (kQuadThreads / 4);
    hipExtLaunchKernelGGL(b3_quad_planned, dim3((unsigned)blocks), dim3(kQuadThreads), 0, s,
                          ev_first, ev_end_groups, 0, data, data_len, chunks, n, ws.cap_g, ws.cv,
                          out, ws.groups, ws.stats, ws.tree_list);
  } else if (!ws.grid_stages && n <= kSmallPlanChunks) {
    // ev_start = END of planning: a start event of hipExtLaunchKernel is a
    // marker packet (~5-10 us on a small layer), a stop event binds to the kernel
    hipExtLaunchKernelGGL(b3_plan_small, dim3(1), dim3(kSmallPlanThreads), 0, s, ev_first, ev_start,
                          0, chunks, n, D, ws.groups, ws.small, ws.group_chunk, ws.cap_g, ws.stats);
  } else {
    // the call's device counters; histogram + cursors + plan ticket + this
    // call's tile words, one memset
    (void)hipMemsetAsync(ws.stats, 0, 16 * sizeof(uint64_t), s);
    const uint64_t nt = (n + kPlanTile - 1) / kPlanTile;
    uint32_t *hist = reinterpret_cast<uint32_t *>(ws.tstat), *cursor = hist + (kMaxKey + 1);
    uint64_t *ts = ws.tstat + kB3Ts;
    (void)hipMemsetAsync(ws.tstat, 0, (kB3Ts + 1 + nt) * sizeof(uint64_t), s);
    hipExtLaunchKernelGGL(b3_plan, dim3((unsigned)nt), dim3(kTileThreads), 0, s, ev_first, nullptr,
                          0, chunks, n, D, ws.groups, hist, ts);
    hipLaunchKernelGGL(b3_small_scatter, dim3((unsigned)nt), dim3(kTileThreads), 0, s, chunks, n,
                       D, (const uint32_t *)hist, cursor, ws.small, ws.stats + 10);
    // lanes per chunk: the groups a chunk of the average size has, 1..64
    const uint64_t per = data_len / (n * ((uint64_t)kLeaf << D)) + 1;
    uint32_t W = 1;
    while (W < 64 && W < per) W <<= 1;
    const uint64_t waves_needed = (n * W + 63) / 64;
    const uint64_t waves = waves_needed < 16384 ? waves_needed : 16384;
    const uint64_t blocks = (waves * 64 + 255) / 256;
    hipExtLaunchKernelGGL(b3_fill_group_chunk, dim3((unsigned)blocks), dim3(256), 0, s, nullptr,
                          ev_start, 0, (const uint64_t *)ws.groups, n, ws.group_chunk, ws.cap_g, W);
  }
  if (blake3_planned_in_leaves(n, data_len, D, ws)) {
    // (leaves done above)
  } else if (quad) {
    const uint64_t blocks = (call_groups(n, data_len, D, ws) + kQuadThreads / 4 - 1) / (kQuadThreads / 4);
    hipExtLaunchKernelGGL(b3_quad_leaves, dim3((unsigned)blocks), dim3(kQuadThreads), 0, s,
                          nullptr, ev_end_groups, 0, data, data_len, chunks, n,
                          (const uint64_t *)ws.groups, (const uint32_t *)ws.group_chunk, ws.cap_g,
                          ws.cv, out, ws.stats + 7, (const uint32_t *)ws.small,
                          (const uint64_t *)(ws.stats + 10), ws.tree_list);
  } else {
    bool ok;
    switch (D) {
      case 0: ok = launch_groups<0>(data, data_len, chunks, n, ws, out, s, nullptr, ev_end_groups); break;
      case 1: ok = launch_groups<1>(data, data_len, chunks, n, ws, out, s, nullptr, ev_end_groups); break;
      case 2: ok = launch_groups<2>(data, data_len, chunks, n, ws, out, s, nullptr, ev_end_groups); break;
      case 3: ok = launch_groups<3>(data, data_len, chunks, n, ws, out, s, nullptr, ev_end_groups); break;
      default: ok = launch_groups<4>(data, data_len, chunks, n, ws, out, s, nullptr, ev_end_groups); break;
    }
    if (!ok) return false;  // (ngpu_create validates the mode; never taken)
  }
  // group CVs of the planned path (at most chunk_size / 4 KiB per chunk) of a
  // layer of many chunks: many small trees, four workgroups per CU.  A layer
  // of few chunks keeps the wide workgroup: its longest tree's widest level
  // is one pass there, two here (C1 206 -> 203, l32m 628 -> 608 narrow;
  // log-normal 30 MB layers of ~2,500 chunks 298 -> 329 GB/s)
  if (B3_QUAD_GROUPS && B3_TREE_NARROW && n >= kTreeNarrowMinChunks &&
      blake3_planned_in_leaves(n, data_len, D, ws) && chunk_size &&
      chunk_size / (4 * kLeaf) <= (uint64_t)kTileNarrow) {
    const uint64_t blocks = n < 8192 ? n : 8192;
    hipExtLaunchKernelGGL((b3_tree<kTreeThreadsNarrow, kTileNarrow>), dim3((unsigned)blocks),
                          dim3(kTreeThreadsNarrow), 0, s, nullptr, ev_end, 0,
                          (const uint64_t *)ws.groups, (const uint32_t *)ws.tree_list,
                          (const uint64_t *)(ws.stats + 9), ws.cap_g, ws.cv, out, quad);
    return true;
  }
  const uint64_t blocks = n < 2048 ? n : 2048;
  hipExtLaunchKernelGGL((b3_tree<kTreeThreads, kTile>), dim3((unsigned)blocks), dim3(kTreeThreads), 0,
                        s, nullptr, ev_end, 0, (const uint64_t *)ws.groups,
                        (const uint32_t *)ws.tree_list, (const uint64_t *)(ws.stats + 9), ws.cap_g,
                        ws.cv, out, quad);
  return true;
}

}  // namespace ngpu
