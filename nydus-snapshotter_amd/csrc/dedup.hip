// dedup.hip — chunk-dict probe and intra-layer dedup decisions on gfx950.
//
// Restates, data-parallel, the stream-order semantics of
// [nydus v2.3.0] Node::deduplicate_chunk + HashChunkDict (external, VERIFY;
// SURVEY.md §8(a) a5/a6):
//   1. global dict (PackOption.ChunkDictPath, builder.go:122-124): hit iff
//      the digest is present and (dict usize == 0 || == chunk size); the dict
//      keeps the FIRST chunk-table entry per digest;
//   2. else the layered dict = earlier NEW chunks of this layer, same size
//      rule, first insertion kept;
//   3. else NEW with the next sequential index; v6 uncompressed offsets are
//      the running sum of 4 KiB-rounded sizes.
// Sequential "first occurrence" becomes an atomic MIN over chunk ids in an
// HBM hash table; sequential index assignment becomes an exclusive scan;
// blob-index allocation in first-hit order becomes a rank over first-hit
// positions.  Results are bit-identical to the sequential restatement
// (oracle/dedup_ref.c) for any schedule.
//
// Hash table: open addressing, linear probing over 8-byte slots
// {tag = digest word 2 : id}; bucket = (digest words 0,1) * golden ratio.
// Roofline: HBM-bound probes.
#include <stddef.h>
#include <stdlib.h>

#include <algorithm>

#include <hip/hip_ext.h>

#include "common.hpp"

namespace ngpu {
namespace {

template <int STRIDE>
__device__ __forceinline__ void load_digest(const uint8_t *keys, uint64_t id,
                                            uint32_t d[8]) {
  const uint4 *p = reinterpret_cast<const uint4 *>(keys + id * STRIDE);
  uint4 a = p[0], b = p[1];
  d[0] = a.x; d[1] = a.y; d[2] = a.z; d[3] = a.w;
  d[4] = b.x; d[5] = b.y; d[6] = b.z; d[7] = b.w;
}

template <int STRIDE>
__device__ __forceinline__ bool digest_eq(const uint8_t *keys, uint64_t id,
                                          const uint32_t d[8]) {
  uint32_t e[8];
  load_digest<STRIDE>(keys, id, e);
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) x |= e[i] ^ d[i];
  return x == 0;
}

// Insert id; for an existing identical digest keep the smallest id.
template <int STRIDE>
__device__ void ht_insert_min(uint64_t *table, uint64_t mask,
                              const uint8_t *keys, uint32_t id) {
  uint32_t d[8];
  load_digest<STRIDE>(keys, id, d);
  const uint32_t tag = digest_tag(d);
  const uint64_t mine = ((uint64_t)tag << 32) | id;
  for (uint64_t p = digest_bucket(d) & mask;; p = (p + 1) & mask) {
    uint64_t s = __hip_atomic_load(table + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (s == kEmpty) {
      const uint64_t old = atomicCAS((unsigned long long *)(table + p),
                                     (unsigned long long)kEmpty,
                                     (unsigned long long)mine);
      if (old == kEmpty) return;
      s = old;
    }
    if ((uint32_t)(s >> 32) == tag && digest_eq<STRIDE>(keys, (uint32_t)s, d)) {
      if ((uint32_t)s > id) atomicMin((unsigned long long *)(table + p), (unsigned long long)mine);
      return;
    }
  }
}

// Returns the stored (smallest) id for digest d, or kNone.
template <int STRIDE>
__device__ uint32_t ht_lookup(const uint64_t *table, uint64_t mask,
                              const uint8_t *keys, const uint32_t d[8]) {
  const uint32_t tag = digest_tag(d);
  for (uint64_t p = digest_bucket(d) & mask;; p = (p + 1) & mask) {
    const uint64_t s = table[p];
    if (s == kEmpty) return kNone;
    if ((uint32_t)(s >> 32) == tag && digest_eq<STRIDE>(keys, (uint32_t)s, d))
      return (uint32_t)s;
  }
}

__global__ void dict_insert(const DictRec *__restrict__ rec, uint64_t m,
                            uint64_t *__restrict__ table, uint64_t mask) {
  const uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (e < m)
    ht_insert_min<sizeof(DictRec)>(table, mask, reinterpret_cast<const uint8_t *>(rec), (uint32_t)e);
}

__device__ __forceinline__ uint32_t dict_lookup(const DictDevice &dict, const uint32_t d[8]) {
  return ht_lookup<sizeof(DictRec)>(dict.table, dict.mask,
                                    reinterpret_cast<const uint8_t *>(dict.rec), d);
}

// The hit record of local entry e (global id through gid for node shards).
__device__ __forceinline__ ngpu_dict_hit dict_hit_of(const DictDevice &dict, uint32_t e) {
  if (e == kNone) return ngpu_dict_hit{kNone, 0, 0, 0, 0};
  // the record's second half: the line the digest compare just brought in
  const uint4 f = reinterpret_cast<const uint4 *>(dict.rec + e)[2];  // usize, blob, index, gid
  const uint64_t uo = dict.rec[e].uoff;
  return ngpu_dict_hit{f.w, f.z, f.y, f.x, uo};
}

// Lookup + hit in one pass: at a tag match the whole 64-B record is read (its
// four loads issued together), compared, and the hit built from registers.
// dict_hit_of(dict_lookup()) re-read the record's second half after the
// probe loop, i.e. after the wave's LONGEST chain had finished; by then the
// line had often left the L2 (random lines turn the L2 over in a few us) and
// the re-read went to HBM: +0.35 line per probe at 30 % hits (1.94 -> 1.60;
// dict_probe_variant RV 2..4 took the probe apart, tools/probe_sweep.py).
__device__ __forceinline__ ngpu_dict_hit dict_find(const DictDevice &dict, const uint32_t d[8]) {
  const uint32_t tag = digest_tag(d);
  for (uint64_t p = digest_bucket(d) & dict.mask;; p = (p + 1) & dict.mask) {
    const uint64_t s = dict.table[p];
    if (s == kEmpty) break;
    if ((uint32_t)(s >> 32) != tag) continue;
    const uint32_t e = (uint32_t)s;
    const uint4 *r = reinterpret_cast<const uint4 *>(dict.rec + e);
    const uint4 a = r[0], b = r[1], f = r[2];
    const uint64_t uo = dict.rec[e].uoff;
    if (((a.x ^ d[0]) | (a.y ^ d[1]) | (a.z ^ d[2]) | (a.w ^ d[3]) | (b.x ^ d[4]) |
         (b.y ^ d[5]) | (b.z ^ d[6]) | (b.w ^ d[7])) == 0)
      return ngpu_dict_hit{f.w, f.z, f.y, f.x, uo};  // gid, index, blob, usize
  }
  return ngpu_dict_hit{kNone, 0, 0, 0, 0};
}

// Look n digests (byte stride `stride`) up in the dict.  The 24-B hits of a
// workgroup are staged in LDS and leave as lane-contiguous 16-B stores, so
// each store instruction writes whole 128-B lines: a lane's own 24-B record
// write covers no line in one instruction, and the L2 then read every hit
// line from HBM before merging (~0.19 of the probe's ~1.96 line requests;
// tools/probe_sweep.py).  256 threads per workgroup (launch_dict_probe).
__global__ __launch_bounds__(256) void dict_probe_records(const uint8_t *__restrict__ digests,
                                                          uint64_t stride, uint64_t n,
                                                          DictDevice dict,
                                                          ngpu_dict_hit *__restrict__ hits) {
  __shared__ uint4 stage[256 * sizeof(ngpu_dict_hit) / 16];
  const uint64_t q0 = blockIdx.x * 256ull;
  const uint64_t q = q0 + threadIdx.x;
  if (q < n) {
    ngpu_dict_hit h{kNone, 0, 0, 0, 0};
    if (dict.m) {
      const uint4 *p = reinterpret_cast<const uint4 *>(digests + q * stride);
      const uint4 a = p[0], b = p[1];
      const uint32_t d[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
      h = dict_find(dict, d);
    }
    reinterpret_cast<ngpu_dict_hit *>(stage)[threadIdx.x] = h;
  }
  __syncthreads();
  const uint64_t m = n - q0 < 256 ? n - q0 : 256;  // this workgroup's hits
  const uint32_t bytes = (uint32_t)m * (uint32_t)sizeof(ngpu_dict_hit);
  uint8_t *dst = reinterpret_cast<uint8_t *>(hits + q0);
  if ((reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
    for (uint32_t i = threadIdx.x; i < bytes / 16; i += 256)
      reinterpret_cast<uint4 *>(dst)[i] = stage[i];
    if ((bytes & 15) && threadIdx.x == 0)  // an odd count leaves one 8-B half
      reinterpret_cast<uint2 *>(dst + (bytes & ~15u))[0] =
          reinterpret_cast<const uint2 *>(stage)[(bytes & ~15u) / 8];
  } else {  // (hit arrays from hipMalloc / torch are 256-B aligned)
    for (uint32_t i = threadIdx.x; i < bytes / 8; i += 256)
      reinterpret_cast<uint2 *>(dst)[i] = reinterpret_cast<const uint2 *>(stage)[i];
  }
}

// Measured-losing A/B probes (dict_probe_multi, dict_probe_multi_lds,
// dict_probe_variant, dict_probe_coop; DESIGN.md §3 "dict probe") are built
// only with -DNGPU_PROBE_AB=1 (scripts/build_ab.sh), never into the product
// library; their launch knobs (NGPU_PROBE_VARIANT / NGPU_PROBE_COOP) exist
// only in such a build.
#ifndef NGPU_PROBE_AB
#define NGPU_PROBE_AB 0
#endif
#if NGPU_PROBE_AB
// K queries per thread, their probe chains stepped in lockstep: each step
// issues the K slot loads (and the K record loads of tag matches) together,
// so a wave has K independent random requests in flight where
// dict_probe_records has one.  Same decisions as dict_find (slots in chain
// order, first equal record, stop at an empty slot).  Hits staged as there.
template <int K>
__global__ __launch_bounds__(256) void dict_probe_multi(const uint8_t *__restrict__ digests,
                                                        uint64_t stride, uint64_t n,
                                                        DictDevice dict,
                                                        ngpu_dict_hit *__restrict__ hits) {
  __shared__ uint4 stage[K * 256 * sizeof(ngpu_dict_hit) / 16];
  const uint64_t q0 = blockIdx.x * (256ull * K);
  uint32_t d[K][8], tag[K];
  uint64_t pos[K];
  bool live[K];
  ngpu_dict_hit h[K];
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const uint64_t q = q0 + threadIdx.x + 256u * j;
    live[j] = q < n && dict.m;
    h[j] = ngpu_dict_hit{kNone, 0, 0, 0, 0};
    uint4 a = make_uint4(0, 0, 0, 0), b = a;
    if (live[j]) {
      const uint4 *p = reinterpret_cast<const uint4 *>(digests + q * stride);
      a = p[0];
      b = p[1];
    }
    d[j][0] = a.x; d[j][1] = a.y; d[j][2] = a.z; d[j][3] = a.w;
    d[j][4] = b.x; d[j][5] = b.y; d[j][6] = b.z; d[j][7] = b.w;
    tag[j] = digest_tag(d[j]);
    pos[j] = digest_bucket(d[j]) & dict.mask;
  }
  for (;;) {
    uint64_t sv[K];
#pragma unroll
    for (int j = 0; j < K; ++j) sv[j] = live[j] ? dict.table[pos[j]] : kEmpty;
    bool cand[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
      if (sv[j] == kEmpty) live[j] = false;
      cand[j] = live[j] && (uint32_t)(sv[j] >> 32) == tag[j];
    }
    uint4 ra[K], rb[K], rf[K];
    uint64_t ru[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
      if (cand[j]) {
        const uint4 *r = reinterpret_cast<const uint4 *>(dict.rec + (uint32_t)sv[j]);
        ra[j] = r[0];
        rb[j] = r[1];
        rf[j] = r[2];
        ru[j] = dict.rec[(uint32_t)sv[j]].uoff;
      }
    }
    bool any = false;
#pragma unroll
    for (int j = 0; j < K; ++j) {
      if (cand[j] && ((ra[j].x ^ d[j][0]) | (ra[j].y ^ d[j][1]) | (ra[j].z ^ d[j][2]) |
                      (ra[j].w ^ d[j][3]) | (rb[j].x ^ d[j][4]) | (rb[j].y ^ d[j][5]) |
                      (rb[j].z ^ d[j][6]) | (rb[j].w ^ d[j][7])) == 0) {
        h[j] = ngpu_dict_hit{rf[j].w, rf[j].z, rf[j].y, rf[j].x, ru[j]};
        live[j] = false;
      }
      if (live[j]) pos[j] = (pos[j] + 1) & dict.mask;
      any |= live[j];
    }
    if (!any) break;
  }
#pragma unroll
  for (int j = 0; j < K; ++j)
    if (q0 + threadIdx.x + 256u * j < n)
      reinterpret_cast<ngpu_dict_hit *>(stage)[threadIdx.x + 256u * j] = h[j];
  __syncthreads();
  const uint64_t m = n - q0 < 256ull * K ? n - q0 : 256ull * K;
  const uint32_t bytes = (uint32_t)m * (uint32_t)sizeof(ngpu_dict_hit);
  uint8_t *dst = reinterpret_cast<uint8_t *>(hits + q0);
  if ((reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
    for (uint32_t i = threadIdx.x; i < bytes / 16; i += 256)
      reinterpret_cast<uint4 *>(dst)[i] = stage[i];
    if ((bytes & 15) && threadIdx.x == 0)
      reinterpret_cast<uint2 *>(dst + (bytes & ~15u))[0] =
          reinterpret_cast<const uint2 *>(stage)[(bytes & ~15u) / 8];
  } else {
    for (uint32_t i = threadIdx.x; i < bytes / 8; i += 256)
      reinterpret_cast<uint2 *>(dst)[i] = reinterpret_cast<const uint2 *>(stage)[i];
  }
}

// dict_probe_multi with the queries kept in LDS instead of registers (the
// compare reads them back), so K = 2 fits 8 waves per SIMD without spills.
template <int K>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void
dict_probe_multi_lds(const uint8_t *__restrict__ digests, uint64_t stride, uint64_t n,
                     DictDevice dict, ngpu_dict_hit *__restrict__ hits) {
  __shared__ uint4 qs[K * 256 * 2];  // the queries, then (after a barrier) the staged hits
  uint4 *stage = qs;
  const uint64_t q0 = blockIdx.x * (256ull * K);
  uint32_t tag[K];
  uint64_t pos[K];
  bool live[K];
  ngpu_dict_hit h[K];
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const uint32_t t = threadIdx.x + 256u * j;
    const uint64_t q = q0 + t;
    live[j] = q < n && dict.m;
    h[j] = ngpu_dict_hit{kNone, 0, 0, 0, 0};
    uint4 a = make_uint4(0, 0, 0, 0), b = a;
    if (live[j]) {
      const uint4 *p = reinterpret_cast<const uint4 *>(digests + q * stride);
      a = p[0];
      b = p[1];
    }
    qs[2 * t] = a;
    qs[2 * t + 1] = b;
    const uint32_t d[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    tag[j] = digest_tag(d);
    pos[j] = digest_bucket(d) & dict.mask;
  }
  for (;;) {
    uint64_t sv[K];
#pragma unroll
    for (int j = 0; j < K; ++j) sv[j] = live[j] ? dict.table[pos[j]] : kEmpty;
    bool any = false;
#pragma unroll
    for (int j = 0; j < K; ++j) {
      if (sv[j] == kEmpty) live[j] = false;
      if (live[j] && (uint32_t)(sv[j] >> 32) == tag[j]) {
        const uint32_t e = (uint32_t)sv[j];
        const uint4 *r = reinterpret_cast<const uint4 *>(dict.rec + e);
        const uint4 ra = r[0], rb = r[1], rf = r[2];
        const uint64_t ru = dict.rec[e].uoff;
        const uint32_t t = threadIdx.x + 256u * j;
        const uint4 a = qs[2 * t], b = qs[2 * t + 1];
        if (((ra.x ^ a.x) | (ra.y ^ a.y) | (ra.z ^ a.z) | (ra.w ^ a.w) | (rb.x ^ b.x) |
             (rb.y ^ b.y) | (rb.z ^ b.z) | (rb.w ^ b.w)) == 0) {
          h[j] = ngpu_dict_hit{rf.w, rf.z, rf.y, rf.x, ru};
          live[j] = false;
        }
      }
      if (live[j]) pos[j] = (pos[j] + 1) & dict.mask;
      any |= live[j];
    }
    if (!any) break;
  }
  __syncthreads();  // every query compare of the workgroup is done with qs
#pragma unroll
  for (int j = 0; j < K; ++j)
    if (q0 + threadIdx.x + 256u * j < n)
      reinterpret_cast<ngpu_dict_hit *>(stage)[threadIdx.x + 256u * j] = h[j];
  __syncthreads();
  const uint64_t m = n - q0 < 256ull * K ? n - q0 : 256ull * K;
  const uint32_t bytes = (uint32_t)m * (uint32_t)sizeof(ngpu_dict_hit);
  uint8_t *dst = reinterpret_cast<uint8_t *>(hits + q0);
  if ((reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
    for (uint32_t i = threadIdx.x; i < bytes / 16; i += 256)
      reinterpret_cast<uint4 *>(dst)[i] = stage[i];
    if ((bytes & 15) && threadIdx.x == 0)
      reinterpret_cast<uint2 *>(dst + (bytes & ~15u))[0] =
          reinterpret_cast<const uint2 *>(stage)[(bytes & ~15u) / 8];
  } else {
    for (uint32_t i = threadIdx.x; i < bytes / 8; i += 256)
      reinterpret_cast<uint2 *>(dst)[i] = reinterpret_cast<const uint2 *>(stage)[i];
  }
}

// A/B variants of the same probe (NGPU_PROBE_VARIANT, read per call; bench /
// tools/probe_sweep.py): where do the line requests beyond query + slot +
// record come from?  QV: the workgroup's queries (stride 32) are read into
// LDS with lane-contiguous 16-B loads -- one instruction per line -- instead
// of two 16-B loads per lane, each touching every query line of the wave.
// RV: a tag-matched record is read and compared 16 B at a time (the second
// half only if the first matched) instead of two loads issued together.
// RV 2..4 take the probe apart (their decisions are NOT the dict's: request
// counting only, never parity): 2 trusts the tag (no compare, the hit record
// still read), 3 trusts the tag and reads no record, 4 reads only the home
// slot (no chain, no record).
template <int QV, int RV>
__global__ __launch_bounds__(256) void dict_probe_variant(const uint8_t *__restrict__ digests,
                                                          uint64_t stride, uint64_t n,
                                                          DictDevice dict,
                                                          ngpu_dict_hit *__restrict__ hits) {
  __shared__ uint4 qs[QV ? 512 : 1];
  const uint64_t q0 = blockIdx.x * 256ull;
  const uint64_t q = q0 + threadIdx.x;
  uint32_t d[8] = {};
  if (QV && stride == 32) {
    const uint64_t m = n - q0 < 256 ? n - q0 : 256;
    const uint4 *src = reinterpret_cast<const uint4 *>(digests + q0 * 32);
    for (uint32_t i = threadIdx.x; i < 2 * m; i += 256) qs[i] = src[i];
    __syncthreads();
    if (q < n) {
      const uint4 a = qs[2 * threadIdx.x], b = qs[2 * threadIdx.x + 1];
      d[0] = a.x; d[1] = a.y; d[2] = a.z; d[3] = a.w; d[4] = b.x; d[5] = b.y; d[6] = b.z; d[7] = b.w;
    }
  } else if (q < n) {
    const uint4 *p = reinterpret_cast<const uint4 *>(digests + q * stride);
    const uint4 a = p[0], b = p[1];
    d[0] = a.x; d[1] = a.y; d[2] = a.z; d[3] = a.w; d[4] = b.x; d[5] = b.y; d[6] = b.z; d[7] = b.w;
  }
  if (q >= n) return;
  uint32_t e = kNone;
  if (dict.m) {
    const uint32_t tag = digest_tag(d);
    for (uint64_t pos = digest_bucket(d) & dict.mask;; pos = (pos + 1) & dict.mask) {
      const uint64_t sv = dict.table[pos];
      if (RV == 4) {
        if (sv != kEmpty && (uint32_t)(sv >> 32) == tag) e = (uint32_t)sv;
        break;
      }
      if (sv == kEmpty) break;
      if ((uint32_t)(sv >> 32) != tag) continue;
      if (RV == 2 || RV == 3) {
        e = (uint32_t)sv;
        break;
      }
      const uint4 *r = reinterpret_cast<const uint4 *>(dict.rec + (uint32_t)sv);
      bool eq;
      if (RV == 1) {
        const uint4 a = r[0];
        eq = ((a.x ^ d[0]) | (a.y ^ d[1]) | (a.z ^ d[2]) | (a.w ^ d[3])) == 0;
        if (eq) {
          const uint4 b = r[1];
          eq = ((b.x ^ d[4]) | (b.y ^ d[5]) | (b.z ^ d[6]) | (b.w ^ d[7])) == 0;
        }
      } else {
        const uint4 a = r[0], b = r[1];
        eq = ((a.x ^ d[0]) | (a.y ^ d[1]) | (a.z ^ d[2]) | (a.w ^ d[3]) | (b.x ^ d[4]) |
              (b.y ^ d[5]) | (b.z ^ d[6]) | (b.w ^ d[7])) == 0;
      }
      if (eq) {
        e = (uint32_t)sv;
        break;
      }
    }
  }
  if (RV >= 3)
    hits[q] = ngpu_dict_hit{e, 0, 0, 0, 0};
  else
    hits[q] = dict_hit_of(dict, e);
}

// The wavefront-cooperative form of the same lookup (the north star's
// "chunk-dict hash table ... probed with wavefront-cooperative open
// addressing"; A/B against dict_probe_records, NGPU_PROBE_COOP=1): 16 lanes
// per query read 16 consecutive slots from the query's bucket in one
// coalesced access, ballot for the first empty slot and the tag matches
// before it, and verify those in probe order -- the decisions of sequential
// linear probing, with the slot reads of a probe run side by side instead of
// one dependent load per slot.
__global__ __launch_bounds__(256) void dict_probe_coop(const uint8_t *__restrict__ digests,
                                                       uint64_t stride, uint64_t n,
                                                       DictDevice dict,
                                                       ngpu_dict_hit *__restrict__ hits) {
  const uint64_t q = (blockIdx.x * 256ull + threadIdx.x) >> 4;
  const uint32_t sub = threadIdx.x & 15, grp = (threadIdx.x & 63) >> 4;
  const bool live = q < n;
  uint32_t e = kNone;
  if (live && dict.m) {
    const uint4 *p = reinterpret_cast<const uint4 *>(digests + q * stride);
    const uint4 a = p[0], b = p[1];
    const uint32_t d[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    const uint32_t tag = digest_tag(d);
    uint64_t pos = digest_bucket(d) & dict.mask;
    for (;;) {
      const uint64_t sv = dict.table[(pos + sub) & dict.mask];
      const bool empty = sv == kEmpty, match = !empty && (uint32_t)(sv >> 32) == tag;
      // this group's 16 bits of the wave's ballots (a wave holds 4 groups;
      // groups of one wave may run different numbers of rounds)
      const uint32_t me = (uint32_t)(__ballot(empty) >> (16 * grp)) & 0xFFFFu;
      uint32_t mm = (uint32_t)(__ballot(match) >> (16 * grp)) & 0xFFFFu;
      const uint32_t fe = me ? (uint32_t)__builtin_ctz(me) : 16u;
      mm &= (1u << fe) - 1u;
      bool found = false;
      while (mm) {
        const uint32_t i = (uint32_t)__builtin_ctz(mm);
        const uint32_t id = (uint32_t)__shfl(sv, (int)(16 * grp + i), 64);
        if (digest_eq<sizeof(DictRec)>(reinterpret_cast<const uint8_t *>(dict.rec), id, d)) {
          e = id;
          found = true;
          break;
        }
        mm &= mm - 1;
      }
      if (found || fe < 16) break;
      pos += 16;
    }
  }
  if (live && sub == 0) hits[q] = dict_hit_of(dict, e);
}

#endif  // NGPU_PROBE_AB

// RAFS v6 chunk-info records (80 B: block_id[32], blob_index, flags,
// compressed_size, uncompressed_size, compressed_offset, uncompressed_offset,
// file_offset, index, reserved) -> dict records.  One thread per record.
__global__ void dict_unpack(const uint8_t *__restrict__ recs, uint64_t n,
                            const uint32_t *__restrict__ gids, uint32_t gid0,
                            DictRec *__restrict__ out) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint4 *r = reinterpret_cast<const uint4 *>(recs + 80 * i);
  const uint4 a = r[0], b = r[1], c = r[2], d = r[3], f = r[4];
  uint4 *o = reinterpret_cast<uint4 *>(out + i);
  o[0] = a;
  o[1] = b;
  o[2] = make_uint4(c.w, c.x, f.z, gids ? gids[i] : gid0 + (uint32_t)i);
  o[3] = make_uint4(d.z, d.w, 0, 0);
}

__global__ void dict_pack(const uint8_t *__restrict__ digests, const uint32_t *__restrict__ usize,
                          const uint32_t *__restrict__ blob, const uint32_t *__restrict__ index,
                          const uint64_t *__restrict__ uoff, const uint32_t *__restrict__ gid,
                          uint64_t n, DictRec *__restrict__ out) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint4 *dg = reinterpret_cast<const uint4 *>(digests + 32 * i);
  uint4 *o = reinterpret_cast<uint4 *>(out + i);
  o[0] = dg[0];
  o[1] = dg[1];
  o[2] = make_uint4(usize[i], blob[i], index ? index[i] : 0, gid ? gid[i] : (uint32_t)i);
  const uint64_t u = uoff ? uoff[i] : 0;
  o[3] = make_uint4((uint32_t)u, (uint32_t)(u >> 32), 0, 0);
}

// ---- layered dedup -----------------------------------------------------------
// A call covers L >= 1 layers; layer l owns chunks [first[l], first[l+1]).
// Everything except the chunk dict restarts per layer: the layered
// (intra-build) dict, NEW indices, uncompressed offsets and blob order.  The
// intra table is shared by all layers of a call: its key is (layer, digest).

__device__ __forceinline__ uint64_t layer_bucket(const uint32_t *d, uint32_t layer) {
  return digest_bucket(d) + (uint64_t)layer * 0xC2B2AE3D27D4EB4Full;
}

// The unwritten-digest guard.  The digest stage stores kind = NGPU_DIGESTED
// next to every digest; a record that reaches dedup without the mark (a
// previous call's record, fresh memory) or with an all-zero digest (no
// BLAKE3 / SHA-256 output, p = 2^-256) was never written by this call's
// digest kernels.  Such a chunk must not take part in dedup: two of them with
// equal lengths would resolve INTRA to each other and one file's bytes would
// silently point at another's.  It is marked NGPU_UNHASHED instead, counted in
// unh[0] with ~(its id) max-ed into unh[1] (stats[kStUnhashed..]), and the
// call fails (NGPU_EDEVICE) when its stats are read.
__device__ __forceinline__ bool digest_unwritten(const ngpu_result &r, const uint32_t d[8]) {
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) x |= d[i];
  return r.kind != NGPU_DIGESTED || x == 0;
}

// unh: two counters, global (grid path) or LDS (one-workgroup paths).
__device__ __forceinline__ void mark_unhashed(ngpu_result &r, uint64_t c, uint64_t *unh) {
  r.kind = NGPU_UNHASHED;
  r.ref = c;
  r.index = kNone;
  r.blob_index = kNone;
  r.dict_blob = 0;
  r.uncompressed_offset = 0;
  atomicAdd((unsigned long long *)unh, 1ull);
  atomicMax((unsigned long long *)(unh + 1), (unsigned long long)~c);
}

// One-workgroup stages: publish the LDS counters into the call's stats words
// and their sticky twins (thread 0, after the last barrier).
__device__ __forceinline__ void publish_unhashed(uint64_t *stats, uint64_t cnt, uint64_t inv_first) {
  stats[kStUnhashed] = cnt;
  stats[kStUnhashedFirst] = inv_first;
  if (cnt) {
    atomicAdd((unsigned long long *)(stats + kStSticky + 2), (unsigned long long)cnt);
    atomicMax((unsigned long long *)(stats + kStSticky + 3), (unsigned long long)inv_first);
  }
}

// Stage 0 (one grid-stride launch instead of four memsets + a map kernel):
// reset the per-layer blob first-hit slots, the layer stats, the intra table
// and the scan tiles, and fill chunk -> layer (binary search in first[0..L]:
// the last layer whose first chunk <= c, so empty layers are skipped).
// single != nullptr: one layer; {0, n} is written there for the later stages.
struct DedupInit {
  const uint64_t *first;
  uint64_t L, n;
  uint64_t *single;
  uint32_t *chunk_layer, *blob_first;
  uint64_t nbf;
  uint64_t *st_words;
  uint64_t nst;
  uint64_t *intra, icap, *tiles, ntw;
  uint64_t *newidx, *uoff, *nbytes, *ndict;
  uint64_t total;
  uint64_t *stats;  // the call's stats words (the grid path's unhashed counters)
};

__device__ __forceinline__ void init_item(const DedupInit &a, uint64_t i) {
  const uint64_t *first = a.first;
  const uint64_t L = a.L, n = a.n, nbf = a.nbf, nst = a.nst, icap = a.icap, ntw = a.ntw;
  uint64_t *single = a.single;
  uint32_t *chunk_layer = a.chunk_layer, *blob_first = a.blob_first;
  uint64_t *st_words = a.st_words, *intra = a.intra, *tiles = a.tiles;
  uint64_t *newidx = a.newidx, *uoff = a.uoff, *nbytes = a.nbytes, *ndict = a.ndict;
  {
    if (i < nbf) blob_first[i] = kNone;
    if (i < nst) st_words[i] = 0;
    if (i < icap) intra[i] = kEmpty;
    if (i < ntw) tiles[i] = 0;
    if (i < n) {
      uint64_t lo = 0;
      if (!single) {
        uint64_t hi = L;  // invariant: first[lo] <= c < first[hi]
        while (hi - lo > 1) {
          const uint64_t mid = (lo + hi) >> 1;
          if (first[mid] <= i) lo = mid;
          else hi = mid;
        }
      }
      chunk_layer[i] = (uint32_t)lo;
    }
    if (i == 0) {  // the scans' totals for n == 0 (the last tile writes them otherwise)
      newidx[n] = 0;
      uoff[n] = 0;
      nbytes[n] = 0;
      ndict[n] = 0;
      if (single) { single[0] = 0; single[1] = n; }
      if (a.stats) a.stats[kStUnhashed] = a.stats[kStUnhashedFirst] = 0;
    }
  }
}

__global__ void dedup_init(DedupInit a) {
  const uint64_t stride = gridDim.x * (uint64_t)blockDim.x;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < a.total; i += stride)
    init_item(a, i);
}

// atomicMin(base[key], v) for the lanes with act set.  Lanes of a wave
// usually share one key (one layer, one dict blob): reduce in the wave and
// issue ONE atomic (per-lane atomics on one address serialise).  Every lane
// of the wave must call this.
__device__ __forceinline__ void wave_min_u32(uint32_t *base, bool act, uint64_t key, uint32_t v) {
  const uint64_t am = __ballot(act);
  if (!am) return;
  const uint64_t k0 = __shfl(key, __builtin_ctzll(am), 64);
  if (__all(!act || key == k0)) {
    uint32_t x = act ? v : kNone;
#pragma unroll
    for (int o = 32; o; o >>= 1) x = min(x, (uint32_t)__shfl_xor((int)x, o, 64));
    if ((threadIdx.x & 63) == 0) atomicMin(base + k0, x);
  } else if (act) {
    atomicMin(base + key, v);
  }
}

__device__ __forceinline__ bool same_key(const ngpu_result *out, const uint32_t *chunk_layer,
                                         uint32_t id, const uint32_t d[8], uint32_t layer) {
  return chunk_layer[id] == layer &&
         digest_eq<sizeof(ngpu_result)>(reinterpret_cast<const uint8_t *>(out), id, d);
}

// Stage 1: dict decision (from given hits, or by probing the local dict);
// a chunk the dict does not take goes into the intra-layer table (CAS into an
// empty slot, or atomic MIN over the slot holding the same (layer, digest):
// the first occurrence wins for any schedule).
// Every lane of the wave must call this (wave_min_u32); c >= n: no chunk.
// unh: the unhashed-chunk counters (digest_unwritten).
__device__ __forceinline__ void probe_insert_item(
    uint64_t c, const ngpu_chunk *__restrict__ chunks, uint64_t n, const DictDevice &dict,
    const ngpu_dict_hit *__restrict__ hits, const uint32_t *__restrict__ chunk_layer,
    ngpu_result *__restrict__ out, uint32_t *__restrict__ blob_first, uint32_t n_blobs,
    uint64_t *__restrict__ table, uint64_t mask, uint64_t *unh) {
  bool live = c < n;
  uint32_t d[8] = {};
  uint32_t layer = 0;
  ngpu_dict_hit h{kNone, 0, 0, 0, 0};
  if (live) {
    load_digest<sizeof(ngpu_result)>(reinterpret_cast<const uint8_t *>(out), c, d);
    if (digest_unwritten(out[c], d)) {
      mark_unhashed(out[c], c, unh);
      live = false;
    }
  }
  if (live) {
    layer = chunk_layer[c];
    if (hits) {
      h = hits[c];
    } else if (dict.m) {
      h = dict_find(dict, d);
    }
  }
  const bool is_dict = live && h.entry != kNone &&
                       (h.usize == 0 || h.usize == chunks[c].length) && h.blob < n_blobs;
  wave_min_u32(blob_first, is_dict, (uint64_t)layer * (n_blobs + 1) + h.blob, (uint32_t)c);
  if (!live) return;
  ngpu_result &r = out[c];
  if (is_dict) {
    r.kind = NGPU_DICT;
    r.ref = h.entry;
    r.index = h.index;
    r.blob_index = h.blob;  // inner index; remapped in finalize
    r.uncompressed_offset = h.uncompressed_offset;  // chunk.copy_from(cached_chunk)
    r.dict_blob = h.blob;
    return;
  }
  r.kind = NGPU_NEW;
  r.dict_blob = 0;
  const uint32_t tag = digest_tag(d);
  const uint32_t id = (uint32_t)c;
  const uint64_t mine = ((uint64_t)tag << 32) | id;
  for (uint64_t p = layer_bucket(d, layer) & mask;; p = (p + 1) & mask) {
    uint64_t s = __hip_atomic_load(table + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (s == kEmpty) {
      const uint64_t old = atomicCAS((unsigned long long *)(table + p),
                                     (unsigned long long)kEmpty, (unsigned long long)mine);
      if (old == kEmpty) return;
      s = old;
    }
    if ((uint32_t)(s >> 32) == tag && same_key(out, chunk_layer, (uint32_t)s, d, layer)) {
      if ((uint32_t)s > id) atomicMin((unsigned long long *)(table + p), (unsigned long long)mine);
      return;
    }
  }
}

__global__ void dedup_probe_insert(const ngpu_chunk *__restrict__ chunks, uint64_t n,
                                   DictDevice dict, const ngpu_dict_hit *__restrict__ hits,
                                   const uint32_t *__restrict__ chunk_layer,
                                   ngpu_result *__restrict__ out,
                                   uint32_t *__restrict__ blob_first, uint32_t n_blobs,
                                   uint64_t *__restrict__ table, uint64_t mask,
                                   uint64_t *__restrict__ stats) {
  __shared__ unsigned long long s_unh[2];  // the workgroup's unhashed chunks, then one atomic
  if (threadIdx.x == 0) s_unh[0] = s_unh[1] = 0;
  __syncthreads();
  probe_insert_item(blockIdx.x * (uint64_t)blockDim.x + threadIdx.x, chunks, n, dict, hits,
                    chunk_layer, out, blob_first, n_blobs, table, mask,
                    reinterpret_cast<uint64_t *>(s_unh));
  __syncthreads();
  if (threadIdx.x == 0 && s_unh[0]) {
    atomicAdd((unsigned long long *)(stats + kStUnhashed), s_unh[0]);
    atomicMax((unsigned long long *)(stats + kStUnhashedFirst), s_unh[1]);
    atomicAdd((unsigned long long *)(stats + kStSticky + 2), s_unh[0]);
    atomicMax((unsigned long long *)(stats + kStSticky + 3), s_unh[1]);
  }
}

// Stage 2: INTRA / NEW per chunk.  Writes the four per-chunk quantities the
// scan turns into prefixes: NEW flag, v6-aligned size, NEW bytes, DICT flag.
// Per-layer figures are differences of these prefixes at layer boundaries,
// so no per-layer atomics are needed anywhere.
__device__ __forceinline__ void resolve_values(
    uint64_t c, const ngpu_chunk *__restrict__ chunks, const uint32_t *__restrict__ chunk_layer,
    const uint64_t *__restrict__ table, uint64_t mask, ngpu_result *__restrict__ out,
    uint32_t align, uint64_t v[kDedupScans]) {
  v[0] = v[1] = v[2] = v[3] = 0;  // NEW, aligned size, bytes, DICT
  ngpu_result &r = out[c];
  const uint32_t layer = chunk_layer[c];
  if (r.kind == NGPU_DICT) {
    v[3] = 1;
  } else if (r.kind == NGPU_UNHASHED) {
    // no digest: no decision, counted nowhere (the call fails)
  } else {
    uint32_t d[8];
    load_digest<sizeof(ngpu_result)>(reinterpret_cast<const uint8_t *>(out), c, d);
    const uint32_t tag = digest_tag(d);
    uint32_t f = kNone;
    for (uint64_t p = layer_bucket(d, layer) & mask;; p = (p + 1) & mask) {
      const uint64_t s = table[p];
      if (s == kEmpty) break;
      if ((uint32_t)(s >> 32) == tag && same_key(out, chunk_layer, (uint32_t)s, d, layer)) {
        f = (uint32_t)s;
        break;
      }
    }
    const uint32_t len = chunks[c].length;
    if (f != (uint32_t)c && f != kNone && chunks[f].length == len) {
      r.kind = NGPU_INTRA;
      r.ref = f;
    } else {
      r.kind = NGPU_NEW;
      r.ref = c;
      v[0] = 1;
      v[1] = ((uint64_t)len + align - 1) & ~(uint64_t)(align - 1);  // (align: 1 or 4096)
      v[2] = len;
    }
  }
}

__device__ __forceinline__ void resolve_item(
    uint64_t c, const ngpu_chunk *__restrict__ chunks, const uint32_t *__restrict__ chunk_layer,
    const uint64_t *__restrict__ table, uint64_t mask, ngpu_result *__restrict__ out,
    uint32_t align, uint64_t *__restrict__ newidx, uint64_t *__restrict__ uoff,
    uint64_t *__restrict__ nbytes, uint64_t *__restrict__ ndict) {
  uint64_t v[kDedupScans];
  resolve_values(c, chunks, chunk_layer, table, mask, out, align, v);
  newidx[c] = v[0];
  uoff[c] = v[1];
  nbytes[c] = v[2];
  ndict[c] = v[3];
}

__global__ void dedup_resolve(const ngpu_chunk *__restrict__ chunks, uint64_t n,
                              const uint32_t *__restrict__ chunk_layer,
                              const uint64_t *__restrict__ table, uint64_t mask,
                              ngpu_result *__restrict__ out, uint32_t align,
                              uint64_t *__restrict__ newidx, uint64_t *__restrict__ uoff,
                              uint64_t *__restrict__ nbytes, uint64_t *__restrict__ ndict) {
  const uint64_t c = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (c < n)
    resolve_item(c, chunks, chunk_layer, table, mask, out, align, newidx, uoff, nbytes, ndict);
}

// Stage 3: the four arrays -> exclusive prefixes over the whole call, in
// place, in one pass (decoupled look-back over tiles of 2048 chunks taken in
// dispatch order; one wave looks back per array).  Large tiles keep the
// tile tickets few: each is a device-scope atomic on one address.
constexpr int kScanItems = 8;
constexpr uint64_t kScanTile = kTileThreads * kScanItems;

__global__ __launch_bounds__(kTileThreads) void dedup_scan(
    uint64_t n, uint64_t *__restrict__ newidx, uint64_t *__restrict__ uoff,
    uint64_t *__restrict__ nbytes, uint64_t *__restrict__ ndict, uint64_t *__restrict__ ts,
    uint64_t nt) {
  __shared__ uint64_t sh_tile, sh_pre[kDedupScans];
  if (threadIdx.x == 0)
    sh_tile = __hip_atomic_fetch_add(ts, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const uint64_t tile = sh_tile;
  const uint64_t c0 = tile * kScanTile + threadIdx.x * kScanItems;
  uint64_t *arr[kDedupScans] = {newidx, uoff, nbytes, ndict};
  uint64_t v[kDedupScans][kScanItems], run[kDedupScans];
#pragma unroll
  for (int k = 0; k < kDedupScans; ++k) {
    uint64_t sum = 0;
#pragma unroll
    for (int i = 0; i < kScanItems; ++i) {
      v[k][i] = c0 + i < n ? arr[k][c0 + i] : 0;
      sum += v[k][i];
    }
    uint64_t tot;
    run[k] = block_exclusive_scan(sum, &tot);
    if (threadIdx.x == 0) sh_pre[k] = tot;  // tile aggregate, replaced by the prefix below
  }
  __syncthreads();
  static_assert(kTileThreads / 64 == kDedupScans, "one wave per array");
  const int w = threadIdx.x >> 6;
  const uint64_t pre = wave_lookback(ts + 1 + w * nt, tile, sh_pre[w]);
  if ((threadIdx.x & 63) == 0) sh_pre[w] = pre;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kDedupScans; ++k) {
    uint64_t x = run[k] + sh_pre[k];
#pragma unroll
    for (int i = 0; i < kScanItems; ++i) {
      const uint64_t c = c0 + i;
      if (c < n) arr[k][c] = x;
      x += v[k][i];
      if (c + 1 == n) arr[k][n] = x;
    }
  }
}

// Blob-table order per layer (one workgroup per layer): each dict blob gets a
// real index at its first hit, the layer's own blob at its first NEW chunk
// ([nydus v2.3.0] BlobManager alloc_index / get_or_create_current_blob).
// The first NEW chunk is found by binary search on the NEW-index scan (the
// smallest c in the layer with newidx[c + 1] > newidx[first]); the layer
// stats are differences of the scans at the layer's ends.
// One workgroup (any multiple of 64 threads) ranks layer l; fl: 1024 words
// of LDS, used_all: one LDS word.
__device__ void blob_rank_layer(uint64_t l, uint32_t *__restrict__ first_all, uint32_t nbo,
                                uint32_t *__restrict__ real_all,
                                const uint64_t *__restrict__ lfirst,
                                const uint64_t *__restrict__ newidx,
                                const uint64_t *__restrict__ uoff,
                                const uint64_t *__restrict__ nbytes,
                                const uint64_t *__restrict__ ndict,
                                ngpu_layer_stats *__restrict__ st, uint32_t *fl,
                                uint32_t *used_all_p) {
  uint32_t &used_all = *used_all_p;
  uint32_t *first = first_all + l * nbo;
  uint32_t *real = real_all + l * nbo;
  const uint64_t a = lfirst[l], e = lfirst[l + 1];
  if (threadIdx.x < 64) {  // 64-ary search by wave 0 (one L2 round trip per 64x)
    const int lane = threadIdx.x;
    uint32_t own = kNone;
    const uint64_t base_new = newidx[a];
    if (newidx[e] > base_new) {
      uint64_t lo = a, hi = e - 1;  // answer in [lo, hi]; pred(hi) holds
      while (lo < hi) {
        const uint64_t span = hi - lo + 1;
        const uint64_t step = (span + 63) / 64;
        const uint64_t p = lo + (uint64_t)lane * step;
        const bool pred = p <= hi && newidx[(p < hi ? p : hi) + 1] > base_new;
        const uint64_t m = __ballot(pred);  // monotone in lane; last lanes may be past hi
        const int k = m ? __builtin_ctzll(m) : 64;
        // k == 64: every probed position fails; x lies past the last one
        const uint64_t kl = k < 64 ? (uint64_t)k : (hi - lo) / step + 1;
        const uint64_t nhi = k < 64 ? lo + kl * step : hi;
        const uint64_t nlo = kl > 0 ? lo + (kl - 1) * step + 1 : lo;
        if (step == 1) { lo = hi = nhi; break; }
        lo = nlo;
        hi = nhi;
      }
      own = (uint32_t)lo;
    }
    if (lane == 0) first[nbo - 1] = own;
  }
  __syncthreads();
  const bool lds = nbo <= 1024;
  if (lds) {
    for (uint32_t b = threadIdx.x; b < nbo; b += blockDim.x) fl[b] = first[b];
    __syncthreads();
  }
  uint32_t used = 0;
  for (uint32_t b = threadIdx.x; b < nbo; b += blockDim.x) {
    const uint32_t fb = lds ? fl[b] : first[b];
    uint32_t rank = kNone;
    if (fb != kNone) {
      rank = 0;
      for (uint32_t o = 0; o < nbo; ++o) rank += (lds ? fl[o] : first[o]) < fb;
      ++used;
    }
    real[b] = rank;
  }
  if (threadIdx.x == 0) used_all = 0;
  __syncthreads();
  if (used) atomicAdd(&used_all, used);
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint64_t chunks = e - a, nw = newidx[e] - newidx[a], nd = ndict[e] - ndict[a];
    ngpu_layer_stats x{};
    x.chunks = chunks;
    x.new_chunks = nw;
    x.dict_chunks = nd;
    x.intra_chunks = chunks - nw - nd;
    x.new_bytes = nbytes[e] - nbytes[a];
    x.own_blob_index = real[nbo - 1];  // kNone -> 0xFFFFFFFF
    x.blobs = used_all;
    x.uncompressed_size = uoff[e] - uoff[a];
    st[l] = x;
  }
}

__global__ void blob_rank(uint32_t *__restrict__ first_all, uint32_t nbo,
                          uint32_t *__restrict__ real_all, const uint64_t *__restrict__ lfirst,
                          const uint64_t *__restrict__ newidx, const uint64_t *__restrict__ uoff,
                          const uint64_t *__restrict__ nbytes, const uint64_t *__restrict__ ndict,
                          ngpu_layer_stats *__restrict__ st) {
  __shared__ uint32_t fl[1024], used_all;
  blob_rank_layer(blockIdx.x, first_all, nbo, real_all, lfirst, newidx, uoff, nbytes, ndict, st,
                  fl, &used_all);
}

__device__ __forceinline__ void finalize_item(uint64_t c, const uint32_t *__restrict__ chunk_layer,
                                              const uint64_t *__restrict__ lfirst,
                                              const uint64_t *__restrict__ newidx,
                                              const uint64_t *__restrict__ uoff,
                                              const uint32_t *__restrict__ real_all, uint32_t nbo,
                                              ngpu_result *__restrict__ out) {
  ngpu_result &r = out[c];
  const uint32_t layer = chunk_layer[c];
  const uint32_t *real = real_all + (uint64_t)layer * nbo;
  const uint64_t a = lfirst[layer];
  const uint64_t ib = newidx[a], ob = uoff[a];
  const uint32_t own = real[nbo - 1];
  if (r.kind == NGPU_NEW) {
    r.index = (uint32_t)(newidx[c] - ib);
    r.uncompressed_offset = uoff[c] - ob;
    r.blob_index = own;
  } else if (r.kind == NGPU_INTRA) {
    const uint64_t f = r.ref;
    r.index = (uint32_t)(newidx[f] - ib);
    r.uncompressed_offset = uoff[f] - ob;
    r.blob_index = own;
  } else if (r.kind == NGPU_DICT) {
    r.blob_index = real[r.blob_index];
  }
}

__global__ void dedup_finalize(const uint64_t n, const uint32_t *__restrict__ chunk_layer,
                               const uint64_t *__restrict__ lfirst,
                               const uint64_t *__restrict__ newidx,
                               const uint64_t *__restrict__ uoff,
                               const uint32_t *__restrict__ real_all, uint32_t nbo,
                               ngpu_result *__restrict__ out) {
  const uint64_t c = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (c < n) finalize_item(c, chunk_layer, lfirst, newidx, uoff, real_all, nbo, out);
}

// ---- small calls: the whole dedup stage in ONE workgroup -----------------------
// A layer of a few thousand chunks (C1: 108) spends ~5 us per launch of the
// six stage kernels above on nothing but dispatch; here the stages run back
// to back inside one 1024-thread workgroup, with barriers between them and
// plain block scans instead of the tile look-back.  The per-chunk work is the
// same device code, so decisions are identical by construction (and by the
// parity tests, which force both paths).  Phases hand data over through
// global memory within ONE workgroup, so the barrier's workgroup-scope
// acquire/release is the whole synchronisation (all waves share the CU's
// vector L1; the hash-table atomics run at L2).  An agent-scope fence here
// would write back and invalidate the L2 at every phase (buffer_wbl2 /
// buffer_inv sc1): measured 29 us per call instead of ~10.
constexpr uint32_t kSmallThreads = 1024;
constexpr uint32_t kSmallItems = 4;

__device__ __forceinline__ void small_phase_end() { __syncthreads(); }

// lfirst and st are NOT __restrict__: for a single-layer call lfirst is
// a.single, and st is a.st_words, both written by the init phase of this same
// kernel.  (With __restrict__ the compiler may hoist the lfirst loads above
// the init writes: an empty layer then reported the previous call's chunk
// count -- tests/test_gpu_parity.py::test_host_reads_see_fresh_results_on_recycled_memory.)
__global__ __launch_bounds__(kSmallThreads) void dedup_small(
    DedupInit a, const ngpu_chunk *__restrict__ chunks, DictDevice dict,
    const ngpu_dict_hit *__restrict__ hits, uint32_t n_blobs, uint32_t align,
    const uint64_t *lfirst, uint32_t *__restrict__ blob_real, ngpu_layer_stats *st,
    ngpu_result *__restrict__ out) {
  __shared__ uint32_t fl[1024], used_all;
  __shared__ uint64_t wsum[2][kDedupScans][kSmallThreads / 64];
  __shared__ unsigned long long s_unh[2];
  const uint64_t n = a.n, mask = a.icap - 1;
  const uint32_t nbo = n_blobs + 1;
  if (threadIdx.x == 0) s_unh[0] = s_unh[1] = 0;
  for (uint64_t i = threadIdx.x; i < a.total; i += kSmallThreads) init_item(a, i);
  small_phase_end();
  const uint64_t n_up = (n + kSmallThreads - 1) / kSmallThreads * kSmallThreads;
  for (uint64_t c = threadIdx.x; c < n_up; c += kSmallThreads)  // whole waves: wave_min_u32
    probe_insert_item(c, chunks, n, dict, hits, a.chunk_layer, out, a.blob_first, n_blobs, a.intra,
                      mask, reinterpret_cast<uint64_t *>(s_unh));
  small_phase_end();
  // Resolve into registers and scan the four arrays together, one row of
  // kSmallThreads chunks at a time (chunk r * kSmallThreads + thread): one
  // barrier per row (C1: one), each array written once, where resolve wrote
  // the arrays and four separate scans re-read them.
  uint64_t *arr[kDedupScans] = {a.newidx, a.uoff, a.nbytes, a.ndict};
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint64_t carry[kDedupScans] = {0, 0, 0, 0};
  for (uint64_t r = 0; r * kSmallThreads < n; ++r) {
    const uint64_t c = r * kSmallThreads + threadIdx.x;
    uint64_t v[kDedupScans] = {0, 0, 0, 0}, x[kDedupScans];
    if (c < n) resolve_values(c, chunks, a.chunk_layer, a.intra, mask, out, align, v);
#pragma unroll
    for (int k = 0; k < kDedupScans; ++k) x[k] = v[k];
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
#pragma unroll
      for (int k = 0; k < kDedupScans; ++k) {
        const uint64_t y = __shfl_up(x[k], o, 64);
        if (lane >= o) x[k] += y;
      }
    }
    const uint32_t b = r & 1;  // double-buffered: one barrier per row
    if (lane == 63) {
#pragma unroll
      for (int k = 0; k < kDedupScans; ++k) wsum[b][k][wid] = x[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kDedupScans; ++k) {
      uint64_t pre = 0, tot = 0;
#pragma unroll 4
      for (int w = 0; w < (int)(kSmallThreads / 64); ++w) {
        const uint64_t t = wsum[b][k][w];
        if (w < wid) pre += t;
        tot += t;
      }
      const uint64_t run = carry[k] + pre + x[k] - v[k];
      if (c < n) arr[k][c] = run;
      if (c + 1 == n) arr[k][n] = run + v[k];
      carry[k] += tot;
    }
  }
  small_phase_end();
  for (uint64_t l = 0; l < a.L; ++l) {
    blob_rank_layer(l, a.blob_first, nbo, blob_real, lfirst, a.newidx, a.uoff, a.nbytes, a.ndict,
                    st, fl, &used_all);
    __syncthreads();  // fl / used_all reused by the next layer
  }
  small_phase_end();
  for (uint64_t c = threadIdx.x; c < n; c += kSmallThreads)
    finalize_item(c, a.chunk_layer, lfirst, a.newidx, a.uoff, blob_real, nbo, out);
  if (threadIdx.x == 0) publish_unhashed(a.stats, s_unh[0], s_unh[1]);
}

// ---- small single-layer calls: the whole stage in LDS --------------------------
// Every Pack and most device calls are one layer of at most a few thousand
// chunks (C1: 108).  dedup_small hands its phases over through global memory:
// each phase waits on several dependent L2 / HBM round trips (digest loads,
// device-scope table atomics, scan arrays, the 64-ary search), ~14 us for C1.
// Here the intra-layer table, the lengths, the NEW-index / offset prefixes
// and the blob ranks live in LDS; global memory is read once per chunk
// (descriptor, digest, dict hit) plus the rare full-digest compare of a tag
// match, and written once per chunk.  Same decisions by construction: the
// same first-occurrence table (LDS CAS / atomic MIN instead of device
// atomics), the same size rule, the same scans in chunk order, the same
// first-hit blob ranking.
constexpr uint32_t kLdsChunks = 4096;   // == kSmallDedupChunks
constexpr uint32_t kLdsSlots = 8192;    // next_pow2(2n) for n <= 4096
constexpr uint32_t kLdsBlobs = 1024;    // dict blobs + own
static_assert(kLdsChunks == kSmallDedupChunks, "one LDS slot per chunk");

// T threads: 1024, or 256 for a layer of at most 256 chunks (C1: 108), whose
// one row of chunks then spans 4 waves instead of 16 (cheaper barriers and
// cross-wave scans; same decisions).
template <uint32_t T>
__global__ __launch_bounds__(T) void dedup_small_lds(
    const ngpu_chunk *__restrict__ chunks, uint64_t n, DictDevice dict,
    const ngpu_dict_hit *__restrict__ hits, uint32_t n_blobs, uint32_t align,
    ngpu_layer_stats *__restrict__ st, ngpu_result *__restrict__ out,
    uint64_t *__restrict__ stats) {
  __shared__ uint64_t table[kLdsSlots];
  __shared__ uint64_t off[kLdsChunks];   // exclusive prefix of aligned NEW sizes
  __shared__ uint32_t len_s[kLdsChunks];
  __shared__ uint32_t nidx[kLdsChunks];  // exclusive prefix of NEW flags
  __shared__ uint32_t bf[kLdsBlobs], real[kLdsBlobs];
  __shared__ uint64_t wsum[2][4][T / 64];
  __shared__ uint32_t used_all;
  __shared__ unsigned long long s_unh[2];  // unhashed chunks: count, ~smallest id
  const uint32_t t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const uint32_t nbo = n_blobs + 1;
  uint32_t mask = 63;
  while (mask + 1 < 2 * n) mask = mask * 2 + 1;
  for (uint32_t i = t; i <= mask; i += T) table[i] = kEmpty;
  for (uint32_t i = t; i < nbo; i += T) bf[i] = kNone;
  if (t == 0) used_all = 0, s_unh[0] = s_unh[1] = 0;
  __syncthreads();
  // A: dict decisions (DICT results written now) and the intra-layer table.
  // Item k of thread t is chunk k * T + t (rows, for the scans).
  // Per chunk, for phase B: len_s = length | DICT flag (bit 31), off = the
  // digest's tag : bucket (overwritten by the chunk's offset prefix in B).
  constexpr uint32_t kDictBit = 0x80000000u;
  constexpr uint32_t kUnhashedBit = 0x20000000u;  // no digest (digest_unwritten)
  // a dict hit's blob, per item: the first hit of every blob is found after
  // the loop, one reduced atomic per wave and item row (wave_min_u32)
  constexpr int kRows = (int)(kLdsChunks / T);
  uint32_t hit_blob[kRows];
#pragma unroll
  for (int k = 0; k < kRows; ++k) hit_blob[k] = kNone;
#pragma unroll 1
  for (int k = 0; k < kRows; ++k) {
    const uint64_t c = (uint64_t)k * T + t;
    if (c >= n) break;
    uint32_t dg[8];
    load_digest<sizeof(ngpu_result)>(reinterpret_cast<const uint8_t *>(out), c, dg);
    if (digest_unwritten(out[c], dg)) {
      len_s[c] = kUnhashedBit;
      mark_unhashed(out[c], c, reinterpret_cast<uint64_t *>(s_unh));
      continue;
    }
    const uint32_t len = chunks[c].length;
    ngpu_dict_hit h{kNone, 0, 0, 0, 0};
    if (hits) h = hits[c];
    else if (dict.m) h = dict_find(dict, dg);
    ngpu_result &r = out[c];
    if (h.entry != kNone && (h.usize == 0 || h.usize == len) && h.blob < n_blobs) {
      len_s[c] = len | kDictBit;
      r.kind = NGPU_DICT;
      r.ref = h.entry;
      r.index = h.index;
      r.blob_index = h.blob;  // inner index; remapped below
      r.uncompressed_offset = h.uncompressed_offset;  // chunk.copy_from(cached_chunk)
      r.dict_blob = h.blob;
      hit_blob[k] = h.blob;
      continue;
    }
    len_s[c] = len;
    r.dict_blob = 0;
    const uint32_t tag = digest_tag(dg), bucket = (uint32_t)digest_bucket(dg);
    off[c] = ((uint64_t)tag << 32) | bucket;
    const uint64_t mine = ((uint64_t)tag << 32) | c;
    for (uint32_t p = bucket & mask;; p = (p + 1) & mask) {
      uint64_t sv = table[p];
      if (sv == kEmpty) {
        const uint64_t old = atomicCAS((unsigned long long *)&table[p], (unsigned long long)kEmpty,
                                       (unsigned long long)mine);
        if (old == kEmpty) break;
        sv = old;
      }
      if ((uint32_t)(sv >> 32) == tag &&
          digest_eq<sizeof(ngpu_result)>(reinterpret_cast<const uint8_t *>(out), (uint32_t)sv, dg)) {
        if ((uint32_t)sv > c) atomicMin((unsigned long long *)&table[p], (unsigned long long)mine);
        break;
      }
    }
  }
  // (every lane of the wave is here: the rows' minima reduce in the wave)
#pragma unroll
  for (int k = 0; k < kRows; ++k) {
    if ((uint64_t)k * T >= n) break;  // (uniform)
    wave_min_u32(bf, hit_blob[k] != kNone, hit_blob[k], (uint32_t)((uint64_t)k * T + t));
  }
  __syncthreads();
  // B: resolve INTRA / NEW and scan the four per-chunk quantities (NEW,
  // aligned size, bytes, DICT) in chunk order.  Here thread t takes the
  // CONTIGUOUS chunks [t R, t R + R): pass 1 resolves them and sums the four
  // values, ONE block scan of the threads' sums follows, and pass 2 writes
  // each chunk's prefix from its thread's.  (Rows of T chunks took a barrier,
  // a wave-sum round and 64 broadcast LDS reads per thread each: 17 of a
  // 30 us stage at ~2,800 chunks, profiles/r6/dedup_phases_r6ab.json.)
  // An INTRA chunk's len_s becomes kIntraBit | its first occurrence once
  // resolved: no other chunk reads it (a first occurrence is always the
  // smallest id of its digest, never an INTRA chunk).
  constexpr uint32_t kIntraBit = 0x40000000u;
  constexpr int W = (int)(T / 64);
  __shared__ uint32_t own_first;
  if (t == 0) own_first = kNone;
  const uint32_t R = (uint32_t)((n + T - 1) / T);
  const uint64_t c0 = (uint64_t)t * R;
  uint64_t sum[4] = {0, 0, 0, 0};
  // this chunk's four values, from its decision in len_s
  auto values = [&](uint32_t lv, uint64_t v[4]) {
    v[0] = v[1] = v[2] = v[3] = 0;
    if (lv & kDictBit) {
      v[3] = 1;
    } else if (!(lv & (kUnhashedBit | kIntraBit))) {  // NEW
      v[0] = 1;
      v[1] = ((uint64_t)lv + align - 1) & ~(uint64_t)(align - 1);  // (align: 1 or 4096)
      v[2] = lv;
    }
  };
#pragma unroll 1
  for (uint32_t j = 0; j < R; ++j) {
    const uint64_t c = c0 + j;
    if (c >= n) break;
    const uint32_t lv = len_s[c];
    if (!(lv & (kDictBit | kUnhashedBit))) {
      const uint64_t tb = off[c];
      const uint32_t tag = (uint32_t)(tb >> 32);
      uint32_t f = kNone;
      for (uint32_t p = (uint32_t)tb & mask;; p = (p + 1) & mask) {
        const uint64_t sv = table[p];
        if (sv == kEmpty) break;
        const uint32_t id = (uint32_t)sv;
        if ((uint32_t)(sv >> 32) != tag) continue;
        if (id == c) {
          f = id;
          break;
        }
        uint32_t dg[8];  // a tag match with another chunk: compare the digests
        load_digest<sizeof(ngpu_result)>(reinterpret_cast<const uint8_t *>(out), c, dg);
        if (digest_eq<sizeof(ngpu_result)>(reinterpret_cast<const uint8_t *>(out), id, dg)) {
          f = id;
          break;
        }
      }
      if (f != (uint32_t)c && f != kNone && (len_s[f] & ~kDictBit) == lv)
        len_s[c] = kIntraBit | f;  // INTRA
    }
    uint64_t v[4];
    values(len_s[c], v);
#pragma unroll
    for (int q = 0; q < 4; ++q) sum[q] += v[q];
  }
  // one block scan of the threads' sums: in the wave, then across the W waves
  uint64_t x[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) x[q] = sum[q];
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint64_t y = __shfl_up(x[q], o, 64);
      if (lane >= o) x[q] += y;
    }
  }
  if (lane == 63) {
#pragma unroll
    for (int q = 0; q < 4; ++q) wsum[0][q][wid] = x[q];
  }
  __syncthreads();
  uint64_t run[4], carry[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint64_t y = lane < (uint32_t)W ? wsum[0][q][lane] : 0;  // lane w: wave w's sum
#pragma unroll
    for (int o = 1; o < W; o <<= 1) {
      const uint64_t z = __shfl_up(y, o, 64);
      if (lane >= (uint32_t)o) y += z;
    }
    carry[q] = __shfl(y, W - 1, 64);                         // the layer's total
    const uint64_t wpre = __shfl(y, wid ? wid - 1 : 0, 64);  // waves before this one
    run[q] = (wid ? wpre : 0) + x[q] - sum[q];               // chunks before c0
  }
#pragma unroll 1
  for (uint32_t j = 0; j < R; ++j) {
    const uint64_t c = c0 + j;
    if (c >= n) break;
    uint64_t v[4];
    values(len_s[c], v);
    nidx[c] = (uint32_t)run[0];
    off[c] = run[1];
    // the layer's first NEW chunk: the one NEW chunk with none before it
    if (v[0] && run[0] == 0) own_first = (uint32_t)c;
#pragma unroll
    for (int q = 0; q < 4; ++q) run[q] += v[q];
  }
  __syncthreads();
  // C: blob order of the layer: dict blobs at their first hit, the own blob
  // at its first NEW chunk ([nydus v2.3.0] alloc_index / get_or_create_current_blob)
  if (t == 0) bf[nbo - 1] = own_first;
  __syncthreads();
  uint32_t used = 0;
  for (uint32_t b = t; b < nbo; b += T) {
    const uint32_t fb = bf[b];
    uint32_t rank = kNone;
    if (fb != kNone) {
      rank = 0;
      for (uint32_t o = 0; o < nbo; ++o) rank += bf[o] < fb;
      ++used;
    }
    real[b] = rank;
  }
  if (used) atomicAdd(&used_all, used);
  __syncthreads();
  // D: final per-chunk fields and the layer stats
  const uint32_t own = real[nbo - 1];
#pragma unroll 1
  for (int k = 0; k < (int)(kLdsChunks / T); ++k) {
    const uint64_t c = (uint64_t)k * T + t;
    if (c >= n) break;
    ngpu_result &r = out[c];
    const uint32_t lv = len_s[c];
    if (lv & kDictBit) {
      r.blob_index = real[r.dict_blob];
    } else if (lv & kUnhashedBit) {
      // marked in phase A
    } else if (lv & kIntraBit) {
      const uint32_t f = lv & ~kIntraBit;
      r.kind = NGPU_INTRA;
      r.ref = f;
      r.index = nidx[f];
      r.uncompressed_offset = off[f];
      r.blob_index = own;
    } else {
      r.kind = NGPU_NEW;
      r.ref = c;
      r.index = nidx[c];
      r.uncompressed_offset = off[c];
      r.blob_index = own;
    }
  }
  if (t == 0) {
    ngpu_layer_stats x{};
    x.chunks = n;
    x.new_chunks = carry[0];
    x.dict_chunks = carry[3];
    x.intra_chunks = n - carry[0] - carry[3];
    x.new_bytes = carry[2];
    x.own_blob_index = own;  // kNone -> 0xFFFFFFFF
    x.blobs = used_all;
    x.uncompressed_size = carry[1];
    st[0] = x;
    publish_unhashed(stats, s_unh[0], s_unh[1]);
  }
}

}  // namespace

void launch_dict_build(const DictRec *rec, uint64_t m, uint64_t *table, uint64_t cap,
                       hipStream_t s) {
  hipMemsetAsync(table, 0xFF, cap * sizeof(uint64_t), s);
  if (m == 0) return;
  const uint64_t blocks = (m + 255) / 256;
  hipLaunchKernelGGL(dict_insert, dim3((unsigned)blocks), dim3(256), 0, s, rec, m, table, cap - 1);
}

void launch_dict_probe(const uint8_t *digests, uint64_t stride, uint64_t n,
                       const DictDevice &dict, ngpu_dict_hit *hits, hipStream_t s) {
  if (n == 0) return;
  const dim3 g((unsigned)((n + 255) / 256));
#if NGPU_PROBE_AB
  // A/B knob, read per call (bench.py probe_roofline; 2.6x slower)
  const char *coop = getenv("NGPU_PROBE_COOP");
  if (coop && coop[0] == '1') {
    hipLaunchKernelGGL(dict_probe_coop, dim3((unsigned)((n * 16 + 255) / 256)), dim3(256), 0, s,
                       digests, stride, n, dict, hits);
    return;
  }
  const char *var = getenv("NGPU_PROBE_VARIANT");
  const int v = var ? atoi(var) : 0;
  switch (v) {
    case 1: hipLaunchKernelGGL((dict_probe_variant<1, 0>), g, dim3(256), 0, s, digests, stride, n, dict, hits); return;
    case 2: hipLaunchKernelGGL((dict_probe_variant<0, 1>), g, dim3(256), 0, s, digests, stride, n, dict, hits); return;
    case 3: hipLaunchKernelGGL((dict_probe_variant<1, 1>), g, dim3(256), 0, s, digests, stride, n, dict, hits); return;
    case 4: hipLaunchKernelGGL((dict_probe_variant<0, 0>), g, dim3(256), 0, s, digests, stride, n, dict, hits); return;
    case 5: hipLaunchKernelGGL((dict_probe_variant<0, 2>), g, dim3(256), 0, s, digests, stride, n, dict, hits); return;
    case 6: hipLaunchKernelGGL((dict_probe_variant<0, 3>), g, dim3(256), 0, s, digests, stride, n, dict, hits); return;
    case 7: hipLaunchKernelGGL((dict_probe_variant<0, 4>), g, dim3(256), 0, s, digests, stride, n, dict, hits); return;
    case 8: hipLaunchKernelGGL((dict_probe_multi<2>), dim3((unsigned)((n + 511) / 512)), dim3(256), 0, s, digests, stride, n, dict, hits); return;
    case 9: hipLaunchKernelGGL((dict_probe_multi<4>), dim3((unsigned)((n + 1023) / 1024)), dim3(256), 0, s, digests, stride, n, dict, hits); return;
    case 10: hipLaunchKernelGGL((dict_probe_multi_lds<2>), dim3((unsigned)((n + 511) / 512)), dim3(256), 0, s, digests, stride, n, dict, hits); return;
    case 11: hipLaunchKernelGGL((dict_probe_multi_lds<3>), dim3((unsigned)((n + 767) / 768)), dim3(256), 0, s, digests, stride, n, dict, hits); return;
    default: break;
  }
#endif
  hipLaunchKernelGGL(dict_probe_records, g, dim3(256), 0, s, digests, stride, n, dict, hits);
}

// ---- node dict exchange (node.hip) -------------------------------------------
namespace {

__device__ __forceinline__ uint32_t owner_of(uint32_t w0, uint32_t W) {
  const uint32_t hi = (w0 & 0xFF) << 8 | ((w0 >> 8) & 0xFF);  // digest bytes 0, 1
  return (uint32_t)(((uint64_t)hi * W) >> 16);
}

__global__ void pack_digests(const uint8_t *__restrict__ src, uint64_t stride, uint64_t n,
                             uint8_t *__restrict__ dst) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint4 *p = reinterpret_cast<const uint4 *>(src + i * stride);
  uint4 *o = reinterpret_cast<uint4 *>(dst + 32 * i);
  o[0] = p[0];
  o[1] = p[1];
}

__global__ void dict_probe_owned(const uint8_t *__restrict__ q, uint64_t n, uint32_t owner,
                                 uint32_t W, DictDevice dict, ngpu_dict_hit *__restrict__ hits) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint4 *p = reinterpret_cast<const uint4 *>(q + 32 * i);
  const uint4 a = p[0];
  if (owner_of(a.x, W) != owner) return;  // another part answers this one
  ngpu_dict_hit h{kNone, 0, 0, 0, 0};
  if (dict.m) {
    const uint4 b = p[1];
    const uint32_t d[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    h = dict_find(dict, d);
  }
  hits[i] = h;
}

__global__ void hits_merge(const uint8_t *__restrict__ q, uint64_t n, uint32_t W,
                           const ngpu_dict_hit *__restrict__ parts,
                           ngpu_dict_hit *__restrict__ hits) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t w0 = reinterpret_cast<const uint32_t *>(q + 32 * i)[0];
  hits[i] = parts[(uint64_t)owner_of(w0, W) * n + i];
}

// ---- digest routing: each digest to its owner only ------
// route_count: per-owner row counts (LDS histogram per workgroup, one global
// atomic per (workgroup, owner)).  route_scatter: each row's 32-B digest and
// its row id to its owner's segment.  Compact layout (seg_cap = 0): owners
// back to back in owner order, owner o at sum(cnt[0..o)).  Padded layout
// (seg_cap > 0, dist.py's equal splits): row of rank k within owner o goes to
// round k / seg_cap, slot [round][o][k % seg_cap].  The order inside a
// segment is the atomics' order: hits return to rows by row id, never by
// position.  cnt[0..W) = counts, cnt[64..64+W) = scatter cursors.
__global__ __launch_bounds__(256) void route_count(const uint8_t *__restrict__ src, uint64_t stride,
                                                   uint64_t n, uint32_t W, uint32_t *__restrict__ cnt) {
  __shared__ uint32_t h[64];
  if (threadIdx.x < 64) h[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
  if (i < n) atomicAdd(&h[owner_of(*reinterpret_cast<const uint32_t *>(src + i * stride), W)], 1u);
  __syncthreads();
  if (threadIdx.x < W && h[threadIdx.x]) atomicAdd(&cnt[threadIdx.x], h[threadIdx.x]);
}

__global__ __launch_bounds__(256) void route_scatter(const uint8_t *__restrict__ src, uint64_t stride,
                                                     uint64_t n, uint32_t W, uint64_t seg_cap,
                                                     uint32_t *__restrict__ cnt,
                                                     uint8_t *__restrict__ out,
                                                     uint32_t *__restrict__ rows) {
  __shared__ uint32_t h[64], base[64];
  if (threadIdx.x < 64) h[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
  uint32_t o = 0, local = 0;
  uint4 a = {}, b = {};
  if (i < n) {
    const uint4 *p = reinterpret_cast<const uint4 *>(src + i * stride);
    a = p[0];
    b = p[1];
    o = owner_of(a.x, W);
    local = atomicAdd(&h[o], 1u);
  }
  __syncthreads();
  if (threadIdx.x < W) {
    const uint32_t t = threadIdx.x;
    uint32_t off = 0;
    if (!seg_cap)
      for (uint32_t k = 0; k < t; ++k) off += cnt[k];
    base[t] = off + (h[t] ? atomicAdd(&cnt[64 + t], h[t]) : 0u);
  }
  __syncthreads();
  if (i >= n) return;
  const uint64_t k = (uint64_t)base[o] + local;
  const uint64_t pos = seg_cap ? (k / seg_cap) * W * seg_cap + (uint64_t)o * seg_cap + k % seg_cap : k;
  uint4 *d = reinterpret_cast<uint4 *>(out + 32 * pos);
  d[0] = a;
  d[1] = b;
  rows[pos] = (uint32_t)i;
}

// An owner's probe of the rows routed to it (compact layout): reads its count
// and segment -- in the requester's HBM when the node spans GPUs (peer loads
// over xGMI) -- and writes each hit straight into the requester's hit array at
// the row's id (peer stores).  Every row has exactly one owner, so the W
// owners together write each hit once and no merge step follows.
__global__ __launch_bounds__(256) void dict_probe_routed(const uint8_t *__restrict__ q,
                                                         const uint32_t *__restrict__ rows,
                                                         const uint32_t *__restrict__ cnt,
                                                         uint32_t owner, DictDevice dict,
                                                         ngpu_dict_hit *__restrict__ hits) {
  __shared__ uint32_t s_off, s_n;
  if (threadIdx.x == 0) {
    uint32_t off = 0;
    for (uint32_t k = 0; k < owner; ++k) off += cnt[k];
    s_off = off;
    s_n = cnt[owner];
  }
  __syncthreads();
  const uint64_t off = s_off, m = s_n;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < m; i += gridDim.x * 256ull) {
    const uint4 *p = reinterpret_cast<const uint4 *>(q + 32 * (off + i));
    ngpu_dict_hit h{kNone, 0, 0, 0, 0};
    if (dict.m) {
      const uint4 a = p[0], b = p[1];
      const uint32_t d[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
      h = dict_find(dict, d);
    }
    hits[rows[off + i]] = h;
  }
}

// An owner's probe of the node step's padded blocks (a2a_plan.hpp
// PaddedStep): requester i's block is rows [off[i], off[i + 1]) of q, its
// first rcnt[i] rows are digests this owner owns, the rest padding (not
// probed, their hits left unwritten: the requester drops them by row id).
// The counts arrived in band, so nothing here waits for the host.
__global__ __launch_bounds__(256) void dict_probe_blocks(const uint8_t *__restrict__ q,
                                                         const uint32_t *__restrict__ rcnt,
                                                         ProbeBlocks b, DictDevice dict,
                                                         ngpu_dict_hit *__restrict__ hits) {
  const uint64_t r = blockIdx.x * 256ull + threadIdx.x;
  if (r >= b.off[b.W]) return;
  uint32_t i = 0;
  while (i + 1 < b.W && b.off[i + 1] <= r) ++i;
  if (r - b.off[i] >= rcnt[i]) return;
  const uint4 *p = reinterpret_cast<const uint4 *>(q + 32 * r);
  ngpu_dict_hit h{kNone, 0, 0, 0, 0};
  if (dict.m) {
    const uint4 x = p[0], y = p[1];
    const uint32_t d[8] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w};
    h = dict_find(dict, d);
  }
  hits[r] = h;
}

// hits of routed rows back to their rows (dist.py: the all-to-all returns
// them in routed order); padding rows (row id ~0) are skipped
__global__ void hits_scatter(const ngpu_dict_hit *__restrict__ routed,
                             const uint32_t *__restrict__ rows, uint64_t m,
                             ngpu_dict_hit *__restrict__ hits) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (i >= m) return;
  const uint32_t r = rows[i];
  if (r != 0xFFFFFFFFu) hits[r] = routed[i];
}

}  // namespace

namespace {
// A record a dedup stage accepted (NEW / INTRA / DICT) gets its digest mark
// back, so a later dedup over a longer prefix of the same layer accepts it
// again; a record the stage rejected (NGPU_UNHASHED) keeps that mark, so the
// digest guard still fires on it (streaming Pack emission, pack.hip).
__global__ void remark_digested(ngpu_result *__restrict__ r, uint64_t n) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (i < n && r[i].kind <= NGPU_DICT) r[i].kind = NGPU_DIGESTED;
}
}  // namespace

void launch_remark_digested(ngpu_result *res, uint64_t n, hipStream_t s) {
  if (n == 0) return;
  hipLaunchKernelGGL(remark_digested, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, res, n);
}

void launch_route(const uint8_t *src, uint64_t stride, uint64_t n, uint32_t W, uint64_t seg_cap,
                  uint32_t *cnt, uint8_t *out, uint32_t *rows, hipStream_t s) {
  hipMemsetAsync(cnt, 0, 128 * sizeof(uint32_t), s);
  if (n == 0) return;
  const unsigned blocks = (unsigned)((n + 255) / 256);
  hipLaunchKernelGGL(route_count, dim3(blocks), dim3(256), 0, s, src, stride, n, W, cnt);
  hipLaunchKernelGGL(route_scatter, dim3(blocks), dim3(256), 0, s, src, stride, n, W, seg_cap, cnt,
                     out, rows);
}

void launch_dict_probe_routed(const uint8_t *q, const uint32_t *rows, const uint32_t *cnt,
                              uint64_t n_max, uint32_t owner, const DictDevice &dict,
                              ngpu_dict_hit *hits, hipStream_t s) {
  if (n_max == 0) return;
  const uint64_t b = std::min<uint64_t>((n_max + 255) / 256, 2048);
  hipLaunchKernelGGL(dict_probe_routed, dim3((unsigned)b), dim3(256), 0, s, q, rows, cnt, owner,
                     dict, hits);
}

void launch_dict_probe_blocks(const uint8_t *q, const uint32_t *rcnt, const ProbeBlocks &b,
                              const DictDevice &dict, ngpu_dict_hit *hits, hipStream_t s) {
  const uint64_t R = b.off[b.W];
  if (R == 0) return;
  hipLaunchKernelGGL(dict_probe_blocks, dim3((unsigned)((R + 255) / 256)), dim3(256), 0, s, q, rcnt,
                     b, dict, hits);
}

void launch_hits_scatter(const ngpu_dict_hit *routed, const uint32_t *rows, uint64_t m,
                         ngpu_dict_hit *hits, hipStream_t s) {
  if (m == 0) return;
  hipLaunchKernelGGL(hits_scatter, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, routed, rows,
                     m, hits);
}

void launch_pack_digests(const uint8_t *src, uint64_t stride, uint64_t n, uint8_t *dst,
                         hipStream_t s) {
  if (n == 0) return;
  hipLaunchKernelGGL(pack_digests, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, src, stride,
                     n, dst);
}

void launch_dict_probe_owned(const uint8_t *q, uint64_t n, uint32_t owner, uint32_t W,
                             const DictDevice &dict, ngpu_dict_hit *hits, hipStream_t s) {
  if (n == 0) return;
  hipLaunchKernelGGL(dict_probe_owned, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, q, n,
                     owner, W, dict, hits);
}

void launch_hits_merge(const uint8_t *q, uint64_t n, uint32_t W, const ngpu_dict_hit *parts,
                       ngpu_dict_hit *hits, hipStream_t s) {
  if (n == 0) return;
  hipLaunchKernelGGL(hits_merge, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, q, n, W, parts,
                     hits);
}

void launch_dict_unpack(const uint8_t *recs, uint64_t n, const uint32_t *gids, uint32_t gid0,
                        DictRec *out, hipStream_t s) {
  if (n == 0) return;
  hipLaunchKernelGGL(dict_unpack, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, recs, n, gids,
                     gid0, out);
}

void launch_dict_pack(const uint8_t *digests, const uint32_t *usize, const uint32_t *blob,
                      const uint32_t *index, const uint64_t *uoff, const uint32_t *gid, uint64_t n,
                      DictRec *out, hipStream_t s) {
  if (n == 0) return;
  hipLaunchKernelGGL(dict_pack, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, digests, usize,
                     blob, index, uoff, gid, n, out);
}

void launch_dedup(const ngpu_chunk *chunks, uint64_t n, const DictDevice &dict,
                  const ngpu_dict_hit *hits, uint32_t n_blobs, uint32_t align,
                  const uint64_t *lfirst, uint64_t L, Workspace &ws, ngpu_result *out,
                  ngpu_layer_stats *st, hipStream_t s, hipEvent_t ev_end) {
  const uint32_t nbo = n_blobs + 1;  // dict blobs + own blob (last slot), per layer
  uint64_t *single = nullptr;
  if (!lfirst) {
    single = ws.lfirst1;
    lfirst = ws.lfirst1;
    L = 1;
  }
  const bool small = !ws.grid_stages && n <= kSmallDedupChunks && L <= kSmallDedupLayers;
  const uint64_t nt = (n + kScanTile - 1) / kScanTile;
  uint64_t *ts = ws.tstat + kDedupTs(ws.tiles);
  const uint64_t nbf = (uint64_t)nbo * L, nst = L * (sizeof(ngpu_layer_stats) / 8);
  // the intra table of this call: its first next_pow2(2(n + 1)) slots (the
  // load the workspace is sized for, <= 0.5), not the
  // workspace's whole table (sized by the largest call the slot has served:
  // after a 16M-chunk layer, zeroing all of it cost a small layer ~0.1 ms).
  // The small path scans in LDS (no tile words to reset).
  uint64_t icap = n ? ws.intra_cap : 0;
  if (n) {
    uint64_t c = 64;
    while (c < 2 * (n + 1)) c <<= 1;
    icap = c < icap ? c : icap;
  }
  const uint64_t ntw = small ? 0 : 1 + kDedupScans * ws.tiles;
  uint64_t total = n + 1;
  for (uint64_t v : {nbf, nst, icap, ntw}) total = v > total ? v : total;
  const DedupInit a{lfirst, L, n, single, ws.chunk_layer, ws.blob_first, nbf,
                    reinterpret_cast<uint64_t *>(st), nst, ws.intra, icap, ts, ntw,
                    ws.newflag, ws.uoff, ws.nbytes, ws.ndict, total, ws.stats};
  if (small && single && nbo <= kLdsBlobs) {  // one layer: the whole stage in LDS
#if NGPU_PROBE_AB
    // NGPU_DEDUP_LDS_THREADS=1024: the wide workgroup for every size (A/B knob)
    static const bool wide = [] {
      const char *v = getenv("NGPU_DEDUP_LDS_THREADS");
      return v && atoi(v) == 1024;
    }();
#else
    constexpr bool wide = false;
#endif
    if (n <= 256 && !wide)
      hipExtLaunchKernelGGL(dedup_small_lds<256>, dim3(1), dim3(256), 0, s, nullptr, ev_end, 0,
                            chunks, n, dict, hits, n_blobs, align, st, out, ws.stats);
    else
      hipExtLaunchKernelGGL(dedup_small_lds<kSmallThreads>, dim3(1), dim3(kSmallThreads), 0, s,
                            nullptr, ev_end, 0, chunks, n, dict, hits, n_blobs, align, st, out,
                            ws.stats);
    return;
  }
  if (small) {
    static_assert(kSmallDedupChunks <= kSmallThreads * kSmallItems, "one scan pass");
    hipExtLaunchKernelGGL(dedup_small, dim3(1), dim3(kSmallThreads), 0, s, nullptr, ev_end, 0, a,
                          chunks, dict, hits, n_blobs, align, lfirst, ws.blob_real, st, out);
    return;
  }
  const uint64_t ib = (total + 255) / 256;
  hipLaunchKernelGGL(dedup_init, dim3((unsigned)(ib < 4096 ? ib : 4096)), dim3(256), 0, s, a);
  if (n) {
    const unsigned blocks = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL(dedup_probe_insert, dim3(blocks), dim3(256), 0, s, chunks, n, dict, hits,
                       ws.chunk_layer, out, ws.blob_first, n_blobs, ws.intra, icap - 1, ws.stats);
    hipLaunchKernelGGL(dedup_resolve, dim3(blocks), dim3(256), 0, s, chunks, n, ws.chunk_layer,
                       ws.intra, icap - 1, out, align, ws.newflag, ws.uoff, ws.nbytes,
                       ws.ndict);
    hipLaunchKernelGGL(dedup_scan, dim3((unsigned)nt), dim3(kTileThreads), 0, s, n, ws.newflag,
                       ws.uoff, ws.nbytes, ws.ndict, ts, ws.tiles);
  }
  // the stage's last kernel carries the end event (no separate marker packet)
  hipExtLaunchKernelGGL(blob_rank, dim3((unsigned)L), dim3(256), 0, s, nullptr,
                        n ? nullptr : ev_end, 0, ws.blob_first, nbo, ws.blob_real, lfirst,
                        (const uint64_t *)ws.newflag, (const uint64_t *)ws.uoff,
                        (const uint64_t *)ws.nbytes, (const uint64_t *)ws.ndict, st);
  if (n)
    hipExtLaunchKernelGGL(dedup_finalize, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                          nullptr, ev_end, 0, n, (const uint32_t *)ws.chunk_layer, lfirst,
                          (const uint64_t *)ws.newflag, (const uint64_t *)ws.uoff,
                          (const uint32_t *)ws.blob_real, nbo, out);
}

}  // namespace ngpu
