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

__global__ void dict_insert(const uint8_t *__restrict__ digests, uint64_t m,
                            uint64_t *__restrict__ table, uint64_t mask) {
  const uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (e < m) ht_insert_min<32>(table, mask, digests, (uint32_t)e);
}

// Look n digests (byte stride `stride`) up in the dict.
__global__ void dict_probe_records(const uint8_t *__restrict__ digests, uint64_t stride,
                                   uint64_t n, DictDevice dict,
                                   ngpu_dict_hit *__restrict__ hits) {
  const uint64_t q = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (q >= n) return;
  ngpu_dict_hit h{kNone, 0, 0, 0};
  if (dict.m) {
    const uint4 *p = reinterpret_cast<const uint4 *>(digests + q * stride);
    const uint4 a = p[0], b = p[1];
    const uint32_t d[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    const uint32_t e = ht_lookup<32>(dict.table, dict.mask, dict.digests, d);
    if (e != kNone) h = ngpu_dict_hit{e, dict.index[e], dict.blob[e], dict.usize[e]};
  }
  hits[q] = h;
}

// ---- layered dedup -----------------------------------------------------------
// A call covers L >= 1 layers; layer l owns chunks [first[l], first[l+1]).
// Everything except the chunk dict restarts per layer: the layered
// (intra-build) dict, NEW indices, uncompressed offsets and blob order.  The
// intra table is shared by all layers of a call: its key is (layer, digest).

__device__ __forceinline__ uint64_t layer_bucket(const uint32_t *d, uint32_t layer) {
  return digest_bucket(d) + (uint64_t)layer * 0xC2B2AE3D27D4EB4Full;
}

// chunk -> layer map: thread per chunk, binary search in lfirst[0..L]
// (last layer whose first chunk <= c; empty layers are skipped naturally).
__global__ void layer_fill(const uint64_t *__restrict__ first, uint64_t L, uint64_t n,
                           uint32_t *__restrict__ chunk_layer) {
  const uint64_t c = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (c >= n) return;
  uint64_t lo = 0, hi = L;  // invariant: first[lo] <= c < first[hi]
  while (hi - lo > 1) {
    const uint64_t mid = (lo + hi) >> 1;
    if (first[mid] <= c) lo = mid;
    else hi = mid;
  }
  chunk_layer[c] = (uint32_t)lo;
}

// Stage 1: dict decision (from given hits, or by probing the local dict) +
// reset of the per-chunk state.
__global__ void dedup_probe(const ngpu_chunk *__restrict__ chunks, uint64_t n,
                            DictDevice dict, const ngpu_dict_hit *__restrict__ hits,
                            const uint32_t *__restrict__ chunk_layer,
                            ngpu_result *__restrict__ out,
                            uint64_t *__restrict__ newflag,
                            uint32_t *__restrict__ blob_first, uint32_t n_blobs) {
  const uint64_t c = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (c >= n) return;
  ngpu_result &r = out[c];
  uint32_t kind = NGPU_NEW;
  ngpu_dict_hit h{kNone, 0, 0, 0};
  if (hits) {
    h = hits[c];
  } else if (dict.m) {
    uint32_t d[8];
    load_digest<sizeof(ngpu_result)>(reinterpret_cast<const uint8_t *>(out), c, d);
    const uint32_t e = ht_lookup<32>(dict.table, dict.mask, dict.digests, d);
    if (e != kNone) h = ngpu_dict_hit{e, dict.index[e], dict.blob[e], dict.usize[e]};
  }
  if (h.entry != kNone && (h.usize == 0 || h.usize == chunks[c].length) && h.blob < n_blobs) {
    kind = NGPU_DICT;
    r.ref = h.entry;
    r.index = h.index;
    r.blob_index = h.blob;  // inner index; remapped in finalize
    r.uncompressed_offset = 0;
    atomicMin(blob_first + (uint64_t)chunk_layer[c] * (n_blobs + 1) + h.blob, (uint32_t)c);
  }
  r.kind = kind;
  r.dict_blob = kind == NGPU_DICT ? h.blob : 0u;
  newflag[c] = 0;
}

// Per-layer counters: lanes of a wave usually share one layer, so reduce in
// the wave and issue ONE atomic (per-lane atomics on one address serialise:
// 16K of them cost ~0.2 ms).  Every lane of the wave must call these.
__device__ __forceinline__ void layer_add_u64(unsigned long long *base, size_t stride_words,
                                              uint32_t layer, uint64_t v) {
  const uint32_t l0 = __builtin_amdgcn_readfirstlane(layer);
  if (__all(layer == l0)) {
#pragma unroll
    for (int o = 32; o; o >>= 1) v += __shfl_xor(v, o, 64);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(base + (size_t)l0 * stride_words, (unsigned long long)v);
  } else if (v) {
    atomicAdd(base + (size_t)layer * stride_words, (unsigned long long)v);
  }
}

__device__ __forceinline__ void layer_min_u32(uint32_t *base, size_t stride, uint32_t layer,
                                              uint32_t v) {
  const uint32_t l0 = __builtin_amdgcn_readfirstlane(layer);
  if (__all(layer == l0)) {
#pragma unroll
    for (int o = 32; o; o >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o, 64));
    if ((threadIdx.x & 63) == 0 && v != kNone) atomicMin(base + (size_t)l0 * stride, v);
  } else if (v != kNone) {
    atomicMin(base + (size_t)layer * stride, v);
  }
}

__device__ __forceinline__ bool same_key(const ngpu_result *out, const uint32_t *chunk_layer,
                                         uint32_t id, const uint32_t d[8], uint32_t layer) {
  return chunk_layer[id] == layer &&
         digest_eq<sizeof(ngpu_result)>(reinterpret_cast<const uint8_t *>(out), id, d);
}

__global__ void dedup_insert(const ngpu_result *__restrict__ out, uint64_t n,
                             const uint32_t *__restrict__ chunk_layer,
                             uint64_t *__restrict__ table, uint64_t mask) {
  const uint64_t c = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (c >= n || out[c].kind == NGPU_DICT) return;
  uint32_t d[8];
  load_digest<sizeof(ngpu_result)>(reinterpret_cast<const uint8_t *>(out), c, d);
  const uint32_t layer = chunk_layer[c];
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

__global__ void dedup_resolve(const ngpu_chunk *__restrict__ chunks, uint64_t n,
                              const uint32_t *__restrict__ chunk_layer,
                              const uint64_t *__restrict__ table, uint64_t mask,
                              ngpu_result *__restrict__ out, uint32_t align,
                              uint64_t *__restrict__ newflag,
                              uint64_t *__restrict__ uoff,
                              uint32_t *__restrict__ blob_first, uint32_t n_blobs) {
  const uint64_t c = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  const bool live = c < n;
  uint32_t layer = 0, first_new = kNone;
  if (live) {
    ngpu_result &r = out[c];
    layer = chunk_layer[c];
    uoff[c] = 0;
    if (c == 0) { newflag[n] = 0; uoff[n] = 0; }
    if (r.kind != NGPU_DICT) {
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
        newflag[c] = 1;
        uoff[c] = ((uint64_t)len + align - 1) / align * align;
        first_new = (uint32_t)c;
      }
    }
  }
  layer_min_u32(blob_first + n_blobs, n_blobs + 1, layer, first_new);
}

// Blob-table order per layer (one workgroup per layer): each dict blob gets a
// real index at its first hit, the layer's own blob at its first NEW chunk
// ([nydus v2.3.0] BlobManager alloc_index / get_or_create_current_blob).
__global__ void blob_rank(const uint32_t *__restrict__ first_all, uint32_t nbo,
                          uint32_t *__restrict__ real_all, const uint64_t *__restrict__ lfirst,
                          const uint64_t *__restrict__ newidx, const uint64_t *__restrict__ uoff,
                          ngpu_layer_stats *__restrict__ st) {
  const uint64_t l = blockIdx.x;
  const uint32_t *first = first_all + l * nbo;
  uint32_t *real = real_all + l * nbo;
  for (uint32_t b = threadIdx.x; b < nbo; b += blockDim.x) {
    const uint32_t fb = first[b];
    uint32_t rank = kNone;
    if (fb != kNone) {
      rank = 0;
      for (uint32_t o = 0; o < nbo; ++o) rank += first[o] < fb;
    }
    real[b] = rank;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t used = 0;
    for (uint32_t b = 0; b < nbo; ++b) used += first[b] != kNone;
    const uint64_t a = lfirst[l], e = lfirst[l + 1];
    st[l].chunks = e - a;
    st[l].new_chunks = newidx[e] - newidx[a];
    st[l].own_blob_index = real[nbo - 1];  // kNone -> 0xFFFFFFFF
    st[l].blobs = used;
    st[l].uncompressed_size = uoff[e] - uoff[a];
  }
}

__global__ void dedup_finalize(const ngpu_chunk *__restrict__ chunks, uint64_t n,
                               const uint32_t *__restrict__ chunk_layer,
                               const uint64_t *__restrict__ lfirst,
                               const uint64_t *__restrict__ newidx,
                               const uint64_t *__restrict__ uoff,
                               const uint32_t *__restrict__ real_all, uint32_t nbo,
                               ngpu_result *__restrict__ out,
                               ngpu_layer_stats *__restrict__ st) {
  const uint64_t c = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint32_t layer = 0;
  uint64_t new_bytes = 0, intra = 0, dict = 0;
  if (c < n) {
    ngpu_result &r = out[c];
    layer = chunk_layer[c];
    const uint32_t *real = real_all + (uint64_t)layer * nbo;
    const uint64_t a = lfirst[layer];
    const uint64_t ib = newidx[a], ob = uoff[a];
    const uint32_t own = real[nbo - 1];
    if (r.kind == NGPU_NEW) {
      r.index = (uint32_t)(newidx[c] - ib);
      r.uncompressed_offset = uoff[c] - ob;
      r.blob_index = own;
      new_bytes = chunks[c].length;
    } else if (r.kind == NGPU_INTRA) {
      const uint64_t f = r.ref;
      r.index = (uint32_t)(newidx[f] - ib);
      r.uncompressed_offset = uoff[f] - ob;
      r.blob_index = own;
      intra = 1;
    } else {
      r.blob_index = real[r.blob_index];
      dict = 1;
    }
  }
  constexpr size_t W = sizeof(ngpu_layer_stats) / 8;
  unsigned long long *base = reinterpret_cast<unsigned long long *>(st);
  layer_add_u64(base + offsetof(ngpu_layer_stats, new_bytes) / 8, W, layer, new_bytes);
  layer_add_u64(base + offsetof(ngpu_layer_stats, intra_chunks) / 8, W, layer, intra);
  layer_add_u64(base + offsetof(ngpu_layer_stats, dict_chunks) / 8, W, layer, dict);
}

// ---- exclusive scan over u64 (n+1 entries, in place) ----------------------
constexpr int kScanThreads = 256;
constexpr int kScanItems = 8;
constexpr int kScanTile = kScanThreads * kScanItems;

__device__ __forceinline__ uint64_t block_exclusive_scan(uint64_t v, uint64_t *total) {
  __shared__ uint64_t wsum[kScanThreads / 64];
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
  for (int w = 0; w < kScanThreads / 64; ++w) {
    if (w < wid) pre += wsum[w];
    tot += wsum[w];
  }
  __syncthreads();
  *total = tot;
  return pre + x - v;
}

__global__ __launch_bounds__(kScanThreads) void scan_reduce(const uint64_t *__restrict__ a,
                                                            uint64_t m, uint64_t *__restrict__ tmp) {
  const uint64_t base = blockIdx.x * (uint64_t)kScanTile + threadIdx.x * kScanItems;
  uint64_t s = 0;
#pragma unroll
  for (int i = 0; i < kScanItems; ++i)
    if (base + i < m) s += a[base + i];
  uint64_t tot;
  block_exclusive_scan(s, &tot);
  if (threadIdx.x == 0) tmp[blockIdx.x] = tot;
}

__global__ __launch_bounds__(kScanThreads) void scan_top(uint64_t *__restrict__ tmp, uint64_t nb) {
  uint64_t carry = 0;
  for (uint64_t t0 = 0; t0 < nb; t0 += kScanThreads) {
    const uint64_t i = t0 + threadIdx.x;
    const uint64_t v = i < nb ? tmp[i] : 0;
    uint64_t tot;
    const uint64_t ex = block_exclusive_scan(v, &tot);
    if (i < nb) tmp[i] = carry + ex;
    carry += tot;
  }
}

__global__ __launch_bounds__(kScanThreads) void scan_apply(uint64_t *__restrict__ a, uint64_t m,
                                                           const uint64_t *__restrict__ tmp) {
  const uint64_t base = blockIdx.x * (uint64_t)kScanTile + threadIdx.x * kScanItems;
  uint64_t v[kScanItems], s = 0;
#pragma unroll
  for (int i = 0; i < kScanItems; ++i) {
    v[i] = base + i < m ? a[base + i] : 0;
    s += v[i];
  }
  uint64_t tot;
  uint64_t run = block_exclusive_scan(s, &tot) + tmp[blockIdx.x];
#pragma unroll
  for (int i = 0; i < kScanItems; ++i) {
    if (base + i < m) a[base + i] = run;
    run += v[i];
  }
}

__global__ void set_single_layer(uint64_t *lfirst, uint64_t n) {
  lfirst[0] = 0;
  lfirst[1] = n;
}

}  // namespace

void launch_set_single_layer(uint64_t *lfirst, uint64_t n, hipStream_t s) {
  hipLaunchKernelGGL(set_single_layer, dim3(1), dim3(1), 0, s, lfirst, n);
}

uint64_t scan_tmp_words(uint64_t n) { return (n + 1 + kScanTile - 1) / kScanTile + 1; }

void launch_scan_u64(uint64_t *a, uint64_t n, uint64_t *tmp, hipStream_t s) {
  const uint64_t m = n + 1;
  const uint64_t nb = (m + kScanTile - 1) / kScanTile;
  hipLaunchKernelGGL(scan_reduce, dim3((unsigned)nb), dim3(kScanThreads), 0, s, a, m, tmp);
  hipLaunchKernelGGL(scan_top, dim3(1), dim3(kScanThreads), 0, s, tmp, nb);
  hipLaunchKernelGGL(scan_apply, dim3((unsigned)nb), dim3(kScanThreads), 0, s, a, m, tmp);
}

void launch_dict_build(const uint8_t *digests, uint64_t m, uint64_t *table,
                       uint64_t cap, hipStream_t s) {
  hipMemsetAsync(table, 0xFF, cap * sizeof(uint64_t), s);
  if (m == 0) return;
  const uint64_t blocks = (m + 255) / 256;
  hipLaunchKernelGGL(dict_insert, dim3((unsigned)blocks), dim3(256), 0, s, digests, m,
                     table, cap - 1);
}

void launch_dict_probe(const uint8_t *digests, uint64_t stride, uint64_t n,
                       const DictDevice &dict, ngpu_dict_hit *hits, hipStream_t s) {
  if (n == 0) return;
  hipLaunchKernelGGL(dict_probe_records, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                     digests, stride, n, dict, hits);
}

void launch_dedup(const ngpu_chunk *chunks, uint64_t n, const DictDevice &dict,
                  const ngpu_dict_hit *hits, uint32_t n_blobs, uint32_t align,
                  const uint64_t *lfirst, uint64_t L, Workspace &ws, ngpu_result *out,
                  ngpu_layer_stats *st, hipStream_t s) {
  const uint32_t nbo = n_blobs + 1;  // dict blobs + own blob (last slot), per layer
  (void)hipMemsetAsync(ws.blob_first, 0xFF, sizeof(uint32_t) * nbo * L, s);
  (void)hipMemsetAsync(st, 0, sizeof(ngpu_layer_stats) * L, s);
  if (n) {
    const unsigned blocks = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL(layer_fill, dim3(blocks), dim3(256), 0, s, lfirst, L, n, ws.chunk_layer);
    (void)hipMemsetAsync(ws.intra, 0xFF, ws.intra_cap * sizeof(uint64_t), s);
    hipLaunchKernelGGL(dedup_probe, dim3(blocks), dim3(256), 0, s, chunks, n, dict, hits,
                       ws.chunk_layer, out, ws.newflag, ws.blob_first, n_blobs);
    hipLaunchKernelGGL(dedup_insert, dim3(blocks), dim3(256), 0, s, out, n, ws.chunk_layer,
                       ws.intra, ws.intra_cap - 1);
    hipLaunchKernelGGL(dedup_resolve, dim3(blocks), dim3(256), 0, s, chunks, n, ws.chunk_layer,
                       ws.intra, ws.intra_cap - 1, out, align, ws.newflag, ws.uoff,
                       ws.blob_first, n_blobs);
  } else {
    (void)hipMemsetAsync(ws.newflag, 0, sizeof(uint64_t), s);
    (void)hipMemsetAsync(ws.uoff, 0, sizeof(uint64_t), s);
  }
  launch_scan_u64(ws.newflag, n, ws.scan_tmp, s);
  launch_scan_u64(ws.uoff, n, ws.scan_tmp, s);
  hipLaunchKernelGGL(blob_rank, dim3((unsigned)L), dim3(256), 0, s, ws.blob_first, nbo,
                     ws.blob_real, lfirst, ws.newflag, ws.uoff, st);
  if (n)
    hipLaunchKernelGGL(dedup_finalize, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                       chunks, n, ws.chunk_layer, lfirst, ws.newflag, ws.uoff, ws.blob_real,
                       nbo, out, st);
}

}  // namespace ngpu
