// common.hpp — shared device/host declarations for libnydusgpu.so (gfx950).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nydus_gpu.h"

namespace ngpu {

constexpr uint32_t kLeaf = 1024;        // BLAKE3 chunk ("leaf" here) bytes
constexpr uint64_t kEmpty = ~0ull;      // empty hash-table slot
constexpr uint32_t kNone = 0xFFFFFFFFu;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// ---- device helpers --------------------------------------------------------
// 16-B streaming load (read-once data: non-temporal).
__device__ __forceinline__ u32x4 load_nt16(const void *p) {
  return __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
}
__device__ __forceinline__ uint32_t rotr32(uint32_t x, uint32_t n) {
  return __builtin_amdgcn_alignbit(x, x, n);
}

// 64-bit hash-table slot: tag (digest word 2) in the high half, id in the low.
// Equal digests give equal tags, so an atomic min over a slot keeps the
// smallest id ("first in stream / table order wins").
__device__ __forceinline__ uint32_t digest_tag(const uint32_t *w) {
  uint32_t t = w[2];
  return t == 0xFFFFFFFFu ? 0xFFFFFFFEu : t;
}
__device__ __forceinline__ uint64_t digest_bucket(const uint32_t *w) {
  return ((uint64_t)w[1] << 32 | w[0]) * 0x9E3779B97F4A7C15ull;
}

// ---- launchers (defined in the .hip files) --------------------------------
struct Workspace;

// blake3.hip
// ev_groups (may be null): recorded right after the leaf-group kernel.
void launch_blake3(const uint8_t *data, const ngpu_chunk *chunks, uint64_t n,
                   uint64_t data_len, int group_log2, Workspace &ws,
                   ngpu_result *out, hipStream_t s, hipEvent_t ev_groups_start,
                   hipEvent_t ev_groups_end);
uint64_t blake3_max_groups(uint64_t n, uint64_t data_len, int group_log2);
// sha256.hip
void launch_sha256(const uint8_t *data, uint64_t data_len,
                   const ngpu_chunk *chunks, uint64_t n, ngpu_result *out,
                   uint64_t *err, int variant, hipStream_t s);

struct DictDevice {
  const uint8_t *digests = nullptr;  // m x 32
  const uint32_t *usize = nullptr;
  const uint32_t *blob = nullptr;    // inner blob index
  const uint32_t *index = nullptr;   // RAFS chunk index
  const uint64_t *table = nullptr;   // hash slots
  uint64_t mask = 0;                 // table capacity - 1
  uint64_t m = 0;
  uint32_t n_blobs = 0;
};

// dedup.hip
void launch_dict_build(const uint8_t *digests, uint64_t m, uint64_t *table,
                       uint64_t cap, hipStream_t s);
// hits == nullptr: probe `dict`; otherwise use the given per-chunk hits.
// n_blobs: inner blobs of the (global) dict.  L layers; layer l owns chunks
// [lfirst[l], lfirst[l+1]) (device array); st: device ngpu_layer_stats[L].
void launch_dedup(const ngpu_chunk *chunks, uint64_t n, const DictDevice &dict,
                  const ngpu_dict_hit *hits, uint32_t n_blobs, uint32_t align,
                  const uint64_t *lfirst, uint64_t L, Workspace &ws, ngpu_result *out,
                  ngpu_layer_stats *st, hipStream_t s);
void launch_set_single_layer(uint64_t *lfirst, uint64_t n, hipStream_t s);
void launch_dict_probe(const uint8_t *digests, uint64_t stride, uint64_t n,
                       const DictDevice &dict, ngpu_dict_hit *hits, hipStream_t s);
void launch_scan_u64(uint64_t *data, uint64_t n, uint64_t *tmp,
                     hipStream_t s);  // exclusive, in place, n+1 entries used
uint64_t scan_tmp_words(uint64_t n);

// Device workspace, grown on demand and owned by the engine.
struct Workspace {
  uint64_t *groups = nullptr;     // n+1: leaf groups per chunk -> exclusive scan
  uint32_t *group_chunk = nullptr;// G_max: chunk id of each leaf group
  uint32_t *cv = nullptr;         // G_max x 8 words: subtree chaining values
  uint32_t *small = nullptr;      // n: single-group chunks sorted by work (blake3.hip)
  uint32_t *small_hist = nullptr; // 2 x (16*16 + 1): block-count histogram + cursors
  uint32_t *tree_list = nullptr;  // n: chunks whose groups straddle a workgroup window
  uint64_t *newflag = nullptr;    // n+1: NEW flag -> scan = NEW index
  uint64_t *uoff = nullptr;       // n+1: aligned NEW size -> scan = offset
  uint64_t *scan_tmp = nullptr;
  uint64_t *intra = nullptr;      // intra-layer hash table
  uint64_t intra_cap = 0;
  uint32_t *blob_first = nullptr; // per layer: dict blobs + 1: first chunk hitting each
  uint32_t *blob_real = nullptr;
  uint32_t *chunk_layer = nullptr;   // n: layer of each chunk
  uint64_t *lfirst1 = nullptr;       // {0, n} for single-layer calls
  ngpu_layer_stats *lstats = nullptr;// per-layer stats (internal, cap_layers)
  uint64_t cap_layers = 0;
  uint64_t *stats = nullptr;      // device-side counters (ngpu_layer_stats)
  uint64_t cap_n = 0, cap_g = 0, cap_blobs = 0;
  int load_mode = 0;              // b3_groups load mode (see blake3.hip)
};

}  // namespace ngpu
