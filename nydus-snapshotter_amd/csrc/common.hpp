// common.hpp — shared device/host declarations for libnydusgpu.so (gfx950).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nydus_gpu.h"

namespace ngpu {

constexpr uint32_t kLeaf = 1024;        // BLAKE3 chunk ("leaf" here) bytes
constexpr uint64_t kEmpty = ~0ull;      // empty hash-table slot
constexpr uint32_t kNone = 0xFFFFFFFFu;

// Workspace::stats words (u64).  The digest stage resets [0, 16) per call;
// the dedup stage resets its own [kStUnhashed, kStUnhashedFirst].  The sticky
// words [16, 20) are never reset by a stage: every error branch adds to them
// too, so a device-pointer call that nobody reads stats for still leaves its
// error for ngpu_device_status (and the next host read of the slot).
constexpr int kStBadDesc = 7;          // descriptors outside the data buffer
constexpr int kStOverlap = 8;          // leaves past the launch (overlapping descriptors)
constexpr int kStTreeQueued = 9;       // chunks queued for b3_tree
constexpr int kStSmall = 10;           // single-group chunks (b3 planning)
constexpr int kStUnhashed = 11;        // chunks that reached dedup without a digest
constexpr int kStUnhashedFirst = 12;   // ~(smallest such chunk id) (atomic max), 0 = none
constexpr int kStSticky = 16;          // + {0 bad desc, 1 overlap, 2 unhashed, 3 ~first unhashed}
constexpr int kStWords = 20;           // words read back per stats read

// Error branch of a kernel: bump the per-call word k and its sticky twin.
// `err` points at stats[kStBadDesc] (the kernels' err argument).
__device__ __forceinline__ void note_bad_desc(uint64_t *err, uint64_t v) {
  atomicAdd((unsigned long long *)err, (unsigned long long)v);
  atomicAdd((unsigned long long *)(err + (kStSticky - kStBadDesc)), (unsigned long long)v);
}
__device__ __forceinline__ void note_overlap(uint64_t *err, uint64_t total) {
  err[kStOverlap - kStBadDesc] = total;
  atomicMax((unsigned long long *)(err + (kStSticky + 1 - kStBadDesc)), (unsigned long long)total);
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Sets the calling thread's HIP device for a scope and restores it after, so
// a library call never changes which device the caller (e.g. PyTorch) is on.
struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
  DeviceGuard(const DeviceGuard &) = delete;
  DeviceGuard &operator=(const DeviceGuard &) = delete;
};

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

// ---- single-pass scan across workgroups (decoupled look-back) -------------
// A workgroup takes a ticket (its tile, in dispatch order), scans its 256
// values in the block, publishes the tile aggregate, then walks back over
// earlier tiles until it meets a published inclusive prefix.  Earlier tickets
// belong to workgroups that are already resident and publish without waiting,
// so the spin always ends.  One 64-bit word per tile carries flag + value, so
// a single atomic load sees a consistent pair.
constexpr int kTileThreads = 256;
constexpr uint64_t kFlagAgg = 1ull << 62, kFlagPre = 2ull << 62, kValMask = kFlagAgg - 1;

static __device__ __forceinline__ uint64_t block_exclusive_scan(uint64_t v, uint64_t *total) {
  __shared__ uint64_t wsum[kTileThreads / 64];
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
  for (int w = 0; w < kTileThreads / 64; ++w) {
    if (w < wid) pre += wsum[w];
    tot += wsum[w];
  }
  __syncthreads();
  *total = tot;
  return pre + x - v;
}

// Called by a whole wave: publish `agg` for `tile` and return the tile's
// exclusive prefix.  Each round the wave reads 8 x 64 predecessors at once
// (lane i, slot j: tile - 1 - i - 64 j; the 8 loads are in flight together),
// waits until each has published, and adds aggregates up to the nearest
// inclusive prefix; only a round without any prefix moves further back.
// (Prefixes appear in dispatch order, so one round usually suffices: a
// window of 64 took one L2 round trip per 64 tiles, 20 us at 1024 tiles.)
static __device__ uint64_t wave_lookback(uint64_t *status, uint64_t tile, uint64_t agg) {
  constexpr int K = 8;
  const int lane = threadIdx.x & 63;
  if (tile == 0) {
    if (lane == 0)
      __hip_atomic_store(status, kFlagPre | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return 0;
  }
  if (lane == 0)
    __hip_atomic_store(status + tile, kFlagAgg | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  uint64_t excl = 0;
  for (int64_t end = (int64_t)tile;; end -= 64 * K) {
    uint64_t s[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const int64_t t = end - 1 - lane - 64 * j;
      s[j] = t >= 0 ? __hip_atomic_load(status + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                    : kFlagPre;  // before tile 0: an inclusive prefix of 0
    }
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const int64_t t = end - 1 - lane - 64 * j;
      while (s[j] == 0) {
        __builtin_amdgcn_s_sleep(1);
        s[j] = __hip_atomic_load(status + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    // nearest inclusive prefix: smallest (slot j, lane) in distance order
    int jp = K, lp = 64;
#pragma unroll
    for (int j = K - 1; j >= 0; --j) {
      const uint64_t pm = __ballot((s[j] & kFlagPre) != 0);
      if (pm) { jp = j; lp = __builtin_ctzll(pm); }
    }
    uint64_t v = 0;
#pragma unroll
    for (int j = 0; j < K; ++j)
      if (j < jp || (j == jp && lane <= lp)) v += s[j] & kValMask;
#pragma unroll
    for (int o = 32; o; o >>= 1) v += __shfl_xor(v, o, 64);
    excl += v;
    if (jp < K) break;
  }
  if (lane == 0)
    __hip_atomic_store(status + tile, kFlagPre | (excl + agg), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  return excl;
}

// Workspace::tstat layout (u64 words), nt = tiles of cap_n chunks:
//   [0, 257)            BLAKE3 small-chunk histogram + cursors (2 x 257 u32)
//   [257]               BLAKE3 plan ticket, [258, 258 + nt) its tile status
//   [kDedupTs(nt)]      dedup ticket, then nt words per dedup scan (kDedupScans)
constexpr uint64_t kB3Ts = 257;
__host__ __device__ constexpr uint64_t tstat_tiles(uint64_t cap_n) {
  return cap_n / kTileThreads + 2;
}
__host__ __device__ constexpr uint64_t kDedupTs(uint64_t nt) { return kB3Ts + 1 + nt; }
constexpr int kDedupScans = 4;  // NEW count, v6 offset, NEW bytes, DICT count
__host__ __device__ constexpr uint64_t tstat_words(uint64_t nt) {
  return kDedupTs(nt) + 1 + kDedupScans * nt;
}

// ---- launchers (defined in the .hip files) --------------------------------
struct Workspace;

// Calls with at most this many chunks (and layers) plan their BLAKE3 groups
// and run their dedup stage in one fused workgroup each (dispatch cost: one
// launch instead of four and six); Workspace::grid_stages turns this off.
constexpr uint64_t kSmallPlanChunks = 4096;
constexpr uint64_t kSmallDedupChunks = 4096;
constexpr uint64_t kSmallDedupLayers = 64;

// blake3.hip.  Events (each may be null) ride on the kernels themselves
// (hipExtLaunchKernelGGL start/stop), so timing and stream ordering add no
// marker packets: ev_first = start of the first kernel (the one start event:
// it IS a marker), ev_groups_start = end of chunk planning (so the digest
// time is the leaf kernel plus its dispatch), ev_groups_end = end of the
// leaf kernel, ev_end = end of the stage.  Returns false when nothing
// was launched (n == 0: ev_end was not recorded).
bool launch_blake3(const uint8_t *data, const ngpu_chunk *chunks, uint64_t n,
                   uint64_t data_len, int group_log2, Workspace &ws,
                   ngpu_result *out, hipStream_t s, hipEvent_t ev_first,
                   hipEvent_t ev_groups_start, hipEvent_t ev_groups_end, hipEvent_t ev_end,
                   uint64_t chunk_size = 0);  // the engine's (0: unknown; picks b3_tree's width)
uint64_t blake3_max_groups(uint64_t n, uint64_t data_len, int group_log2);
// ngpu_config load-mode override (flags bits 8..10 minus one) this build runs.
bool blake3_load_mode_ok(int lm);
// True when the call's chunk planning runs inside its leaf kernel
// (b3_quad_planned: small layers on the quad path) -- there is no planning
// kernel, so ev_groups_start is not recorded.
bool blake3_planned_in_leaves(uint64_t n, uint64_t data_len, int group_log2, const Workspace &ws);
// Leaves + chunks up to which D = 0 calls hash one leaf per lane quad.
uint64_t blake3_quad_max_leaves();
// sha256.hip
// mixed: the chunks' lengths vary (round waves run wave-uniform, sha256_pair U)
void launch_sha256(const uint8_t *data, uint64_t data_len,
                   const ngpu_chunk *chunks, uint64_t n, ngpu_result *out,
                   uint64_t *err, int variant, bool mixed, hipStream_t s);

// One chunk-dict entry in HBM (64 B, 64-B aligned): the key and every field
// a hit returns, so a probe that hits reads one hash-slot line and one record
// line (SoA arrays cost a line per field: six random lines per hit).
struct alignas(64) DictRec {
  uint32_t digest[8];
  uint32_t usize;  // uncompressed size (0 = any)
  uint32_t blob;   // inner blob index
  uint32_t index;  // RAFS chunk index
  uint32_t gid;    // global entry id (table order; differs from the slot in node shards)
  uint64_t uoff;   // uncompressed offset in its blob
  uint64_t pad;
};
static_assert(sizeof(DictRec) == 64, "DictRec is 64 bytes");

struct DictDevice {
  const DictRec *rec = nullptr;      // m records, table order
  const uint64_t *table = nullptr;   // hash slots {tag : local id}
  uint64_t mask = 0;                 // table capacity - 1
  uint64_t m = 0;
  uint32_t n_blobs = 0;
};

// dedup.hip
void launch_dict_build(const DictRec *rec, uint64_t m, uint64_t *table, uint64_t cap,
                       hipStream_t s);
// hits == nullptr: probe `dict`; otherwise use the given per-chunk hits.
// n_blobs: inner blobs of the (global) dict.  L layers; layer l owns chunks
// [lfirst[l], lfirst[l+1]) (device array; nullptr = one layer, {0, n} is
// written to ws.lfirst1); st: device ngpu_layer_stats[L].
// ev_end (may be null): recorded by the stage's last kernel.
void launch_dedup(const ngpu_chunk *chunks, uint64_t n, const DictDevice &dict,
                  const ngpu_dict_hit *hits, uint32_t n_blobs, uint32_t align,
                  const uint64_t *lfirst, uint64_t L, Workspace &ws, ngpu_result *out,
                  ngpu_layer_stats *st, hipStream_t s, hipEvent_t ev_end);
void launch_dict_probe(const uint8_t *digests, uint64_t stride, uint64_t n,
                       const DictDevice &dict, ngpu_dict_hit *hits, hipStream_t s);
// Node dict exchange (node.hip): pack n digests (byte stride) to 32-B rows;
// probe the rows a part owns (owner = ((d0 << 8 | d1) * W) >> 16); merge the
// W parts' hit arrays (W x n) by owner.
void launch_pack_digests(const uint8_t *src, uint64_t stride, uint64_t n, uint8_t *dst,
                         hipStream_t s);
void launch_dict_probe_owned(const uint8_t *q, uint64_t n, uint32_t owner, uint32_t W,
                             const DictDevice &dict, ngpu_dict_hit *hits, hipStream_t s);
void launch_hits_merge(const uint8_t *q, uint64_t n, uint32_t W, const ngpu_dict_hit *parts,
                       ngpu_dict_hit *hits, hipStream_t s);
// Digest routing (W <= 64): n digests (byte stride) to their owners' segments
// of `out` (32 B each) with their row ids in `rows`; cnt: 128 u32 (counts at
// 0..W, cursors at 64..64+W), zeroed here.  seg_cap 0: compact, owners back to
// back; > 0: [round][owner][seg_cap] slots (the caller pre-fills padding).
void launch_route(const uint8_t *src, uint64_t stride, uint64_t n, uint32_t W, uint64_t seg_cap,
                  uint32_t *cnt, uint8_t *out, uint32_t *rows, hipStream_t s);
// Owner `owner` probes its compact segment (q, rows, cnt may live on a peer
// GPU) and writes hits[rows[i]]; n_max bounds the segment (grid size).
void launch_dict_probe_routed(const uint8_t *q, const uint32_t *rows, const uint32_t *cnt,
                              uint64_t n_max, uint32_t owner, const DictDevice &dict,
                              ngpu_dict_hit *hits, hipStream_t s);
// Owner side of the node step's padded all-to-all (a2a_plan.hpp): W blocks
// of q (32-B rows), block i = rows [off[i], off[i + 1]), of which the first
// rcnt[i] (device u32[W]) are probed into hits[row]; padding rows are skipped.
struct ProbeBlocks {
  uint32_t W;
  uint64_t off[65];
};
void launch_dict_probe_blocks(const uint8_t *q, const uint32_t *rcnt, const ProbeBlocks &b,
                              const DictDevice &dict, ngpu_dict_hit *hits, hipStream_t s);
// Records [0, n) a dedup stage accepted get kind = NGPU_DIGESTED again
// (rejected ones keep NGPU_UNHASHED): a later dedup over a longer prefix.
void launch_remark_digested(ngpu_result *res, uint64_t n, hipStream_t s);
// hits[rows[i]] = routed[i] for rows[i] != ~0.
void launch_hits_scatter(const ngpu_dict_hit *routed, const uint32_t *rows, uint64_t m,
                         ngpu_dict_hit *hits, hipStream_t s);
// RAFS v6 chunk records (80 B, device) -> dict records; gid = gids[i] (device
// array) or gid0 + i.
void launch_dict_unpack(const uint8_t *recs, uint64_t n, const uint32_t *gids, uint32_t gid0,
                        DictRec *out, hipStream_t s);
// Device SoA arrays -> dict records (index / uoff may be null: 0), gid =
// gid[i] (null: i).
void launch_dict_pack(const uint8_t *digests, const uint32_t *usize, const uint32_t *blob,
                      const uint32_t *index, const uint64_t *uoff, const uint32_t *gid, uint64_t n,
                      DictRec *out, hipStream_t s);

// Device workspace, grown on demand and owned by the engine.
struct Workspace {
  uint64_t *groups = nullptr;     // n+1: leaf groups per chunk -> exclusive scan
  uint32_t *group_chunk = nullptr;// G_max: chunk id of each leaf group
  uint32_t *cv = nullptr;         // G_max x 8 words: subtree chaining values
  uint32_t *small = nullptr;      // n: single-group chunks sorted by work (blake3.hip)
  uint32_t *tree_list = nullptr;  // n: chunks whose groups straddle a workgroup window
  uint64_t *newflag = nullptr;    // n+1: NEW flag -> scan = NEW index
  uint64_t *uoff = nullptr;       // n+1: aligned NEW size -> scan = offset
  uint64_t *nbytes = nullptr;     // n+1: scan of NEW chunk bytes (layer stats)
  uint64_t *ndict = nullptr;      // n+1: scan of DICT flags (layer stats)
  uint64_t *tstat = nullptr;      // tile tickets/status of the single-pass scans (+ histogram)
  uint64_t tiles = 0;             // tiles the tstat layout is sized for
  uint64_t *intra = nullptr;      // intra-layer hash table
  uint64_t intra_cap = 0;
  uint32_t *blob_first = nullptr; // per layer: dict blobs + 1: first chunk hitting each
  uint32_t *blob_real = nullptr;
  uint32_t *chunk_layer = nullptr;   // n: layer of each chunk
  uint64_t *lfirst1 = nullptr;       // {0, n} for single-layer calls
  ngpu_layer_stats *lstats = nullptr;// per-layer stats (internal, cap_layers)
  uint64_t cap_layers = 0;
  uint64_t *stats = nullptr;      // device-side counters (kSt* words above)
  uint64_t cap_n = 0, cap_g = 0, cap_blobs = 0;
  // node dict exchange: packed digests (n x 32; routed: owner-ordered), per-part
  // hits (W x n, copy exchange only), hits (n), routed row ids (n) and the
  // route counters (128 u32)
  uint8_t *xq = nullptr;
  ngpu_dict_hit *xparts = nullptr, *xhits = nullptr;
  uint32_t *xrow = nullptr, *xcnt = nullptr;
  uint64_t cap_x = 0, cap_xparts = 0;
  int load_mode = 0;              // b3_groups load mode (see blake3.hip)
  bool grid_stages = false;       // NGPU_FLAG_GRID_STAGES: no fused small-call path
};

}  // namespace ngpu
