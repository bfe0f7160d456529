// engine_internal.hpp — engine / chunk-dict state and stage helpers shared by
// engine.hip (C ABI), dict.hip (chunk dicts), pack.hip (streaming Pack
// writer) and node.hip (multi-GPU node).  Not installed.
#pragma once

#include <atomic>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "blob.hpp"
#include "common.hpp"

// Pinned staging + device buffers of one streaming-Pack slot, kept by the
// engine between packs (pinning 64 MiB costs milliseconds: per-pack
// allocation cost the streaming path a third of its rate).
struct ngpu_staging_buf {
  void *h = nullptr, *h_ch = nullptr, *d = nullptr, *d_ch = nullptr;
  hipEvent_t copied = nullptr, done = nullptr;
  uint64_t cap = 0;
};

// Per-pack device buffers and streams, kept by the engine between packs
// (a stream create/destroy and two hipMalloc/hipFree pairs per pack were most
// of a small layer's streaming Pack: 0.9 ms for C1's 10 MB).  `stream` is the
// pack's compute stream: packs open at once run side by side on the GPU.
// Compute streams live until the engine is destroyed (ngpu_engine::streams).
// The double-buffered gather windows of a Pack's blob stream: device window
// + descriptors and the pinned descriptor staging, per buffer (allocated per
// Pack close until round 3: two hipMalloc/hipHostMalloc pairs of 5 MB and a
// staging-sized window each time).
struct BlobWindows {
  uint8_t *dwin[2] = {}, *ddesc[2] = {}, *hdesc[2] = {};
  hipEvent_t ev[2] = {};        // the window's bytes landed (D2H done)
  hipEvent_t gathered[2] = {};  // the window's gather kernel done (its D2H may start)
  uint64_t cap = 0, kcap = 0;  // window bytes, descriptors per window
};
void blob_windows_free(BlobWindows &w);  // (pack.hip)

struct ngpu_pack_bufs {
  hipStream_t stream = nullptr;
  hipEvent_t fence = nullptr;  // the pack's host_fence marker
  uint64_t *h_stats = nullptr;  // pinned, 32 words: the pack's stats read back
  uint8_t *h_io = nullptr;      // pinned: chunk table out, results back (no pageable copies
  uint64_t io_cap = 0;          // under the engine lock)
  ngpu_result *d_res = nullptr;
  uint64_t res_cap = 0;
  ngpu_chunk *d_all = nullptr;
  uint64_t all_cap = 0;
  BlobWindows win;              // the blob stream's gather windows (ngpu_pack_finish)
};

// A chunk dict ([nydus v2.3.0] HashChunkDict): HBM-resident, read-only once
// built, reference counted (the engine's default slot, its open cache, every
// pack using it and the caller each hold one).
struct ngpu_dict {
  std::atomic<int> refs{1};
  int device = 0;
  uint32_t digester = 0, chunk_size = 0;
  ngpu::DictDevice dev;                // device arrays + hash table
  std::vector<void *> allocs;          // device allocations owned
  std::vector<uint8_t> blob_table;     // 256-B RAFS v6 blob records (inner-index order)
  std::vector<ngpu::DictPlace> place;  // per entry: compressed placement (empty: unknown)
  // identity of the bootstrap file it was opened from (ngpu_dict_open cache)
  std::string path;
  uint64_t st_dev = 0, st_ino = 0, st_size = 0;
  int64_t st_mtime_ns = 0;
  uint32_t node_mode = 0;  // ngpu_node_dict_open cache: the mode it was opened with
  // node dicts (node.hip): one part per node device -- a digest-prefix shard
  // (its records carry their global entry ids) or a full replica.
  // dev.m / dev.n_blobs are the global counts; dev.rec / dev.table stay null.
  // The exchange runs over one channel per (owner part, requester engine):
  // a probe stream, the query/hit buffers and a cached `done` event on the
  // owner's device, so requesters never share a buffer, stream or lock.
  struct PartIO {
    hipStream_t stream = nullptr;
    uint8_t *q = nullptr;        // requester digests (n x 32), copied in
    ngpu_dict_hit *h = nullptr;  // this part's hits (n), copied back
    uint64_t cap = 0;
    hipEvent_t done = nullptr;   // recorded on `stream` after the hits copy back
  };
  struct Requester {
    uint64_t engine_uid = 0;
    int device = 0;
    hipEvent_t ready = nullptr;  // on the requester's device: its queries are packed
    std::vector<PartIO> io;      // one per owner part
    std::mutex mu;               // one exchange at a time per requester
  };
  std::vector<ngpu_dict *> parts;
  // one entry per engine that has exchanged through this dict (the node's
  // engines, normally W of them); freed with the dict
  std::vector<std::unique_ptr<Requester>> req;
  std::mutex req_mu;  // held only to find or add a requester
  bool replicated = false;
  bool routed = false;  // partitioned: routed exchange (peer kernels), else copy exchange
};

// One HBM workspace and its cross-stream ordering state.  Every stage that
// uses the workspace ends with an event on its stream (last_ev; null = not
// recorded yet, only while `last` is a stream that lives as long as the
// engine); a stage on another stream waits for it first, so calls on
// different streams never run over one workspace concurrently.  An engine
// keeps several (NGPU_WS_SLOTS, default 8, plus one of its own per batch lane,
// batch.hip): a call on a stream keeps the slot
// its stream used last (stream order is the ordering), a call on another
// stream takes an idle slot, so independent layers on different streams --
// containerd converting an image's layers concurrently -- run side by side
// on the GPU instead of queueing behind one workspace.
struct ngpu_ws_slot {
  ngpu::Workspace ws;
  hipEvent_t done = nullptr;     // stage-end event when no kernel carries one
  hipEvent_t last_ev = nullptr;  // the event that ended the last stage
  hipStream_t last = nullptr;    // stream of the last stage
  bool pending = false;          // a stage has been enqueued on this slot
  uint64_t *h_stats = nullptr;   // pinned: counters + layer stats read back
  uint64_t tick = 0;             // last use (LRU)
  char path[48] = "";            // digest kernels of its last digest stage (error messages)
  bool lane = false;             // one of the batch lanes' own slots (never taken by others)
  hipStream_t owner = nullptr;   // lane slot: the batch lane stream it belongs to
};

namespace ngpu {
constexpr int kBatchLanes = 4;  // concurrent batch lanes (batch.hip) = GPU_MAX_HW_QUEUES
struct Batcher;
struct BatchEvent;
// One pack's layer in a batch (batch.hip): its bytes and chunk table already
// in HBM / pinned host memory, where its results and stats go.
struct BatchJob {
  const uint8_t *d_data = nullptr;  // the layer's bytes in HBM (slot-relative chunk offsets)
  uint64_t len = 0;
  const ngpu_chunk *h_ch = nullptr;  // n descriptors (host)
  uint64_t n = 0;
  hipEvent_t ready = nullptr;        // d_data is complete after this event
  const ngpu_dict *dict = nullptr;
  void *h_res = nullptr;             // pinned (hipHostMalloc), n results, written by the batch
  uint64_t *h_stats = nullptr;       // pinned (hipHostMalloc), 32 words (read_stats_parse layout)
  int rc = 0;
  bool enqueued = false;
  uint32_t batch_layers = 0;         // layers in the launch set it joined
  int lane = 0;                      // the batch lane it ran on
  uint64_t seq = 0;                  // its batch's number (the lane's end marker)
  bool uncounted = false;            // taken: the leader took it out of e->batch_waitable
  char path[48] = "";                // the batch's digest kernels (error messages)
  std::shared_ptr<BatchEvent> done;
};
}  // namespace ngpu

struct ngpu_engine {
  std::atomic<int> refs{1};  // the creator + every open pack
  ngpu::Batcher *batcher = nullptr;  // concurrent small Packs' launch sets (batch.hip)
  hipMemPool_t seg_pool = nullptr;   // retained Pack segments (stream-ordered, own pool)
  // The packs' bulk copies go through a few shared engine streams, each
  // enqueued under its mutex: staging H2D on h2d[k], blob-window D2H on
  // d2h[k], pack k-th opened on lane k % kCopyLanes.  Measured on MI355X
  // (tools/h2d_streams, profiles/r5/h2d_streams_r5k4.jsonl): 32 streams
  // copying at once stall hipMemcpyAsync on the host for up to 46 ms and
  // carry 27 GB/s; 2 streams carry 45 GB/s with no call over 0.1 ms.
  static constexpr int kCopyLanes = 2;
  hipStream_t h2d[kCopyLanes] = {}, d2h[kCopyLanes] = {};
  std::mutex h2d_mu[kCopyLanes], d2h_mu[kCopyLanes];
  uint32_t copy_rr = 0;  // next pack's lane (e->mu)
  std::atomic<int> open_packs{0};    // packs opened and not yet ended
  // open packs that may still join a batch at close (one staging slot of tar
  // so far, not OCIRef, batching on): what a batch leader waits for
  std::atomic<int> batch_waitable{0};
  uint64_t uid = 0;          // unique for the process's lifetime (node exchange channels)
  ngpu_config cfg{};
  int device = 0;
  hipStream_t stream = nullptr;
  std::vector<ngpu_ws_slot> slots;  // fixed at create
  ngpu_ws_slot *cur = nullptr;      // the slot of the call being enqueued (e->mu held)
  uint64_t tick = 0;
  // streams that live as long as the engine (its own + every pack compute
  // stream): a stage on one of them may leave its end event unrecorded
  std::vector<hipStream_t> streams;  // guarded by mu
  ngpu_dict *dict = nullptr;              // default dict (one reference), may be null
  std::vector<ngpu_dict *> dict_cache;    // dicts opened by path (one reference each)
  // host-path device buffers
  uint8_t *d_data = nullptr;
  uint64_t d_data_cap = 0;
  ngpu_chunk *d_chunks = nullptr;
  ngpu_result *d_results = nullptr;
  uint64_t d_chunk_cap = 0;
  // pinned landing buffer of the host-buffer calls' result tables (copied to
  // the caller's pageable memory after the stream sync, as packs do with h_io)
  ngpu_result *h_results = nullptr;
  uint64_t h_results_cap = 0;
  // NGPU_FLAG_TIMING: a ring of per-call event sets (0 start, 1 digest start,
  // 2 digest end, 3 tree end, 4 end), so timing a call never makes the next
  // one wait: ngpu_timing_at reads any of the last kTimingRing calls.
  static constexpr int kTimingRing = 64;
  hipEvent_t ev[kTimingRing][5] = {};
  bool timed[kTimingRing] = {};
  int slot_D[kTimingRing] = {};
  bool slot_fused[kTimingRing] = {};  // planning inside the leaf kernel: digest from ev[0]
  uint64_t tcalls = 0;  // calls recorded so far; the current slot is (tcalls - 1) % ring
  int tslot = 0;
  // the digest stage that took ring entry tslot: a dedup stage on the same
  // workspace slot and stream completes that entry (ev[tslot][4]); any other
  // dedup stage records no timing (it must not re-record another stage's event)
  ngpu_ws_slot *tshare_slot = nullptr;
  hipStream_t tshare_stream = nullptr;
  bool tshare_open = false;
  hipEvent_t host_ev = nullptr;  // host_fence marker (system scope)
  std::vector<ngpu_staging_buf> staging_pool;  // guarded by pool_mu, <= kStagingPool
  // 128 packs open at once keep their two slots (bench.py --packs 128 with
  // 16 MiB slots); the pinned bytes kept are bounded too (64 default 256 MiB
  // slots would pin 16 GiB)
  static constexpr size_t kStagingPool = 256;
  static constexpr uint64_t kStagingPoolBytes = 8ull << 30;
  uint64_t staging_pool_bytes = 0;  // guarded by pool_mu
  std::vector<ngpu_pack_bufs> pack_pool;        // guarded by pool_mu
  // pinned landing buffers of early-emission Packs that did not come from the
  // staging pool (ngpu_pack_set_output): kept, not hipHostFree'd (~5 ms each)
  std::vector<std::pair<void *, uint64_t>> land_pool;  // guarded by pool_mu, <= kStagingPool
  std::mutex pool_mu;
  std::string err;
  std::mutex err_mu;  // fail() may run outside mu (a pack's blob stream)
  std::mutex mu;
};


namespace ngpu {

int fail(ngpu_engine *e, int code, const char *fmt, ...);
// Batched close of a small Pack (batch.hip): blocks until the batch it joined
// has run and its results / stats are in j.h_res / j.h_stats.
int batch_run(ngpu_engine *e, BatchJob &j);
void batch_stats(ngpu_engine *e, uint64_t out[3]);  // batches, layers, most layers in one
// A waiting batch leader re-checks its wait (e->batch_waitable went down).
void batch_wake(ngpu_engine *e);
Batcher *batcher_new();
void batcher_free(ngpu_engine *e);
// Pick the workspace slot for a stage on stream s and make it e->cur (e->mu
// held): the slot s used last, else an idle slot, else the least recently
// used one (ws_acquire then orders s after its last stage).
ngpu_ws_slot *use_slot(ngpu_engine *e, hipStream_t s);
int pick_group_log2(const ngpu_engine *e, uint64_t data_len);
int ensure_workspace(ngpu_engine *e, uint64_t n, uint64_t data_len, int D, uint32_t n_blobs,
                     uint64_t L);
// Host-wait until the current slot's last stage has finished (before any of
// its buffers is freed).
int slot_quiesce(ngpu_engine *e);
// chained: the caller enqueues the dedup stage next on the same stream (under
// the same lock), so the digest stage binds no end event (ws_lazy_end).
int enqueue_digest(ngpu_engine *e, const uint8_t *d_data, uint64_t len,
                   const ngpu_chunk *d_chunks, uint64_t n, ngpu_result *d_out, hipStream_t s,
                   bool chained = false);
// d_hits == nullptr: probe `dict` (may be null: no chunk dict).
// d_lfirst == nullptr: one layer of n chunks (stats -> internal lstats[0]).
int enqueue_dedup(ngpu_engine *e, const ngpu_dict *dict, const ngpu_chunk *d_chunks, uint64_t n,
                  ngpu_result *d_out, const ngpu_dict_hit *d_hits, uint32_t n_blobs,
                  hipStream_t s, const uint64_t *d_lfirst, uint64_t L, ngpu_layer_stats *d_stats);
// A system-scope release on s before the host reads device results (ev: a
// marker event of the caller's; null = the engine's, e->mu held).
int host_fence(ngpu_engine *e, hipStream_t s, hipEvent_t ev = nullptr);
// fenced: host_fence already recorded after the last kernel.
int read_stats(ngpu_engine *e, hipStream_t s, ngpu_layer_stats *st, bool fenced);
// The same in two halves, for callers that wait outside e->mu: enqueue the
// copies of the current slot's counters (kStWords) + layer stats (at
// kStatsLayer) into pinned h (32 words) on s (e->mu held); after s is
// synchronised, check and unpack them.
constexpr int kStatsLayer = 24;
int read_stats_enqueue(ngpu_engine *e, hipStream_t s, uint64_t *h);
int read_stats_parse(ngpu_engine *e, const uint64_t *h, ngpu_layer_stats *st,
                     const char *path = nullptr);
// Order a workspace stage on stream s after the previous one (any stream).
int ws_acquire(ngpu_engine *e, hipStream_t s);
// Digest then dedup on one stream (digest chained).
int enqueue_chain(ngpu_engine *e, const ngpu_dict *dict, const uint8_t *d_data, uint64_t len,
                  const ngpu_chunk *d_chunks, uint64_t n, ngpu_result *d_out, hipStream_t s,
                  const uint64_t *d_lfirst, uint64_t L, ngpu_layer_stats *d_stats);
// May the stage on s leave its end event unrecorded (chained, or s is the
// engine's own stream)?  ws_acquire records it when another stream needs it.
bool ws_lazy_end(const ngpu_engine *e, hipStream_t s, bool chained);
// bound: the stage-end event its last kernel records (null: record ws_done,
// or nothing when ws_lazy_end).
int ws_release(ngpu_engine *e, hipStream_t s, hipEvent_t bound, bool chained);

// Reference counts.  engine_unref frees the engine when the last holder (the
// creator's ngpu_destroy or the last open pack) lets go.
void engine_ref(ngpu_engine *e);
void engine_unref(ngpu_engine *e);
void dict_ref(ngpu_dict *d);
void dict_unref(ngpu_dict *d);
// A dict usable by engine e (same device, digester and chunk size), or an
// error message.
int dict_check(ngpu_engine *e, const ngpu_dict *d);
// The engine's default dict with one more reference (null if none).
ngpu_dict *default_dict(ngpu_engine *e);
inline uint32_t dict_blobs(const ngpu_dict *d) { return d ? d->dev.n_blobs : 0; }
uint64_t next_pow2(uint64_t x);
// From 80-B RAFS v6 records in host memory on engine e's device (own stream, no lock).
int dict_from_records(ngpu_engine *e, const uint8_t *recs, uint64_t m, const uint8_t *blobs,
                      uint32_t n_blobs, ngpu_dict **out, const uint32_t *gids);
int read_dict_bootstrap(ngpu_engine *e, const char *path, uint64_t file_size,
                        std::vector<uint8_t> *recs_out, std::vector<uint8_t> *blobs_out,
                        uint64_t *table_at = nullptr);
// Node dicts: the replica on e's device, or (partitioned) route the probe of
// n digests (byte stride) over the parts into e's workspace hits, ordered on
// stream s.  *hits = the per-chunk hits with global entry ids.
int node_dict_hits(ngpu_engine *e, ngpu_dict *d, const uint8_t *digests, uint64_t stride,
                   uint64_t n, hipStream_t s, const ngpu_dict_hit **hits, ngpu_dict **replica);

}  // namespace ngpu

#define HIP_TRY(e, call)                                                        \
  do {                                                                          \
    hipError_t _st = (call);                                                    \
    if (_st != hipSuccess)                                                      \
      return ::ngpu::fail((e), _st == hipErrorOutOfMemory ? NGPU_ENOMEM : NGPU_EHIP, \
                          "%s: %s (%s:%d)", #call, hipGetErrorString(_st), __FILE__, \
                          __LINE__);                                            \
  } while (0)
