// batch.hip — concurrent small Packs closed as ONE multi-layer launch set
// (VERDICT r4 item 3).
//
// The reference converts an image's layers concurrently, one goroutine and
// one nydus-image process per layer (pkg/converter/convert_unix.go:467-538,
// LayerConvertFunc :822).  Behind the ABI each of those layers is a Pack on
// one shared engine, and a small layer (C1: ~10 MB, a few dozen chunks)
// leaves most of the chip idle: its digest is bound by one chunk's chain (16
// compressions per BLAKE3 leaf + the tree levels; for SHA-256 the whole
// chunk, ~21 ms for 1 MiB), and at most GPU_MAX_HW_QUEUES (4) packs' kernels
// run side by side.  So Packs that close within a short window share one
// launch set: their layers' bytes are gathered into one HBM buffer (D2D),
// their chunk tables concatenated with layer boundaries, and ONE digest
// stage + ONE multi-layer dedup stage (the C5 path, per-layer semantics:
// every layer keeps its own intra-layer dict, NEW indices, offsets and blob
// order) decide them all; each pack gets its own results and stats back.
// Decisions are identical to one launch per pack (the multi-layer dedup is
// the per-layer algorithm with layer boundaries).
//
// Window: the first pack to close leads; it waits until every pack open on
// the engine has joined, or kWindowUs (SHA-256: kWindowShaUs), whichever
// comes first (a lone pack goes at once), and until one of the kLanes batch
// lanes is idle.  Batches on different lanes run concurrently (each lane: its
// own stream, buffers and workspace slot), so a small batch's chain latency
// -- a SHA-256 batch holds the device ~21 ms whatever its size -- does not
// hold the next one back.  Each pack's results and stats are written into
// its pinned read-back buffers by the lane's last two kernels.
// Only packs whose layer fit one staging slot join (their bytes are all in
// HBM at close); packs with another chunk dict than the leader's wait for
// the next batch.  NGPU_FLAG_NO_BATCH turns it off.
#include <algorithm>
#include <chrono>
#include <condition_variable>

#include "batch_lanes.hpp"
#include "batch_stats.hpp"
#include "engine_internal.hpp"

namespace ngpu {

// The end of one batch: every pack in it waits for this event, the last one
// to drop its reference destroys it.
struct BatchEvent {
  hipEvent_t ev = nullptr;
  int device = 0;
  ~BatchEvent() {
    if (ev) {
      DeviceGuard g(device);
      (void)hipEventDestroy(ev);
    }
  }
};

// One batch lane: a stream and the buffers of the batch running on it
// (reused batch after batch: a lane takes a new batch only when its last one
// has ended).
struct BatchLane {
  hipStream_t s = nullptr;
  double mark[6] = {};  // NGPU_BATCH_TRACE: launch_batch's steps (µs, batch_now_us)
  uint8_t *d_data = nullptr;
  uint64_t data_cap = 0;
  ngpu_chunk *d_ch = nullptr;
  uint64_t ch_cap = 0;
  ngpu_result *d_res = nullptr;
  uint64_t res_cap = 0;
  uint64_t *d_lfirst = nullptr;
  void **d_dst = nullptr;  // per layer: its pack's pinned results, then its pinned stats
  uint64_t dst_cap = 0;
  ngpu_layer_stats *d_lst = nullptr;
  uint64_t l_cap = 0, lst_cap = 0;
  uint8_t *h_tab = nullptr;  // pinned: chunk table + layer boundaries of one batch
  uint64_t h_cap = 0;
};

constexpr int kLanes = kBatchLanes;  // = GPU_MAX_HW_QUEUES: more lanes would share hardware queues

struct Batcher {
  std::mutex m;
  std::condition_variable cv;
  std::vector<BatchJob *> open;  // packs waiting for a batch
  bool leading = false;
  BatchLane lane[kLanes];
  LaneTable<kLanes> lanes;  // which lane is free (batch_lanes.hpp), under m
  uint64_t batches = 0, jobs = 0, max_jobs = 0;
};

static bool batch_trace_on();
static double batch_now_us();

namespace {

// One layer's results out of the batch: a multi-layer call numbers chunks
// across the whole call, so the chunk ids in NEW / INTRA `ref` fields are
// rebased to the layer's own (what the layer packed alone reports).  They go
// straight into each pack's pinned read-back buffer (mapped host memory), so
// a batch of K layers ends in two launches instead of 3K small D2H copies.
// One kernel for all layers: chunk i of the call belongs to layer k with
// lfirst[k] <= i < lfirst[k + 1] (binary search) and goes to dst[k][i - lfirst[k]].
__global__ void batch_results_out(const ngpu_result *__restrict__ src, uint64_t n,
                                  const uint64_t *__restrict__ lfirst, uint32_t K,
                                  ngpu_result *const *__restrict__ dst) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t lo = 0, hi = K;  // the last layer whose first chunk is <= i
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) / 2;
    if (lfirst[mid] <= i) lo = mid; else hi = mid;
  }
  const uint64_t base = lfirst[lo];
  ngpu_result r = src[i];
  if (r.kind == NGPU_NEW || r.kind == NGPU_INTRA) r.ref -= base;
  dst[lo][i - base] = r;
}

// The batch's inputs in ONE launch (row y = blockIdx.y): rows 0..K-1 copy the
// layers' staged bytes into the lane buffer, the last rows the host-built
// tables (chunk table, layer firsts, result pointers) straight from mapped
// pinned memory.  32+ hipMemcpyAsync calls per batch stalled the leader's
// enqueue for ~8 ms on every other round (NGPU_BATCH_TRACE steps, r5tr): the
// copy engines are busy with the next packs' H2D.  A row's bytes move in
// 16-B words when both ends are 16-B aligned, else bytewise.
struct GatherRow {
  const uint8_t *src;
  uint8_t *dst;
  uint64_t len;
};

__global__ __launch_bounds__(256) void batch_gather(const GatherRow *__restrict__ rows) {
  const GatherRow r = rows[blockIdx.y];
  const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t head = 0;
  if ((((uintptr_t)r.src | (uintptr_t)r.dst) & 15) == 0) {
    const uint64_t w = r.len / 16;
    const uint4 *s4 = reinterpret_cast<const uint4 *>(r.src);
    uint4 *d4 = reinterpret_cast<uint4 *>(r.dst);
    for (uint64_t i = t; i < w; i += stride) d4[i] = s4[i];
    head = w * 16;
  }
  for (uint64_t i = head + t; i < r.len; i += stride) r.dst[i] = r.src[i];
}

constexpr int kWindowUs = 250;
// SHA-256: a batch holds its lane for one 1 MiB chunk's chain (~21 ms)
// whatever its size, so a longer wait for more packs costs < 10 % of that and
// saves a whole chain time for every pack it adds (32 C1 packs closing over
// ~3 ms went out as 4-5 batches in 250 µs windows).
constexpr int kWindowShaUs = 2000;
// ... and each pack that joins restarts it, up to this much after the lead:
// 32 C1 packs join over ~7 ms behind the shared H2D lanes, so a fixed 2 ms
// window split them into 2-4 batches whose chains did not overlap
// (37-42 ms a round against one chain's 21 ms)
constexpr int kWindowShaCapUs = 12000;
constexpr size_t kMaxJobs = 256;
constexpr uint64_t kMaxBytes = 2ull << 30;  // a lane buffer (4 lanes: 8 GiB of HBM at most)
constexpr uint64_t kMaxChunks = 1ull << 20;
// a lane's buffers and workspace start at these sizes (4 lanes: ~1.1 GiB of HBM)
constexpr uint64_t kLaneBytesMin = 256ull << 20;
constexpr uint64_t kLaneChunksMin = 1ull << 16;

// A lane buffer of at least `want` elements (powers of two).  Stream-ordered
// on the lane's own stream from the engine's pool: hipFree would wait for the
// whole device -- every other lane's running batch and every pack's copies --
// under the engine lock.
template <class T>
int grow_dev(ngpu_engine *e, hipStream_t s, T **p, uint64_t &cap, uint64_t want) {
  if (want <= cap && *p) return 0;  // (the lane is idle: its last batch has ended)
  if (*p) (void)hipFreeAsync(*p, s), *p = nullptr, cap = 0;
  uint64_t c = 4096;
  while (c < want) c *= 2;
  const hipError_t r = e->seg_pool ? hipMallocFromPoolAsync((void **)p, c * sizeof(T), e->seg_pool, s)
                                   : hipMallocAsync((void **)p, c * sizeof(T), s);
  if (r != hipSuccess) {
    (void)hipGetLastError();
    *p = nullptr;
    return fail(e, NGPU_ENOMEM, "batch: device buffer allocation failed");
  }
  cap = c;
  return 0;
}

// (A batch's end is seen by the first of its packs whose hipEventSynchronize
// returns, batch_run, not by polling: hipEventQuery on an event other threads
// synchronize on blocked for the whole batch, ~30 ms for SHA-256; HIP API
// trace, profiles/r5/pack_api_trace_r5j.md.)

// Enqueue one batch on an idle lane (the leader, e->mu taken here).
int launch_batch(ngpu_engine *e, BatchLane &b, const std::vector<BatchJob *> &jobs) {
  const bool tr = batch_trace_on();
  std::lock_guard<std::mutex> g(e->mu);
  if (tr) b.mark[0] = batch_now_us();
  DeviceGuard dg(e->device);
  if (!b.s) {
    HIP_TRY(e, hipStreamCreateWithFlags(&b.s, hipStreamNonBlocking));
    e->streams.push_back(b.s);  // lives as long as the engine (ws_lazy_end)
    for (auto &sl : e->slots)   // the lane's own workspace slot
      if (sl.lane && !sl.owner) {
        sl.owner = b.s;
        break;
      }
  }
  const uint64_t K = jobs.size();
  std::vector<uint64_t> off(K), first(K + 1, 0);
  uint64_t bytes = 0;
  for (uint64_t k = 0; k < K; ++k) {
    off[k] = bytes;
    bytes += (jobs[k]->len + 255) & ~255ull;
    first[k + 1] = first[k] + jobs[k]->n;
  }
  const uint64_t N = first[K];
  // floors: batches vary in size from one to the next, and each regrowth (or
  // workspace growth below) held a leader's enqueue for 1-8 ms (r5g3 trace)
  if (int rc = grow_dev(e, b.s, &b.d_data, b.data_cap, std::max<uint64_t>(bytes + 64, kLaneBytesMin))) return rc;
  if (int rc = grow_dev(e, b.s, &b.d_ch, b.ch_cap, std::max<uint64_t>(N + 1, kLaneChunksMin))) return rc;
  if (int rc = grow_dev(e, b.s, &b.d_res, b.res_cap, std::max<uint64_t>(N + 1, kLaneChunksMin))) return rc;
  if (int rc = grow_dev(e, b.s, &b.d_lfirst, b.l_cap, K + 2)) return rc;
  if (int rc = grow_dev(e, b.s, &b.d_lst, b.lst_cap, K + 2)) return rc;
  if (int rc = grow_dev(e, b.s, &b.d_dst, b.dst_cap, 2 * K + 2)) return rc;
  const uint64_t tab_data = N * sizeof(ngpu_chunk) + (K + 1) * sizeof(uint64_t) + 2 * K * sizeof(void *);
  const uint64_t rows_at = (tab_data + 15) & ~15ull;
  const uint64_t tab = rows_at + (K + 3) * sizeof(GatherRow);
  if (tab > b.h_cap) {
    if (b.h_tab) (void)hipHostFree(b.h_tab), b.h_tab = nullptr, b.h_cap = 0;
    uint64_t c = 4 << 20;
    while (c < tab) c *= 2;
    HIP_TRY(e, hipHostMalloc((void **)&b.h_tab, c, hipHostMallocDefault));
    b.h_cap = c;
  }
  ngpu_chunk *hc = reinterpret_cast<ngpu_chunk *>(b.h_tab);
  for (uint64_t k = 0; k < K; ++k)
    for (uint64_t i = 0; i < jobs[k]->n; ++i) {
      ngpu_chunk c = jobs[k]->h_ch[i];
      c.offset += off[k];
      hc[first[k] + i] = c;
    }
  memcpy(b.h_tab + N * sizeof(ngpu_chunk), first.data(), (K + 1) * sizeof(uint64_t));
  void **hd = reinterpret_cast<void **>(b.h_tab + N * sizeof(ngpu_chunk) + (K + 1) * sizeof(uint64_t));
  for (uint64_t k = 0; k < K; ++k) {  // the packs' pinned buffers as the device sees them
    HIP_TRY(e, hipHostGetDevicePointer(&hd[k], jobs[k]->h_res, 0));
    HIP_TRY(e, hipHostGetDevicePointer(&hd[K + k], jobs[k]->h_stats, 0));
  }
  if (tr) b.mark[1] = batch_now_us();
  // gather: every layer's bytes behind its own copy, and the tables, in one
  // launch (batch_gather)
  uint8_t *tab_dev = nullptr;  // h_tab as the device sees it
  HIP_TRY(e, hipHostGetDevicePointer((void **)&tab_dev, b.h_tab, 0));
  GatherRow *rows = reinterpret_cast<GatherRow *>(b.h_tab + rows_at);
  uint64_t most = 0;
  for (uint64_t k = 0; k < K; ++k) {
    HIP_TRY(e, hipStreamWaitEvent(b.s, jobs[k]->ready, 0));
    rows[k] = GatherRow{jobs[k]->d_data, b.d_data + off[k], jobs[k]->len};
    most = std::max(most, jobs[k]->len);
  }
  rows[K] = GatherRow{tab_dev, reinterpret_cast<uint8_t *>(b.d_ch), N * sizeof(ngpu_chunk)};
  rows[K + 1] = GatherRow{tab_dev + N * sizeof(ngpu_chunk), reinterpret_cast<uint8_t *>(b.d_lfirst),
                          (K + 1) * sizeof(uint64_t)};
  rows[K + 2] = GatherRow{tab_dev + N * sizeof(ngpu_chunk) + (K + 1) * sizeof(uint64_t),
                          reinterpret_cast<uint8_t *>(b.d_dst), 2 * K * sizeof(void *)};
  most = std::max(most, N * sizeof(ngpu_chunk));
  // blocks per row: one 16-B word per thread per pass, at most 1,024 blocks
  const uint64_t bx = std::min<uint64_t>(1024, std::max<uint64_t>(1, (most / 16 + 255) / 256));
  hipLaunchKernelGGL(batch_gather, dim3((unsigned)bx, (unsigned)(K + 3)), dim3(256), 0, b.s,
                     reinterpret_cast<const GatherRow *>(tab_dev + rows_at));
  HIP_TRY(e, hipGetLastError());
  if (tr) b.mark[2] = batch_now_us();
  // the lane's own workspace sized with headroom (powers of two), so batches
  // of varying size seldom regrow it
  {
    use_slot(e, b.s);
    const uint64_t n2 = next_pow2(std::max<uint64_t>(N + 1, kLaneChunksMin)),
                   len2 = next_pow2(std::max<uint64_t>(bytes + 1, kLaneBytesMin));
    if (int rc = ensure_workspace(e, n2, len2, pick_group_log2(e, bytes), dict_blobs(jobs[0]->dict),
                                  next_pow2(K)))
      return rc;
    // the slot is this lane's now (the digest below finds it by its stream)
    if (int rc = ws_acquire(e, b.s)) return rc;
    if (int rc = ws_release(e, b.s, nullptr, true)) return rc;
  }
  if (tr) b.mark[3] = batch_now_us();
  // ONE digest stage over all layers, ONE multi-layer dedup stage
  if (int rc = enqueue_digest(e, b.d_data, bytes, b.d_ch, N, b.d_res, b.s, true)) return rc;
  if (tr) b.mark[4] = batch_now_us();
  if (int rc = enqueue_dedup(e, jobs[0]->dict, b.d_ch, N, b.d_res, nullptr, 0, b.s, b.d_lfirst, K,
                             b.d_lst)) {
    (void)ws_release(e, b.s, nullptr, false);
    return rc;
  }
  if (tr) b.mark[5] = batch_now_us();
  // each pack's results (chunk ids rebased to its layer) and stats, into its
  // pinned read-back buffers
  const ngpu_ws_slot &sl = *e->cur;
  if (N) {
    hipLaunchKernelGGL(batch_results_out, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, b.s,
                       b.d_res, N, b.d_lfirst, (uint32_t)K, reinterpret_cast<ngpu_result **>(b.d_dst));
    HIP_TRY(e, hipGetLastError());
  }
  // (each layer's own error words: batch_stats.hpp)
  hipLaunchKernelGGL(batch_stats_out, dim3((unsigned)K), dim3(256), 0, b.s, sl.ws.stats, b.d_lst,
                     b.d_res, b.d_lfirst, reinterpret_cast<uint64_t **>(b.d_dst + K));
  HIP_TRY(e, hipGetLastError());
  if (int rc = host_fence(e, b.s)) return rc;
  for (uint64_t k = 0; k < K; ++k) snprintf(jobs[k]->path, sizeof jobs[k]->path, "%s", sl.path);
  auto done = std::make_shared<BatchEvent>();
  done->device = e->device;
  HIP_TRY(e, hipEventCreateWithFlags(&done->ev, hipEventDisableTiming));
  HIP_TRY(e, hipEventRecord(done->ev, b.s));
  for (BatchJob *j : jobs) {
    j->done = done;
    j->batch_layers = (uint32_t)K;
  }
  return 0;
}

}  // namespace

// NGPU_BATCH_TRACE=1: one line per launch set on stderr (diagnostic): when
// its leader arrived, stopped waiting and had it enqueued, the layers it took
// and how many packs were open, microseconds since the engine's first batch.
static bool batch_trace_on() {
  static const bool on = [] {
    const char *v = getenv("NGPU_BATCH_TRACE");
    return v && *v == '1';
  }();
  return on;
}

static double batch_now_us() {
  static const auto t0 = std::chrono::steady_clock::now();
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
}

int batch_run(ngpu_engine *e, BatchJob &j) {
  Batcher &b = *e->batcher;
  std::unique_lock<std::mutex> lk(b.m);
  b.open.push_back(&j);
  b.cv.notify_all();  // a leader waiting for more packs
  while (!j.enqueued) {
    if (b.leading) {
      b.cv.wait(lk);
      continue;
    }
    b.leading = true;
    const double t_lead = batch_trace_on() ? batch_now_us() : 0;
    // wait for the open packs to join -- until all have, or kWindowUs has
    // passed -- and for an idle lane (while every lane runs a batch, a new
    // one would only queue behind them: better to let more packs join it)
    const bool sha = e->cfg.digester == NGPU_DIGEST_SHA256;
    const auto t0 = std::chrono::steady_clock::now();
    const auto window = std::chrono::microseconds(sha ? kWindowShaUs : kWindowUs);
    const auto cap = t0 + std::chrono::microseconds(sha ? kWindowShaCapUs : kWindowUs);
    auto until = t0 + window;
    size_t joined = b.open.size();
    int ln = -1;
    for (;;) {
      ln = b.lanes.idle();
      // every pack that may still join has (packs already in a running
      // batch, grown past one slot, OCIRef or closing alone are not counted)
      const bool all_in = (int)b.open.size() >= e->batch_waitable.load() || b.open.size() >= kMaxJobs;
      if (sha && b.open.size() > joined) {  // a pack joined: restart the window
        joined = b.open.size();
        until = std::min(cap, std::chrono::steady_clock::now() + window);
      }
      if (ln >= 0 && (all_in || std::chrono::steady_clock::now() >= until)) break;
      if (ln >= 0)
        b.cv.wait_until(lk, until);
      else
        b.cv.wait(lk);  // a lane's end (batch_run) or a new pack wakes it
    }
    const uint64_t seq = b.lanes.take(ln);  // under b.m (batch_lanes.hpp: why)
    // this leader's batch: the open packs sharing its dict, within the caps
    std::vector<BatchJob *> take;
    uint64_t bytes = 0, chunks = 0;
    for (size_t i = 0; i < b.open.size();) {
      BatchJob *x = b.open[i];
      const bool fits = take.size() < kMaxJobs && bytes + x->len <= kMaxBytes &&
                        chunks + x->n <= kMaxChunks;
      if (x->dict == j.dict && (fits || x == &j)) {
        take.push_back(x);
        bytes += x->len;
        chunks += x->n;
        b.open.erase(b.open.begin() + (long)i);
      } else {
        ++i;
      }
    }
    for (BatchJob *x : take) x->uncounted = true;  // (read by its pack after `enqueued`)
    e->batch_waitable.fetch_sub((int)take.size());
    const int open_now = e->open_packs.load();
    lk.unlock();
    const double t_take = batch_trace_on() ? batch_now_us() : 0;
    for (BatchJob *x : take) {  // (read by their packs only after `enqueued`, under b.m)
      x->lane = ln;
      x->seq = seq;
    }
    const int rc = launch_batch(e, b.lane[ln], take);
    if (batch_trace_on())
      fprintf(stderr, "{\"batch_trace\": %llu, \"lane\": %d, \"lead_us\": %.1f, \"take_us\": %.1f, "
              "\"enqueued_us\": %.1f, \"layers\": %zu, \"open_packs\": %d, \"rc\": %d, "
              "\"steps_us\": [%.1f, %.1f, %.1f, %.1f, %.1f, %.1f]}\n",
              (unsigned long long)seq, ln, t_lead, t_take, batch_now_us(), take.size(), open_now, rc,
              b.lane[ln].mark[0], b.lane[ln].mark[1], b.lane[ln].mark[2], b.lane[ln].mark[3],
              b.lane[ln].mark[4], b.lane[ln].mark[5]);
    if (rc && b.lane[ln].s) {  // part of it may be enqueued: let it drain before the packs free their buffers
      DeviceGuard dg(e->device);
      (void)hipStreamSynchronize(b.lane[ln].s);
    }
    lk.lock();
    if (rc) {
      b.lanes.drop(ln);  // drained above
    } else {
      ++b.batches;
      b.jobs += take.size();
      b.max_jobs = std::max<uint64_t>(b.max_jobs, take.size());
    }
    for (BatchJob *x : take) {
      x->rc = rc;
      x->enqueued = true;
    }
    b.leading = false;
    b.cv.notify_all();
  }
  lk.unlock();
  if (j.rc) return j.rc;
  DeviceGuard dg(e->device);
  const bool ok = hipEventSynchronize(j.done->ev) == hipSuccess;
  {
    std::lock_guard<std::mutex> g(b.m);  // the first pack back frees the lane for the next leader
    if (b.lanes.end(j.lane, j.seq)) b.cv.notify_all();
  }
  if (!ok) return fail(e, NGPU_EHIP, "batch: stream failed");
  return 0;
}

void batch_wake(ngpu_engine *e) {
  if (!e->batcher) return;
  std::lock_guard<std::mutex> g(e->batcher->m);
  e->batcher->cv.notify_all();
}

void batch_stats(ngpu_engine *e, uint64_t out[3]) {
  out[0] = out[1] = out[2] = 0;
  if (!e->batcher) return;
  std::lock_guard<std::mutex> g(e->batcher->m);
  out[0] = e->batcher->batches;
  out[1] = e->batcher->jobs;
  out[2] = e->batcher->max_jobs;
}

void batcher_free(ngpu_engine *e) {
  Batcher *b = e->batcher;
  if (!b) return;
  DeviceGuard dg(e->device);
  for (BatchLane &l : b->lane) {
    if (!l.s) continue;  // (a lane that never ran has no buffers)
    for (void *p : {(void *)l.d_data, (void *)l.d_ch, (void *)l.d_res, (void *)l.d_lfirst,
                    (void *)l.d_lst, (void *)l.d_dst})
      if (p) (void)hipFreeAsync(p, l.s);
    (void)hipStreamSynchronize(l.s);
    if (l.h_tab) (void)hipHostFree(l.h_tab);
    // l.s is one of e->streams: destroyed with them
  }
  delete b;
  e->batcher = nullptr;
}

Batcher *batcher_new() { return new Batcher(); }

}  // namespace ngpu
