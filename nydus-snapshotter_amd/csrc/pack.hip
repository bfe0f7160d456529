// pack.hip — streaming Pack writer: the in-process replacement for the
// FIFO + `nydus-image create` pair behind converter.Pack
// (pkg/converter/convert_unix.go:325-362, packFromTar :443-539).
//
// Pack returns an io.WriteCloser in the reference; here ngpu_pack_write (or
// the zero-copy ngpu_pack_reserve / ngpu_pack_commit pair) accepts the
// uncompressed layer tar in any split and ngpu_pack_close returns the chunk
// list and per-chunk digests + dedup decisions.
//
// Pipeline (two staging slots):
//   host bytes -> pinned slot (raw tar stream; the incremental TarScanner
//   records chunks as they start) -> when a slot is full, every chunk that
//   ends inside it is dispatched: hipMemcpyAsync H2D on a copy stream, then
//   the digest kernels on the engine stream write digests straight into the
//   layer's device result array.  The bytes of the one chunk still in
//   progress are carried to the front of the other slot, so every chunk is
//   contiguous in exactly one slot.  While slot A is copied and hashed the
//   caller fills slot B.  Dedup needs stream order over the whole layer, so it
//   runs once at close over the device-resident digests.
//
// NGPU_PACK_RETAIN (ngpu_pack_finish): each slot is
// copied into its own device segment that stays resident until the end (the
// whole layer lives in HBM), so after dedup the NEW chunks are gathered on the
// GPU into window buffers in blob (index) order and only those bytes cross
// PCIe, window k+1's gather + D2H overlapping the host compression of window k
// (blob.cpp BlobWriter).
//
// ngpu_pack_set_output (early emission): with the output
// known when the Pack opens (converter.Pack's `dest`, convert_unix.go:325), an
// emitter thread writes the blob stream while the caller is still writing the
// tar.  A chunk's decision depends only on the chunks before it (stream order),
// so after each staging slot is digested the emitter dedups the whole prefix
// dispatched so far and the NEW chunks of the new part are final: they are
// gathered, copied back and handed to the BlobWriter, whose sequential
// SHA-256 -- the bound of converter.Pack end to end -- then runs alongside the
// H2D copies and digests of the rest of the layer instead of after them.
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "blob.hpp"
#include "engine_internal.hpp"
#include "tarstream.hpp"
#include "zran.hpp"

using namespace ngpu;

extern "C" const char *ngpu_host_error(void);

namespace {

struct Slot {
  uint8_t *h = nullptr;       // pinned raw stream bytes
  uint8_t *d = nullptr;       // device copy
  ngpu_chunk *h_ch = nullptr; // pinned slot-relative descriptors
  ngpu_chunk *d_ch = nullptr;
  uint64_t base = 0, fill = 0;
  uint64_t sent = 0;          // bytes [0, sent) already queued H2D (eager copies)
  hipEvent_t copied = nullptr, done = nullptr;
  bool busy = false;
};

// A retained device copy of one dispatched slot (NGPU_PACK_RETAIN).
struct Seg {
  uint8_t *d = nullptr;
  uint64_t base = 0;     // stream offset of d[0]
  uint64_t a = 0, b = 0; // chunks [a, b) live here
};

// Early emission state (ngpu_pack_set_output).  ch / dptr / avail / deduped
// are guarded by the engine lock (dispatch appends under it); emitted and rc
// belong to the emitter thread until it is joined.
struct Emit {
  ngpu_blob_options opt{};
  std::string prefetch;
  std::unique_ptr<BlobWriter> bw;
  std::vector<ngpu_chunk> ch;    // dispatched chunks (stream offsets)
  std::vector<uint64_t> dptr;    // device address of each dispatched chunk's bytes
  uint64_t avail = 0;            // chunks dispatched
  uint64_t deduped = 0;          // prefix covered by the last dedup stage (remarked before the next)
  uint64_t emitted = 0;          // chunks whose NEW bytes went to the writer
  uint64_t new_emitted = 0;      // NEW chunks among them
  std::atomic<uint64_t> hint{0}; // = avail, for the emitter's wait
  std::atomic<int> rc{0};
  std::thread th;
  std::mutex m;
  std::condition_variable cv;
  bool stop = false;
  ngpu_result *h_res = nullptr;  // pinned landing of the prefix results
  uint64_t h_cap = 0;
  uint64_t *h_stats = nullptr;   // pinned: the prefix stage's counters (digest guard)
  hipEvent_t ev = nullptr;
  ngpu_staging_buf land[2];      // pinned landing of the blob windows (engine staging pool)
};

// Copies chunk k (src[k], len[k] bytes) to dst + doff[k] (16-B aligned).
// One workgroup per chunk, grid-stride over chunks.
__global__ __launch_bounds__(256) void gather_chunks(const uint64_t *__restrict__ src,
                                                     const uint32_t *__restrict__ len,
                                                     const uint64_t *__restrict__ doff,
                                                     uint64_t count, uint8_t *__restrict__ dst) {
  for (uint64_t k = blockIdx.x; k < count; k += gridDim.x) {
    const uint8_t *s = reinterpret_cast<const uint8_t *>(src[k]);
    uint8_t *d = dst + doff[k];
    const uint32_t n = len[k];
    uint32_t done = 0;
    if ((reinterpret_cast<uintptr_t>(s) & 15) == 0) {
      const uint32_t v = n >> 4;
      const uint4 *s4 = reinterpret_cast<const uint4 *>(s);
      uint4 *d4 = reinterpret_cast<uint4 *>(d);
      for (uint32_t i = threadIdx.x; i < v; i += blockDim.x) d4[i] = s4[i];
      done = v << 4;
    }
    for (uint32_t i = done + threadIdx.x; i < n; i += blockDim.x) d[i] = s[i];
  }
}

// A few persistent threads that split large host copies into the pinned
// staging slot (one memcpy thread tops out well below PCIe Gen5 H2D).
class CopyPool {
 public:
  explicit CopyPool(unsigned n) {
    for (unsigned i = 0; i < n; ++i) th_.emplace_back([this] { work(); });
  }
  ~CopyPool() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto &t : th_) t.join();
  }
  unsigned size() const { return (unsigned)th_.size(); }
  void copy(uint8_t *dst, const uint8_t *src, uint64_t n) {
    const unsigned parts = size() + 1;
    const uint64_t step = ((n + parts - 1) / parts + 4095) & ~4095ull;
    std::unique_lock<std::mutex> g(m_);
    for (uint64_t off = step; off < n; off += step)
      jobs_.push_back({dst + off, src + off, off + step < n ? step : n - off});
    pending_ = jobs_.size();
    g.unlock();
    cv_.notify_all();
    memcpy(dst, src, step < n ? step : n);  // the caller takes the first part
    g.lock();
    done_.wait(g, [this] { return pending_ == 0; });
  }

 private:
  struct Job { uint8_t *dst; const uint8_t *src; uint64_t n; };
  void work() {
    std::unique_lock<std::mutex> g(m_);
    for (;;) {
      cv_.wait(g, [this] { return stop_ || !jobs_.empty(); });
      if (stop_) return;
      Job j = jobs_.back();
      jobs_.pop_back();
      g.unlock();
      memcpy(j.dst, j.src, j.n);
      g.lock();
      if (--pending_ == 0) done_.notify_all();
    }
  }
  std::vector<std::thread> th_;
  std::vector<Job> jobs_;
  uint64_t pending_ = 0;
  bool stop_ = false;
  std::mutex m_;
  std::condition_variable cv_, done_;
};

}  // namespace

struct ngpu_pack : TarSink {
  ngpu_engine *e = nullptr;    // one reference, dropped when the pack ends
  ngpu_dict *dict = nullptr;   // the chunk dict it dedups against (one reference)
  const volatile int32_t *cancel = nullptr;  // caller-owned cancel flag
  TarScanner sc;
  Slot slot[2];
  int cur = 0;
  uint64_t cap = 0, max_ch = 0;
  std::vector<ngpu_chunk> chunks;  // stream offsets
  uint64_t dispatched = 0;
  ngpu_result *d_res = nullptr;
  uint64_t res_cap = 0;
  ngpu_chunk *d_all = nullptr;
  uint64_t all_cap = 0;
  hipStream_t copy = nullptr;    // shared H2D lane (engine h2d[k]), enqueued under *copy_mu
  std::mutex *copy_mu = nullptr;
  hipStream_t d2h = nullptr;     // shared D2H lane (engine d2h[k]), enqueued under *d2h_mu
  std::mutex *d2h_mu = nullptr;
  hipStream_t stream = nullptr;  // compute: digest, dedup, gather (lives as long as the engine)
  hipEvent_t fence = nullptr;    // host_fence marker of this pack
  uint64_t *h_stats = nullptr;   // pinned: its stats, read after the engine lock is let go
  uint8_t *h_io = nullptr;       // pinned staging of the chunk table / results at close
  uint64_t io_cap = 0;
  BlobWindows win;           // blob stream gather windows (kept by the engine's pack_pool)
  CopyPool *pool = nullptr;  // created on the first large write
  bool retain = false;       // NGPU_PACK_RETAIN: device segments kept to the end
  bool ws_sized = false;     // its stream's workspace sized for a whole slot (first digest)
  std::vector<Seg> segs;
  // NGPU_PACK_RETAIN: the segments are carved out of arenas that double in
  // size (1 slot, 2, 4, ... up to 1 GiB): a 2 GiB layer frees 6 arenas at the end
  // instead of 32 slot-sized segments (~0.17 ms per free)
  struct Arena { uint8_t *d = nullptr; uint64_t cap = 0, used = 0; };
  std::vector<Arena> arenas;
  std::vector<TarEntry> entries;  // NGPU_PACK_RETAIN: the tar's entries (the bootstrap's inode tree)
  Emit *em = nullptr;              // ngpu_pack_set_output: the stream leaves while the tar arrives
  std::unique_ptr<GzipIndexer> gz; // NGPU_PACK_OCIREF: the gzip blob is inflated and indexed
  // counted in e->batch_waitable: it may still join a batch at its close, so
  // a batch leader waits for it (batch.hip)
  bool waitable = false;
  int err = 0;

  std::chrono::steady_clock::time_point born = std::chrono::steady_clock::now();

  explicit ngpu_pack(ngpu_engine *eng) : e(eng), sc(eng->cfg.chunk_size) {}

  int chunk(uint64_t off, uint32_t len, uint32_t fi, uint64_t fo) override {
    chunks.push_back(ngpu_chunk{off, len, fi, fo});
    return 0;
  }
  int data(const uint8_t *, uint64_t) override { return 0; }  // bytes already in the slot
};

namespace {

// NGPU_PACK_TRACE=1: phase timestamps of a Pack's close, on stderr (diagnostic)
void ptrace(const ngpu_pack *p, const char *what) {
  static const bool on = [] {
    const char *v = getenv("NGPU_PACK_TRACE");
    return v && *v == '1';
  }();
  if (!on) return;
  const double t = std::chrono::duration<double>(std::chrono::steady_clock::now() - p->born).count();
  fprintf(stderr, "{\"pack_trace\": \"%s\", \"t_s\": %.4f}\n", what, t);
}

bool cancelled(const ngpu_pack *p) {
  return p->cancel && __atomic_load_n(p->cancel, __ATOMIC_RELAXED) != 0;
}

// The pack can no longer join a batch (its layer outgrew one staging slot, it
// closes outside one, or it ends): a leader stops waiting for it.
void not_waitable(ngpu_pack *p) {
  if (!p->waitable) return;
  p->waitable = false;
  p->e->batch_waitable.fetch_sub(1);
  batch_wake(p->e);
}

void emit_stop(ngpu_pack *p);  // below

void release(ngpu_pack *p) {
  if (!p) return;
  ngpu_engine *e = p->e;
  ngpu_dict *dict = p->dict;
  DeviceGuard dg(e->device);
  ptrace(p, "release");
  not_waitable(p);
  emit_stop(p);
  // the stream's writer goes first: its sink may still hold raw pieces of the
  // pinned staging slots (src_stable, emit_range_host) until it has drained
  if (p->em) p->em->bw.reset();
  for (Slot &s : p->slot) {
    if (s.done) (void)hipEventSynchronize(s.done);
  }
  if (p->copy) {  // this pack's copies on its shared lane: everything enqueued before this marker
    hipEvent_t m = p->slot[0].copied;
    bool marked = false;
    if (m) {
      std::lock_guard<std::mutex> g(*p->copy_mu);
      marked = hipEventRecord(m, p->copy) == hipSuccess;
    }
    (void)(marked ? hipEventSynchronize(m) : hipStreamSynchronize(p->copy));
  }
  if (p->stream) (void)hipStreamSynchronize(p->stream);
  ptrace(p, "release_synced");
  {
    std::lock_guard<std::mutex> g(p->e->pool_mu);
    for (Slot &s : p->slot) {
      if (!s.h || !s.h_ch || !s.d_ch || !s.copied || !s.done ||
          p->e->staging_pool.size() >= ngpu_engine::kStagingPool ||
          p->e->staging_pool_bytes + p->cap > ngpu_engine::kStagingPoolBytes)
        continue;
      p->e->staging_pool.push_back({s.h, s.h_ch, s.d, s.d_ch, s.copied, s.done, p->cap});
      p->e->staging_pool_bytes += p->cap;
      s = Slot{};
    }
  }
  for (Slot &s : p->slot) {
    if (s.h) (void)hipHostFree(s.h);
    if (s.h_ch) (void)hipHostFree(s.h_ch);
    if (s.d) (void)hipFree(s.d);
    if (s.d_ch) (void)hipFree(s.d_ch);
    if (s.copied) (void)hipEventDestroy(s.copied);
    if (s.done) (void)hipEventDestroy(s.done);
  }
  for (ngpu_pack::Arena &ar : p->arenas) (void)hipFreeAsync(ar.d, p->stream);  // the streams are idle
  ptrace(p, "release_segments");
  if (Emit *em = p->em) {  // its landing buffers go back to the staging pool
    std::lock_guard<std::mutex> g(e->pool_mu);
    for (ngpu_staging_buf &b : em->land) {
      if (!b.h) continue;
      const bool whole = b.h_ch && b.d_ch && b.copied && b.done;  // a pool entry (else: own landing)
      if (whole && e->staging_pool.size() < ngpu_engine::kStagingPool &&
          e->staging_pool_bytes + b.cap <= ngpu_engine::kStagingPoolBytes) {
        e->staging_pool.push_back(b);
        e->staging_pool_bytes += b.cap;
      } else if (!whole && !b.d && e->land_pool.size() < ngpu_engine::kStagingPool) {
        e->land_pool.push_back({b.h, b.cap});  // an own landing: kept for the next Pack
      } else {
        (void)hipHostFree(b.h);
        if (b.h_ch) (void)hipHostFree(b.h_ch);
        if (b.d) (void)hipFree(b.d);
        if (b.d_ch) (void)hipFree(b.d_ch);
        if (b.copied) (void)hipEventDestroy(b.copied);
        if (b.done) (void)hipEventDestroy(b.done);
      }
      b = ngpu_staging_buf{};
    }
  }
  ptrace(p, "release_landing");
  if (Emit *em = p->em) {
    if (em->h_res) (void)hipHostFree(em->h_res);
    if (em->h_stats) (void)hipHostFree(em->h_stats);
    if (em->ev) (void)hipEventDestroy(em->ev);
    delete em;
    p->em = nullptr;
    ptrace(p, "release_writer_gone");
  }
  {
    // the streams are idle (synchronised above).  Every compute stream goes
    // back to the pool: the engine's workspace slots may still name it as
    // the stream of their last stage (ws_lazy_end), so it lives until the
    // engine does.  The pool holds as many as packs were ever open at once.
    std::lock_guard<std::mutex> g(p->e->pool_mu);
    if (p->stream) {
      p->e->pack_pool.push_back({p->stream, p->fence, p->h_stats, p->h_io, p->io_cap,
                                 p->d_res, p->res_cap, p->d_all, p->all_cap, p->win});
      p->win = BlobWindows{};
      p->h_io = nullptr;
      p->stream = nullptr;
      p->fence = nullptr;
      p->h_stats = nullptr;
      p->d_res = nullptr;
      p->d_all = nullptr;
    }
  }
  if (p->d_res) (void)hipFree(p->d_res);
  if (p->d_all) (void)hipFree(p->d_all);
  if (p->fence) (void)hipEventDestroy(p->fence);
  if (p->h_stats) (void)hipHostFree(p->h_stats);
  if (p->h_io) (void)hipHostFree(p->h_io);
  blob_windows_free(p->win);
  delete p->pool;
  delete p;
  dict_unref(dict);
  e->open_packs.fetch_sub(1);
  engine_unref(e);  // may free the engine if its creator already destroyed it
}

int grow_results(ngpu_pack *p, uint64_t want) {
  if (want <= p->res_cap) return 0;
  uint64_t c = p->res_cap ? p->res_cap : 4096;
  while (c < want) c *= 2;
  ngpu_result *n = nullptr;
  HIP_TRY(p->e, hipMalloc((void **)&n, c * sizeof(ngpu_result)));
  if (p->d_res) {
    HIP_TRY(p->e, hipMemcpyAsync(n, p->d_res, p->dispatched * sizeof(ngpu_result),
                                 hipMemcpyDeviceToDevice, p->stream));
    HIP_TRY(p->e, hipStreamSynchronize(p->stream));
    (void)hipFree(p->d_res);
  }
  p->d_res = n;
  p->res_cap = c;
  return 0;
}

// The layer's device chunk table (p->d_all) holds at least `want` entries,
// its contents kept (e->mu held; a regrow waits for the pack's stream).
int grow_all(ngpu_pack *p, uint64_t want) {
  if (want <= p->all_cap) return 0;
  uint64_t c = p->all_cap ? p->all_cap : 4096;
  while (c < want) c *= 2;
  ngpu_chunk *n = nullptr;
  HIP_TRY(p->e, hipMalloc((void **)&n, c * sizeof(ngpu_chunk)));
  if (p->d_all) {
    HIP_TRY(p->e, hipMemcpyAsync(n, p->d_all, p->all_cap * sizeof(ngpu_chunk),
                                 hipMemcpyDeviceToDevice, p->stream));
    HIP_TRY(p->e, hipStreamSynchronize(p->stream));
    (void)hipFree(p->d_all);
  }
  p->d_all = n;
  p->all_cap = c;
  return 0;
}

// Copy the slot to HBM and digest chunks [a, b) (all inside the slot).
// digest == false: the copies only (a batched close digests the slot's bytes
// in its launch set, batch.hip); *dev_out = where the bytes land.
// Take a workspace slot for the pack's stream and size it once for a whole
// staging slot, so no later dispatch of the pack reallocates it (e->mu held).
int size_workspace(ngpu_pack *p) {
  if (p->ws_sized) return 0;
  ngpu_engine *e = p->e;
  use_slot(e, p->stream);
  if (int rc = ensure_workspace(e, p->max_ch, p->cap, pick_group_log2(e, p->cap), dict_blobs(p->dict), 1))
    return rc;
  if (int rc = ws_acquire(e, p->stream)) return rc;
  if (int rc = ws_release(e, p->stream, nullptr, true)) return rc;
  p->ws_sized = true;
  return 0;
}

int dispatch(ngpu_pack *p, Slot &s, uint64_t a, uint64_t b, bool digest = true,
             uint8_t **dev_out = nullptr) {
  if (b == a) return 0;
  ngpu_engine *e = p->e;
  const uint64_t nch = b - a;
  if (nch > p->max_ch) return fail(e, NGPU_EINVAL, "too many chunks in one staging slot");
  for (uint64_t k = 0; k < nch; ++k) {
    s.h_ch[k] = p->chunks[a + k];
    s.h_ch[k].offset -= s.base;
  }
  int rc = grow_results(p, b);
  if (rc) return rc;
  if (digest && (rc = size_workspace(p))) return rc;
  uint8_t *dev = s.d;
  {  // the copies go out on the pack's shared H2D lane
    std::lock_guard<std::mutex> cg(*p->copy_mu);
    if (p->retain) {  // this slot's bytes get their own resident segment
      Seg g;
      const uint64_t need = (s.fill + 255) & ~255ull;
      if (p->arenas.empty() || p->arenas.back().cap - p->arenas.back().used < need) {
        // stream-ordered (the device pool, engine.hip): freed without a device-wide wait
        uint64_t cap = p->arenas.empty() ? p->cap : std::min<uint64_t>(2 * p->arenas.back().cap, 1ull << 30);
        if (cap < need) cap = need;
        ngpu_pack::Arena ar;
        if (e->seg_pool)
          HIP_TRY(e, hipMallocFromPoolAsync((void **)&ar.d, cap, e->seg_pool, p->copy));
        else
          HIP_TRY(e, hipMallocAsync((void **)&ar.d, cap, p->copy));
        ar.cap = cap;
        p->arenas.push_back(ar);
      }
      ngpu_pack::Arena &ar = p->arenas.back();
      g.d = ar.d + ar.used;
      ar.used += need;
      g.base = s.base;
      g.a = a;
      g.b = b;
      p->segs.push_back(g);
      dev = g.d;
    }
    // bytes [0, sent) went H2D as they were committed (eager_copy); the copy
    // stream is in order, so s.copied covers them too
    const uint64_t from = p->retain ? 0 : s.sent;
    if (s.fill > from)
      HIP_TRY(e, hipMemcpyAsync(dev + from, s.h + from, s.fill - from, hipMemcpyHostToDevice, p->copy));
    s.sent = s.fill;
    HIP_TRY(e, hipMemcpyAsync(s.d_ch, s.h_ch, nch * sizeof(ngpu_chunk), hipMemcpyHostToDevice,
                              p->copy));
    HIP_TRY(e, hipEventRecord(s.copied, p->copy));
    HIP_TRY(e, hipStreamWaitEvent(p->stream, s.copied, 0));  // (later copies of the lane are not waited for)
  }
  if (p->em && !p->gz) {  // the prefix dedups read lengths from the layer's device chunk table
    if ((rc = grow_all(p, b + 1))) return rc;
    HIP_TRY(e, hipMemcpyAsync(p->d_all + a, s.d_ch, nch * sizeof(ngpu_chunk),
                              hipMemcpyDeviceToDevice, p->stream));
  }
  if (dev_out) *dev_out = dev;
  if (digest) {
    rc = enqueue_digest(e, dev, s.fill, s.d_ch, nch, p->d_res + a, p->stream);
    if (rc) return rc;
  }
  HIP_TRY(e, hipEventRecord(s.done, p->stream));
  s.busy = true;
  p->dispatched = b;
  if (Emit *em = p->gz ? nullptr : p->em) {  // the new range is the emitter's (e->mu held)
    for (uint64_t k = a; k < b; ++k) {
      em->ch.push_back(p->chunks[k]);
      em->dptr.push_back((uint64_t)(uintptr_t)(dev + (p->chunks[k].offset - s.base)));
    }
    em->avail = b;
    {
      std::lock_guard<std::mutex> g(em->m);
      em->hint.store(b);
    }
    em->cv.notify_one();
  }
  return 0;
}

// Current slot is full: dispatch its complete chunks (under the engine lock),
// carry the chunk in progress to the other slot and make that one current.
int switch_slot(ngpu_pack *p) {
  Slot &s = p->slot[p->cur];
  Slot &t = p->slot[p->cur ^ 1];
  const uint64_t end = s.base + s.fill;
  uint64_t k = p->dispatched;
  while (k < p->chunks.size() && p->chunks[k].offset + p->chunks[k].length <= end) ++k;
  const uint64_t carry_from = k < p->chunks.size() ? p->chunks[k].offset : end;
  const uint64_t carry = end - carry_from;
  if (carry >= p->cap) return fail(p->e, NGPU_EINVAL, "chunk larger than a staging slot");
  not_waitable(p);  // more than one slot of tar: its close cannot batch
  {
    std::lock_guard<std::mutex> g(p->e->mu);  // the engine lock covers the enqueue only
    int rc = dispatch(p, s, p->dispatched, k);
    if (rc) return rc;
  }
  if (t.busy) {  // the other slot's copy + digest, waited for without the lock
    HIP_TRY(p->e, hipEventSynchronize(t.done));
    t.busy = false;
  }
  memcpy(t.h, s.h + (carry_from - s.base), carry);
  t.base = carry_from;
  t.fill = carry;
  t.sent = 0;
  p->cur ^= 1;
  return 0;
}

// Queue the slot's newly committed bytes H2D once kEagerCopy of them have
// gathered, so the layer's copy runs while the caller is still writing and
// only the tail is left for the dispatch (C1 through 1 MiB writes: the whole
// 10 MB copy used to start at close).  Not with NGPU_PACK_RETAIN, whose
// device segment is sized and allocated at dispatch.  4 MiB: 32 concurrent C1
// Packs (ReadFrom) move 38.3 / 40.5 / 42.9 / 42.7 / 43.5 GB/s at 1 / 2 / 4 / 8
// / 16 MiB granules (profiles/r6/packs_eager_granule_r6d.json; the copy lanes'
// H2D rate grows with the piece size, profiles/r5/h2d_streams_granule_r5w.jsonl).
constexpr uint64_t kEagerCopy = 4ull << 20;

// NGPU_EAGER_COPY (bytes, tuning knob): the eager copy granule.
uint64_t eager_granule() {
  static const uint64_t g = [] {
    if (const char *v = getenv("NGPU_EAGER_COPY")) {
      const unsigned long long x = strtoull(v, nullptr, 0);
      if (x >= 4096) return (uint64_t)x;
    }
    return kEagerCopy;
  }();
  return g;
}

int eager_copy(ngpu_pack *p, Slot &s) {
  if (p->retain || s.fill - s.sent < eager_granule()) return 0;
  DeviceGuard dg(p->e->device);
  std::lock_guard<std::mutex> g(*p->copy_mu);
  HIP_TRY(p->e, hipMemcpyAsync(s.d + s.sent, s.h + s.sent, s.fill - s.sent, hipMemcpyHostToDevice,
                               p->copy));
  s.sent = s.fill;
  return 0;
}

// The pack's BlobWriter: dict blob table and compressed placements from the
// caller's options or the pack's dict (RAFS options from the engine).
int make_writer(ngpu_pack *p, const ngpu_blob_options &opt, ngpu_write_fn w, void *ctx,
                std::unique_ptr<BlobWriter> *out) {
  ngpu_engine *e = p->e;
  ngpu_blob_options o = opt;
  o.digester = e->cfg.digester;
  o.chunk_size = e->cfg.chunk_size;
  o.fs_version = e->cfg.fs_version;
  std::vector<RafsV6BlobInfo> dict;
  const uint8_t *rec = opt.dict_blobs;
  uint64_t nrec = opt.n_dict_blobs;
  if ((!rec || !nrec) && p->dict) {
    rec = p->dict->blob_table.data();
    nrec = p->dict->blob_table.size() / sizeof(RafsV6BlobInfo);
  }
  dict.resize(nrec);
  if (nrec) memcpy(dict.data(), rec, nrec * sizeof(RafsV6BlobInfo));
  const DictPlace *place = nullptr;
  uint64_t nplace = 0;
  if (p->dict && !p->dict->place.empty()) {
    place = p->dict->place.data();
    nplace = p->dict->place.size();
  }
  out->reset(new BlobWriter(o, w, ctx, std::move(dict), place, nplace));
  (*out)->set_cancel(p->cancel);
  if (int rc = (*out)->init()) return fail(e, rc, "pack: %s", ngpu_host_error());
  return 0;
}

// Gather the NEW chunks among `count` decided chunks (device address dptr[i],
// stream descriptor ch[i], decision res[i]; index order == stream order) into
// window buffers on the GPU, copy each window to a pinned landing buffer
// (land[0/1], alternating) and hand it to the BlobWriter; window k+1's gather
// + D2H run while the host compresses window k.  Enqueues on the pack's
// stream without the engine lock (pack-owned buffers only).
int emit_range(ngpu_pack *p, BlobWriter &bw, const ngpu_chunk *ch, const uint64_t *dptr,
               const ngpu_result *res, uint64_t count, uint8_t *const land[2],
               uint64_t *new_out) {
  ngpu_engine *e = p->e;
  std::vector<uint64_t> src;
  std::vector<uint32_t> len;
  for (uint64_t i = 0; i < count; ++i) {
    if (res[i].kind != NGPU_NEW) continue;
    src.push_back(dptr[i]);
    len.push_back(ch[i].length);
  }
  const uint64_t k = src.size();
  if (new_out) *new_out += k;
  // windows of <= cap bytes (16-B aligned placement) and <= maxk chunks
  const uint64_t cap = p->cap, maxk = 1ull << 18;
  std::vector<uint64_t> wstart{0};
  std::vector<uint64_t> doff(k);
  for (uint64_t i = 0, used = 0, cnt = 0; i < k; ++i) {
    const uint64_t need = (len[i] + 15) & ~15ull;
    if (cnt && (used + need > cap || cnt == maxk)) {
      wstart.push_back(i);
      used = cnt = 0;
    }
    doff[i] = used;
    used += need;
    ++cnt;
  }
  wstart.push_back(k);
  const uint64_t nw = k ? wstart.size() - 1 : 0;  // no NEW chunk: no window
  // the gather windows (pooled with the pack's other buffers): descriptors
  // sized to the layer's NEW chunks, at least 4K, at most maxk per window
  uint64_t kneed = 4096;
  while (kneed < k && kneed < maxk) kneed *= 2;
  BlobWindows &bw_ = p->win;
  if (nw && (bw_.cap < cap || bw_.kcap < kneed || !bw_.ev[0] || !bw_.gathered[0])) {
    (void)hipStreamSynchronize(p->stream);  // a previous range's windows may still be read
    for (int b = 0; b < 2; ++b)
      if (bw_.ev[b]) (void)hipEventSynchronize(bw_.ev[b]);
    blob_windows_free(bw_);
    bool ok = true;
    for (int i = 0; i < 2 && ok; ++i)
      ok = hipMalloc((void **)&bw_.dwin[i], cap) == hipSuccess &&
           hipMalloc((void **)&bw_.ddesc[i], kneed * 20) == hipSuccess &&
           hipHostMalloc((void **)&bw_.hdesc[i], kneed * 20, hipHostMallocDefault) == hipSuccess &&
           hipEventCreateWithFlags(&bw_.ev[i], hipEventDisableTiming) == hipSuccess &&
           hipEventCreateWithFlags(&bw_.gathered[i], hipEventDisableTiming) == hipSuccess;
    if (!ok) {
      (void)hipGetLastError();
      blob_windows_free(bw_);
      return fail(e, NGPU_ENOMEM, "pack: blob window allocation failed");
    }
    bw_.cap = cap;
    bw_.kcap = kneed;
  }
  uint8_t *const *dwin = bw_.dwin, *const *ddesc = bw_.ddesc, *const *hdesc = bw_.hdesc;
  const hipEvent_t *ev = bw_.ev, *gathered = bw_.gathered;
  auto enqueue = [&](uint64_t wi) -> int {
    const int b = wi & 1;
    const uint64_t a = wstart[wi], c = wstart[wi + 1] - a;
    // one descriptor block per window: c sources, c offsets, c lengths
    uint64_t *hs = (uint64_t *)hdesc[b];
    uint64_t *ho = hs + c;
    uint32_t *hl = (uint32_t *)(ho + c);
    memcpy(hs, &src[a], c * 8);
    for (uint64_t i = 0; i < c; ++i) ho[i] = doff[a + i];
    memcpy(hl, &len[a], c * 4);
    uint64_t *ds = (uint64_t *)ddesc[b];
    hipStream_t ps = p->stream;
    HIP_TRY(e, hipMemcpyAsync(ds, hs, c * 20, hipMemcpyHostToDevice, ps));
    const unsigned grid = (unsigned)(c < 2048 ? c : 2048);
    hipLaunchKernelGGL(gather_chunks, dim3(grid), dim3(256), 0, ps, ds, (uint32_t *)(ds + 2 * c),
                       ds + c, c, dwin[b]);
    HIP_TRY(e, hipGetLastError());
    const uint64_t bytes = doff[a + c - 1] + len[a + c - 1];
    if (int rc = host_fence(e, ps, p->fence)) return rc;
    HIP_TRY(e, hipEventRecord(gathered[b], ps));
    // the window's bytes come back on the pack's shared D2H lane
    std::lock_guard<std::mutex> g(*p->d2h_mu);
    HIP_TRY(e, hipStreamWaitEvent(p->d2h, gathered[b], 0));
    HIP_TRY(e, hipMemcpyAsync(land[b], dwin[b], bytes, hipMemcpyDeviceToHost, p->d2h));
    HIP_TRY(e, hipEventRecord(ev[b], p->d2h));
    return 0;
  };
  int rc = 0;
  std::vector<const uint8_t *> hp;
  if (nw) rc = enqueue(0);
  for (uint64_t wi = 0; wi < nw && !rc; ++wi) {
    if (cancelled(p)) {
      rc = fail(e, NGPU_ECANCELED, "pack: cancelled");
      break;
    }
    if (wi + 1 < nw && (rc = enqueue(wi + 1))) break;
    const int b = wi & 1;
    if (hipEventSynchronize(ev[b]) != hipSuccess) {
      rc = fail(e, NGPU_EHIP, "pack: blob window copy failed");
      break;
    }
    const uint64_t a = wstart[wi], c = wstart[wi + 1] - a;
    hp.resize(c);
    for (uint64_t i = 0; i < c; ++i) hp[i] = land[b] + doff[a + i];
    if ((rc = bw.add(hp.data(), &len[a], c))) rc = fail(e, rc, "pack: %s", ngpu_host_error());
  }
  // every window was waited for on success; after an error the next one may
  // still be in flight
  if (rc) {
    (void)hipStreamSynchronize(p->stream);
    for (int b = 0; b < 2; ++b) (void)hipEventSynchronize(ev[b]);
  }
  return rc;
}

// Device address of every chunk of the layer in the retained segments.
int chunk_addresses(ngpu_pack *p, const ngpu_chunk *ch, uint64_t from, uint64_t n,
                    std::vector<uint64_t> *dptr) {
  dptr->resize(n - from);
  size_t g = 0;
  for (uint64_t i = from; i < n; ++i) {
    while (g < p->segs.size() && p->segs[g].b <= i) ++g;
    if (g == p->segs.size())
      return fail(p->e, NGPU_EINVAL, "pack: chunk %llu has no segment", (unsigned long long)i);
    const Seg &sg = p->segs[g];
    (*dptr)[i - from] = (uint64_t)(uintptr_t)(sg.d + (ch[i].offset - sg.base));
  }
  return 0;
}

// When every chunk of [from, n) lies in the current staging slot -- a layer
// that fit one slot, or the tail still in the last one -- their bytes are in
// pinned host memory as the caller wrote them: *hp = their host addresses,
// and the NEW chunks are compressed from there, with no GPU gather and no D2H
// of bytes the host already holds (32 concurrent C1 streams moved 330 MB back
// over PCIe per round for that).  false: some chunk is only in HBM.
bool host_addresses(const ngpu_pack *p, const ngpu_chunk *ch, uint64_t from, uint64_t n,
                    std::vector<const uint8_t *> *hp) {
  const Slot &s = p->slot[p->cur];
  if (!s.h) return false;
  hp->resize(n - from);
  for (uint64_t i = from; i < n; ++i) {
    if (ch[i].offset < s.base || ch[i].offset + ch[i].length > s.base + s.fill) return false;
    (*hp)[i - from] = s.h + (ch[i].offset - s.base);
  }
  return true;
}

// The NEW chunks of a range from host memory (host_addresses) into the writer.
int emit_range_host(ngpu_pack *p, BlobWriter &bw, const ngpu_chunk *ch, const uint8_t *const *hp,
                    const ngpu_result *res, uint64_t count, uint64_t *new_out) {
  std::vector<const uint8_t *> src;
  std::vector<uint32_t> len;
  for (uint64_t i = 0; i < count; ++i) {
    if (res[i].kind != NGPU_NEW) continue;
    src.push_back(hp[i]);
    len.push_back(ch[i].length);
  }
  if (new_out) *new_out += src.size();
  if (src.empty()) return 0;
  // (src_stable: the slot stays this pack's until release, after the writer's finish)
  if (int rc = bw.add(src.data(), len.data(), src.size(), true))
    return fail(p->e, rc, "pack: %s", ngpu_host_error());
  return 0;
}

// The whole stream at close (no early emission): every NEW chunk, then the
// headers, blob.meta, image.boot and TOC.  The landing buffers are the pinned
// staging slots (the layer's bytes are all written by now).
int write_stream(ngpu_pack *p, const ngpu_blob_options &opt, ngpu_write_fn w, void *ctx,
                 const ngpu_chunk *ch, const ngpu_result *res, uint64_t n,
                 const ngpu_layer_stats &st, ngpu_blob_info *info) {
  std::unique_ptr<BlobWriter> bw;
  if (int rc = make_writer(p, opt, w, ctx, &bw)) return rc;
  std::vector<const uint8_t *> hp;
  if (host_addresses(p, ch, 0, n, &hp)) {
    if (int rc = emit_range_host(p, *bw, ch, hp.data(), res, n, nullptr)) return rc;
  } else {
    std::vector<uint64_t> dptr;
    if (int rc = chunk_addresses(p, ch, 0, n, &dptr)) return rc;
    uint8_t *const land[2] = {p->slot[0].h, p->slot[1].h};
    if (int rc = emit_range(p, *bw, ch, dptr.data(), res, n, land, nullptr)) return rc;
  }
  if (int rc = bw->finish(ch, res, n, st, p->entries, info))
    return fail(p->e, rc, "pack: %s", ngpu_host_error());
  return 0;
}

// ---- early emission -----------------------------------------------------------
// One iteration of the emitter: dedup the dispatched prefix [0, k) (its
// records from the previous prefix remarked first), copy the decisions of
// [emitted, k) back, check the digest guard, write their NEW chunks.
int emit_step(ngpu_pack *p, Emit *em) {
  ngpu_engine *e = p->e;
  const uint64_t a = em->emitted;
  uint64_t k = 0;
  std::vector<ngpu_chunk> ch;
  std::vector<uint64_t> dptr;
  std::string path;
  {
    std::lock_guard<std::mutex> g(e->mu);
    DeviceGuard dg(e->device);
    k = em->avail;
    if (k <= a) return 0;
    ch.assign(em->ch.begin() + (long)a, em->ch.begin() + (long)k);
    dptr.assign(em->dptr.begin() + (long)a, em->dptr.begin() + (long)k);
    if (k - a > em->h_cap) {
      uint64_t c = em->h_cap ? em->h_cap : 4096;
      while (c < k - a) c *= 2;
      if (em->h_res) (void)hipHostFree(em->h_res), em->h_res = nullptr, em->h_cap = 0;
      HIP_TRY(e, hipHostMalloc((void **)&em->h_res, c * sizeof(ngpu_result), hipHostMallocDefault));
      em->h_cap = c;
    }
    hipStream_t ps = p->stream;
    launch_remark_digested(p->d_res, em->deduped, ps);
    HIP_TRY(e, hipGetLastError());
    if (int rc = enqueue_dedup(e, p->dict, p->d_all, k, p->d_res, nullptr, 0, ps, nullptr, 1, nullptr))
      return rc;
    em->deduped = k;
    if (int rc = host_fence(e, ps, p->fence)) return rc;
    HIP_TRY(e, hipMemcpyAsync(em->h_res, p->d_res + a, (k - a) * sizeof(ngpu_result),
                              hipMemcpyDeviceToHost, ps));
    if (int rc = read_stats_enqueue(e, ps, em->h_stats)) return rc;
    HIP_TRY(e, hipEventRecord(em->ev, ps));
    path = e->cur->path;
  }
  HIP_TRY(e, hipEventSynchronize(em->ev));
  ngpu_layer_stats st{};
  if (int rc = read_stats_parse(e, em->h_stats, &st, path.c_str())) return rc;  // digest guard
  uint8_t *const land[2] = {(uint8_t *)em->land[0].h, (uint8_t *)em->land[1].h};
  if (int rc = emit_range(p, *em->bw, ch.data(), dptr.data(), em->h_res, k - a, land,
                          &em->new_emitted))
    return rc;
  em->emitted = k;
  return 0;
}

void emit_loop(ngpu_pack *p, Emit *em) {
  DeviceGuard dg(p->e->device);
  for (;;) {
    {
      std::unique_lock<std::mutex> g(em->m);
      em->cv.wait(g, [&] { return em->stop || em->hint.load() > em->emitted; });
      if (em->stop) return;
    }
    if (cancelled(p)) {
      em->rc = fail(p->e, NGPU_ECANCELED, "pack: cancelled");
      return;
    }
    if (int rc = emit_step(p, em)) {
      em->rc = rc;
      return;
    }
  }
}

// Close of an OCIRef Pack (targz-ref): the gzip stream must have ended; the
// own blob is the gzip blob, each NEW chunk addressed by the checkpoint it
// starts after and the deflate range that produces it (ZranRef, blob.hpp).
int ref_finish(ngpu_pack *p, BlobWriter &bw, const ngpu_chunk *ch, const ngpu_result *res,
               uint64_t n, const ngpu_layer_stats &st, ngpu_blob_info *info) {
  ngpu_engine *e = p->e;
  GzipIndexer &gz = *p->gz;
  if (int rc = gz.finish()) return fail(e, rc, "pack: %s", ngpu_host_error());
  ZranRef zr;
  gz.blob_digest(zr.digest);
  zr.gz_size = gz.in_bytes();
  zr.tar_size = gz.out_bytes();
  const std::vector<ZranPoint> &pts = gz.points();
  zr.n_points = pts.size();
  zr.dicts = gz.dicts();
  // ZranInflateContext records, 40 B (restated, VERIFY): in_offset u64,
  // out_offset u64, in_len u32, out_len u32 (to the next checkpoint), ctx_byte
  // u8, ctx_bits u8, reserved u16, dict_size u32, dict_offset u64
  zr.table.assign(40 * pts.size(), 0);
  for (size_t i = 0; i < pts.size(); ++i) {
    const ZranPoint &x = pts[i];
    const uint64_t in_next = i + 1 < pts.size() ? pts[i + 1].in_offset : zr.gz_size;
    const uint64_t out_next = i + 1 < pts.size() ? pts[i + 1].out_offset : zr.tar_size;
    const uint32_t in_len = (uint32_t)(in_next - x.in_offset), out_len = (uint32_t)(out_next - x.out_offset);
    uint8_t *r = zr.table.data() + 40 * i;
    memcpy(r, &x.in_offset, 8);
    memcpy(r + 8, &x.out_offset, 8);
    memcpy(r + 16, &in_len, 4);
    memcpy(r + 20, &out_len, 4);
    r[24] = (uint8_t)x.byte;
    r[25] = (uint8_t)x.bits;
    memcpy(r + 28, &x.dict_size, 4);
    memcpy(r + 32, &x.dict_offset, 8);
  }
  for (uint64_t i = 0; i < n; ++i) {
    if (res[i].kind != NGPU_NEW) continue;
    const uint64_t off = ch[i].offset, end = off + ch[i].length;
    if (pts.empty() || end > zr.tar_size)
      return fail(e, NGPU_EINVAL, "pack: OCIRef chunk %llu outside the inflated stream",
                  (unsigned long long)i);
    const uint64_t k = gz.point_of(off);
    const ZranPoint &x = pts[k];
    const uint64_t coff = x.in_offset - (x.bits ? 1 : 0);
    zr.coff.push_back(coff);
    zr.csize.push_back(gz.in_end_of(end) - coff);
    if (k > 0xFFFFFFFFull || off - x.out_offset > 0xFFFFFFFFull)  // 32-bit fields: refused, not truncated
      return fail(e, NGPU_EFORMAT, "pack: OCIRef chunk %llu lies %llu B past its checkpoint (32-bit field)",
                  (unsigned long long)i, (unsigned long long)(off - x.out_offset));
    zr.ctx.push_back((uint32_t)k);
    zr.ctx_off.push_back((uint32_t)(off - x.out_offset));
  }
  bw.set_zran(&zr);
  if (int rc = bw.finish(ch, res, n, st, p->entries, info))
    return fail(e, rc, "pack: %s", ngpu_host_error());
  return 0;
}

// Close of an early-emission Pack: the final dedup over the whole layer gave
// the same decisions for the chunks already written (stream order; checked by
// their NEW count), so the rest [emitted, n) follows and the writer finishes.
int emit_finish(ngpu_pack *p, Emit *em, const ngpu_chunk *ch, const ngpu_result *res, uint64_t n,
                const ngpu_layer_stats &st, ngpu_blob_info *info) {
  ngpu_engine *e = p->e;
  uint64_t same = 0;
  for (uint64_t i = 0; i < em->emitted && i < n; ++i) same += res[i].kind == NGPU_NEW;
  if (em->emitted > n || same != em->new_emitted)
    return fail(e, NGPU_EDEVICE, "pack: %llu NEW chunks written early, %llu in the final decisions",
                (unsigned long long)em->new_emitted, (unsigned long long)same);
  std::vector<const uint8_t *> hp;
  if (host_addresses(p, ch, em->emitted, n, &hp)) {
    if (int rc = emit_range_host(p, *em->bw, ch + em->emitted, hp.data(), res + em->emitted,
                                 n - em->emitted, &em->new_emitted))
      return rc;
  } else {
    std::vector<uint64_t> dptr;
    if (int rc = chunk_addresses(p, ch, em->emitted, n, &dptr)) return rc;
    uint8_t *const land[2] = {(uint8_t *)em->land[0].h, (uint8_t *)em->land[1].h};
    if (int rc = emit_range(p, *em->bw, ch + em->emitted, dptr.data(), res + em->emitted,
                            n - em->emitted, land, &em->new_emitted))
      return rc;
  }
  ptrace(p, "finish_rest_emitted");
  if (int rc = em->bw->finish(ch, res, n, st, p->entries, info))
    return fail(e, rc, "pack: %s", ngpu_host_error());
  return 0;
}

void emit_stop(ngpu_pack *p) {
  Emit *em = p->em;
  if (!em || !em->th.joinable()) return;
  {
    std::lock_guard<std::mutex> g(em->m);
    em->stop = true;
  }
  em->cv.notify_all();
  em->th.join();
}

}  // namespace

void blob_windows_free(BlobWindows &w) {
  for (int i = 0; i < 2; ++i) {
    if (w.dwin[i]) (void)hipFree(w.dwin[i]);
    if (w.ddesc[i]) (void)hipFree(w.ddesc[i]);
    if (w.hdesc[i]) (void)hipHostFree(w.hdesc[i]);
    if (w.ev[i]) (void)hipEventDestroy(w.ev[i]);
    if (w.gathered[i]) (void)hipEventDestroy(w.gathered[i]);
  }
  w = BlobWindows{};
}

extern "C" {

int ngpu_pack_open(ngpu_engine *e, ngpu_pack **out) { return ngpu_pack_open_ex(e, 0, out); }

static ngpu_dict *const kDefaultDict = reinterpret_cast<ngpu_dict *>(1);

static int pack_open(ngpu_engine *e, ngpu_dict *dict, uint32_t flags, ngpu_pack **out) {
  if (!e || !out || (flags & ~(NGPU_PACK_RETAIN | NGPU_PACK_OCIREF))) return NGPU_EINVAL;
  *out = nullptr;
  const bool ociref = (flags & NGPU_PACK_OCIREF) != 0;
  std::unique_ptr<GzipIndexer> gz;
  if (ociref) {  // packRef (builder.go:180-218) passes no --chunk-dict
    if (dict != kDefaultDict && dict)
      return fail(e, NGPU_EINVAL, "OCIRef (targz-ref) takes no chunk dict");
    dict = nullptr;
    gz.reset(new GzipIndexer(std::max<uint64_t>(e->cfg.chunk_size, 1ull << 20)));
    if (int rc = gz->init()) return fail(e, rc, "pack: %s", ngpu_host_error());
  }
  std::lock_guard<std::mutex> g(e->mu);
  DeviceGuard dg(e->device);
  if (dict == kDefaultDict) dict = e->dict;
  if (int rc = dict_check(e, dict)) return rc;
  ngpu_pack *p = new ngpu_pack(e);
  engine_ref(e);
  e->open_packs.fetch_add(1);
  dict_ref(dict);
  p->dict = dict;
  p->retain = flags & NGPU_PACK_RETAIN;
  p->gz = std::move(gz);
  if (!p->gz && !(e->cfg.flags & NGPU_FLAG_NO_BATCH)) {
    p->waitable = true;
    e->batch_waitable.fetch_add(1);
  }
  // the stream's bootstrap lists every entry (OCIRef: the bootstrap is all it carries)
  if (p->retain || p->gz) p->sc.record(&p->entries);
  uint64_t cap = e->cfg.staging_bytes;
  if (cap < 4ull * e->cfg.chunk_size) cap = 4ull * e->cfg.chunk_size;
  p->cap = cap;
  p->max_ch = cap / 1024 + 16;  // a chunk costs >= 1 KiB of tar stream unless it is a file's last
  bool ok = true;
  {
    std::lock_guard<std::mutex> pg(e->pool_mu);
    if (!e->pack_pool.empty()) {
      const ngpu_pack_bufs b = e->pack_pool.back();
      e->pack_pool.pop_back();
      p->stream = b.stream;
      p->fence = b.fence;
      p->h_stats = b.h_stats;
      p->h_io = b.h_io;
      p->io_cap = b.io_cap;
      p->d_res = b.d_res;
      p->res_cap = b.res_cap;
      p->d_all = b.d_all;
      p->all_cap = b.all_cap;
      p->win = b.win;
    }
    for (Slot &s : p->slot) {
      auto &pool = e->staging_pool;
      for (size_t i = 0; i < pool.size(); ++i) {
        if (pool[i].cap != cap) continue;
        const ngpu_staging_buf b = pool[i];
        pool.erase(pool.begin() + (long)i);
        e->staging_pool_bytes -= b.cap;
        s.h = (uint8_t *)b.h;
        s.h_ch = (ngpu_chunk *)b.h_ch;
        s.d = (uint8_t *)b.d;
        s.d_ch = (ngpu_chunk *)b.d_ch;
        s.copied = b.copied;
        s.done = b.done;
        break;
      }
    }
  }
  {  // the pack's shared copy lanes (created with the engine's first pack)
    const uint32_t k = e->copy_rr++ % ngpu_engine::kCopyLanes;
    if (!e->h2d[k]) {
      ok = hipStreamCreateWithFlags(&e->h2d[k], hipStreamNonBlocking) == hipSuccess;
      if (ok) e->streams.push_back(e->h2d[k]);  // destroyed with the engine
    }
    if (ok && !e->d2h[k]) {
      ok = hipStreamCreateWithFlags(&e->d2h[k], hipStreamNonBlocking) == hipSuccess;
      if (ok) e->streams.push_back(e->d2h[k]);
    }
    p->copy = e->h2d[k];
    p->copy_mu = &e->h2d_mu[k];
    p->d2h = e->d2h[k];
    p->d2h_mu = &e->d2h_mu[k];
  }
  if (ok && !p->fence) ok = hipEventCreateWithFlags(&p->fence, hipEventDisableTiming) == hipSuccess;
  if (ok && !p->h_stats)
    ok = hipHostMalloc((void **)&p->h_stats, 32 * sizeof(uint64_t), hipHostMallocDefault) ==
         hipSuccess;
  if (ok && !p->stream) {
    ok = hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking) == hipSuccess;
    if (ok) e->streams.push_back(p->stream);  // lives until the engine does (e->mu held)
  }
  for (Slot &s : p->slot) {
    if (s.h) {  // from the engine's pool: only the device copy may be missing
      if (!p->retain && !s.d) ok = ok && hipMalloc((void **)&s.d, cap) == hipSuccess;
      continue;
    }
    ok = ok && hipHostMalloc((void **)&s.h, cap, hipHostMallocDefault) == hipSuccess &&
         hipHostMalloc((void **)&s.h_ch, p->max_ch * sizeof(ngpu_chunk), hipHostMallocDefault) ==
             hipSuccess &&
         (p->retain || hipMalloc((void **)&s.d, cap) == hipSuccess) &&
         hipMalloc((void **)&s.d_ch, p->max_ch * sizeof(ngpu_chunk)) == hipSuccess &&
         hipEventCreateWithFlags(&s.copied, hipEventDisableTiming) == hipSuccess &&
         hipEventCreateWithFlags(&s.done, hipEventDisableTiming) == hipSuccess;
  }
  // (the pack's workspace is sized at its first digest on its own stream,
  // size_workspace: a pack whose close joins a batch never takes one -- at
  // open, the GPU-side wait on the slot's last stage tied the pack's events
  // to an unrelated running batch)
  if (!ok) {
    (void)hipGetLastError();
    release(p);
    return fail(e, NGPU_ENOMEM, "pack: staging allocation failed");
  }
  *out = p;
  return 0;
}

int ngpu_pack_open_ex(ngpu_engine *e, uint32_t flags, ngpu_pack **out) {
  return pack_open(e, kDefaultDict, flags, out);
}

int ngpu_pack_open_dict(ngpu_engine *e, ngpu_dict *dict, uint32_t flags, ngpu_pack **out) {
  return pack_open(e, dict, flags, out);
}

int ngpu_pack_set_output(ngpu_pack *p, const ngpu_blob_options *opt, ngpu_write_fn w, void *ctx) {
  if (!p || !opt || !w) return NGPU_EINVAL;
  return guarded([&]() -> int {
    ngpu_engine *e = p->e;
    if (!p->retain && !p->gz)
      return fail(e, NGPU_EINVAL, "pack: early output needs NGPU_PACK_RETAIN");
    if (p->em || !p->chunks.empty() || p->slot[p->cur].fill || p->dispatched)
      return fail(e, NGPU_EINVAL, "pack: the output is set once, before the first write");
    DeviceGuard dg(e->device);
    Emit *em = new Emit();
    p->em = em;
    em->opt = *opt;
    em->prefetch = opt->prefetch_patterns ? opt->prefetch_patterns : "";
    // NULL stays NULL: the writer's default patterns ("/") apply to it
    em->opt.prefetch_patterns = opt->prefetch_patterns ? em->prefetch.c_str() : nullptr;
    if (int rc = make_writer(p, em->opt, w, ctx, &em->bw)) return rc;
    HIP_TRY(e, hipHostMalloc((void **)&em->h_stats, 32 * sizeof(uint64_t), hipHostMallocDefault));
    HIP_TRY(e, hipEventCreateWithFlags(&em->ev, hipEventDisableTiming));
    {  // window landing buffers: staging slots from the engine's pool when it has them
      std::lock_guard<std::mutex> g(e->pool_mu);
      auto &pool = e->staging_pool;
      for (ngpu_staging_buf &b : em->land) {
        for (size_t i = 0; i < pool.size(); ++i)
          if (pool[i].cap == p->cap) {
            b = pool[i];
            pool.erase(pool.begin() + (long)i);
            e->staging_pool_bytes -= b.cap;
            break;
          }
        auto &lp = e->land_pool;  // else a landing kept by an earlier Pack
        for (size_t i = 0; !b.h && i < lp.size(); ++i)
          if (lp[i].second == p->cap) {
            b.h = lp[i].first;
            b.cap = lp[i].second;
            lp.erase(lp.begin() + (long)i);
          }
      }
    }
    for (ngpu_staging_buf &b : em->land)
      if (!b.h) {
        HIP_TRY(e, hipHostMalloc(&b.h, p->cap, hipHostMallocDefault));
        b.cap = p->cap;
      }
    // OCIRef: the stream carries no chunk data, nothing leaves before the close
    if (!p->gz) em->th = std::thread([p, em] { emit_loop(p, em); });
    return 0;
  });
}

int ngpu_pack_set_cancel(ngpu_pack *p, const volatile int32_t *flag) {
  if (!p) return NGPU_EINVAL;
  p->cancel = flag;
  return 0;
}

static int pack_reserve(ngpu_pack *p, void **ptr, uint64_t *avail);
static int pack_commit(ngpu_pack *p, uint64_t n);

int ngpu_pack_reserve(ngpu_pack *p, void **ptr, uint64_t *avail) {
  if (!p || !ptr || !avail) return NGPU_EINVAL;
  if (p->gz) return fail(p->e, NGPU_EINVAL, "pack: an OCIRef pack takes gzip bytes through ngpu_pack_write");
  return pack_reserve(p, ptr, avail);
}

int ngpu_pack_commit(ngpu_pack *p, uint64_t n) {
  if (!p) return NGPU_EINVAL;
  if (p->gz) return fail(p->e, NGPU_EINVAL, "pack: an OCIRef pack takes gzip bytes through ngpu_pack_write");
  return pack_commit(p, n);
}

static int pack_reserve(ngpu_pack *p, void **ptr, uint64_t *avail) {
  if (p->err) return p->err;
  if (p->em && p->em->rc.load()) return p->err = p->em->rc.load();  // the emitter failed
  if (cancelled(p)) return p->err = fail(p->e, NGPU_ECANCELED, "pack: cancelled");
  Slot &s = p->slot[p->cur];
  if (s.fill == p->cap) {
    DeviceGuard dg(p->e->device);
    int rc = switch_slot(p);
    if (rc) return p->err = rc;
  }
  Slot &c = p->slot[p->cur];
  *ptr = c.h + c.fill;
  *avail = p->cap - c.fill;
  return 0;
}

static int pack_commit(ngpu_pack *p, uint64_t n) {
  if (p->err) return p->err;
  if (cancelled(p)) return p->err = fail(p->e, NGPU_ECANCELED, "pack: cancelled");
  Slot &s = p->slot[p->cur];
  if (n > p->cap - s.fill) return p->err = NGPU_EINVAL;
  int rc = guarded([&] { return p->sc.feed(s.h + s.fill, n, *p); });
  s.fill += n;
  if (!rc) rc = eager_copy(p, s);
  if (rc) return p->err = rc;
  return 0;
}

static int pack_write_plain(ngpu_pack *p, const void *buf, uint64_t len);

int ngpu_pack_write(ngpu_pack *p, const void *buf, uint64_t len) {
  if (!p) return NGPU_EINVAL;
  if (p->gz) {  // OCIRef: inflate the gzip blob into the tar path, indexing as it goes
    if (p->err) return p->err;
    if (!len) return 0;
    const int rc = guarded([&] {
      return p->gz->feed((const uint8_t *)buf, len,
                         [&](const uint8_t *t, uint64_t n) { return pack_write_plain(p, t, n); });
    });
    if (rc) {
      if (!p->err) p->err = fail(p->e, rc, "OCIRef: %s", ngpu_host_error());
      return p->err;
    }
    return 0;
  }
  return pack_write_plain(p, buf, len);
}

static int pack_write_plain(ngpu_pack *p, const void *buf, uint64_t len) {
  const uint8_t *b = (const uint8_t *)buf;
  while (len) {
    void *dst;
    uint64_t avail;
    int rc = pack_reserve(p, &dst, &avail);
    if (rc) return rc;
    const uint64_t take = len < avail ? len : avail;
    if (take >= (8ull << 20)) {
      if (!p->pool) {
        unsigned hw = std::thread::hardware_concurrency();
        unsigned nt = hw >= 16 ? 7 : (hw > 2 ? hw / 2 - 1 : 1);
        // NGPU_COPY_THREADS: helper threads besides the caller (tuning knob)
        if (const char *v = getenv("NGPU_COPY_THREADS")) {
          const long x = strtol(v, nullptr, 10);
          if (x >= 1 && x <= 63) nt = (unsigned)x;
        }
        p->pool = new CopyPool(nt);
      }
      p->pool->copy((uint8_t *)dst, b, take);
    } else {
      memcpy(dst, b, take);
    }
    rc = pack_commit(p, take);
    if (rc) return rc;
    b += take;
    len -= take;
  }
  return 0;
}

void ngpu_pack_abort(ngpu_pack *p) { release(p); }

ngpu_engine *ngpu_pack_engine(const ngpu_pack *p) { return p ? p->e : nullptr; }

int ngpu_pack_close(ngpu_pack *p, ngpu_chunk **chunks_out, ngpu_result **results_out,
                    uint64_t *n_out, ngpu_layer_stats *stats) {
  return ngpu_pack_finish(p, nullptr, nullptr, nullptr, chunks_out, results_out, n_out, stats,
                          nullptr);
}

static int pack_finish(ngpu_pack *p, const ngpu_blob_options *opt, ngpu_write_fn w, void *ctx,
                       ngpu_chunk **chunks_out, ngpu_result **results_out, uint64_t *n_out,
                       ngpu_layer_stats *stats, ngpu_blob_info *info) {
  if (!p || !chunks_out || !results_out || !n_out || (w && !opt)) {
    release(p);
    return NGPU_EINVAL;
  }
  *chunks_out = nullptr;
  *results_out = nullptr;
  *n_out = 0;
  ngpu_engine *e = p->e;
  Emit *em = p->em;
  ptrace(p, "finish");
  emit_stop(p);  // the emitter stops after its current range; the rest is written below
  ptrace(p, "finish_emitter_stopped");
  int rc = p->err ? p->err : (em && em->rc.load()) ? em->rc.load() : p->sc.finish();
  if (!rc && cancelled(p)) rc = fail(e, NGPU_ECANCELED, "pack: cancelled");
  if (!rc && w && !p->retain && !p->gz)
    rc = fail(e, NGPU_EINVAL, "pack: writing the blob stream needs ngpu_pack_open_ex(NGPU_PACK_RETAIN)");
  if (!rc && w && em)
    rc = fail(e, NGPU_EINVAL, "pack: the output was set by ngpu_pack_set_output");
  const uint64_t n = p->chunks.size();
  ngpu_chunk *ch = nullptr;
  ngpu_result *res = nullptr;
  ngpu_layer_stats st{};
  std::string path;
  bool batched = false;
  uint8_t *batch_dev = nullptr;
  if (!rc) {
    DeviceGuard dg(e->device);
    {
      std::lock_guard<std::mutex> g(e->mu);
      hipStream_t ps = p->stream;
      // a layer that fit one staging slot goes out in this one dispatch, so
      // the slot's device chunk table already lists every chunk: the dedup
      // reads only lengths from it (the offsets are slot-relative), and the
      // second copy of the table is skipped
      Slot &cs = p->slot[p->cur];
      const bool one_slot = p->dispatched == 0 && n > 0;
      // a layer that fit one staging slot, closing while other packs are
      // open on the engine, joins a batch (batch.hip): ONE launch set for
      // every such pack closing at about this time
      batched = one_slot && !p->gz && !(e->cfg.flags & NGPU_FLAG_NO_BATCH) &&
                e->batch_waitable.load() > 1;
      rc = dispatch(p, cs, p->dispatched, n, !batched, &batch_dev);
      const ngpu_chunk *d_dedup = one_slot ? cs.d_ch : p->d_all;
      if (!rc) rc = grow_results(p, n + 1);
      if (!rc && !one_slot && p->all_cap < n + 1) {  // kept between packs (engine pack_pool)
        if (p->d_all) (void)hipFree(p->d_all), p->d_all = nullptr, p->all_cap = 0;
        uint64_t c = 4096;
        while (c < n + 1) c *= 2;
        if (hipMalloc((void **)&p->d_all, c * sizeof(ngpu_chunk)) != hipSuccess)
          rc = fail(e, NGPU_ENOMEM, "pack: chunk table allocation failed");
        else
          p->all_cap = c;
      }
      ch = (ngpu_chunk *)malloc(sizeof(ngpu_chunk) * (n ? n : 1));
      res = (ngpu_result *)malloc(sizeof(ngpu_result) * (n ? n : 1));
      if (!rc && (!ch || !res)) rc = NGPU_ENOMEM;
      // the chunk table goes out and the results come back through pinned
      // memory: a pageable copy would block this thread under the lock
      const uint64_t io = n * (sizeof(ngpu_chunk) > sizeof(ngpu_result) ? sizeof(ngpu_chunk)
                                                                         : sizeof(ngpu_result));
      if (!rc && io > p->io_cap) {
        if (p->h_io) (void)hipHostFree(p->h_io), p->h_io = nullptr, p->io_cap = 0;
        uint64_t c = 64 << 10;
        while (c < io) c *= 2;
        if (hipHostMalloc((void **)&p->h_io, c, hipHostMallocDefault) != hipSuccess)
          rc = fail(e, NGPU_ENOMEM, "pack: pinned result buffer allocation failed");
        else
          p->io_cap = c;
      }
      if (!rc && n) memcpy(ch, p->chunks.data(), n * sizeof(ngpu_chunk));
      if (!rc && n && !one_slot) {
        memcpy(p->h_io, ch, n * sizeof(ngpu_chunk));
        if (hipMemcpyAsync(p->d_all, p->h_io, n * sizeof(ngpu_chunk), hipMemcpyHostToDevice,
                           ps) != hipSuccess)
          rc = fail(e, NGPU_EHIP, "pack: chunk table copy failed");
        d_dedup = p->d_all;
      }
      if (!rc && em && !batched) {  // records the emitter's last prefix stage decided get their mark back
        launch_remark_digested(p->d_res, em->deduped, ps);
        if (hipGetLastError() != hipSuccess) rc = fail(e, NGPU_EHIP, "pack: remark failed");
      }
      if (batched) {
        // the rest runs in the batch, after the engine lock is let go
      } else {
      if (!rc) rc = size_workspace(p);
      if (!rc)
        rc = enqueue_dedup(e, p->dict, d_dedup, n, p->d_res, nullptr, 0, ps, nullptr, 1, nullptr);
      if (!rc) rc = host_fence(e, ps, p->fence);
      // (stream order: the results overwrite h_io after the chunk table left it)
      if (!rc && n &&
          hipMemcpyAsync(p->h_io, p->d_res, n * sizeof(ngpu_result), hipMemcpyDeviceToHost, ps) !=
              hipSuccess)
        rc = fail(e, NGPU_EHIP, "pack: result copy failed");
      if (!rc) rc = read_stats_enqueue(e, ps, p->h_stats);
      path = e->cur->path;  // the digest kernels, for a guard error (read outside the lock)
      }
    }
    if (!batched) not_waitable(p);  // a leader waiting for it stops now
    if (batched && !rc) {  // the slot's bytes are in HBM (or on their way: cs.copied)
      Slot &cs = p->slot[p->cur];
      BatchJob job;
      job.d_data = batch_dev;
      job.len = cs.fill;
      job.h_ch = cs.h_ch;
      job.n = n;
      job.ready = cs.copied;
      job.dict = p->dict;
      job.h_res = p->h_io;
      job.h_stats = p->h_stats;
      rc = batch_run(e, job);
      if (job.uncounted) p->waitable = false;  // (batch_waitable dropped when its batch was taken)
      path = job.path;
    }
    // wait for the pack's own stream without the engine lock (other packs
    // and calls keep enqueueing meanwhile), then check its stats
    if (!rc && hipStreamSynchronize(p->stream) != hipSuccess)
      rc = fail(e, NGPU_EHIP, "pack: stream failed");
    ptrace(p, "finish_dedup_done");
    if (!rc) rc = read_stats_parse(e, p->h_stats, &st, path.c_str());
    if (!rc && n) memcpy(res, p->h_io, n * sizeof(ngpu_result));
    // the blob stream is host work on the pack's own buffers: no engine lock
    if (!rc && w && p->gz) {
      std::unique_ptr<BlobWriter> bw;
      rc = make_writer(p, *opt, w, ctx, &bw);
      if (!rc) rc = ref_finish(p, *bw, ch, res, n, st, info);
    } else if (!rc && w) {
      rc = write_stream(p, *opt, w, ctx, ch, res, n, st, info);
    }
    if (!rc && em) rc = p->gz ? ref_finish(p, *em->bw, ch, res, n, st, info)
                              : emit_finish(p, em, ch, res, n, st, info);
    ptrace(p, "finish_stream_done");
  }
  release(p);
  if (rc) {
    free(ch);
    free(res);
    return rc;
  }
  if (stats) *stats = st;
  *chunks_out = ch;
  *results_out = res;
  *n_out = n;
  return 0;
}

int ngpu_pack_finish(ngpu_pack *p, const ngpu_blob_options *opt, ngpu_write_fn w, void *ctx,
                     ngpu_chunk **chunks_out, ngpu_result **results_out, uint64_t *n_out,
                     ngpu_layer_stats *stats, ngpu_blob_info *info) {
  return guarded([&] { return pack_finish(p, opt, w, ctx, chunks_out, results_out, n_out, stats, info); });
}

}  // extern "C"
