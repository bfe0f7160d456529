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
#include <stdlib.h>
#include <string.h>

#include <condition_variable>
#include <thread>
#include <vector>

#include "engine_internal.hpp"
#include "tarstream.hpp"

using namespace ngpu;

namespace {

struct Slot {
  uint8_t *h = nullptr;       // pinned raw stream bytes
  uint8_t *d = nullptr;       // device copy
  ngpu_chunk *h_ch = nullptr; // pinned slot-relative descriptors
  ngpu_chunk *d_ch = nullptr;
  uint64_t base = 0, fill = 0;
  hipEvent_t copied = nullptr, done = nullptr;
  bool busy = false;
};

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
  ngpu_engine *e = nullptr;
  TarScanner sc;
  Slot slot[2];
  int cur = 0;
  uint64_t cap = 0, max_ch = 0;
  std::vector<ngpu_chunk> chunks;  // stream offsets
  uint64_t dispatched = 0;
  ngpu_result *d_res = nullptr;
  uint64_t res_cap = 0;
  ngpu_chunk *d_all = nullptr;
  hipStream_t copy = nullptr;
  CopyPool *pool = nullptr;  // created on the first large write
  int err = 0;

  explicit ngpu_pack(ngpu_engine *eng) : e(eng), sc(eng->cfg.chunk_size) {}

  int chunk(uint64_t off, uint32_t len, uint32_t fi, uint64_t fo) override {
    chunks.push_back(ngpu_chunk{off, len, fi, fo});
    return 0;
  }
  int data(const uint8_t *, uint64_t) override { return 0; }  // bytes already in the slot
};

namespace {

void release(ngpu_pack *p) {
  if (!p) return;
  (void)hipSetDevice(p->e->device);
  for (Slot &s : p->slot) {
    if (s.done) (void)hipEventSynchronize(s.done);
  }
  if (p->copy) (void)hipStreamSynchronize(p->copy);
  (void)hipStreamSynchronize(p->e->stream);
  for (Slot &s : p->slot) {
    if (s.h) (void)hipHostFree(s.h);
    if (s.h_ch) (void)hipHostFree(s.h_ch);
    if (s.d) (void)hipFree(s.d);
    if (s.d_ch) (void)hipFree(s.d_ch);
    if (s.copied) (void)hipEventDestroy(s.copied);
    if (s.done) (void)hipEventDestroy(s.done);
  }
  if (p->d_res) (void)hipFree(p->d_res);
  if (p->d_all) (void)hipFree(p->d_all);
  if (p->copy) (void)hipStreamDestroy(p->copy);
  delete p->pool;
  delete p;
}

int grow_results(ngpu_pack *p, uint64_t want) {
  if (want <= p->res_cap) return 0;
  uint64_t c = p->res_cap ? p->res_cap : 4096;
  while (c < want) c *= 2;
  ngpu_result *n = nullptr;
  HIP_TRY(p->e, hipMalloc((void **)&n, c * sizeof(ngpu_result)));
  if (p->d_res) {
    HIP_TRY(p->e, hipMemcpyAsync(n, p->d_res, p->dispatched * sizeof(ngpu_result),
                                 hipMemcpyDeviceToDevice, p->e->stream));
    HIP_TRY(p->e, hipStreamSynchronize(p->e->stream));
    (void)hipFree(p->d_res);
  }
  p->d_res = n;
  p->res_cap = c;
  return 0;
}

// Copy the slot to HBM and digest chunks [a, b) (all inside the slot).
int dispatch(ngpu_pack *p, Slot &s, uint64_t a, uint64_t b) {
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
  HIP_TRY(e, hipMemcpyAsync(s.d, s.h, s.fill, hipMemcpyHostToDevice, p->copy));
  HIP_TRY(e, hipMemcpyAsync(s.d_ch, s.h_ch, nch * sizeof(ngpu_chunk), hipMemcpyHostToDevice,
                            p->copy));
  HIP_TRY(e, hipEventRecord(s.copied, p->copy));
  HIP_TRY(e, hipStreamWaitEvent(e->stream, s.copied, 0));
  rc = enqueue_digest(e, s.d, s.fill, s.d_ch, nch, p->d_res + a, e->stream);
  if (rc) return rc;
  HIP_TRY(e, hipEventRecord(s.done, e->stream));
  s.busy = true;
  p->dispatched = b;
  return 0;
}

// Current slot is full: dispatch its complete chunks, carry the chunk in
// progress to the other slot and make that one current.
int switch_slot(ngpu_pack *p) {
  Slot &s = p->slot[p->cur];
  Slot &t = p->slot[p->cur ^ 1];
  const uint64_t end = s.base + s.fill;
  uint64_t k = p->dispatched;
  while (k < p->chunks.size() && p->chunks[k].offset + p->chunks[k].length <= end) ++k;
  const uint64_t carry_from = k < p->chunks.size() ? p->chunks[k].offset : end;
  const uint64_t carry = end - carry_from;
  if (carry >= p->cap) return fail(p->e, NGPU_EINVAL, "chunk larger than a staging slot");
  int rc = dispatch(p, s, p->dispatched, k);
  if (rc) return rc;
  if (t.busy) {
    HIP_TRY(p->e, hipEventSynchronize(t.done));
    t.busy = false;
  }
  memcpy(t.h, s.h + (carry_from - s.base), carry);
  t.base = carry_from;
  t.fill = carry;
  p->cur ^= 1;
  return 0;
}

}  // namespace

extern "C" {

int ngpu_pack_open(ngpu_engine *e, ngpu_pack **out) {
  if (!e || !out) return NGPU_EINVAL;
  *out = nullptr;
  std::lock_guard<std::mutex> g(e->mu);
  HIP_TRY(e, hipSetDevice(e->device));
  ngpu_pack *p = new ngpu_pack(e);
  uint64_t cap = e->cfg.staging_bytes;
  if (cap < 4ull * e->cfg.chunk_size) cap = 4ull * e->cfg.chunk_size;
  p->cap = cap;
  p->max_ch = cap / 1024 + 16;  // a chunk costs >= 1 KiB of tar stream unless it is a file's last
  bool ok = hipStreamCreateWithFlags(&p->copy, hipStreamNonBlocking) == hipSuccess;
  for (Slot &s : p->slot) {
    ok = ok && hipHostMalloc((void **)&s.h, cap, hipHostMallocDefault) == hipSuccess &&
         hipHostMalloc((void **)&s.h_ch, p->max_ch * sizeof(ngpu_chunk), hipHostMallocDefault) ==
             hipSuccess &&
         hipMalloc((void **)&s.d, cap) == hipSuccess &&
         hipMalloc((void **)&s.d_ch, p->max_ch * sizeof(ngpu_chunk)) == hipSuccess &&
         hipEventCreateWithFlags(&s.copied, hipEventDisableTiming) == hipSuccess &&
         hipEventCreateWithFlags(&s.done, hipEventDisableTiming) == hipSuccess;
  }
  // size the digest workspace once so no slot dispatch reallocates it
  if (ok) ok = ensure_workspace(e, p->max_ch, cap, pick_group_log2(e, cap), e->dict.n_blobs, 1) == 0;
  if (!ok) {
    release(p);
    return fail(e, NGPU_ENOMEM, "pack: staging allocation failed");
  }
  *out = p;
  return 0;
}

int ngpu_pack_reserve(ngpu_pack *p, void **ptr, uint64_t *avail) {
  if (!p || !ptr || !avail) return NGPU_EINVAL;
  if (p->err) return p->err;
  Slot &s = p->slot[p->cur];
  if (s.fill == p->cap) {
    std::lock_guard<std::mutex> g(p->e->mu);
    (void)hipSetDevice(p->e->device);
    int rc = switch_slot(p);
    if (rc) return p->err = rc;
  }
  Slot &c = p->slot[p->cur];
  *ptr = c.h + c.fill;
  *avail = p->cap - c.fill;
  return 0;
}

int ngpu_pack_commit(ngpu_pack *p, uint64_t n) {
  if (!p) return NGPU_EINVAL;
  if (p->err) return p->err;
  Slot &s = p->slot[p->cur];
  if (n > p->cap - s.fill) return p->err = NGPU_EINVAL;
  const int rc = p->sc.feed(s.h + s.fill, n, *p);
  s.fill += n;
  if (rc) return p->err = rc;
  return 0;
}

int ngpu_pack_write(ngpu_pack *p, const void *buf, uint64_t len) {
  const uint8_t *b = (const uint8_t *)buf;
  while (len) {
    void *dst;
    uint64_t avail;
    int rc = ngpu_pack_reserve(p, &dst, &avail);
    if (rc) return rc;
    const uint64_t take = len < avail ? len : avail;
    if (take >= (8ull << 20)) {
      if (!p->pool) {
        unsigned hw = std::thread::hardware_concurrency();
        p->pool = new CopyPool(hw >= 16 ? 7 : (hw > 2 ? hw / 2 - 1 : 1));
      }
      p->pool->copy((uint8_t *)dst, b, take);
    } else {
      memcpy(dst, b, take);
    }
    rc = ngpu_pack_commit(p, take);
    if (rc) return rc;
    b += take;
    len -= take;
  }
  return 0;
}

void ngpu_pack_abort(ngpu_pack *p) { release(p); }

int ngpu_pack_close(ngpu_pack *p, ngpu_chunk **chunks_out, ngpu_result **results_out,
                    uint64_t *n_out, ngpu_layer_stats *stats) {
  if (!p || !chunks_out || !results_out || !n_out) {
    release(p);
    return NGPU_EINVAL;
  }
  *chunks_out = nullptr;
  *results_out = nullptr;
  *n_out = 0;
  ngpu_engine *e = p->e;
  int rc = p->err ? p->err : p->sc.finish();
  const uint64_t n = p->chunks.size();
  ngpu_chunk *ch = nullptr;
  ngpu_result *res = nullptr;
  if (!rc) {
    std::lock_guard<std::mutex> g(e->mu);
    (void)hipSetDevice(e->device);
    rc = dispatch(p, p->slot[p->cur], p->dispatched, n);
    if (!rc) rc = grow_results(p, n + 1);
    if (!rc && hipMalloc((void **)&p->d_all, (n + 1) * sizeof(ngpu_chunk)) != hipSuccess)
      rc = fail(e, NGPU_ENOMEM, "pack: chunk table allocation failed");
    ch = (ngpu_chunk *)malloc(sizeof(ngpu_chunk) * (n ? n : 1));
    res = (ngpu_result *)malloc(sizeof(ngpu_result) * (n ? n : 1));
    if (!rc && (!ch || !res)) rc = NGPU_ENOMEM;
    if (!rc && n) {
      memcpy(ch, p->chunks.data(), n * sizeof(ngpu_chunk));
      if (hipMemcpyAsync(p->d_all, ch, n * sizeof(ngpu_chunk), hipMemcpyHostToDevice,
                         e->stream) != hipSuccess)
        rc = fail(e, NGPU_EHIP, "pack: chunk table copy failed");
    }
    if (!rc) rc = enqueue_dedup(e, p->d_all, n, p->d_res, nullptr, 0, e->stream, nullptr, 1, nullptr);
    if (!rc && n &&
        hipMemcpyAsync(res, p->d_res, n * sizeof(ngpu_result), hipMemcpyDeviceToHost,
                       e->stream) != hipSuccess)
      rc = fail(e, NGPU_EHIP, "pack: result copy failed");
    if (!rc) rc = read_stats(e, e->stream, stats);
  }
  release(p);
  if (rc) {
    free(ch);
    free(res);
    return rc;
  }
  *chunks_out = ch;
  *results_out = res;
  *n_out = n;
  return 0;
}

}  // extern "C"
