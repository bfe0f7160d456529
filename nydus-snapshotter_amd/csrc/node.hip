// node.hip — one process driving the GPUs of a node, and
// node chunk dicts: partitioned by digest prefix, or replicated.
//
// The reference converts layers concurrently in one process (goroutines,
// pkg/converter/convert_unix.go:467-538) and hands each to its own
// nydus-image; the chunk dict is loaded by every one of them.  Here a node
// keeps one engine per GPU and one dict for all of them.  A partitioned dict
// keeps the entries whose digest prefix maps to device o on device o
// (owner = ((d[0] << 8 | d[1]) * n) >> 16, nydus_gpu/dist.py's rule), in
// global table order, with their global entry ids, so "first entry wins" and
// the DICT results are the same as with the whole dict on one GPU.
//
// The exchange (the north star's digest-prefix all-to-all, in-process): the
// requester packs its chunk digests (n x 32 B), every owner receives them over
// xGMI with hipMemcpyPeerAsync, probes the rows it owns, and its hit array
// (n x 24 B) goes back the same way; the requester merges the W arrays by
// owner.  Every (owner, requester) pair has its own channel -- probe stream,
// buffers and cached done event on the owner -- so W requesters exchange at
// once with no shared lock, buffer or queue between them; an owner's W
// probes run concurrently on its CUs.  Copies, not peer loads/stores from kernels:
// the DMA engines keep coarse-grained HBM coherent across the GPUs, and the
// payload is tiny (16K chunks of a 16 GiB layer = 512 KiB out, 384 KiB back
// per owner), so the exchange is latency-bound, not link-bound.
//
// The node step (ngpu_node_process_step) is the bulk form: every part at
// once, one all-to-all-v of digests and one of hits, over RCCL or peer
// copies.  It routes into padded per-owner segments (a2a_plan.hpp) so that
// no transfer size depends on a device-side count: the counts cross in band
// and the whole step enqueues without a host wait.
#include <dlfcn.h>
#include <stdio.h>
#include <string.h>
#include <sys/stat.h>

#include <algorithm>

#include <rccl/rccl.h>

#include "a2a_plan.hpp"
#include "engine_internal.hpp"

using namespace ngpu;

namespace {
// Buffers of one part of a node step (ngpu_node_process_step), on its device.
struct StepBuf {
  uint8_t *xq = nullptr;          // its digests bucketed by owner, padded: W x n rows of 32 B
  uint32_t *xrow = nullptr;       // their row ids (~0: padding)
  ngpu_dict_hit *sh = nullptr;    // hits returned, same (owner-bucketed, padded) order
  ngpu_dict_hit *hits = nullptr;  // hits by row
  uint64_t cap = 0;               // rows of xq / xrow / sh / hits
  uint8_t *rq = nullptr;          // digests it received as owner (R x 32)
  ngpu_dict_hit *rh = nullptr;    // its hits for them
  uint64_t rcap = 0;
  uint32_t *cnt = nullptr;        // 128 u32: per-owner counts (+ scatter cursors)
  uint32_t *rcnt = nullptr;       // 64 u32: as owner, each requester's count (in band)
  hipEvent_t counted = nullptr, sent = nullptr, returned = nullptr, done = nullptr;
};
}  // namespace

struct ngpu_node {
  std::vector<ngpu_engine *> eng;  // one per listed device (a reference each)
  std::vector<int> dev;
  std::atomic<uint64_t> rr{0};     // where a Pack's least-loaded search starts (ties)
  std::mutex place_mu;             // one placement at a time: concurrent opens spread evenly
  // node dicts opened by path (one reference each; ngpu_node_dict_open)
  std::vector<ngpu_dict *> dict_cache;
  std::mutex cache_mu;
  bool peer_ok = true;             // every pair of distinct devices has peer access
  // node steps (ngpu_node_process_step): one at a time, buffers per part,
  // the RCCL communicator of the node's devices once a step asked for it
  std::mutex step_mu;
  std::vector<StepBuf> sb;
  bool stepped = false;            // sb[*].done recorded by a previous step
  std::vector<ncclComm_t> comms;
};

namespace ngpu {

static uint32_t owner_of(const uint8_t *d, uint32_t W) {
  return (uint32_t)((((uint64_t)d[0] << 8 | d[1]) * W) >> 16);
}

static void free_io(ngpu_dict::PartIO &io, int device) {
  DeviceGuard g(device);
  if (io.stream) (void)hipStreamSynchronize(io.stream);
  if (io.q) (void)hipFree(io.q);
  if (io.h) (void)hipFree(io.h);
  io.q = nullptr;
  io.h = nullptr;
  io.cap = 0;
}

// The requester's channel set: found (or added) under req_mu, which is held
// for the lookup only -- the enqueue itself runs under the requester's own mu.
static ngpu_dict::Requester *requester_of(ngpu_engine *e, ngpu_dict *d) {
  std::lock_guard<std::mutex> g(d->req_mu);
  for (auto &r : d->req)
    if (r->engine_uid == e->uid) return r.get();
  d->req.emplace_back(new ngpu_dict::Requester());
  ngpu_dict::Requester *r = d->req.back().get();
  r->engine_uid = e->uid;
  r->device = e->device;
  r->io.resize(d->parts.size());
  return r;
}

// One owner's channel for this requester: stream, buffers for n rows and the
// done event on the owner's device (created once, reused by every call).
static int channel_ready(ngpu_engine *e, ngpu_dict::PartIO &io, int device, uint64_t n,
                         uint64_t cap) {
  DeviceGuard dg(device);
  if (!io.stream && hipStreamCreateWithFlags(&io.stream, hipStreamNonBlocking) != hipSuccess)
    return fail(e, NGPU_EHIP, "node dict: probe stream on device %d", device);
  if (!io.done && hipEventCreateWithFlags(&io.done, hipEventDisableTiming) != hipSuccess)
    return fail(e, NGPU_EHIP, "node dict: exchange event on device %d", device);
  if (n > io.cap) {
    free_io(io, device);  // the stream's earlier exchanges finish first
    if (hipMalloc((void **)&io.q, cap * 32) != hipSuccess ||
        hipMalloc((void **)&io.h, cap * sizeof(ngpu_dict_hit)) != hipSuccess) {
      free_io(io, device);
      return fail(e, NGPU_ENOMEM, "node dict: exchange buffers on device %d", device);
    }
    io.cap = cap;
  }
  return 0;
}

// The routed exchange (ABI 4): the requester buckets its n digests by owner in
// its own HBM (ws.xq rows, ws.xrow row ids, ws.xcnt counts); owner o's probe
// kernel, launched on o's device after the requester's `ready` event, reads
// only its own segment (peer loads over xGMI) and stores each hit at its row
// in the requester's ws.xhits (peer stores).  The requester's stream waits for
// every owner's `done`.  Bytes over the links per call: n x 36 out and n x 24
// back in total, against W x n x 56 for the copy exchange below it.
// Reuse is stream-ordered: the next call's routing on s runs after this call's
// waits on every `done`, so no owner still reads ws.xq when it is rewritten.
static int routed_hits(ngpu_engine *e, ngpu_dict *d, const uint8_t *digests, uint64_t stride,
                       uint64_t n, hipStream_t s, const ngpu_dict_hit **hits) {
  const uint32_t W = (uint32_t)d->parts.size();
  Workspace &ws = e->cur->ws;
  const bool regrow = n > ws.cap_x || !ws.xq || !ws.xrow || !ws.xhits;
  if (regrow && (ws.xq || ws.xrow || ws.xhits))
    if (int rc = slot_quiesce(e)) return rc;  // no buffer freed under a running stage
  if (regrow) {
    if (ws.xq) (void)hipFree(ws.xq), ws.xq = nullptr;
    if (ws.xhits) (void)hipFree(ws.xhits), ws.xhits = nullptr;
    if (ws.xrow) (void)hipFree(ws.xrow), ws.xrow = nullptr;
    const uint64_t c = next_pow2(n < 1024 ? 1024 : n);
    HIP_TRY(e, hipMalloc((void **)&ws.xq, c * 32));
    HIP_TRY(e, hipMalloc((void **)&ws.xhits, c * sizeof(ngpu_dict_hit)));
    HIP_TRY(e, hipMalloc((void **)&ws.xrow, c * 4));
    ws.cap_x = c;
  }
  if (!ws.xcnt) HIP_TRY(e, hipMalloc((void **)&ws.xcnt, 128 * sizeof(uint32_t)));
  *hits = ws.xhits;
  if (n == 0) return 0;
  ngpu_dict::Requester *r = requester_of(e, d);
  std::lock_guard<std::mutex> g(r->mu);  // this requester's channels only
  if (!r->ready) HIP_TRY(e, hipEventCreateWithFlags(&r->ready, hipEventDisableTiming));
  launch_route(digests, stride, n, W, 0, ws.xcnt, ws.xq, ws.xrow, s);
  HIP_TRY(e, hipGetLastError());
  HIP_TRY(e, hipEventRecord(r->ready, s));
  int rc = 0;
  uint32_t sent = 0;
  for (uint32_t o = 0; o < W && !rc; ++o, ++sent) {
    ngpu_dict *p = d->parts[o];
    ngpu_dict::PartIO &io = r->io[o];
    if ((rc = channel_ready(e, io, p->device, 0, 0))) break;
    DeviceGuard dg(p->device);
    if (hipStreamWaitEvent(io.stream, r->ready, 0) != hipSuccess) {
      rc = fail(e, NGPU_EHIP, "node dict: wait on the requester failed (device %d)", p->device);
      break;
    }
    launch_dict_probe_routed(ws.xq, ws.xrow, ws.xcnt, n, o, p->dev, ws.xhits, io.stream);
    if (hipGetLastError() != hipSuccess || hipEventRecord(io.done, io.stream) != hipSuccess)
      rc = fail(e, NGPU_EHIP, "node dict: routed probe on device %d failed", p->device);
  }
  // the requester's stream waits for every owner it enqueued, even on failure,
  // so no later stage reuses ws.xq / ws.xhits under a probe still in flight
  for (uint32_t o = 0; o < sent && o < W; ++o)
    if (r->io[o].done && hipStreamWaitEvent(s, r->io[o].done, 0) != hipSuccess && !rc)
      rc = fail(e, NGPU_EHIP, "node dict: cross-device wait failed");
  return rc;
}

int node_dict_hits(ngpu_engine *e, ngpu_dict *d, const uint8_t *digests, uint64_t stride,
                   uint64_t n, hipStream_t s, const ngpu_dict_hit **hits, ngpu_dict **replica) {
  *hits = nullptr;
  *replica = nullptr;
  if (d->replicated) {  // no exchange: the copy on this engine's device
    for (ngpu_dict *p : d->parts)
      if (p->device == e->device) {
        *replica = p;
        return 0;
      }
    return fail(e, NGPU_EINVAL, "node chunk dict has no replica on device %d", e->device);
  }
  const uint32_t W = (uint32_t)d->parts.size();
  Workspace &ws = e->cur->ws;  // the dedup stage's slot (use_slot)
  if (d->routed) return routed_hits(e, d, digests, stride, n, s, hits);
  if (((n > ws.cap_x && ws.xq) || ((uint64_t)W * n > ws.cap_xparts && ws.xparts)))
    if (int rc = slot_quiesce(e)) return rc;  // no buffer freed under a running stage
  if (n > ws.cap_x || !ws.xq) {
    if (ws.xq) (void)hipFree(ws.xq), ws.xq = nullptr;
    if (ws.xhits) (void)hipFree(ws.xhits), ws.xhits = nullptr;
    const uint64_t c = next_pow2(n < 1024 ? 1024 : n);
    HIP_TRY(e, hipMalloc((void **)&ws.xq, c * 32));
    HIP_TRY(e, hipMalloc((void **)&ws.xhits, c * sizeof(ngpu_dict_hit)));
    ws.cap_x = c;
  }
  if ((uint64_t)W * n > ws.cap_xparts || !ws.xparts) {
    if (ws.xparts) (void)hipFree(ws.xparts), ws.xparts = nullptr;
    const uint64_t c = (uint64_t)W * ws.cap_x;
    HIP_TRY(e, hipMalloc((void **)&ws.xparts, c * sizeof(ngpu_dict_hit)));
    ws.cap_xparts = c;
  }
  *hits = ws.xhits;
  if (n == 0) return 0;
  ngpu_dict::Requester *r = requester_of(e, d);
  std::lock_guard<std::mutex> g(r->mu);  // this requester's channels only
  if (!r->ready) HIP_TRY(e, hipEventCreateWithFlags(&r->ready, hipEventDisableTiming));
  launch_pack_digests(digests, stride, n, ws.xq, s);
  HIP_TRY(e, hipEventRecord(r->ready, s));
  int rc = 0;
  uint32_t sent = 0;
  for (uint32_t o = 0; o < W && !rc; ++o, ++sent) {
    ngpu_dict *p = d->parts[o];
    ngpu_dict::PartIO &io = r->io[o];
    if ((rc = channel_ready(e, io, p->device, n, ws.cap_x))) break;
    DeviceGuard dg(p->device);
    const bool ok =
        hipStreamWaitEvent(io.stream, r->ready, 0) == hipSuccess &&
        hipMemcpyPeerAsync(io.q, p->device, ws.xq, e->device, n * 32, io.stream) == hipSuccess;
    if (ok) launch_dict_probe_owned(io.q, n, o, W, p->dev, io.h, io.stream);
    if (!ok || hipGetLastError() != hipSuccess ||
        hipMemcpyPeerAsync(ws.xparts + (uint64_t)o * n, e->device, io.h, p->device,
                           n * sizeof(ngpu_dict_hit), io.stream) != hipSuccess ||
        hipEventRecord(io.done, io.stream) != hipSuccess)
      rc = fail(e, NGPU_EHIP, "node dict: exchange with device %d failed", p->device);
  }
  // the requester's stream waits for every owner it enqueued, even on failure,
  // so no later stage reuses ws.xq / ws.xparts under a copy still in flight
  for (uint32_t o = 0; o < sent && o < W; ++o)
    if (r->io[o].done && hipStreamWaitEvent(s, r->io[o].done, 0) != hipSuccess && !rc)
      rc = fail(e, NGPU_EHIP, "node dict: cross-device wait failed");
  if (rc) return rc;
  launch_hits_merge(ws.xq, n, W, ws.xparts, ws.xhits, s);
  HIP_TRY(e, hipGetLastError());
  return 0;
}

namespace {

// A node dict over records in host memory (each part built on its device's
// own build stream, no engine lock held).
int node_dict_build(ngpu_node *node, const uint8_t *recs, uint64_t m, const uint8_t *blobs,
                    uint32_t n_blobs, uint32_t mode, ngpu_dict **out) {
  ngpu_engine *e0 = node->eng[0];
  const bool routed = (mode & NGPU_NODE_EXCHANGE_ROUTED) != 0;
  if ((mode & NGPU_NODE_EXCHANGE_COPY) && routed)
    return fail(e0, NGPU_EINVAL, "node dict: copy and routed exchange both asked for");
  mode &= ~(NGPU_NODE_EXCHANGE_COPY | NGPU_NODE_EXCHANGE_ROUTED);
  if (mode != NGPU_NODE_DICT_PARTITION && mode != NGPU_NODE_DICT_REPLICATE)
    return fail(e0, NGPU_EINVAL, "bad node dict mode %u", mode);
  if (m >= 0xFFFFFFFFull) return fail(e0, NGPU_EINVAL, "chunk dict too large");
  uint32_t nb = 0;
  for (uint64_t i = 0; i < m; ++i) {
    const RafsV6ChunkInfo *r = reinterpret_cast<const RafsV6ChunkInfo *>(recs + 80 * i);
    nb = std::max(nb, r->blob_index + 1);
  }
  if (n_blobs) {
    if (nb > n_blobs) return fail(e0, NGPU_EFORMAT, "chunk dict record points at blob %u of %u",
                                  nb - 1, n_blobs);
    nb = n_blobs;
  }
  ngpu_dict *d = new ngpu_dict();
  d->device = node->dev[0];
  d->digester = e0->cfg.digester;
  d->chunk_size = e0->cfg.chunk_size;
  d->replicated = mode == NGPU_NODE_DICT_REPLICATE;
  // the copy exchange (DMA peer copies) unless the routed one was asked for
  // and every pair of devices has peer access (its kernels reach the
  // requester's HBM): the routed exchange's peer stores have not met two
  // distinct GPUs yet
  d->routed = !d->replicated && routed && node->peer_ok;
  d->dev.m = m;
  d->dev.n_blobs = nb;
  d->place.resize(m);
  for (uint64_t i = 0; i < m; ++i) {
    const RafsV6ChunkInfo *r = reinterpret_cast<const RafsV6ChunkInfo *>(recs + 80 * i);
    d->place[i] = DictPlace{r->compressed_offset, r->compressed_size, r->flags};
  }
  if (blobs && n_blobs) d->blob_table.assign(blobs, blobs + 256ull * n_blobs);
  const uint32_t W = (uint32_t)node->eng.size();
  // partition: rows per owner in global table order, with their global ids
  std::vector<std::vector<uint8_t>> part_recs(W);
  std::vector<std::vector<uint32_t>> gid(W);
  if (!d->replicated) {
    for (uint64_t i = 0; i < m; ++i) {
      const uint32_t o = owner_of(recs + 80 * i, W);
      part_recs[o].insert(part_recs[o].end(), recs + 80 * i, recs + 80 * (i + 1));
      gid[o].push_back((uint32_t)i);
    }
  }
  int rc = 0;
  for (uint32_t o = 0; o < W && !rc; ++o) {
    ngpu_engine *e = node->eng[o];
    DeviceGuard dg(e->device);
    ngpu_dict *p = nullptr;
    const uint8_t *pr = d->replicated ? recs : part_recs[o].data();
    const uint64_t pm = d->replicated ? m : gid[o].size();
    if ((rc = dict_from_records(e, pr, pm, blobs, nb, &p, d->replicated ? nullptr : gid[o].data())))
      break;
    p->dev.n_blobs = nb;
    p->place.clear();  // the global table (d->place) answers the writer
    d->parts.push_back(p);
  }
  if (rc) {
    dict_unref(d);
    return rc;
  }
  *out = d;
  return 0;
}

}  // namespace

// Called by dict_unref for a node dict.
void node_dict_free(ngpu_dict *d) {
  for (auto &r : d->req) {
    for (size_t o = 0; o < r->io.size() && o < d->parts.size(); ++o) {
      ngpu_dict::PartIO &io = r->io[o];
      const int dev = d->parts[o]->device;
      free_io(io, dev);
      DeviceGuard g(dev);
      if (io.stream) (void)hipStreamDestroy(io.stream);
      if (io.done) (void)hipEventDestroy(io.done);
    }
    if (r->ready) {
      DeviceGuard g(r->device);
      (void)hipEventDestroy(r->ready);
    }
  }
  d->req.clear();
  for (ngpu_dict *p : d->parts) dict_unref(p);
  d->parts.clear();
}

// ---- node step ---------------------------------------------------------------
namespace {

// RCCL is loaded when a step first asks for it (dlopen): processes that never
// run an RCCL step do not map its 570 MB library or register its kernels.
struct Rccl {
  decltype(&ncclCommInitAll) init = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclAllToAllv) alltoallv = nullptr;
  decltype(&ncclGetErrorString) err = nullptr;
  bool ok = false;
};
const Rccl &rccl() {
  static const Rccl r = [] {
    Rccl x;
    void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) return x;
    x.init = (decltype(x.init))dlsym(h, "ncclCommInitAll");
    x.destroy = (decltype(x.destroy))dlsym(h, "ncclCommDestroy");
    x.group_start = (decltype(x.group_start))dlsym(h, "ncclGroupStart");
    x.group_end = (decltype(x.group_end))dlsym(h, "ncclGroupEnd");
    x.alltoallv = (decltype(x.alltoallv))dlsym(h, "ncclAllToAllv");
    x.err = (decltype(x.err))dlsym(h, "ncclGetErrorString");
    x.ok = x.init && x.destroy && x.group_start && x.group_end && x.alltoallv && x.err;
    return x;
  }();
  return r;
}

void step_free(ngpu_node *node) {
  for (size_t i = 0; i < node->sb.size(); ++i) {
    StepBuf &b = node->sb[i];
    DeviceGuard g(node->dev[i]);
    if (b.done) (void)hipEventSynchronize(b.done);
    for (void *p : {(void *)b.xq, (void *)b.xrow, (void *)b.sh, (void *)b.hits, (void *)b.rq,
                    (void *)b.rh, (void *)b.cnt, (void *)b.rcnt})
      if (p) (void)hipFree(p);
    for (hipEvent_t ev : {b.counted, b.sent, b.returned, b.done})
      if (ev) (void)hipEventDestroy(ev);
  }
  node->sb.clear();
  for (ncclComm_t c : node->comms)
    if (c) (void)rccl().destroy(c);
  node->comms.clear();
}

// The node's RCCL communicator (one rank per device), created on first use.
int step_comms(ngpu_node *node) {
  ngpu_engine *e0 = node->eng[0];
  if (!node->comms.empty()) return 0;
  if (!rccl().ok) return fail(e0, NGPU_EUNSUPP, "node step over RCCL: librccl.so.1 not loadable");
  const int W = (int)node->dev.size();
  for (int a = 0; a < W; ++a)
    for (int b = a + 1; b < W; ++b)
      if (node->dev[a] == node->dev[b])
        return fail(e0, NGPU_EUNSUPP, "node step over RCCL: device %d is listed twice (RCCL "
                    "takes one rank per GPU)", node->dev[a]);
  std::vector<ncclComm_t> c((size_t)W);
  const ncclResult_t r = rccl().init(c.data(), W, node->dev.data());
  if (r != ncclSuccess)
    return fail(e0, NGPU_EHIP, "node step: ncclCommInitAll over %d devices: %s", W,
                rccl().err(r));
  node->comms = std::move(c);
  return 0;
}

// quiesce: waits for the previous step before a buffer it may still use is freed
template <class Q>
int step_grow(ngpu_engine *e, StepBuf &b, uint64_t n, uint64_t r, Q &&quiesce) {
  if (!b.cnt) HIP_TRY(e, hipMalloc((void **)&b.cnt, 128 * sizeof(uint32_t)));
  if (!b.rcnt) HIP_TRY(e, hipMalloc((void **)&b.rcnt, 64 * sizeof(uint32_t)));
  for (hipEvent_t *ev : {&b.counted, &b.sent, &b.returned, &b.done})
    if (!*ev) HIP_TRY(e, hipEventCreateWithFlags(ev, hipEventDisableTiming));
  if ((n > b.cap && b.xq) || (r > b.rcap && b.rq))
    if (int rc = quiesce()) return rc;
  if (n > b.cap || !b.xq) {
    for (void *p : {(void *)b.xq, (void *)b.xrow, (void *)b.sh, (void *)b.hits})
      if (p) (void)hipFree(p);
    b.xq = nullptr, b.xrow = nullptr, b.sh = nullptr, b.hits = nullptr, b.cap = 0;
    const uint64_t c = next_pow2(n < 1024 ? 1024 : n);
    HIP_TRY(e, hipMalloc((void **)&b.xq, c * 32));
    HIP_TRY(e, hipMalloc((void **)&b.xrow, c * 4));
    HIP_TRY(e, hipMalloc((void **)&b.sh, c * sizeof(ngpu_dict_hit)));
    HIP_TRY(e, hipMalloc((void **)&b.hits, c * sizeof(ngpu_dict_hit)));
    b.cap = c;
  }
  if (r > b.rcap || !b.rq) {
    if (b.rq) (void)hipFree(b.rq);
    if (b.rh) (void)hipFree(b.rh);
    b.rq = nullptr, b.rh = nullptr, b.rcap = 0;
    const uint64_t c = next_pow2(r < 1024 ? 1024 : r);
    HIP_TRY(e, hipMalloc((void **)&b.rq, c * 32));
    HIP_TRY(e, hipMalloc((void **)&b.rh, c * sizeof(ngpu_dict_hit)));
    b.rcap = c;
  }
  return 0;
}

#define NCCL_TRY(e, x)                                                                  \
  do {                                                                                  \
    const ncclResult_t r_ = (x);                                                        \
    if (r_ != ncclSuccess) return fail(e, NGPU_EHIP, "node step: %s: %s", #x, rccl().err(r_)); \
  } while (0)

// One all-to-all-v of `row`-byte rows: part i sends cnt_send(i, j) rows from
// src[i] + sdis(i, j) to part j, which stores them at dst[j] + rdis(j, i).
template <class CntF, class SdisF, class RdisF>
int step_alltoallv(ngpu_node *node, bool use_rccl, const std::vector<hipStream_t> &s,
                   const std::vector<const uint8_t *> &src, const std::vector<uint8_t *> &dst,
                   uint64_t row, CntF cnt_send, SdisF sdis, RdisF rdis, hipEvent_t StepBuf::*mark) {
  ngpu_engine *e0 = node->eng[0];
  const uint32_t W = (uint32_t)node->eng.size();
  if (use_rccl) {
    std::vector<size_t> sc(W), sd(W), rc(W), rd(W);
    NCCL_TRY(e0, rccl().group_start());
    for (uint32_t i = 0; i < W; ++i) {
      a2a_rank_args(W, i, row, cnt_send, sdis, rdis, sc.data(), sd.data(), rc.data(), rd.data());
      const ncclResult_t r = rccl().alltoallv(src[i], sc.data(), sd.data(), dst[i], rc.data(),
                                              rd.data(), ncclUint8, node->comms[i], s[i]);
      if (r != ncclSuccess) {
        (void)rccl().group_end();
        return fail(e0, NGPU_EHIP, "node step: ncclAllToAllv: %s", rccl().err(r));
      }
    }
    NCCL_TRY(e0, rccl().group_end());
    return 0;
  }
  // peer copies on the sender's stream; every receiver waits for every sender
  for (uint32_t i = 0; i < W; ++i) {
    DeviceGuard g(node->dev[i]);
    for (uint32_t j = 0; j < W; ++j) {
      const uint64_t c = cnt_send(i, j);
      if (c)
        HIP_TRY(e0, hipMemcpyPeerAsync(dst[j] + rdis(j, i) * row, node->dev[j],
                                       src[i] + sdis(i, j) * row, node->dev[i], c * row, s[i]));
    }
    HIP_TRY(e0, hipEventRecord(node->sb[i].*mark, s[i]));
  }
  for (uint32_t j = 0; j < W; ++j) {
    DeviceGuard g(node->dev[j]);
    for (uint32_t i = 0; i < W; ++i)
      if (i != j) HIP_TRY(e0, hipStreamWaitEvent(s[j], node->sb[i].*mark, 0));
  }
  return 0;
}

int node_step_enqueue(ngpu_node *node, ngpu_dict *d, const ngpu_node_part *pt, uint32_t W,
                      bool use_rccl);

// A failed step may have enqueued part of its work on the parts' streams: it
// is waited for before the step buffers can be reused (or freed).
int node_step(ngpu_node *node, ngpu_dict *d, const ngpu_node_part *pt, uint32_t np, uint32_t flags) {
  ngpu_engine *e0 = node->eng[0];
  const uint32_t W = (uint32_t)node->eng.size();
  if (np != W) return fail(e0, NGPU_EINVAL, "node step: %u parts for a node of %u devices", np, W);
  for (uint32_t i = 0; i < W; ++i) {
    const ngpu_node_part &p = pt[i];
    if ((p.n && (!p.d_data || !p.d_chunks || !p.d_out)) || (p.d_layer_first && !p.n_layers) ||
        p.n >= 0xFFFFFFFFull)
      return fail(e0, NGPU_EINVAL, "node step: bad part %u", i);
  }
  if (!d || d->parts.empty() || d->replicated) {  // no exchange: each part on its own
    for (uint32_t i = 0; i < W; ++i) {
      const ngpu_node_part &p = pt[i];
      if (int rc = ngpu_process_dict_device(node->eng[i], d, p.d_data, p.len, p.d_chunks, p.n,
                                            p.d_out, p.d_layer_first, p.n_layers, p.d_stats,
                                            p.stream, nullptr))
        return rc;
    }
    return 0;
  }
  if (d->parts.size() != W) return fail(e0, NGPU_EINVAL, "node step: the dict has %zu parts, the node %u devices",
                                        d->parts.size(), W);
  for (uint32_t i = 0; i < W; ++i)
    if (d->parts[i]->device != node->dev[i])
      return fail(e0, NGPU_EINVAL, "node step: dict part %u is not on node device %u", i, i);
  const bool use_rccl = (flags & NGPU_NODE_STEP_RCCL) != 0;
  std::lock_guard<std::mutex> g(node->step_mu);
  if (use_rccl)
    if (int rc = step_comms(node)) return rc;
  const int rc = node_step_enqueue(node, d, pt, W, use_rccl);
  if (rc) {
    for (uint32_t i = 0; i < W; ++i) {
      DeviceGuard dg(node->dev[i]);
      (void)hipStreamSynchronize((hipStream_t)pt[i].stream);
    }
    node->stepped = false;  // nothing of this step is still in flight
  }
  return rc;
}

int node_step_enqueue(ngpu_node *node, ngpu_dict *d, const ngpu_node_part *pt, uint32_t W,
                      bool use_rccl) {
  ngpu_engine *e0 = node->eng[0];
  node->sb.resize(W);
  bool quiet = !node->stepped;
  auto quiesce = [&]() -> int {  // the previous step done on every device
    for (uint32_t j = 0; j < W && !quiet; ++j) {
      DeviceGuard dg(node->dev[j]);
      HIP_TRY(e0, hipEventSynchronize(node->sb[j].done));
    }
    quiet = true;
    return 0;
  };
  std::vector<hipStream_t> s(W);
  for (uint32_t i = 0; i < W; ++i) s[i] = (hipStream_t)pt[i].stream;
  // the padded layout (a2a_plan.hpp): every transfer size is known here, the
  // per-owner counts travel in band, and nothing below waits for the device
  std::vector<uint64_t> n(W), off(W + 1, 0);
  for (uint32_t i = 0; i < W; ++i) n[i] = pt[i].n, off[i + 1] = off[i] + n[i];
  if (W > 64) return fail(e0, NGPU_EINVAL, "node step: %u parts (at most 64)", W);
  const PaddedStep ps{W, n.data(), off.data()};
  // buffers are reused: this step's streams start after every part of the last
  for (uint32_t i = 0; i < W; ++i) {
    DeviceGuard dg(node->dev[i]);
    if (int rc = step_grow(node->eng[i], node->sb[i], (uint64_t)W * n[i], off[W], quiesce))
      return rc;
    if (node->stepped)
      for (uint32_t j = 0; j < W; ++j) HIP_TRY(e0, hipStreamWaitEvent(s[i], node->sb[j].done, 0));
  }
  // 1. digests; 2. bucketed by owner into padded segments (seg_cap = n), the
  // padding rows' ids ~0
  for (uint32_t i = 0; i < W; ++i) {
    const ngpu_node_part &p = pt[i];
    StepBuf &b = node->sb[i];
    if (p.n)
      if (int rc = ngpu_digest_device(node->eng[i], p.d_data, p.len, p.d_chunks, p.n, p.d_out, p.stream))
        return rc;
    DeviceGuard dg(node->dev[i]);
    if (p.n) HIP_TRY(e0, hipMemsetAsync(b.xrow, 0xFF, (size_t)W * p.n * sizeof(uint32_t), s[i]));
    launch_route(reinterpret_cast<const uint8_t *>(p.d_out), sizeof(ngpu_result), p.n, W, p.n,
                 b.cnt, b.xq, b.xrow, s[i]);
    HIP_TRY(e0, hipGetLastError());
  }
  std::vector<const uint8_t *> src(W);
  std::vector<uint8_t *> dst(W);
  // 3. counts (requester i's cnt[j] -> owner j's rcnt[i]) and digests to their owners
  for (uint32_t i = 0; i < W; ++i)
    src[i] = reinterpret_cast<const uint8_t *>(node->sb[i].cnt),
    dst[i] = reinterpret_cast<uint8_t *>(node->sb[i].rcnt);
  if (int rc = step_alltoallv(node, use_rccl, s, src, dst, sizeof(uint32_t), PaddedStep::cnt_cnt,
                              PaddedStep::cnt_sdis, PaddedStep::cnt_rdis, &StepBuf::counted))
    return rc;
  for (uint32_t i = 0; i < W; ++i) src[i] = node->sb[i].xq, dst[i] = node->sb[i].rq;
  if (int rc = step_alltoallv(
          node, use_rccl, s, src, dst, 32, [&](uint32_t i, uint32_t j) { return ps.fwd_cnt(i, j); },
          [&](uint32_t i, uint32_t j) { return ps.fwd_sdis(i, j); },
          [&](uint32_t j, uint32_t i) { return ps.fwd_rdis(j, i); }, &StepBuf::sent))
    return rc;
  // 4. owners probe the counted rows of each requester's block
  ProbeBlocks pb{};
  pb.W = W;
  for (uint32_t i = 0; i <= W; ++i) pb.off[i] = off[i];
  for (uint32_t j = 0; j < W; ++j) {
    DeviceGuard dg(node->dev[j]);
    launch_dict_probe_blocks(node->sb[j].rq, node->sb[j].rcnt, pb, d->parts[j]->dev, node->sb[j].rh,
                             s[j]);
    HIP_TRY(e0, hipGetLastError());
  }
  // 5. hits back: owner j sends requester i's block to i's segment j
  for (uint32_t j = 0; j < W; ++j)
    src[j] = reinterpret_cast<const uint8_t *>(node->sb[j].rh),
    dst[j] = reinterpret_cast<uint8_t *>(node->sb[j].sh);
  if (int rc = step_alltoallv(
          node, use_rccl, s, src, dst, sizeof(ngpu_dict_hit),
          [&](uint32_t j, uint32_t i) { return ps.back_cnt(j, i); },
          [&](uint32_t j, uint32_t i) { return ps.back_sdis(j, i); },
          [&](uint32_t i, uint32_t j) { return ps.back_rdis(i, j); }, &StepBuf::returned))
    return rc;
  // 6. hits to their rows (padding rows dropped by their ~0 id), then each
  // part's own dedup
  const uint32_t nb = d->dev.n_blobs ? d->dev.n_blobs : 1;
  for (uint32_t i = 0; i < W; ++i) {
    const ngpu_node_part &p = pt[i];
    StepBuf &b = node->sb[i];
    ngpu_engine *e = node->eng[i];
    if (p.n) {
      DeviceGuard dg(e->device);
      launch_hits_scatter(b.sh, b.xrow, (uint64_t)W * p.n, b.hits, s[i]);
      HIP_TRY(e0, hipGetLastError());
      std::lock_guard<std::mutex> eg(e->mu);
      if (int rc = enqueue_dedup(e, nullptr, p.d_chunks, p.n, p.d_out, b.hits, nb, s[i],
                                 p.d_layer_first, p.d_layer_first ? p.n_layers : 1, p.d_stats))
        return rc;
    }
    DeviceGuard dg(node->dev[i]);
    HIP_TRY(e0, hipEventRecord(b.done, s[i]));
  }
  node->stepped = true;
  return 0;
}

}  // namespace

}  // namespace ngpu

extern "C" {

int ngpu_node_create(const int32_t *devices, uint32_t n, const ngpu_config *cfg, ngpu_node **out) {
  if (!devices || !n || n > 64 || !out) return NGPU_EINVAL;
  *out = nullptr;
  ngpu_node *node = new ngpu_node();
  for (uint32_t i = 0; i < n; ++i) {
    ngpu_config c{};
    if (cfg) c = *cfg;
    c.device = devices[i];
    ngpu_engine *e = nullptr;
    const int rc = ngpu_create(&c, &e);
    if (rc) {
      ngpu_node_destroy(node);
      return rc;
    }
    node->eng.push_back(e);
    node->dev.push_back(devices[i]);
  }
  // xGMI peer access between every pair of distinct devices (the exchange
  // copies go device to device)
  for (uint32_t a = 0; a < n; ++a)
    for (uint32_t b = 0; b < n; ++b) {
      if (node->dev[a] == node->dev[b]) continue;
      int can = 0;
      if (hipDeviceCanAccessPeer(&can, node->dev[a], node->dev[b]) != hipSuccess || !can) {
        (void)hipGetLastError();
        node->peer_ok = false;  // partitioned dicts fall back to the copy exchange
        continue;
      }
      DeviceGuard g(node->dev[a]);
      const hipError_t st = hipDeviceEnablePeerAccess(node->dev[b], 0);
      if (st != hipSuccess && st != hipErrorPeerAccessAlreadyEnabled) {
        ngpu_node_destroy(node);
        return NGPU_EHIP;
      }
      (void)hipGetLastError();
    }
  *out = node;
  return 0;
}

void ngpu_node_destroy(ngpu_node *node) {
  if (!node) return;
  {
    std::vector<ngpu_dict *> cache;
    {
      std::lock_guard<std::mutex> g(node->cache_mu);
      cache.swap(node->dict_cache);
    }
    for (ngpu_dict *d : cache) dict_unref(d);  // the cache's references (packs keep their own)
  }
  step_free(node);
  for (ngpu_engine *e : node->eng) ngpu_destroy(e);
  delete node;
}

uint32_t ngpu_node_size(const ngpu_node *node) { return node ? (uint32_t)node->eng.size() : 0; }

ngpu_engine *ngpu_node_engine(ngpu_node *node, uint32_t i) {
  return node && i < node->eng.size() ? node->eng[i] : nullptr;
}

uint32_t ngpu_node_owner(const ngpu_node *node, const uint8_t *digest) {
  return node && digest ? owner_of(digest, (uint32_t)node->eng.size()) : 0;
}

int ngpu_node_dict_create(ngpu_node *node, const void *records, uint64_t n,
                          const void *blob_table, uint32_t n_blobs, uint32_t mode,
                          ngpu_dict **out) {
  if (!node || !out || (n && !records) || (n_blobs && !blob_table)) return NGPU_EINVAL;
  *out = nullptr;
  return guarded([&] {
    return node_dict_build(node, (const uint8_t *)records, n, (const uint8_t *)blob_table, n_blobs,
                           mode, out);
  });
}

int ngpu_node_dict_open(ngpu_node *node, const char *path, uint32_t mode, ngpu_dict **out) {
  if (!node || !path || !out) return NGPU_EINVAL;
  *out = nullptr;
  return guarded([&] {
    struct stat st;
    ngpu_engine *e0 = node->eng[0];
    if (stat(path, &st) != 0) return fail(e0, NGPU_EIO, "stat chunk dict %s", path);
    const int64_t mt = (int64_t)st.st_mtim.tv_sec * 1000000000 + st.st_mtim.tv_nsec;
    auto same = [&](const ngpu_dict *d) {
      return d->path == path && d->node_mode == mode && d->st_dev == (uint64_t)st.st_dev &&
             d->st_ino == (uint64_t)st.st_ino && d->st_size == (uint64_t)st.st_size &&
             d->st_mtime_ns == mt;
    };
    std::vector<ngpu_dict *> drop;
    {
      std::lock_guard<std::mutex> g(node->cache_mu);
      for (ngpu_dict *d : node->dict_cache)
        if (same(d)) {
          dict_ref(d);
          *out = d;
          return 0;
        }
    }
    std::vector<uint8_t> recs, blobs;
    if (int rc = read_dict_bootstrap(e0, path, (uint64_t)st.st_size, &recs, &blobs)) return rc;
    ngpu_dict *d = nullptr;
    if (int rc = node_dict_build(node, recs.data(), recs.size() / 80, blobs.data(),
                                 (uint32_t)(blobs.size() / 256), mode, &d))
      return rc;
    d->path = path;
    d->node_mode = mode;
    d->st_dev = (uint64_t)st.st_dev;
    d->st_ino = (uint64_t)st.st_ino;
    d->st_size = (uint64_t)st.st_size;
    d->st_mtime_ns = mt;
    {
      std::lock_guard<std::mutex> g(node->cache_mu);
      auto &c = node->dict_cache;
      for (ngpu_dict *x : c)
        if (same(x)) {  // another thread loaded it meanwhile: share that one
          dict_ref(x);
          drop.push_back(d);
          d = x;
          break;
        }
      if (std::find(c.begin(), c.end(), d) == c.end()) {
        for (size_t i = 0; i < c.size();)  // older loads of the path (same mode) go
          if (c[i]->path == path && c[i]->node_mode == mode) {
            drop.push_back(c[i]);
            c.erase(c.begin() + (long)i);
          } else {
            ++i;
          }
        if (c.size() >= 8) {
          drop.push_back(c.front());
          c.erase(c.begin());
        }
        dict_ref(d);  // the cache's reference
        c.push_back(d);
      }
    }
    for (ngpu_dict *x : drop) dict_unref(x);
    *out = d;
    return 0;
  });
}

// Layers shard over the node's GPUs (north star; convert_unix.go:467-538 runs
// one per goroutine): each Pack goes to the engine with the fewest open packs,
// the search starting one further each time so that ties rotate.
int ngpu_node_pack_open(ngpu_node *node, ngpu_dict *dict, uint32_t flags, ngpu_pack **out) {
  if (!node || !out) return NGPU_EINVAL;
  const size_t W = node->eng.size();
  std::lock_guard<std::mutex> g(node->place_mu);
  const uint64_t r = node->rr.fetch_add(1, std::memory_order_relaxed);
  size_t best = r % W;
  int load = node->eng[best]->open_packs.load();
  for (size_t k = 1; k < W; ++k) {
    const size_t i = (r + k) % W;
    const int l = node->eng[i]->open_packs.load();
    if (l < load) best = i, load = l;
  }
  return ngpu_pack_open_dict(node->eng[best], dict, flags, out);
}

int ngpu_node_process_device(ngpu_node *node, uint32_t i, ngpu_dict *dict, const void *d_data,
                             uint64_t len, const ngpu_chunk *d_chunks, uint64_t n,
                             ngpu_result *d_out, const uint64_t *d_layer_first,
                             uint64_t n_layers, ngpu_layer_stats *d_stats, void *stream) {
  if (!node || i >= node->eng.size()) return NGPU_EINVAL;
  return ngpu_process_dict_device(node->eng[i], dict, d_data, len, d_chunks, n, d_out,
                                  d_layer_first, n_layers, d_stats, stream, nullptr);
}

int ngpu_node_process_step(ngpu_node *node, ngpu_dict *dict, const ngpu_node_part *parts,
                           uint32_t n_parts, uint32_t flags) {
  if (!node || !parts || (flags & ~NGPU_NODE_STEP_RCCL)) return NGPU_EINVAL;
  return guarded([&] { return node_step(node, dict, parts, n_parts, flags); });
}

}  // extern "C"
