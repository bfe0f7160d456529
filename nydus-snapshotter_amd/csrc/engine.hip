// engine.hip — the C ABI of libnydusgpu.so (include/nydus_gpu.h): engine
// lifetime, HBM workspace, chunk dict residency and the per-layer
// digest -> dedup pipeline on one HIP stream.
//
// Replaces the per-layer `nydus-image create` process of
// pkg/converter/tool/builder.go:148-178 for the digest/dedup stage; the
// option validation mirrors pkg/converter/types.go:58-90 (ChunkSize power of
// two in [0x1000, 0x1000000], FsVersion "5"/"6", default "6").
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <string>
#include <vector>

#include "engine_internal.hpp"
#include "tarstream.hpp"

using namespace ngpu;

namespace ngpu {

int fail(ngpu_engine *e, int code, const char *fmt, ...) {
  if (e) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    std::lock_guard<std::mutex> g(e->err_mu);
    e->err = buf;
  }
  return code;
}

template <typename T>
int grow(ngpu_engine *e, T **p, uint64_t &cap, uint64_t want, uint64_t elem_bytes = sizeof(T)) {
  if (want <= cap && *p) return 0;
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  cap = 0;
  uint64_t c = want < 1024 ? 1024 : want;
  HIP_TRY(e, hipMalloc((void **)p, c * elem_bytes));
  cap = c;
  return 0;
}

uint64_t next_pow2(uint64_t x) {
  uint64_t p = 1;
  while (p < x) p <<= 1;
  return p;
}

int pick_group_log2(const ngpu_engine *e, uint64_t data_len) {
  switch (e->cfg.leaves_per_lane) {
    case 1: return 0;
    case 2: return 1;
    case 4: return 2;
    case 8: return 3;
    case 16: return 4;
    default: break;
  }
  // auto: up to 8 leaves per lane (tuned: profiles/r1/tune_*) (never more than a chunk holds), fewer
  // when the layer is too small to give >= 4 waves per SIMD at that size.
  int D = 0;
  while (D < 3 && (2ull << D) * kLeaf <= e->cfg.chunk_size) ++D;
  const uint64_t leaves = data_len / kLeaf + 1;
  while (D > 0 && (leaves >> D) < (1ull << 18)) --D;
  return D;
}

// The event after which nothing reads the slot any more, recorded into
// sl.last_ev.  A stage's end event (a timing stop event, the dedup's last
// kernel) does not cover the reads its call enqueues after it -- the stats
// read-back copies, a batch's stats-out kernel -- so when the slot's last
// stream lives as long as the engine (ws_lazy_end) the fence is recorded on
// it now, after all of them.  (A regrow freed the stats of a slot whose
// read-back copy was still queued behind a timing stop event: an illegal
// memory access in the timed packs bench, r5n.)  A caller's stream may be
// gone, so its stage's own end event stays the fence.
int slot_fence(ngpu_engine *e, ngpu_ws_slot &sl) {
  if (!sl.last_ev || ws_lazy_end(e, sl.last, false)) {
    HIP_TRY(e, hipEventRecord(sl.done, sl.last));
    sl.last_ev = sl.done;
  }
  return 0;
}

// Before a slot's buffers are freed: its last stage has finished.  (The
// stage is on another stream; a buffer freed under it could be handed to
// another slot's allocation and written by a stage unordered with it.)
int slot_quiesce(ngpu_engine *e) {
  ngpu_ws_slot &sl = *e->cur;
  if (!sl.pending) return 0;
  if (int rc = slot_fence(e, sl)) return rc;
  HIP_TRY(e, hipEventSynchronize(sl.last_ev));
  return 0;
}

int ensure_workspace(ngpu_engine *e, uint64_t n, uint64_t data_len, int D,
                     uint32_t n_blobs, uint64_t L) {
  Workspace &ws = e->cur->ws;
  {
    const uint64_t nb = ((uint64_t)n_blobs + 1) * (L ? L : 1);
    const bool regrow =
        n + 1 > ws.cap_n || L > ws.cap_layers || nb > ws.cap_blobs ||
        (e->cfg.digester == NGPU_DIGEST_BLAKE3 && blake3_max_groups(n, data_len, D) > ws.cap_g);
    if (regrow && ws.groups)
      if (int rc = slot_quiesce(e)) return rc;
  }
  if (n + 1 > ws.cap_n || !ws.groups) {
    uint64_t cn = n + 1 < 4096 ? 4096 : n + 1;
    uint64_t c0 = 0, c1 = 0, c2 = 0, c3 = 0, c4 = 0;
    if (grow(e, &ws.chunk_layer, c4, cn)) return NGPU_ENOMEM;
    uint64_t c5 = 0;
    if (grow(e, &ws.small, c5, cn)) return NGPU_ENOMEM;
    uint64_t c7 = 0;
    if (grow(e, &ws.tree_list, c7, cn)) return NGPU_ENOMEM;
    if (grow(e, &ws.groups, c0, cn)) return NGPU_ENOMEM;
    if (grow(e, &ws.newflag, c1, cn)) return NGPU_ENOMEM;
    if (grow(e, &ws.uoff, c2, cn)) return NGPU_ENOMEM;
    uint64_t c8 = 0, c9 = 0;
    if (grow(e, &ws.nbytes, c8, cn)) return NGPU_ENOMEM;
    if (grow(e, &ws.ndict, c9, cn)) return NGPU_ENOMEM;
    ws.tiles = tstat_tiles(cn);
    if (grow(e, &ws.tstat, c3, tstat_words(ws.tiles))) return NGPU_ENOMEM;
    uint64_t icap = next_pow2(2 * cn);
    uint64_t ic = 0;
    if (ws.intra) (void)hipFree(ws.intra), ws.intra = nullptr;
    if (grow(e, &ws.intra, ic, icap)) return NGPU_ENOMEM;
    ws.intra_cap = icap;
    ws.cap_n = cn;
  }
  if (!ws.stats) {
    uint64_t c = 0, c1 = 0;
    if (grow(e, &ws.stats, c, 16)) return NGPU_ENOMEM;
    if (grow(e, &ws.lfirst1, c1, 2)) return NGPU_ENOMEM;
    // no stale error counter.  hipMemset is asynchronous to the host and runs on
    // the null stream, which does not order against a caller's non-blocking
    // stream: unwaited, the zeroing could land AFTER this call's first digest
    // kernel wrote the counters -- b3_tree then found its queue count zeroed
    // and the multi-leaf chunks kept no digest (the digest guard's NGPU_EDEVICE;
    // reproduced by the first node step on 8 streams, tools/step_diag.py).
    // The counters are zeroed and waited for here, before any stage uses them.
    HIP_TRY(e, hipMemsetAsync(ws.stats, 0, c * sizeof(uint64_t), nullptr));
    HIP_TRY(e, hipStreamSynchronize(nullptr));
  }
  if (L > ws.cap_layers || !ws.lstats) {
    uint64_t c = ws.cap_layers;
    if (grow(e, &ws.lstats, c, L)) return NGPU_ENOMEM;
    ws.cap_layers = c;
  }
  const uint64_t nb = ((uint64_t)n_blobs + 1) * (L ? L : 1);
  if (nb > ws.cap_blobs || !ws.blob_first) {
    uint64_t c0 = 0, c1 = 0;
    if (ws.blob_first) (void)hipFree(ws.blob_first), ws.blob_first = nullptr;
    if (ws.blob_real) (void)hipFree(ws.blob_real), ws.blob_real = nullptr;
    if (grow(e, &ws.blob_first, c0, nb)) return NGPU_ENOMEM;
    if (grow(e, &ws.blob_real, c1, nb)) return NGPU_ENOMEM;
    ws.cap_blobs = c0;
  }
  if (e->cfg.digester == NGPU_DIGEST_BLAKE3) {
    const uint64_t g = blake3_max_groups(n, data_len, D);
    if (g > ws.cap_g || !ws.cv) {
      uint64_t c0 = 0, c1 = 0;
      if (ws.cv) hipFree(ws.cv), ws.cv = nullptr;
      if (ws.group_chunk) hipFree(ws.group_chunk), ws.group_chunk = nullptr;
      if (grow(e, &ws.cv, c0, g, 32)) return NGPU_ENOMEM;
      if (grow(e, &ws.group_chunk, c1, g)) return NGPU_ENOMEM;
      ws.cap_g = c0 < c1 ? c0 : c1;
    }
  }
  return 0;
}

ngpu_ws_slot *use_slot(ngpu_engine *e, hipStream_t s) {
  ngpu_ws_slot *pick = nullptr;
  for (auto &sl : e->slots)  // a batch lane's own slot
    if (sl.lane && sl.owner == s) {
      pick = &sl;
      break;
    }
  if (!pick)
    for (auto &sl : e->slots)  // the slot this stream used last: stream order
      if (!sl.lane && sl.pending && sl.last == s) {
        pick = &sl;
        break;
      }
  if (!pick)  // a slot never used yet
    for (auto &sl : e->slots)
      if (!sl.lane && !sl.pending) {
        pick = &sl;
        break;
      }
  // else the least recently used: with streams taking turns it is the one
  // most likely finished, and ws_acquire's GPU-side wait costs nothing then.
  // (Querying every slot's event first cost ~1-2 us of host time per slot
  // and call, on a path the host enqueue already bounds.)
  if (!pick)
    for (auto &sl : e->slots)
      if (!sl.lane && (!pick || sl.tick < pick->tick)) pick = &sl;
  pick->tick = ++e->tick;
  e->cur = pick;
  return pick;
}

int ws_acquire(ngpu_engine *e, hipStream_t s) {
  ngpu_ws_slot &sl = *e->cur;
  if (!sl.pending || sl.last == s) return 0;
  if (int rc = slot_fence(e, sl)) return rc;  // a lazy stage end, or reads after the end event
  HIP_TRY(e, hipStreamWaitEvent(s, sl.last_ev, 0));
  return 0;
}

// A kernel that carries an event (a stop event of hipExtLaunchKernelGGL, or a
// marker after it) holds the next kernel on its stream back by ~4.4 us
// (rocprofv3 trace of back-to-back C1 calls), so a stage binds no end event
// when none is needed yet:
//  * chained: the next stage of the same call follows on the same stream;
//  * s lives as long as the engine (its own stream, a pack compute stream),
//    so the event can be recorded later, by the ws_acquire of a stage on
//    another stream (recorded then, it also covers later work on s: safe,
//    not tight).
bool ws_lazy_end(const ngpu_engine *e, hipStream_t s, bool chained) {
  if (chained) return true;
  if (!s) return false;
  for (hipStream_t x : e->streams)
    if (x == s) return true;
  return false;
}

// bound: an event the stage's last kernel already records at its end (a
// stop event of hipExtLaunchKernelGGL), or null to record the slot's done event now --
// unless the end may be lazy (ws_lazy_end), then ws_acquire records it.
int ws_release(ngpu_engine *e, hipStream_t s, hipEvent_t bound, bool chained) {
  ngpu_ws_slot &sl = *e->cur;
  if (!bound && !ws_lazy_end(e, s, chained)) {
    HIP_TRY(e, hipEventRecord(sl.done, s));
    bound = sl.done;
  }
  sl.last_ev = bound;
  sl.last = s;
  sl.pending = true;
  return 0;
}

// Before timing-ring entry k is recorded again: a workspace slot whose last
// stage ended on one of k's events must not keep that event as its fence (a
// later wait on it would wait for the new record, not the slot's stage).  The
// entry was recorded kTimingRing calls ago, so the host wait is for work long
// done; the slot is then idle.
static int ring_reclaim(ngpu_engine *e, int k) {
  for (auto &sl : e->slots) {
    if (!sl.pending || !sl.last_ev) continue;
    for (hipEvent_t ev : e->ev[k])
      if (sl.last_ev == ev) {
        if (ws_lazy_end(e, sl.last, false)) {  // an engine stream: fenced afresh when next needed
          sl.last_ev = nullptr;                // (slot_fence), after every read of the slot
          break;
        }
        HIP_TRY(e, hipEventSynchronize(ev));
        sl.pending = false;
        sl.last_ev = nullptr;
        break;
      }
  }
  return 0;
}

// Digest stage: resets the layer stats, runs the digest kernels.
int enqueue_digest(ngpu_engine *e, const uint8_t *d_data, uint64_t len,
                   const ngpu_chunk *d_chunks, uint64_t n, ngpu_result *d_out,
                   hipStream_t s, bool chained) {
  const int D = pick_group_log2(e, len);
  use_slot(e, s);
  Workspace &ws = e->cur->ws;
  int rc = ensure_workspace(e, n, len, D, 0, 1);
  if (rc) return rc;
  if ((rc = ws_acquire(e, s))) return rc;
  const bool tm = (e->cfg.flags & NGPU_FLAG_TIMING) != 0;
  // tuning override: flags bits 8..10 = 1 + BLAKE3 load mode (0 = default;
  // validated by ngpu_create)
  const uint32_t lm = (e->cfg.flags >> NGPU_FLAG_LOAD_MODE_SHIFT) & 7;
  ws.load_mode = lm ? (int)(lm - 1) : 0;
  hipEvent_t *ev = nullptr;
  if (tm) {
    const int k = (int)(e->tcalls % ngpu_engine::kTimingRing);
    if ((rc = ring_reclaim(e, k))) return rc;
    e->tslot = k;
    ++e->tcalls;
    e->tshare_slot = e->cur;
    e->tshare_stream = s;
    e->tshare_open = true;
    ev = e->ev[e->tslot];
    e->timed[e->tslot] = false;
    e->slot_D[e->tslot] = D;
    e->slot_fused[e->tslot] =
        e->cfg.digester == NGPU_DIGEST_BLAKE3 && blake3_planned_in_leaves(n, len, D, ws);
  }
  hipEvent_t bound = nullptr;  // the stage-end event a kernel records
  if (e->cfg.digester == NGPU_DIGEST_SHA256) {
    if (tm) HIP_TRY(e, hipEventRecord(ev[0], s));
    HIP_TRY(e, hipMemsetAsync(ws.stats, 0, 16 * sizeof(uint64_t), s));
    if (tm) HIP_TRY(e, hipEventRecord(ev[1], s));
    // tuning override: flags bits 11..13 = 1 + SHA-256 variant (0 split,
    // 1 pair, 2 lane, 4/5 pair layouts)
    const uint32_t sv = (e->cfg.flags >> NGPU_FLAG_SHA_MODE_SHIFT) & 7;
    // mixed lengths unless the data averages >= 15/16 of a full chunk per
    // chunk and fills every 32-chunk wave (a raw stream cut at chunk_size,
    // C3); tar layers and batches mix file-sized chunks with full ones
    const bool mixed = n % 32 != 0 || len < n * (uint64_t)e->cfg.chunk_size / 16 * 15;
    launch_sha256(d_data, len, d_chunks, n, d_out, ws.stats + kStBadDesc, sv ? (int)sv - 1 : -1,
                  mixed, s);
    snprintf(e->cur->path, sizeof e->cur->path, "sha256 variant %d, %llu chunks",
             sv ? (int)sv - 1 : -1, (unsigned long long)n);
    if (tm) {
      HIP_TRY(e, hipEventRecord(ev[2], s));
      HIP_TRY(e, hipEventRecord(ev[3], s));
      bound = ev[3];
    }
  } else {
    // events ride on the kernels: no marker packets between the launches
    hipEvent_t end = tm ? ev[3] : ws_lazy_end(e, s, chained) ? nullptr : e->cur->done;
    if (launch_blake3(d_data, d_chunks, n, len, D, ws, d_out, s, tm ? ev[0] : nullptr,
                      tm ? ev[1] : nullptr, tm ? ev[2] : nullptr, end, e->cfg.chunk_size))
      bound = end;
    snprintf(e->cur->path, sizeof e->cur->path, "blake3 %s D=%d, %llu chunks",
             blake3_planned_in_leaves(n, len, D, ws) ? "quad_planned"
             : (D == 0 && !ws.grid_stages && len / kLeaf + n <= blake3_quad_max_leaves()) ? "quad_leaves"
                                                                        : "groups",
             D, (unsigned long long)n);
  }
  HIP_TRY(e, hipGetLastError());
  if ((rc = ws_release(e, s, bound, chained))) return rc;
  return 0;
}

// Dedup stage: dict decisions (given hits or the engine's dict), intra-layer
// dedup, NEW indices / offsets, blob order, stats.
int enqueue_dedup(ngpu_engine *e, const ngpu_dict *dict, const ngpu_chunk *d_chunks, uint64_t n,
                  ngpu_result *d_out, const ngpu_dict_hit *d_hits, uint32_t n_blobs,
                  hipStream_t s, const uint64_t *d_lfirst, uint64_t L, ngpu_layer_stats *d_stats) {
  if (!d_hits) n_blobs = dict_blobs(dict);
  if (!d_lfirst) L = 1;
  use_slot(e, s);
  int rc = ensure_workspace(e, n, 0, 0, n_blobs, L);
  if (rc) return rc;
  if ((rc = ws_acquire(e, s))) return rc;
  if (!d_hits && dict && !dict->parts.empty()) {  // node dict (node.hip)
    ngpu_dict *replica = nullptr;
    rc = node_dict_hits(e, const_cast<ngpu_dict *>(dict), reinterpret_cast<const uint8_t *>(d_out),
                        sizeof(ngpu_result), n, s, &d_hits, &replica);
    if (rc) return rc;
    if (replica) dict = replica;
  }
  if (!d_stats) d_stats = e->cur->ws.lstats;
  const bool tm = (e->cfg.flags & NGPU_FLAG_TIMING) != 0;
  const uint32_t align =
      (e->cfg.fs_version == 6 || (e->cfg.flags & NGPU_FLAG_ALIGNED_CHUNK)) ? 4096u : 1u;
  // d_lfirst == nullptr: the init kernel writes {0, n} into ws.lfirst1
  // the last dedup kernel records the stage end (timing slot or the slot's done event)
  const bool timed = tm && e->tshare_open && e->tshare_slot == e->cur && e->tshare_stream == s;
  hipEvent_t end = timed                      ? e->ev[e->tslot][4]
                   : ws_lazy_end(e, s, false) ? nullptr
                                              : e->cur->done;
  launch_dedup(d_chunks, n, dict ? dict->dev : DictDevice{}, d_hits, n_blobs, align, d_lfirst, L,
               e->cur->ws, d_out, d_stats, s, end);
  HIP_TRY(e, hipGetLastError());
  if (timed) e->timed[e->tslot] = n > 0, e->tshare_open = false;
  if ((rc = ws_release(e, s, end, false))) return rc;
  return 0;
}

int enqueue_chain(ngpu_engine *e, const ngpu_dict *dict, const uint8_t *d_data, uint64_t len,
                  const ngpu_chunk *d_chunks, uint64_t n, ngpu_result *d_out, hipStream_t s,
                  const uint64_t *d_lfirst, uint64_t L, ngpu_layer_stats *d_stats) {
  int rc = enqueue_digest(e, d_data, len, d_chunks, n, d_out, s, true);
  if (rc) return rc;
  rc = enqueue_dedup(e, dict, d_chunks, n, d_out, nullptr, 0, s, d_lfirst, L, d_stats);
  // the chained digest left its end unrecorded: s may be gone after the call
  if (rc) (void)ws_release(e, s, nullptr, false);
  return rc;
}

int enqueue(ngpu_engine *e, const ngpu_dict *dict, const uint8_t *d_data, uint64_t len,
            const ngpu_chunk *d_chunks, uint64_t n, ngpu_result *d_out, hipStream_t s) {
  return enqueue_chain(e, dict, d_data, len, d_chunks, n, d_out, s, nullptr, 1, nullptr);
}

void engine_ref(ngpu_engine *e) { e->refs.fetch_add(1, std::memory_order_relaxed); }

void engine_unref(ngpu_engine *e) {
  if (!e || e->refs.fetch_sub(1, std::memory_order_acq_rel) != 1) return;
  DeviceGuard g(e->device);
  if (e->stream) (void)hipStreamSynchronize(e->stream);
  for (hipStream_t x : e->streams)
    if (x != e->stream) (void)hipStreamSynchronize(x);
  for (auto &sl : e->slots) {
    Workspace &ws = sl.ws;
    void *bufs[] = {ws.groups, ws.group_chunk, ws.cv, ws.newflag, ws.uoff, ws.nbytes, ws.ndict,
                    ws.tstat, ws.intra, ws.blob_first, ws.blob_real, ws.stats, ws.chunk_layer,
                    ws.lfirst1, ws.lstats, ws.small, ws.tree_list, ws.xq, ws.xparts, ws.xhits,
                    ws.xrow, ws.xcnt};
    for (void *p : bufs)
      if (p) (void)hipFree(p);
    if (sl.h_stats) (void)hipHostFree(sl.h_stats);
    if (sl.done) (void)hipEventDestroy(sl.done);
  }
  for (void *p : {(void *)e->d_data, (void *)e->d_chunks, (void *)e->d_results})
    if (p) (void)hipFree(p);
  for (auto &set : e->ev)
    for (auto ev : set)
      if (ev) (void)hipEventDestroy(ev);
  for (auto &b : e->staging_pool) {
    if (b.h) (void)hipHostFree(b.h);
    if (b.h_ch) (void)hipHostFree(b.h_ch);
    if (b.d) (void)hipFree(b.d);
    if (b.d_ch) (void)hipFree(b.d_ch);
    if (b.copied) (void)hipEventDestroy(b.copied);
    if (b.done) (void)hipEventDestroy(b.done);
  }
  for (auto &b : e->land_pool) (void)hipHostFree(b.first);
  for (auto &b : e->pack_pool) {
    if (b.d_res) (void)hipFree(b.d_res);
    if (b.d_all) (void)hipFree(b.d_all);
    if (b.fence) (void)hipEventDestroy(b.fence);
    if (b.h_stats) (void)hipHostFree(b.h_stats);
    if (b.h_io) (void)hipHostFree(b.h_io);
    blob_windows_free(b.win);
  }
  batcher_free(e);  // syncs its stream (one of e->streams, destroyed below)
  if (e->seg_pool) {  // every segment went back at its Pack's end (streams synced above)
    (void)hipMemPoolTrimTo(e->seg_pool, 0);
    (void)hipMemPoolDestroy(e->seg_pool);
  }
  for (hipStream_t x : e->streams)  // every pack compute stream (+ the engine's)
    if (x != e->stream) (void)hipStreamDestroy(x);
  if (e->h_results) (void)hipHostFree(e->h_results);
  if (e->host_ev) (void)hipEventDestroy(e->host_ev);
  if (e->stream) (void)hipStreamDestroy(e->stream);
  delete e;
}

// Layer stats of a single-layer call (internal lstats[0]) + the digest
// stage's bad-descriptor counter.
// Before the host reads what the stream's kernels wrote: a system-scope
// release on the stream.  A stage with a lazy end (ws_lazy_end) leaves no
// event after its last kernel, so nothing else on the stream is guaranteed to
// be system-scoped before the copy; one marker per host read is cheap next to
// the PCIe transfer around it.
int host_fence(ngpu_engine *e, hipStream_t s, hipEvent_t ev) {
  HIP_TRY(e, hipEventRecord(ev ? ev : e->host_ev, s));
  return 0;
}

int read_stats(ngpu_engine *e, hipStream_t s, ngpu_layer_stats *st, bool fenced) {
  if (!fenced) {
    if (int rc = host_fence(e, s)) return rc;
  }
  uint64_t *h = e->cur->h_stats;  // the slot the call's stages used (e->mu held)
  if (int rc = read_stats_enqueue(e, s, h)) return rc;
  HIP_TRY(e, hipStreamSynchronize(s));
  return read_stats_parse(e, h, st, e->cur->path);
}

int read_stats_enqueue(ngpu_engine *e, hipStream_t s, uint64_t *h) {
  const ngpu_ws_slot &sl = *e->cur;
  static_assert(kStWords <= kStatsLayer && kStatsLayer * 8 + sizeof(ngpu_layer_stats) <= 32 * 8,
                "stats read-back layout fits the 32-word pinned buffers");
  HIP_TRY(e, hipMemcpyAsync(h, sl.ws.stats, kStWords * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
  HIP_TRY(e, hipMemcpyAsync(h + kStatsLayer, sl.ws.lstats, sizeof(ngpu_layer_stats),
                            hipMemcpyDeviceToHost, s));
  return 0;
}

// Errors recorded by a stage, in order of precedence (one message).
static int stats_error(ngpu_engine *e, uint64_t bad, uint64_t over, uint64_t unh,
                       uint64_t inv_first, const char *path) {
  if (bad)
    return fail(e, NGPU_EINVAL, "%llu chunk descriptor(s) outside the data buffer",
                (unsigned long long)bad);
  if (over)
    return fail(e, NGPU_EINVAL, "chunk descriptors overlap (%llu leaves, more than the buffer holds)",
                (unsigned long long)over);
  if (unh)
    return fail(e, NGPU_EDEVICE,
                "%llu chunk(s) reached the dedup stage without a digest, first chunk %llu "
                "(digest stage: %s); results marked NGPU_UNHASHED",
                (unsigned long long)unh, (unsigned long long)~inv_first,
                path && *path ? path : "caller-supplied digests");
  return 0;
}

int read_stats_parse(ngpu_engine *e, const uint64_t *h, ngpu_layer_stats *st, const char *path) {
  if (int rc = stats_error(e, h[kStBadDesc], h[kStOverlap], h[kStUnhashed], h[kStUnhashedFirst],
                           path))
    return rc;
  if (st) memcpy(st, h + kStatsLayer, sizeof(ngpu_layer_stats));
  return 0;
}

}  // namespace ngpu

extern "C" {

int ngpu_abi_version(void) { return NGPU_ABI_VERSION; }

// internal (host.cpp), not part of nydus_gpu.h
uint32_t ngpu_engine_chunk_size(const ngpu_engine *e) { return e->cfg.chunk_size; }

int ngpu_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int ngpu_create(const ngpu_config *cfg, ngpu_engine **out) {
  if (!out) return NGPU_EINVAL;
  *out = nullptr;
  ngpu_config c{};
  if (cfg) c = *cfg;
  if (c.chunk_size == 0) c.chunk_size = 0x100000;
  if (c.fs_version == 0) c.fs_version = 6;
  if (c.staging_bytes == 0) c.staging_bytes = 256ull << 20;
  if ((c.chunk_size & (c.chunk_size - 1)) || c.chunk_size < 0x1000 || c.chunk_size > 0x1000000)
    return NGPU_EINVAL;  // types.go:76
  if (c.fs_version != 5 && c.fs_version != 6) return NGPU_EINVAL;
  if (c.digester != NGPU_DIGEST_BLAKE3 && c.digester != NGPU_DIGEST_SHA256) return NGPU_EINVAL;
  if (c.leaves_per_lane & (c.leaves_per_lane - 1) || c.leaves_per_lane > 16) return NGPU_EINVAL;
  // SHA-256 kernel override (benchmarks): 1 + {0 split, 1 pair, 2 lane, 4 pair
  // one group per workgroup, 5 pair four groups}; anything else is rejected
  switch ((c.flags >> NGPU_FLAG_SHA_MODE_SHIFT) & 7) {
    case 0: case 1: case 2: case 3: case 5: case 6: break;
    default: return NGPU_EINVAL;
  }
  // BLAKE3 load-mode override: only modes this build has a kernel for, all of
  // which compute the reference digests (the no-load diagnostic is not built)
  if (const uint32_t lm = (c.flags >> NGPU_FLAG_LOAD_MODE_SHIFT) & 7)
    if (!blake3_load_mode_ok((int)lm - 1)) return NGPU_EINVAL;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return NGPU_ENODEV;
  if (c.device < 0 || c.device >= ndev) return NGPU_ENODEV;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, c.device) != hipSuccess) return NGPU_ENODEV;
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return NGPU_ENODEV;
  static std::atomic<uint64_t> next_uid{1};
  ngpu_engine *e = new ngpu_engine();
  e->batcher = batcher_new();
  e->uid = next_uid.fetch_add(1, std::memory_order_relaxed);
  e->cfg = c;
  // NGPU_WS_SLOTS: workspace slots = calls on distinct streams that may run
  // at once (default 8: 32 unbatched concurrent Packs measured 17 GB/s on 4
  // slots, 26 on 8 -- fewer slots, more GPU-side waits on a slot's last
  // stage), plus one slot of its own per batch lane (a lane never waits on
  // another call's slot, nor regrows one under it).  A slot allocates on
  // first use.
  int nslots = 8;
  if (const char *v = getenv("NGPU_WS_SLOTS")) {
    const long x = strtol(v, nullptr, 10);
    if (x >= 1 && x <= 64) nslots = (int)x;
  }
  e->slots.resize((size_t)nslots + kBatchLanes);
  for (size_t i = (size_t)nslots; i < e->slots.size(); ++i) e->slots[i].lane = true;
  for (auto &sl : e->slots) sl.ws.grid_stages = (c.flags & NGPU_FLAG_GRID_STAGES) != 0;
  e->cur = &e->slots[0];
  e->device = c.device;
  DeviceGuard dg(c.device);
  // Events keep the default system-scope fence: the end event of a call on a
  // caller's stream is also what makes its results visible to the host's
  // copies.  (hipEventDisableSystemFence measured +2 % on C1 and is not
  // worth that: profiles/r2/ab_event_fence_r2ef.json.)
  if (c.flags & NGPU_FLAG_TIMING)
    for (auto &set : e->ev)
      for (auto &ev : set)
        if (hipEventCreate(&ev) != hipSuccess) {
          ngpu_destroy(e);
          return NGPU_EHIP;
        }
  // Retained Pack segments (pack.hip) come from the engine's own
  // stream-ordered pool: a layer's 64 MiB segments go back to it at the
  // Pack's end without hipFree's device-wide wait (~0.5 ms each), and the
  // next Pack reuses them.  The pool keeps up to NGPU_SEG_POOL_MIB (default
  // 4096) cached and is trimmed and destroyed with the engine; the device's
  // default pool (the host application's) is left as it was.
  {
    hipMemPoolProps pp;
    memset(&pp, 0, sizeof pp);
    pp.allocType = hipMemAllocationTypePinned;
    pp.handleTypes = hipMemHandleTypeNone;
    pp.location.type = hipMemLocationTypeDevice;
    pp.location.id = c.device;
    uint64_t keep = 4096ull << 20;
    if (const char *v = getenv("NGPU_SEG_POOL_MIB")) keep = strtoull(v, nullptr, 10) << 20;
    DeviceGuard g(c.device);
    if (hipMemPoolCreate(&e->seg_pool, &pp) == hipSuccess && e->seg_pool)
      (void)hipMemPoolSetAttribute(e->seg_pool, hipMemPoolAttrReleaseThreshold, &keep);
    else
      e->seg_pool = nullptr;  // segments then come from hipMallocAsync's default pool
    (void)hipGetLastError();
  }
  bool ok = hipEventCreateWithFlags(&e->host_ev, hipEventDisableTiming) == hipSuccess &&
            hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) == hipSuccess;
  if (ok) e->streams.push_back(e->stream);
  for (auto &sl : e->slots)
    ok = ok && hipEventCreateWithFlags(&sl.done, hipEventDisableTiming) == hipSuccess &&
         hipHostMalloc((void **)&sl.h_stats, 32 * sizeof(uint64_t), hipHostMallocDefault) ==
             hipSuccess;
  if (!ok) {
    ngpu_destroy(e);
    return NGPU_EHIP;
  }
  *out = e;
  return NGPU_OK;
}

void ngpu_destroy(ngpu_engine *e) {
  if (!e) return;
  ngpu_dict *d;
  std::vector<ngpu_dict *> cache;
  {
    std::lock_guard<std::mutex> g(e->mu);
    d = e->dict;
    e->dict = nullptr;
    cache.swap(e->dict_cache);
  }
  dict_unref(d);
  for (ngpu_dict *c : cache) dict_unref(c);
  engine_unref(e);  // open packs keep the engine until they end
}

const char *ngpu_last_error(const ngpu_engine *e) { return e ? e->err.c_str() : "null engine"; }

int ngpu_device_status(ngpu_engine *e) {
  if (!e) return NGPU_EINVAL;
  return guarded([&]() -> int {
    std::lock_guard<std::mutex> g(e->mu);
    DeviceGuard dg(e->device);
    int first = 0;
    for (auto &sl : e->slots) {
      if (!sl.ws.stats) continue;
      if (sl.pending) {  // wait for the slot's last stage (its stream may be a caller's)
        if (!sl.last_ev) {  // lazy end: its stream lives as long as the engine
          HIP_TRY(e, hipEventRecord(sl.done, sl.last));
          sl.last_ev = sl.done;
        }
        HIP_TRY(e, hipEventSynchronize(sl.last_ev));
      }
      uint64_t w[4];
      HIP_TRY(e, hipMemcpy(w, sl.ws.stats + kStSticky, sizeof w, hipMemcpyDeviceToHost));
      if (!(w[0] | w[1] | w[2])) continue;
      // waited for (see ensure_workspace): a later stage's error counts on a
      // non-blocking stream must not be cleared by a null-stream memset still queued
      HIP_TRY(e, hipMemsetAsync(sl.ws.stats + kStSticky, 0, sizeof w, nullptr));
      HIP_TRY(e, hipStreamSynchronize(nullptr));
      if (!first) first = stats_error(e, w[0], w[1], w[2], w[3], sl.path);  // its message kept
    }
    return first;
  });
}

int ngpu_alloc_pinned(ngpu_engine *e, uint64_t bytes, void **out) {
  if (!e || !out) return NGPU_EINVAL;
  std::lock_guard<std::mutex> g(e->mu);
  DeviceGuard dg(e->device);
  HIP_TRY(e, hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault));
  return 0;
}

int ngpu_free_pinned(ngpu_engine *e, void *p) {
  if (!e) return NGPU_EINVAL;
  HIP_TRY(e, hipHostFree(p));
  return 0;
}

// Device-pointer entry points run on the caller's stream.  NULL is the null
// (default) stream, as everywhere in HIP — it used to mean the engine's own
// non-blocking stream, which ran unordered with a caller (e.g. PyTorch on its
// default stream, whose handle is 0) still producing the inputs.
static inline hipStream_t dev_stream(void *s) { return (hipStream_t)s; }

int ngpu_digest_device(ngpu_engine *e, const void *d_data, uint64_t len,
                       const ngpu_chunk *d_chunks, uint64_t n, ngpu_result *d_out,
                       void *stream) {
  if (!e || (n && (!d_data || !d_chunks || !d_out))) return NGPU_EINVAL;
  if (n >= 0xFFFFFFFFull) return fail(e, NGPU_EINVAL, "too many chunks in one call");
  std::lock_guard<std::mutex> g(e->mu);
  DeviceGuard dg(e->device);
  return enqueue_digest(e, (const uint8_t *)d_data, len, d_chunks, n, d_out,
                        dev_stream(stream));
}

int ngpu_dedup_device(ngpu_engine *e, const ngpu_chunk *d_chunks, uint64_t n,
                      ngpu_result *d_out, const ngpu_dict_hit *d_hits, uint32_t n_dict_blobs,
                      void *stream, ngpu_layer_stats *stats) {
  if (!e || (n && (!d_chunks || !d_out))) return NGPU_EINVAL;
  if (n >= 0xFFFFFFFFull) return fail(e, NGPU_EINVAL, "too many chunks in one call");
  std::lock_guard<std::mutex> g(e->mu);
  DeviceGuard dg(e->device);
  if (d_hits && n_dict_blobs == 0) n_dict_blobs = dict_blobs(e->dict) ? dict_blobs(e->dict) : 1;
  hipStream_t s = dev_stream(stream);
  int rc = enqueue_dedup(e, e->dict, d_chunks, n, d_out, d_hits, n_dict_blobs, s, nullptr, 1,
                         nullptr);
  if (rc) return rc;
  if (stats) return read_stats(e, s, stats, false);
  return 0;
}

int ngpu_dedup_layers_device(ngpu_engine *e, const ngpu_chunk *d_chunks, uint64_t n,
                             ngpu_result *d_out, const ngpu_dict_hit *d_hits,
                             uint32_t n_dict_blobs, const uint64_t *d_layer_first,
                             uint64_t n_layers, ngpu_layer_stats *d_stats, void *stream) {
  if (!e || !d_layer_first || n_layers == 0 || (n && (!d_chunks || !d_out))) return NGPU_EINVAL;
  if (n >= 0xFFFFFFFFull || n_layers >= 0xFFFFFFFFull) return fail(e, NGPU_EINVAL, "too large");
  std::lock_guard<std::mutex> g(e->mu);
  DeviceGuard dg(e->device);
  if (d_hits && n_dict_blobs == 0) n_dict_blobs = dict_blobs(e->dict) ? dict_blobs(e->dict) : 1;
  return enqueue_dedup(e, e->dict, d_chunks, n, d_out, d_hits, n_dict_blobs, dev_stream(stream),
                       d_layer_first, n_layers, d_stats);
}

// dict == kDefault: the engine's default dict (read under e->mu).
static ngpu_dict *const kDefault = reinterpret_cast<ngpu_dict *>(1);

static int process_device(ngpu_engine *e, ngpu_dict *dict, const void *d_data, uint64_t len,
                          const ngpu_chunk *d_chunks, uint64_t n, ngpu_result *d_out,
                          const uint64_t *d_layer_first, uint64_t n_layers,
                          ngpu_layer_stats *d_stats, void *stream, ngpu_layer_stats *stats) {
  if (!e || (d_layer_first && n_layers == 0) || (n && (!d_data || !d_chunks || !d_out)))
    return NGPU_EINVAL;
  if (n >= 0xFFFFFFFFull || n_layers >= 0xFFFFFFFFull)
    return fail(e, NGPU_EINVAL, "too many chunks in one call");
  if (stats && d_layer_first) return fail(e, NGPU_EINVAL, "host stats are for one-layer calls");
  std::lock_guard<std::mutex> g(e->mu);
  DeviceGuard dg(e->device);
  if (dict == kDefault) dict = e->dict;
  if (int rc = dict_check(e, dict)) return rc;
  hipStream_t s = dev_stream(stream);
  int rc = enqueue_chain(e, dict, (const uint8_t *)d_data, len, d_chunks, n, d_out, s,
                         d_layer_first, d_layer_first ? n_layers : 1, d_stats);
  if (rc) return rc;
  if (stats) return read_stats(e, s, stats, false);
  return 0;
}

int ngpu_process_layers_device(ngpu_engine *e, const void *d_data, uint64_t len,
                               const ngpu_chunk *d_chunks, uint64_t n, ngpu_result *d_out,
                               const uint64_t *d_layer_first, uint64_t n_layers,
                               ngpu_layer_stats *d_stats, void *stream) {
  if (!d_layer_first) return NGPU_EINVAL;
  return process_device(e, kDefault, d_data, len, d_chunks, n, d_out, d_layer_first, n_layers,
                        d_stats, stream, nullptr);
}

int ngpu_process_device(ngpu_engine *e, const void *d_data, uint64_t len,
                        const ngpu_chunk *d_chunks, uint64_t n, ngpu_result *d_out,
                        void *stream, ngpu_layer_stats *stats) {
  return process_device(e, kDefault, d_data, len, d_chunks, n, d_out, nullptr, 1, nullptr, stream,
                        stats);
}

int ngpu_process_dict_device(ngpu_engine *e, ngpu_dict *dict, const void *d_data, uint64_t len,
                             const ngpu_chunk *d_chunks, uint64_t n, ngpu_result *d_out,
                             const uint64_t *d_layer_first, uint64_t n_layers,
                             ngpu_layer_stats *d_stats, void *stream, ngpu_layer_stats *stats) {
  return process_device(e, dict, d_data, len, d_chunks, n, d_out, d_layer_first, n_layers, d_stats,
                        stream, stats);
}

// Results of a host-buffer call come back through pinned memory: a D2H
// hipMemcpyAsync into pageable memory takes the runtime's staging path.
static int pinned_results(ngpu_engine *e, uint64_t n) {
  if (n <= e->h_results_cap) return 0;
  uint64_t c = 4096;
  while (c < n) c *= 2;
  if (e->h_results) (void)hipHostFree(e->h_results), e->h_results = nullptr, e->h_results_cap = 0;
  HIP_TRY(e, hipHostMalloc((void **)&e->h_results, c * sizeof(ngpu_result), hipHostMallocDefault));
  e->h_results_cap = c;
  return 0;
}

static int process_host(ngpu_engine *e, ngpu_dict *dict, const void *data, uint64_t len,
                        const ngpu_chunk *chunks, uint64_t n, ngpu_result *out,
                        ngpu_layer_stats *stats) {
  if (!e || (n && (!data || !chunks || !out))) return NGPU_EINVAL;
  if (n >= 0xFFFFFFFFull) return fail(e, NGPU_EINVAL, "too many chunks in one call");
  for (uint64_t i = 0; i < n; ++i) {
    if (chunks[i].offset > len || chunks[i].length > len - chunks[i].offset)
      return fail(e, NGPU_EINVAL, "chunk %llu outside the data buffer", (unsigned long long)i);
    if (chunks[i].length > e->cfg.chunk_size)
      return fail(e, NGPU_EINVAL, "chunk %llu longer than chunk_size", (unsigned long long)i);
  }
  std::lock_guard<std::mutex> g(e->mu);
  DeviceGuard dg(e->device);
  if (dict == kDefault) dict = e->dict;
  if (int rc = dict_check(e, dict)) return rc;
  hipStream_t s = e->stream;
  uint64_t c0 = e->d_data_cap;
  if (grow(e, &e->d_data, c0, len + 64)) return NGPU_ENOMEM;
  e->d_data_cap = c0;
  if (n + 1 > e->d_chunk_cap || !e->d_chunks) {
    uint64_t a = 0, b = 0;
    if (e->d_chunks) hipFree(e->d_chunks), e->d_chunks = nullptr;
    if (e->d_results) hipFree(e->d_results), e->d_results = nullptr;
    if (grow(e, &e->d_chunks, a, n + 1)) return NGPU_ENOMEM;
    if (grow(e, &e->d_results, b, n + 1)) return NGPU_ENOMEM;
    e->d_chunk_cap = a < b ? a : b;
  }
  if (len) HIP_TRY(e, hipMemcpyAsync(e->d_data, data, len, hipMemcpyHostToDevice, s));
  if (n) HIP_TRY(e, hipMemcpyAsync(e->d_chunks, chunks, n * sizeof(ngpu_chunk),
                                   hipMemcpyHostToDevice, s));
  int rc = pinned_results(e, n);
  if (rc) return rc;
  rc = enqueue(e, dict, e->d_data, len, e->d_chunks, n, e->d_results, s);
  if (rc) return rc;
  if ((rc = host_fence(e, s))) return rc;
  if (n) HIP_TRY(e, hipMemcpyAsync(e->h_results, e->d_results, n * sizeof(ngpu_result),
                                   hipMemcpyDeviceToHost, s));
  if ((rc = read_stats(e, s, stats, true))) return rc;  // synchronises s
  if (n) memcpy(out, e->h_results, n * sizeof(ngpu_result));
  return 0;
}

int ngpu_process(ngpu_engine *e, const void *data, uint64_t len, const ngpu_chunk *chunks,
                 uint64_t n, ngpu_result *out, ngpu_layer_stats *stats) {
  return process_host(e, kDefault, data, len, chunks, n, out, stats);
}

// A whole layer tar in host memory.  Its bytes start crossing PCIe before the
// host walks the headers, so with a pinned buffer the walk (tarstream.hpp)
// overlaps the H2D DMA; then the chunk table follows, the stages run and the
// results come back.  Single walk (one pass collects the chunks).
int ngpu_pack_tar(ngpu_engine *e, const void *tar, uint64_t len, ngpu_chunk **chunks_out,
                  ngpu_result **results_out, uint64_t *n_out, ngpu_layer_stats *stats) {
  return guarded([&]() -> int {
    if (!e || !chunks_out || !results_out || !n_out || (!tar && len)) return NGPU_EINVAL;
    *chunks_out = nullptr;
    *results_out = nullptr;
    *n_out = 0;
    std::lock_guard<std::mutex> g(e->mu);
    DeviceGuard dg(e->device);
    ngpu_dict *dict = e->dict;
    if (int rc = dict_check(e, dict)) return rc;
    hipStream_t s = e->stream;
    uint64_t c0 = e->d_data_cap;
    if (grow(e, &e->d_data, c0, len + 64)) return NGPU_ENOMEM;
    e->d_data_cap = c0;
    if (len) HIP_TRY(e, hipMemcpyAsync(e->d_data, tar, len, hipMemcpyHostToDevice, s));
    struct Vec : TarSink {
      std::vector<ngpu_chunk> v;
      int chunk(uint64_t off, uint32_t l, uint32_t fi, uint64_t fo) override {
        v.push_back(ngpu_chunk{off, l, fi, fo});
        return 0;
      }
      int data(const uint8_t *, uint64_t) override { return 0; }
    } vec;
    TarScanner sc(e->cfg.chunk_size);
    int rc = sc.feed(static_cast<const uint8_t *>(tar), len, vec);
    if (!rc) rc = sc.finish();
    const uint64_t n = vec.v.size();
    if (!rc && n >= 0xFFFFFFFFull) rc = fail(e, NGPU_EINVAL, "too many chunks in one call");
    if (rc) {
      (void)hipStreamSynchronize(s);  // the DMA may still read the caller's buffer
      return rc;
    }
    if (n + 1 > e->d_chunk_cap || !e->d_chunks) {
      uint64_t a = 0, b = 0;
      (void)hipStreamSynchronize(s);  // buffers about to be replaced may be in use
      if (e->d_chunks) hipFree(e->d_chunks), e->d_chunks = nullptr;
      if (e->d_results) hipFree(e->d_results), e->d_results = nullptr;
      if (grow(e, &e->d_chunks, a, n + 1)) return NGPU_ENOMEM;
      if (grow(e, &e->d_results, b, n + 1)) return NGPU_ENOMEM;
      e->d_chunk_cap = a < b ? a : b;
    }
    ngpu_chunk *ch = (ngpu_chunk *)malloc(sizeof(ngpu_chunk) * (n ? n : 1));
    ngpu_result *res = (ngpu_result *)malloc(sizeof(ngpu_result) * (n ? n : 1));
    if (!ch || !res) {
      (void)hipStreamSynchronize(s);
      free(ch);
      free(res);
      return NGPU_ENOMEM;
    }
    if (n) memcpy(ch, vec.v.data(), n * sizeof(ngpu_chunk));
    auto bail = [&](int code) {
      (void)hipStreamSynchronize(s);
      free(ch);
      free(res);
      return code;
    };
    if (n && hipMemcpyAsync(e->d_chunks, ch, n * sizeof(ngpu_chunk), hipMemcpyHostToDevice, s) !=
                 hipSuccess)
      return bail(fail(e, NGPU_EHIP, "chunk table H2D failed"));
    if ((rc = pinned_results(e, n))) return bail(rc);
    if ((rc = enqueue(e, dict, e->d_data, len, e->d_chunks, n, e->d_results, s))) return bail(rc);
    if ((rc = host_fence(e, s))) return bail(rc);
    if (n && hipMemcpyAsync(e->h_results, e->d_results, n * sizeof(ngpu_result),
                            hipMemcpyDeviceToHost, s) != hipSuccess)
      return bail(fail(e, NGPU_EHIP, "results D2H failed"));
    if ((rc = read_stats(e, s, stats, true))) return bail(rc);  // synchronises s
    if (n) memcpy(res, e->h_results, n * sizeof(ngpu_result));
    *chunks_out = ch;
    *results_out = res;
    *n_out = n;
    return NGPU_OK;
  });
}

int ngpu_process_dict(ngpu_engine *e, ngpu_dict *dict, const void *data, uint64_t len,
                      const ngpu_chunk *chunks, uint64_t n, ngpu_result *out,
                      ngpu_layer_stats *stats) {
  return process_host(e, dict, data, len, chunks, n, out, stats);
}

int ngpu_timing_at(ngpu_engine *e, uint32_t back, ngpu_timing *out) {
  if (!e || !out) return NGPU_EINVAL;
  if (!(e->cfg.flags & NGPU_FLAG_TIMING))
    return fail(e, NGPU_EINVAL, "engine created without NGPU_FLAG_TIMING");
  std::lock_guard<std::mutex> g(e->mu);
  memset(out, 0, sizeof *out);
  const uint64_t have = e->tcalls < (uint64_t)ngpu_engine::kTimingRing
                            ? e->tcalls : (uint64_t)ngpu_engine::kTimingRing;
  if (back >= have) {
    if (back == 0) return 0;  // nothing recorded yet
    return fail(e, NGPU_EINVAL, "timing %u calls back: only %llu kept", back,
                (unsigned long long)have);
  }
  const int k = (int)((e->tcalls - 1 - back) % ngpu_engine::kTimingRing);
  if (!e->timed[k]) return 0;
  hipEvent_t *ev = e->ev[k];
  HIP_TRY(e, hipEventSynchronize(ev[4]));
  HIP_TRY(e, hipEventElapsedTime(&out->digest_ms, e->slot_fused[k] ? ev[0] : ev[1], ev[2]));
  HIP_TRY(e, hipEventElapsedTime(&out->tree_ms, ev[2], ev[3]));
  HIP_TRY(e, hipEventElapsedTime(&out->dedup_ms, ev[3], ev[4]));
  HIP_TRY(e, hipEventElapsedTime(&out->total_ms, ev[0], ev[4]));
  out->group_log2 = (uint32_t)e->slot_D[k];
  return 0;
}

int ngpu_last_timing(ngpu_engine *e, ngpu_timing *out) { return ngpu_timing_at(e, 0, out); }

int ngpu_batch_stats(ngpu_engine *e, uint64_t out[3]) {
  if (!e || !out) return NGPU_EINVAL;
  batch_stats(e, out);
  return 0;
}

int ngpu_engine_counters_get(ngpu_engine *e, ngpu_engine_counters *out) {
  if (!e || !out) return NGPU_EINVAL;
  memset(out, 0, sizeof *out);
  out->open_packs = (uint64_t)e->open_packs.load();
  out->batch_waitable = (uint64_t)e->batch_waitable.load();
  std::lock_guard<std::mutex> g(e->pool_mu);
  out->staging_pool_bufs = e->staging_pool.size();
  out->staging_pool_bytes = e->staging_pool_bytes;
  out->pack_pool = e->pack_pool.size();
  out->land_pool = e->land_pool.size();
  return 0;
}

}  // extern "C"
