// packs_drive.cpp — K layers converted concurrently through ONE engine, driven
// from native threads the way containerd's Go converter drives the drop-in:
// one goroutine per layer (LayerConvertFunc, pkg/converter/convert_unix.go:822)
// each calling converter.Pack over cgo.  No Python (and no GIL) on the submit
// path: bench.py --packs times the Pack API through this harness and, beside
// it, through Python threads.
//
// A round: every thread opens a pack, feeds its layer, closes it (mode bit 0
// clear: decisions back) or finishes the early-emission stream (bit 0 set:
// ngpu_pack_set_output before the first write, zstd, into a counting sink),
// then all meet; round_s[r] = the wall time from the round's start (every
// thread released) to its last close.  Feed (mode bit 1): clear = Write, the
// layer from pageable memory in `piece`-byte ngpu_pack_write calls; set =
// ReadFrom, what the Go drop-in does for io.Copy(tw, tr) (convert_unix.go:881,
// integration/go/pkg/gpu/gpu.go PackWriter.ReadFrom): ngpu_pack_reserve, the
// source's Read of at most `piece` bytes straight into the pinned staging,
// ngpu_pack_commit.  node (or NULL): the packs open on that node's
// least-loaded engine (ngpu_node_pack_open) instead of on eng; part (or
// NULL): per layer, the node index its last round's pack ran on.  trace (or
// NULL): per round and layer, seconds from the round's start to the pack's
// open, its last write and its close returning (rounds x k x 3).
//
// build: nydus-snapshotter_amd/Makefile (build/libpacks_drive.so)
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "nydus_gpu.h"

namespace {

// generation barrier for n parties; abort() releases every waiter with false
class Barrier {
 public:
  explicit Barrier(unsigned n) : n_(n) {}
  bool wait() {
    std::unique_lock<std::mutex> g(m_);
    if (broken_) return false;
    const uint64_t gen = gen_;
    if (++in_ == n_) {
      in_ = 0;
      ++gen_;
      cv_.notify_all();
      return true;
    }
    cv_.wait(g, [&] { return gen_ != gen || broken_; });
    return !broken_;
  }
  void abort() {
    std::lock_guard<std::mutex> g(m_);
    broken_ = true;
    cv_.notify_all();
  }

 private:
  std::mutex m_;
  std::condition_variable cv_;
  unsigned n_, in_ = 0;
  uint64_t gen_ = 0;
  bool broken_ = false;
};

int count_sink(void *ctx, const void *, uint64_t len) {
  *static_cast<uint64_t *>(ctx) += len;
  return 0;
}

}  // namespace

extern "C" int packs_drive(ngpu_engine *eng, uint32_t k, const uint8_t *const *tars,
                           const uint64_t *lens, uint64_t piece, uint32_t mode, uint32_t digester,
                           uint32_t chunk_size, uint32_t rounds, double *round_s,
                           uint64_t *per_layer, double *trace, char *err, uint64_t err_len,
                           ngpu_node *node, int32_t *part) {
  if ((!eng && !node) || !k || !tars || !lens || !piece || !rounds || !round_s || !per_layer)
    return NGPU_EINVAL;
  if (!eng) eng = ngpu_node_engine(node, 0);  // (error messages)
  const bool stream = mode & 1, read_from = mode & 2;
  Barrier meet(k + 1);
  std::mutex em;
  std::string first_err;
  std::atomic<int> rc_all{0};
  auto fail = [&](int rc, const char *what) {
    std::lock_guard<std::mutex> g(em);
    if (!rc_all.load()) {
      rc_all = rc;
      first_err = std::string(what) + ": " + ngpu_last_error(eng);
    }
    meet.abort();
  };
  using clk = std::chrono::steady_clock;
  std::vector<clk::time_point> t_round(rounds);
  auto mark = [&](uint32_t r, uint32_t i, int what) {
    if (trace)
      trace[((uint64_t)r * k + i) * 3 + what] =
          std::chrono::duration<double>(clk::now() - t_round[r]).count();
  };
  std::vector<std::thread> th;
  for (uint32_t i = 0; i < k; ++i)
    th.emplace_back([&, i] {
      for (uint32_t r = 0; r < rounds; ++r) {
        if (!meet.wait()) return;
        ngpu_pack *p = nullptr;
        uint64_t out_bytes = 0;
        const uint32_t flags = stream ? NGPU_PACK_RETAIN : 0;
        int rc = node ? ngpu_node_pack_open(node, nullptr, flags, &p) : ngpu_pack_open_ex(eng, flags, &p);
        if (rc) return fail(rc, "pack_open");
        mark(r, i, 0);
        if (part && node && r + 1 == rounds) {
          part[i] = -1;
          for (uint32_t j = 0; j < ngpu_node_size(node); ++j)
            if (ngpu_node_engine(node, j) == ngpu_pack_engine(p)) part[i] = (int32_t)j;
        }
        if (stream) {
          ngpu_blob_options o;
          memset(&o, 0, sizeof o);
          o.compressor = NGPU_COMPRESSOR_ZSTD;
          o.digester = digester;
          o.chunk_size = chunk_size;
          o.fs_version = 6;
          if ((rc = ngpu_pack_set_output(p, &o, count_sink, &out_bytes))) {
            ngpu_pack_abort(p);
            return fail(rc, "pack_set_output");
          }
        }
        if (read_from) {  // io.Copy -> PackWriter.ReadFrom: reads land in pinned staging
          for (uint64_t a = 0; a < lens[i];) {
            void *dst = nullptr;
            uint64_t avail = 0;
            if ((rc = ngpu_pack_reserve(p, &dst, &avail))) {
              ngpu_pack_abort(p);
              return fail(rc, "pack_reserve");
            }
            uint64_t n = lens[i] - a < piece ? lens[i] - a : piece;  // the source's Read
            if (n > avail) n = avail;
            memcpy(dst, tars[i] + a, n);
            if ((rc = ngpu_pack_commit(p, n))) {
              ngpu_pack_abort(p);
              return fail(rc, "pack_commit");
            }
            a += n;
          }
        } else {
          for (uint64_t a = 0; a < lens[i]; a += piece) {
            const uint64_t n = lens[i] - a < piece ? lens[i] - a : piece;
            if ((rc = ngpu_pack_write(p, tars[i] + a, n))) {
              ngpu_pack_abort(p);
              return fail(rc, "pack_write");
            }
          }
        }
        mark(r, i, 1);
        ngpu_chunk *ch = nullptr;
        ngpu_result *res = nullptr;
        uint64_t n = 0;
        ngpu_layer_stats st;
        if (stream) {
          ngpu_blob_info info;
          rc = ngpu_pack_finish(p, nullptr, nullptr, nullptr, &ch, &res, &n, &st, &info);
        } else {
          rc = ngpu_pack_close(p, &ch, &res, &n, &st);
        }
        if (rc) return fail(rc, stream ? "pack_finish" : "pack_close");
        mark(r, i, 2);
        if (r + 1 == rounds) {
          uint64_t *o = per_layer + 4 * (uint64_t)i;
          o[0] = o[1] = o[2] = 0;
          for (uint64_t c = 0; c < n; ++c)
            if (res[c].kind < 3) ++o[res[c].kind];
          o[3] = out_bytes;
        }
        ngpu_free_host(ch);
        ngpu_free_host(res);
        if (!meet.wait()) return;
      }
    });
  for (uint32_t r = 0; r < rounds; ++r) {
    t_round[r] = clk::now();  // (before the release: the threads read it after the barrier)
    if (!meet.wait()) break;  // round r starts
    const auto t0 = t_round[r];
    if (!meet.wait()) break;  // every pack of round r closed
    round_s[r] = std::chrono::duration<double>(clk::now() - t0).count();
  }
  for (auto &t : th) t.join();
  if (rc_all.load() && err && err_len) snprintf(err, err_len, "%s", first_err.c_str());
  return rc_all.load();
}
