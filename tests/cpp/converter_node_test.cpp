// converter_node_test.cpp — the C++ converter mirror (host/converter.hpp) on a
// multi-GPU node, as containerd drives converter.Pack:
// one goroutine per layer (convert_unix.go:467-538), io.Copy into the Pack
// (ReadFrom, :881) or Write in pieces, then Close.
//
// 1. N layer tars packed at once on N threads (a barrier lines them up):
//    every output stream is written to WORKDIR/out_<i>.bin for the Python
//    side to compare with the oracle, and the node part each Pack ran on is
//    printed ("pack <i> part <p> ...").
// 2. The reference's error paths that never reach tw.Close()
//    (convert_unix.go:885-907): ctx.Done() with no Close, a source read
//    error inside io.Copy, a writer dropped without Close, Cancel then Close,
//    and Cancel racing a running Write.  After each, every engine of the node
//    must hold exactly what it held before (open packs, pooled staging and
//    stream sets): nothing of the aborted Pack is left behind.
// usage: converter_node_test WORKDIR COMPRESSOR DICT_BOOTSTRAP|- TAR...
// Prints lines and "PASS"; exit 1 on failure.  NYDUS_GPU_DEVICES picks the node.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "converter.hpp"

using namespace nydus::converter;

#define REQUIRE(c, ...)                                                         \
  do {                                                                          \
    if (!(c)) {                                                                 \
      fprintf(stderr, "REQUIRE failed at %s:%d: %s: ", __FILE__, __LINE__, #c); \
      fprintf(stderr, __VA_ARGS__);                                             \
      fprintf(stderr, "\n");                                                    \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)
#define REQUIRE_NOERR(e) REQUIRE(!(e), "error %d: %s", (e).code, (e).msg.c_str())

static std::vector<uint8_t> read_file(const std::string &p) {
  FILE *f = fopen(p.c_str(), "rb");
  REQUIRE(f, "open %s", p.c_str());
  std::vector<uint8_t> v;
  uint8_t b[1 << 16];
  size_t r;
  while ((r = fread(b, 1, sizeof b, f)) > 0) v.insert(v.end(), b, b + r);
  fclose(f);
  return v;
}

static void write_file(const std::string &p, const std::vector<uint8_t> &v) {
  FILE *f = fopen(p.c_str(), "wb");
  REQUIRE(f && fwrite(v.data(), 1, v.size(), f) == v.size(), "write %s", p.c_str());
  fclose(f);
}

// A tar reader for io.Copy: up to `piece` bytes per Read; with fail_at, the
// read that would pass that offset fails instead (a broken source).
class TarReader : public Reader {
 public:
  TarReader(const std::vector<uint8_t> &b, size_t piece, size_t fail_at = SIZE_MAX)
      : b_(b), piece_(piece), fail_at_(fail_at) {}
  int64_t Read(void *p, size_t n) override {
    if (off_ >= b_.size()) return 0;
    size_t k = std::min({n, piece_, b_.size() - off_});
    if (off_ + k > fail_at_) return -1;
    memcpy(p, b_.data() + off_, k);
    off_ += k;
    return (int64_t)k;
  }

 private:
  const std::vector<uint8_t> &b_;
  size_t piece_, off_ = 0, fail_at_;
};

// A ustar header of one regular file (the racing writer's endless layer).
static void file_header(uint8_t h[512], const char *name, uint64_t size) {
  memset(h, 0, 512);
  char *b = (char *)h;
  snprintf(b, 100, "%s", name);
  snprintf(b + 100, 8, "%07o", 0644);
  snprintf(b + 108, 8, "%07o", 0);
  snprintf(b + 116, 8, "%07o", 0);
  snprintf(b + 124, 12, "%011llo", (unsigned long long)size);
  snprintf(b + 136, 12, "%011o", 0);
  b[156] = '0';
  memcpy(b + 257, "ustar\0" "00", 8);
  memset(b + 148, ' ', 8);
  unsigned sum = 0;
  for (int i = 0; i < 512; ++i) sum += h[i];
  snprintf(b + 148, 8, "%06o", sum);
}

static std::vector<EngineCounters> counters(const PackOption &opt) {
  std::vector<EngineCounters> c;
  REQUIRE_NOERR(GpuCounters(opt, &c));
  return c;
}

static std::string show(const std::vector<EngineCounters> &v) {
  std::string s;
  char b[160];
  for (const EngineCounters &c : v) {
    snprintf(b, sizeof b, "[open %llu staging %llu/%llu B packsets %llu landing %llu]",
             (unsigned long long)c.OpenPacks, (unsigned long long)c.StagingPoolBufs,
             (unsigned long long)c.StagingPoolBytes, (unsigned long long)c.PackPool,
             (unsigned long long)c.LandPool);
    s += b;
  }
  return s;
}

static void expect_back(const PackOption &opt, const std::vector<EngineCounters> &before,
                        const char *what) {
  const std::vector<EngineCounters> now = counters(opt);
  REQUIRE(now == before, "%s left something behind: before %s now %s", what, show(before).c_str(),
          show(now).c_str());
  printf("%s ok %s\n", what, show(now).c_str());
}

int main(int argc, char **argv) {
  if (argc < 5) return 2;
  const std::string work = argv[1], comp = argv[2], dict = argv[3];
  std::vector<std::vector<uint8_t>> tars;
  for (int i = 4; i < argc; ++i) tars.push_back(read_file(argv[i]));
  PackOption opt;
  opt.Compressor = comp;
  if (dict != "-") opt.ChunkDictPath = dict;

  // 1. every layer at once, one thread each (LayerConvertFunc per goroutine)
  const size_t N = tars.size();
  std::vector<BufferWriter> outs(N);
  std::vector<PackStats> stats(N);
  std::vector<Error> errs(N);
  std::mutex m;
  std::condition_variable cv;
  size_t ready = 0;
  std::vector<std::thread> th;
  for (size_t i = 0; i < N; ++i)
    th.emplace_back([&, i] {
      std::unique_ptr<PackWriteCloser> w;
      errs[i] = Pack(outs[i], opt, &w);
      {
        std::unique_lock<std::mutex> g(m);
        ++ready;
        cv.notify_all();
        cv.wait(g, [&] { return ready == N; });  // all open before any writes
      }
      if (errs[i]) return;
      if (i % 2 == 0) {  // io.Copy -> ReadFrom (zero-copy into staging)
        TarReader r(tars[i], 100000 + 4096 * i);
        uint64_t n = 0;
        errs[i] = w->ReadFrom(r, &n);
        if (!errs[i] && n != tars[i].size()) errs[i] = Error{-1, "short ReadFrom"};
      } else {  // Write in pieces
        for (size_t a = 0; !errs[i] && a < tars[i].size(); a += 65536)
          errs[i] = w->Write(tars[i].data() + a, std::min<size_t>(65536, tars[i].size() - a));
      }
      if (!errs[i]) errs[i] = w->Close();
      if (!errs[i]) stats[i] = w->Stats();
    });
  for (auto &t : th) t.join();
  std::vector<int> per_part;
  for (size_t i = 0; i < N; ++i) {
    REQUIRE_NOERR(errs[i]);
    write_file(work + "/out_" + std::to_string(i) + ".bin", outs[i].data);
    printf("pack %zu part %d digest %s chunks %llu new %llu dict %llu\n", i, stats[i].Part,
           stats[i].Digest.c_str(), (unsigned long long)stats[i].Chunks,
           (unsigned long long)stats[i].NewChunks, (unsigned long long)stats[i].DictChunks);
    REQUIRE(stats[i].Part >= 0, "pack %zu: not on a node part", i);
    if ((size_t)stats[i].Part >= per_part.size()) per_part.resize(stats[i].Part + 1, 0);
    ++per_part[stats[i].Part];
  }
  printf("parts");
  for (int c : per_part) printf(" %d", c);
  printf("\n");

  // 2. the paths that never reach Close
  const std::vector<uint8_t> &big = tars[0];
  const std::vector<EngineCounters> base = counters(opt);
  printf("base %s\n", show(base).c_str());
  for (const EngineCounters &c : base) REQUIRE(c.OpenPacks == 0, "a pack still open after step 1");
  {  // ctx.Done() with no Close to follow (the copy goroutine finished, the
     // select took ctx.Done(): convert_unix.go:885-893)
    BufferWriter o;
    std::unique_ptr<PackWriteCloser> w;
    REQUIRE_NOERR(Pack(o, opt, &w));
    REQUIRE_NOERR(w->Write(big.data(), big.size() / 2));
    w->Cancel();
    expect_back(opt, base, "cancel_without_close");
    Error e = w->Write(big.data(), 10);
    REQUIRE(e.code == -10, "write after cancel: %d %s", e.code, e.msg.c_str());
    e = w->Close();
    REQUIRE(e.code == -10 && e.msg.find("signal: killed") == 0, "close after cancel: %d %s", e.code,
            e.msg.c_str());
  }
  {  // a source error inside io.Copy (copyBufferDone gets it; no tw.Close())
    BufferWriter o;
    std::unique_ptr<PackWriteCloser> w;
    REQUIRE_NOERR(Pack(o, opt, &w));
    TarReader r(big, 50000, big.size() / 2);
    uint64_t n = 0;
    Error e = w->ReadFrom(r, &n);
    REQUIRE(e && n > 0 && n <= big.size() / 2, "ReadFrom of a failing source: %d after %llu", e.code,
            (unsigned long long)n);
    expect_back(opt, base, "readfrom_source_error");
  }
  {  // the writer dropped without Close (the Go binding's finalizer)
    BufferWriter o;
    std::unique_ptr<PackWriteCloser> w;
    REQUIRE_NOERR(Pack(o, opt, &w));
    REQUIRE_NOERR(w->Write(big.data(), big.size() / 2));
    w.reset();
    expect_back(opt, base, "dropped_without_close");
  }
  {  // Cancel racing a running Write from another thread
    BufferWriter o;
    std::unique_ptr<PackWriteCloser> w;
    REQUIRE_NOERR(Pack(o, opt, &w));
    std::atomic<bool> started{false};
    Error we;
    std::thread wr([&] {  // one 4 GiB file: still being written when Cancel comes
      uint8_t h[512];
      file_header(h, "big.bin", 4ull << 30);
      we = w->Write(h, 512);
      static const std::vector<uint8_t> zeros(1 << 20, 0);
      for (uint64_t a = 0; !we && a < (4ull << 30); a += zeros.size()) {
        we = w->Write(zeros.data(), zeros.size());
        started = true;
      }
    });
    while (!started) std::this_thread::yield();
    std::this_thread::sleep_for(std::chrono::milliseconds(2));
    w->Cancel();
    wr.join();
    REQUIRE(we.code == -10, "the racing write: %d %s", we.code, we.msg.c_str());
    expect_back(opt, base, "cancel_during_write");
  }
  {  // and the normal path still works afterwards, on the warm pools
    BufferWriter o;
    std::unique_ptr<PackWriteCloser> w;
    REQUIRE_NOERR(Pack(o, opt, &w));
    TarReader r(big, 1 << 20);
    uint64_t n = 0;
    REQUIRE_NOERR(w->ReadFrom(r, &n));
    REQUIRE_NOERR(w->Close());
    REQUIRE(o.data == outs[0].data, "a Pack after the aborts differs from the first one");
    expect_back(opt, base, "pack_after_aborts");
  }
  printf("PASS\n");
  return 0;
}
