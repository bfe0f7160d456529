// converter.cpp — see converter.hpp.  Only the C ABI is used.
#include "converter.hpp"

#include <openssl/sha.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <map>
#include <mutex>
#include <thread>
#include <tuple>

#include "nydus_gpu.h"

namespace nydus {
namespace converter {

const char *const EntryBlob = "image.blob";
const char *const EntryBootstrap = "image.boot";
const char *const EntryBlobMeta = "blob.meta";
const char *const EntryTOC = "rafs.blob.toc";

namespace {

Error err(int code, const std::string &msg) { return Error{code ? code : NGPU_EINVAL, msg}; }

std::string hex(const uint8_t *d, int n) {
  static const char *x = "0123456789abcdef";
  std::string s;
  for (int i = 0; i < n; ++i) {
    s += x[d[i] >> 4];
    s += x[d[i] & 15];
  }
  return s;
}

int write_trampoline(void *ctx, const void *buf, uint64_t len) {
  Writer *w = static_cast<Writer *>(ctx);
  return w->Write(buf, (size_t)len) ? 1 : 0;
}

int64_t read_trampoline(void *ctx, void *buf, uint64_t len, uint64_t off) {
  return static_cast<ReaderAt *>(ctx)->ReadAt(buf, (size_t)len, off);
}

Error parse_chunk_size(const std::string &s, uint32_t *out) {
  if (s.empty()) {
    *out = 0x100000;
    return {};
  }
  char *end = nullptr;
  const unsigned long long v = strtoull(s.c_str(), &end, 0);
  if (!end || *end || (v & (v - 1)) || v < 0x1000 || v > 0x1000000)
    return err(NGPU_EINVAL, "invalid chunk size " + s + ": must be power of two in [0x1000, 0x1000000]");
  *out = (uint32_t)v;
  return {};
}

Error compressor_of(const std::string &s, uint32_t *out) {
  if (s.empty() || s == "zstd") *out = NGPU_COMPRESSOR_ZSTD;  // nydus-image default
  else if (s == "none") *out = NGPU_COMPRESSOR_NONE;
  else if (s == "lz4_block") *out = NGPU_COMPRESSOR_LZ4_BLOCK;
  else return err(NGPU_EINVAL, "unsupported compressor " + s);
  return {};
}

// tool.DetectFeatures (pkg/converter/tool/feature.go:114-146): the features a
// Pack requires, checked once per process against what the builder supports.
// The builder emulated is the pinned nydus-image v2.3.0
// (misc/snapshotter/Dockerfile:5), whose `create -h` lists all three
// features (feature_test.go:255, 379), so all are detected and none is
// ignored.  The GPU builder then refuses what it does not implement
// (`--batch-size`, `--encrypt`) with NGPU_EUNSUPP at Pack(): the reference
// passes both flags to the builder unconditionally (builder.go:137-142), so it
// never returns a blob without them.  A later Pack requiring a different set
// fails ("features changed"), as the reference's process-global sync.Once
// makes it.
const char *const kFeatureTar2Rafs = "--type tar-rafs";
const char *const kFeatureBatchSize = "--batch-size";
const char *const kFeatureEncrypt = "--encrypt";
std::mutex g_feat_mu;
bool g_feat_done = false;
std::vector<std::string> g_feat_required, g_feat_detected;

Error detect_features(const std::vector<std::string> &required, std::vector<std::string> *detected) {
  std::lock_guard<std::mutex> g(g_feat_mu);
  if (!g_feat_done) {
    g_feat_done = true;
    g_feat_required = required;
    for (const std::string &f : required)
      if (f == kFeatureTar2Rafs || f == kFeatureBatchSize || f == kFeatureEncrypt)
        g_feat_detected.push_back(f);
  }
  if (g_feat_required != required) {
    std::string a, b;
    for (auto &f : g_feat_required) a += (a.empty() ? "" : ",") + f;
    for (auto &f : required) b += (b.empty() ? "" : ",") + f;
    return err(NGPU_EINVAL, "features changed: [" + a + "] -> [" + b + "]");
  }
  *detected = g_feat_detected;
  return {};
}

// Where Packs run.  The reference runs one nydus-image process per layer,
// concurrently (convert_unix.go:467-538 -- one goroutine per layer); here the
// layers of a process shard over the node's GPUs (north star): one node per
// option set (digester, chunk size, fs version, aligned chunk) over every
// device -- NYDUS_GPU_DEVICES ("0,1,..."; a device may repeat, e.g. "0,0" to
// rehearse a 2-GPU node on one) or all the devices the library sees -- and
// each Pack goes to its least-loaded engine (ngpu_node_pack_open).
// PackOption.Device >= 0 pins every Pack of the option set to one engine on
// that device instead.  Engines serialise their own calls and every Pack holds
// its own chunk dict handle, so Packs share engines safely.
using OptKey = std::tuple<int, uint32_t, uint32_t, uint32_t, bool>;
std::mutex g_mu;
std::map<OptKey, ngpu_engine *> g_engines;  // PackOption.Device >= 0
std::map<OptKey, ngpu_node *> g_nodes;      // PackOption.Device < 0 (default)

std::vector<int32_t> node_devices() {
  std::vector<int32_t> d;
  if (const char *v = getenv("NYDUS_GPU_DEVICES")) {
    for (const char *p = v; *p;) {
      char *end = nullptr;
      const long x = strtol(p, &end, 10);
      if (end == p) break;
      d.push_back((int32_t)x);
      p = *end == ',' ? end + 1 : end;
    }
  }
  if (d.empty())
    for (int i = 0, n = ngpu_device_count(); i < n; ++i) d.push_back(i);
  return d;
}

// Where a Pack opens: the node of its option set, or one engine (Device >= 0).
struct Target {
  ngpu_node *node = nullptr;
  ngpu_engine *eng = nullptr;
  ngpu_engine *first() const { return node ? ngpu_node_engine(node, 0) : eng; }
};

Error target_for(const PackOption &opt, Target *out) {
  uint32_t cs = 0;
  if (Error e = parse_chunk_size(opt.ChunkSize, &cs)) return e;
  const std::string fv = opt.FsVersion.empty() ? "6" : opt.FsVersion;  // convert_unix.go:326-328
  if (fv != "5" && fv != "6") return err(NGPU_EINVAL, "invalid fs version " + opt.FsVersion);
  uint32_t dg;
  if (opt.Digester.empty() || opt.Digester == "blake3") dg = NGPU_DIGEST_BLAKE3;
  else if (opt.Digester == "sha256") dg = NGPU_DIGEST_SHA256;
  else return err(NGPU_EINVAL, "unsupported digester " + opt.Digester);
  // AlignedChunk only matters for RAFS v5 (types.go:73-74; builder.go:131-133)
  const bool aligned = opt.AlignedChunk && fv == "5";
  const int dev = opt.Device < 0 ? -1 : opt.Device;
  const OptKey key = std::make_tuple(dev, dg, cs, (uint32_t)(fv[0] - '0'), aligned);
  ngpu_config cfg;
  memset(&cfg, 0, sizeof cfg);
  cfg.device = dev < 0 ? 0 : dev;
  cfg.digester = dg;
  cfg.chunk_size = cs;
  cfg.fs_version = std::get<3>(key);
  if (aligned) cfg.flags |= NGPU_FLAG_ALIGNED_CHUNK;
  std::lock_guard<std::mutex> g(g_mu);
  if (dev >= 0) {
    auto it = g_engines.find(key);
    if (it == g_engines.end()) {
      ngpu_engine *e = nullptr;
      if (int rc = ngpu_create(&cfg, &e)) return err(rc, "gpu engine: create failed");
      it = g_engines.emplace(key, e).first;
    }
    out->eng = it->second;
    return {};
  }
  auto it = g_nodes.find(key);
  if (it == g_nodes.end()) {
    const std::vector<int32_t> devs = node_devices();
    if (devs.empty()) return err(NGPU_ENODEV, "gpu node: no device");
    ngpu_node *n = nullptr;
    if (int rc = ngpu_node_create(devs.data(), (uint32_t)devs.size(), &cfg, &n))
      return err(rc, "gpu node: create failed");
    it = g_nodes.emplace(key, n).first;
  }
  out->node = it->second;
  return {};
}

// Node index of the engine a pack runs on (-1: a pinned engine).
int part_of(const Target &t, ngpu_pack *p) {
  if (!t.node) return -1;
  ngpu_engine *e = ngpu_pack_engine(p);
  for (uint32_t i = 0, n = ngpu_node_size(t.node); i < n; ++i)
    if (ngpu_node_engine(t.node, i) == e) return (int)i;
  return -1;
}

// Every end of a Pack releases it exactly once: Close (finish), a failed
// Write / ReadFrom, a source read error, Cancel (ctx.Done() -- also when no
// Close follows: LayerConvertFunc skips tw.Close() on its error paths,
// convert_unix.go:885-907) and the destructor (the Go binding's finalizer).
// mu_ is held across every call on the pack, so Cancel from another thread
// aborts it only between them; the cancel flag, stored first, makes a running
// Write or Close return at its next slot.
class GpuPackWriteCloser : public PackWriteCloser {
 public:
  GpuPackWriteCloser(ngpu_engine *e, ngpu_pack *p, int part, Writer &dest, uint32_t comp,
                     double timeout, std::string prefetch, bool ociref = false)
      : e_(e), p_(p), dest_(dest), comp_(comp), timeout_(timeout), prefetch_(std::move(prefetch)) {
    stats_.Part = part;
    ngpu_pack_set_cancel(p_, &cancel_);
    // `dest` is known at Pack() (convert_unix.go:325): the stream leaves while
    // the tar arrives (ngpu_pack_set_output, early emission); Close finishes it.
    // PrefetchPatterns: the builder's stdin, "/" by default (builder.go:125-127, 166)
    ngpu_blob_options o;
    memset(&o, 0, sizeof o);
    o.compressor = comp_;
    o.prefetch_patterns = ociref ? nullptr : prefetch_.c_str();
    out_rc_ = ngpu_pack_set_output(p_, &o, write_trampoline, &dest_);
    if (timeout_ > 0)  // builder.go:153-158: the builder runs under ctx.WithTimeout
      timer_ = std::thread([this] {
        std::unique_lock<std::mutex> g(tm_);
        if (!tcv_.wait_for(g, std::chrono::duration<double>(timeout_), [this] { return done_; })) {
          g.unlock();
          Cancel();
        }
      });
  }
  ~GpuPackWriteCloser() override {
    StopTimer();
    std::lock_guard<std::mutex> g(mu_);
    End();
  }
  void Cancel() override {
    __atomic_store_n(&cancel_, 1, __ATOMIC_RELAXED);
    std::lock_guard<std::mutex> g(mu_);  // after the running call, if any
    End();
  }
  Error Write(const void *p, size_t n) override {
    Error e;
    {
      std::lock_guard<std::mutex> g(mu_);
      e = WriteLocked(p, n);
    }
    if (e) StopTimer();
    return e;
  }
  Error ReadFrom(Reader &src, uint64_t *total) override {
    *total = 0;
    Error e;
    {
      std::lock_guard<std::mutex> g(mu_);
      e = ReadFromLocked(src, total);
    }
    if (e) StopTimer();
    return e;
  }
  Error Close() override {
    Error e;
    {
      std::lock_guard<std::mutex> g(mu_);
      e = CloseLocked();
    }
    StopTimer();
    return e;
  }
  const PackStats &Stats() const override { return stats_; }

 private:
  // the pack ends here (mu_ held): nothing more reads the flag or the staging
  void End() {
    if (p_) ngpu_pack_abort(p_);
    p_ = nullptr;
  }
  Error Gone() const {
    if (__atomic_load_n(&cancel_, __ATOMIC_RELAXED))
      return Killed(NGPU_ECANCELED, "pack: cancelled");
    return err(NGPU_EINVAL, "pack already ended");
  }
  Error OutputFailed() {
    Error e = err(out_rc_, std::string("pack output: ") + ngpu_last_error(e_));
    End();
    return e;
  }
  Error WriteLocked(const void *p, size_t n) {
    if (!p_) return Gone();
    if (out_rc_) return OutputFailed();
    if (!n) return {};
    if (int rc = ngpu_pack_write(p_, p, n)) {
      Error e = Killed(rc, std::string("pack write: ") + ngpu_last_error(e_));
      End();  // a failed write leaves the pack open
      return e;
    }
    return {};
  }
  // Go's PackWriter.ReadFrom (io.Copy's path into a Pack): the source reads
  // straight into the engine's pinned staging (ngpu_pack_reserve / commit)
  Error ReadFromLocked(Reader &src, uint64_t *total) {
    if (!p_) return Gone();
    if (out_rc_) return OutputFailed();
    for (;;) {
      void *dst = nullptr;
      uint64_t avail = 0;
      if (int rc = ngpu_pack_reserve(p_, &dst, &avail)) {
        Error e = Killed(rc, std::string("pack reserve: ") + ngpu_last_error(e_));
        End();
        return e;
      }
      const int64_t r = src.Read(dst, (size_t)avail);
      if (r < 0) {  // the source failed: no Close will come for this pack
        End();
        return err(NGPU_EIO, "read source");
      }
      if (r == 0) return {};  // io.EOF
      if (int rc = ngpu_pack_commit(p_, (uint64_t)r)) {
        Error e = Killed(rc, std::string("pack commit: ") + ngpu_last_error(e_));
        End();
        return e;
      }
      *total += (uint64_t)r;
    }
  }
  Error CloseLocked() {
    if (!p_) return Gone();
    if (out_rc_) return OutputFailed();
    ngpu_chunk *ch = nullptr;
    ngpu_result *res = nullptr;
    uint64_t n = 0;
    ngpu_layer_stats st;
    ngpu_blob_info info;
    ngpu_pack *p = p_;
    p_ = nullptr;  // finish releases it on every outcome
    const int rc = ngpu_pack_finish(p, nullptr, nullptr, nullptr, &ch, &res, &n, &st, &info);
    if (rc) return Killed(rc, std::string("convert nydus ref: ") + ngpu_last_error(e_));
    ngpu_free_host(ch);
    ngpu_free_host(res);
    stats_.Digest = "sha256:" + hex(info.stream_digest, 32);
    stats_.Chunks = st.chunks;
    stats_.NewChunks = st.new_chunks;
    stats_.IntraChunks = st.intra_chunks;
    stats_.DictChunks = st.dict_chunks;
    stats_.StreamBytes = info.stream_bytes;
    stats_.BlobBytes = info.blob_bytes;
    return {};
  }
  // builder.go:169-171: a timed-out builder fails with "signal: killed"
  Error Killed(int rc, const std::string &msg) const {
    if (rc != NGPU_ECANCELED) return err(rc, msg);
    char b[96] = "";
    if (timeout_ > 0) snprintf(b, sizeof b, ", possibly due to timeout %gs", timeout_);
    return err(rc, std::string("signal: killed") + b + ": " + msg);
  }
  void StopTimer() {
    if (!timer_.joinable() || timer_.get_id() == std::this_thread::get_id()) return;
    {
      std::lock_guard<std::mutex> g(tm_);
      done_ = true;
    }
    tcv_.notify_all();
    timer_.join();
  }
  ngpu_engine *e_;
  ngpu_pack *p_;  // mu_
  Writer &dest_;
  uint32_t comp_;
  double timeout_;
  std::string prefetch_;
  alignas(4) volatile int32_t cancel_ = 0;
  int out_rc_ = 0;  // ngpu_pack_set_output at construction
  std::mutex mu_;   // held across every call on p_
  std::thread timer_;
  std::mutex tm_;
  std::condition_variable tcv_;
  bool done_ = false;
  PackStats stats_;
};

// packToTar (utils.go:92-160) without compression: image/ + image/<name>.
void tar_header(uint8_t h[512], const char *name, uint64_t size, char type, unsigned mode) {
  memset(h, 0, 512);
  char *b = (char *)h;
  snprintf(b, 100, "%s", name);
  snprintf(b + 100, 8, "%07o", mode);
  snprintf(b + 108, 8, "%07o", 0);
  snprintf(b + 116, 8, "%07o", 0);
  snprintf(b + 124, 12, "%011llo", (unsigned long long)size);
  snprintf(b + 136, 12, "%011o", 0);
  b[156] = type;
  memcpy(b + 257, "ustar\0" "00", 8);
  memset(b + 148, ' ', 8);
  unsigned sum = 0;
  for (int i = 0; i < 512; ++i) sum += h[i];
  snprintf(b + 148, 8, "%06o", sum);
  b[155] = ' ';
}

}  // namespace

Error BufferWriter::Write(const void *p, size_t n) {
  const uint8_t *b = static_cast<const uint8_t *>(p);
  data.insert(data.end(), b, b + n);
  return {};
}

int64_t BytesReaderAt::ReadAt(void *p, size_t n, uint64_t off) {
  if (off >= n_) return -1;
  if (n > n_ - off) n = (size_t)(n_ - off);
  memcpy(p, p_ + off, n);
  return (int64_t)n;
}

std::string TOCEntry::GetName() const {  // types.go:181-191
  std::string s;
  for (uint8_t c : Name) {
    if (!c) break;
    s += (char)c;
  }
  return s;
}

Error TOCEntry::GetCompressor(Compressor *out) const {  // types.go:167-179
  switch (Flags & CompressorMask) {
    case CompressorNone: *out = CompressorNone; return {};
    case CompressorZstd: *out = CompressorZstd; return {};
    case CompressorLz4Block: *out = CompressorLz4Block; return {};
  }
  char b[64];
  snprintf(b, sizeof b, "unsupported compressor, entry flags %x", Flags);
  return err(NGPU_EUNSUPP, b);
}

std::string TOCEntry::GetUncompressedDigest() const { return hex(UncompressedDigest, 32); }

bool IsNotFound(const Error &e) { return e.code == NGPU_ENOTFOUND; }

Error GpuCounters(const PackOption &opt, std::vector<EngineCounters> *out) {
  out->clear();
  Target t;
  if (Error e = target_for(opt, &t)) return e;
  const uint32_t n = t.node ? ngpu_node_size(t.node) : 1;
  for (uint32_t i = 0; i < n; ++i) {
    ngpu_engine_counters c;
    if (int rc = ngpu_engine_counters_get(t.node ? ngpu_node_engine(t.node, i) : t.eng, &c))
      return err(rc, "engine counters");
    out->push_back(EngineCounters{c.open_packs, c.staging_pool_bufs, c.staging_pool_bytes,
                                  c.pack_pool, c.land_pool});
  }
  return {};
}

Error Pack(Writer &dest, const PackOption &opt, std::unique_ptr<PackWriteCloser> *out) {
  out->reset();
  const std::string fv = opt.FsVersion.empty() ? "6" : opt.FsVersion;  // convert_unix.go:326-328
  // convert_unix.go:332-356: required features, detected once per process
  std::vector<std::string> required{kFeatureTar2Rafs}, detected;
  if (!opt.BatchSize.empty() && opt.BatchSize != "0") required.push_back(kFeatureBatchSize);
  if (opt.Encrypt) required.push_back(kFeatureEncrypt);
  if (Error e = detect_features(required, &detected)) return e;
  if (opt.OCIRef) {
    if (fv != "6") return err(NGPU_EINVAL, "oci ref can only be supported by fs version 6");
    // packRef (builder.go:180-218): `nydus-image create --type targz-ref` with
    // nydus-image's defaults (v6, 1 MiB chunks, blake3, no chunk dict).  The
    // writer takes the ORIGINAL gzip layer (convert_unix.go:857-859):
    // inflated and indexed on the host, digested and deduped on the GPU; the
    // stream holds blob.meta (chunk infos + gzip checkpoints), image.boot, TOC.
    PackOption ref;
    ref.Device = opt.Device;
    Target t;
    if (Error x = target_for(ref, &t)) return x;
    ngpu_pack *p = nullptr;
    const int rc = t.node ? ngpu_node_pack_open(t.node, nullptr, NGPU_PACK_OCIREF, &p)
                          : ngpu_pack_open_dict(t.eng, nullptr, NGPU_PACK_OCIREF, &p);
    if (rc) return err(rc, std::string("pack open: ") + ngpu_last_error(t.first()));
    out->reset(new GpuPackWriteCloser(ngpu_pack_engine(p), p, part_of(t, p), dest,
                                      NGPU_COMPRESSOR_NONE, opt.Timeout, "", true));
    return {};
  }
  const bool batch = std::find(detected.begin(), detected.end(), kFeatureBatchSize) != detected.end();
  if (batch && fv != "6") return err(NGPU_EINVAL, "'--batch-size' can only be supported by fs version 6");
  // v2.3.0 would write batch chunks (several small chunks compressed as one,
  // a different blob.meta) or an encrypted blob; this builder writes neither,
  // so it refuses instead of returning a blob the reference would not produce
  if (batch)
    return err(NGPU_EUNSUPP, "batch chunks (--batch-size " + opt.BatchSize +
                                 ") not implemented by the GPU builder");
  if (opt.Encrypt) return err(NGPU_EUNSUPP, "blob encryption (--encrypt) not implemented by the GPU builder");
  uint32_t comp = 0;
  if (Error e = compressor_of(opt.Compressor, &comp)) return e;
  Target t;
  if (Error x = target_for(opt, &t)) return x;
  // the Pack's own dict handle (loaded once per unchanged ChunkDictPath and
  // shared by every Pack naming it; builder.go:122-124 passes it per process).
  // On a node: one replica on every GPU (a probe needs no exchange; the
  // partitioned dict's exchange has not met two distinct GPUs yet).
  ngpu_dict *d = nullptr;
  int rc = 0;
  if (!opt.ChunkDictPath.empty() &&
      (rc = t.node ? ngpu_node_dict_open(t.node, opt.ChunkDictPath.c_str(), NGPU_NODE_DICT_REPLICATE, &d)
                   : ngpu_dict_open(t.eng, opt.ChunkDictPath.c_str(), &d)))
    return err(rc, "load chunk dict " + opt.ChunkDictPath + ": " + ngpu_last_error(t.first()));
  ngpu_pack *p = nullptr;
  rc = t.node ? ngpu_node_pack_open(t.node, d, NGPU_PACK_RETAIN, &p)
              : ngpu_pack_open_dict(t.eng, d, NGPU_PACK_RETAIN, &p);
  ngpu_dict_release(d);  // the pack holds its own reference
  if (rc) return err(rc, std::string("pack open: ") + ngpu_last_error(t.first()));
  out->reset(new GpuPackWriteCloser(ngpu_pack_engine(p), p, part_of(t, p), dest, comp, opt.Timeout,
                                    opt.PrefetchPatterns));
  return {};
}

Error Unpack(ReaderAt &ra, Writer &dest, const UnpackOption &opt) {
  (void)opt;  // Stream / WorkDir / BuilderPath / Timeout: the in-process unpack reads ra directly
  if (int rc = ngpu_unpack(read_trampoline, &ra, ra.Size(), write_trampoline, &dest))
    return err(rc, std::string("unpack nydus tar: ") + ngpu_host_error());
  return {};
}

Error UnpackEntry(ReaderAt &ra, const std::string &targetName, Writer &target, TOCEntry *entry) {
  TOCEntry t;
  const int rc = ngpu_unpack_entry(read_trampoline, &ra, ra.Size(), targetName.c_str(),
                                   write_trampoline, &target, reinterpret_cast<uint8_t *>(&t));
  if (rc) return err(rc, ngpu_host_error());
  if (entry) *entry = t;
  return {};
}

Error Merge(const std::vector<Layer> &layers, Writer &dest, const MergeOption &opt,
            std::vector<std::string> *blobDigests) {
  blobDigests->clear();
  std::vector<BufferWriter> boots(layers.size());
  std::vector<std::string> hexes(layers.size()), ref_digest(layers.size()), ref_toc(layers.size());
  std::vector<uint64_t> ref_size(layers.size(), 0);
  bool any_ref = false;
  for (size_t i = 0; i < layers.size(); ++i) {
    if (!layers[i].ReaderAt) return err(NGPU_EINVAL, "layer without reader");
    if (Error e = UnpackEntry(*layers[i].ReaderAt, EntryBootstrap, boots[i], nullptr))
      return err(e.code, "unpack all bootstraps: unpack nydus tar: " + e.msg);
    // an OCIRef layer's blob is its original gzip blob, named by its
    // OriginalDigest (getBootstrapPath, convert_unix.go:567-573)
    const std::string &d = layers[i].OriginalDigest.empty() ? layers[i].Digest : layers[i].OriginalDigest;
    hexes[i] = d.compare(0, 7, "sha256:") == 0 ? d.substr(7) : d;
    if (!layers[i].OriginalDigest.empty()) {
      // --blob-digests / --blob-sizes / --blob-toc-digests (convert_unix.go:
      // 579-587): the nydus stream's digest and size, and calcBlobTOCDigest
      // (:541-554): sha256 of the TOC entry's data
      BufferWriter toc;
      if (Error e = UnpackEntry(*layers[i].ReaderAt, EntryTOC, toc, nullptr))
        return err(e.code, "calc blob toc digest for layer " + layers[i].Digest + ": " + e.msg);
      uint8_t md[32];
      SHA256(toc.data.data(), toc.data.size(), md);
      static const char *hx = "0123456789abcdef";
      std::string th(64, '0');
      for (int k = 0; k < 32; ++k) th[2 * k] = hx[md[k] >> 4], th[2 * k + 1] = hx[md[k] & 15];
      const std::string &ld = layers[i].Digest;
      ref_digest[i] = ld.compare(0, 7, "sha256:") == 0 ? ld.substr(7) : ld;
      ref_toc[i] = th;
      ref_size[i] = layers[i].ReaderAt->Size();
      any_ref = true;
    }
  }
  std::vector<uint8_t> dict;
  if (!opt.ChunkDictPath.empty()) {
    FILE *f = fopen(opt.ChunkDictPath.c_str(), "rb");
    if (!f) return err(NGPU_EIO, "open chunk dict " + opt.ChunkDictPath);
    uint8_t buf[1 << 16];
    size_t r;
    while ((r = fread(buf, 1, sizeof buf, f)) > 0) dict.insert(dict.end(), buf, buf + r);
    fclose(f);
  }
  std::vector<const void *> ptrs;
  std::vector<uint64_t> sizes;
  std::vector<const char *> names;
  for (size_t i = 0; i < layers.size(); ++i) {
    ptrs.push_back(boots[i].data.data());
    sizes.push_back(boots[i].data.size());
    names.push_back(hexes[i].c_str());
  }
  std::vector<uint8_t> parent;  // --parent-bootstrap (builder.go:235-237)
  if (!opt.ParentBootstrapPath.empty()) {
    FILE *f = fopen(opt.ParentBootstrapPath.c_str(), "rb");
    if (!f) return err(NGPU_EIO, "open parent bootstrap " + opt.ParentBootstrapPath);
    uint8_t buf[1 << 16];
    size_t r;
    while ((r = fread(buf, 1, sizeof buf, f)) > 0) parent.insert(parent.end(), buf, buf + r);
    fclose(f);
  }
  ngpu_merge_options mo;
  memset(&mo, 0, sizeof mo);
  mo.parent_bootstrap = parent.empty() ? nullptr : parent.data();
  mo.parent_size = parent.size();
  mo.prefetch_patterns = opt.PrefetchPatterns.c_str();  // the builder's stdin (builder.go:238-240)
  std::vector<const char *> rd(layers.size(), nullptr), rt(layers.size(), nullptr);
  for (size_t i = 0; any_ref && i < layers.size(); ++i)
    if (!ref_toc[i].empty()) rd[i] = ref_digest[i].c_str(), rt[i] = ref_toc[i].c_str();
  BufferWriter merged;
  char *ids = nullptr;
  const int rc = ngpu_merge_ex2(ptrs.data(), sizes.data(), names.data(), layers.size(),
                                dict.empty() ? nullptr : dict.data(), dict.size(), &mo,
                                any_ref ? rd.data() : nullptr, any_ref ? ref_size.data() : nullptr,
                                any_ref ? rt.data() : nullptr, write_trampoline, &merged, &ids);
  if (rc) return err(rc, std::string("merge bootstrap: ") + ngpu_host_error());
  for (const char *s = ids; s && *s;) {
    const char *c = strchr(s, ',');
    const std::string id = c ? std::string(s, c - s) : std::string(s);
    blobDigests->push_back("sha256:" + id);
    s = c ? c + 1 : nullptr;
  }
  ngpu_free_host(ids);
  if (!opt.WithTar) return dest.Write(merged.data.data(), merged.data.size());
  uint8_t h[512];
  tar_header(h, "image", 0, '5', 0755);
  if (Error e = dest.Write(h, 512)) return e;
  tar_header(h, "image/image.boot", merged.data.size(), '0', 0444);
  if (Error e = dest.Write(h, 512)) return e;
  if (Error e = dest.Write(merged.data.data(), merged.data.size())) return e;
  static const uint8_t zeros[1024] = {};
  const size_t pad = (512 - merged.data.size() % 512) % 512;
  if (Error e = dest.Write(zeros, pad)) return e;
  return dest.Write(zeros, 1024);  // end-of-archive (tar.Writer.Close)
}

}  // namespace converter
}  // namespace nydus
