// converter.hpp — C++ mirror of the reference's pkg/converter API for the
// accelerated path, written only against the C ABI (include/nydus_gpu.h).
//
// Same names, argument meaning and error behaviour as the Go package
// (pkg/converter/types.go, convert_unix.go), so that host code written against
// the reference reads the same:
//   Pack(dest, opt)            convert_unix.go:325   -> WriteCloser; Close() must be checked
//   Merge(layers, dest, opt)   convert_unix.go:560   -> referenced blob digests
//   UnpackEntry(ra, name, w)   convert_unix.go:284   -> TOCEntry (ErrNotFound)
//   Unpack(ra, dest, opt)      convert_unix.go:669   -> the layer's OCI tar
// Go's `error` is `Error` (code 0 == nil); nothing throws.  Digest/dedup run on
// the GPU (libnydusgpu.so); compression, SHA-256 and Merge bookkeeping on the
// host inside the same library.
#pragma once

#include <stdint.h>

#include <memory>
#include <string>
#include <vector>

namespace nydus {
namespace converter {

struct Error {
  int code = 0;  // negative NGPU_E* code; 0 = nil
  std::string msg;
  explicit operator bool() const { return code != 0; }
};

// io.Writer / io.WriteCloser / content.ReaderAt
class Writer {
 public:
  virtual ~Writer() = default;
  virtual Error Write(const void *p, size_t n) = 0;
};
class WriteCloser : public Writer {
 public:
  virtual Error Close() = 0;
};
class Reader {  // io.Reader: bytes read (> 0), 0 at io.EOF, < 0 on error
 public:
  virtual ~Reader() = default;
  virtual int64_t Read(void *p, size_t n) = 0;
};
class ReaderAt {
 public:
  virtual ~ReaderAt() = default;
  // bytes read (> 0) or < 0 on error
  virtual int64_t ReadAt(void *p, size_t n, uint64_t off) = 0;
  virtual uint64_t Size() const = 0;
};

class BufferWriter : public Writer {  // bytes.Buffer
 public:
  Error Write(const void *p, size_t n) override;
  std::vector<uint8_t> data;
};
class BytesReaderAt : public ReaderAt {  // over caller-owned bytes
 public:
  BytesReaderAt(const uint8_t *p, uint64_t n) : p_(p), n_(n) {}
  int64_t ReadAt(void *p, size_t n, uint64_t off) override;
  uint64_t Size() const override { return n_; }

 private:
  const uint8_t *p_;
  uint64_t n_;
};

using Compressor = uint32_t;  // types.go:22-31
constexpr Compressor CompressorNone = 0x0000'0001;
constexpr Compressor CompressorZstd = 0x0000'0002;
constexpr Compressor CompressorLz4Block = 0x0000'0004;
constexpr Compressor CompressorMask = 0x0000'000f;

extern const char *const EntryBlob;        // "image.blob"      convert_unix.go:45
extern const char *const EntryBootstrap;   // "image.boot"      :46
extern const char *const EntryBlobMeta;    // "blob.meta"       :47
extern const char *const EntryTOC;         // "rafs.blob.toc"   :49

struct TOCEntry {  // types.go:147-202 (128 B on disk)
  uint32_t Flags = 0;
  uint32_t Reserved1 = 0;
  uint8_t Name[16] = {};
  uint8_t UncompressedDigest[32] = {};
  uint64_t CompressedOffset = 0;
  uint64_t CompressedSize = 0;
  uint64_t UncompressedSize = 0;
  uint8_t Reserved2[48] = {};
  std::string GetName() const;
  Error GetCompressor(Compressor *out) const;
  std::string GetUncompressedDigest() const;
};
static_assert(sizeof(TOCEntry) == 128, "TOCEntry is 128 bytes on disk");

struct PackOption {  // types.go:58-90
  std::string WorkDir, BuilderPath;
  std::string FsVersion;       // "5" | "6" (default "6")
  std::string ChunkDictPath;   // bootstrap of the chunk dict image
  std::string PrefetchPatterns;
  std::string Compressor;      // "" (zstd) | "none" | "zstd" | "lz4_block"
  bool OCIRef = false, AlignedChunk = false;
  std::string ChunkSize;       // power of two in [0x1000, 0x1000000] (types.go:76)
  std::string BatchSize;
  double Timeout = 0;           // seconds; 0 = none (the builder's ctx.WithTimeout)
  bool Encrypt = false;
  std::string Digester;        // API extension: "blake3" (default) | "sha256"
  // -1 (default): the process's node -- every GPU (or NYDUS_GPU_DEVICES,
  // e.g. "0,1,2,3"), each Pack on the least-loaded one (layers shard over the
  // node, as the reference's per-layer goroutines shard its builder processes);
  // >= 0: every Pack of this option set on that one GPU
  int Device = -1;
};

struct MergeOption {  // types.go:92-133
  std::string WorkDir, BuilderPath, FsVersion, ChunkDictPath, ParentBootstrapPath,
      PrefetchPatterns;
  bool WithTar = false, OCI = false, OCIRef = false;
  double Timeout = 0;
};

struct UnpackOption {  // types.go:135-145
  std::string WorkDir, BuilderPath;
  double Timeout = 0;
  bool Stream = false;
};

struct Layer {  // types.go:37-44
  std::string Digest;  // "sha256:<hex>" of the whole nydus tar blob
  std::shared_ptr<converter::ReaderAt> ReaderAt;
  std::string OriginalDigest;  // OCIRef: "sha256:<hex>" of the original gzip layer (or empty)
};

// Pack result details beyond the Go API (the digest LayerConvertFunc computes
// over dest, convert_unix.go:870-914, and the dedup counts).
struct PackStats {
  std::string Digest;  // "sha256:<hex>" of everything written to dest
  uint64_t Chunks = 0, NewChunks = 0, IntraChunks = 0, DictChunks = 0;
  uint64_t StreamBytes = 0, BlobBytes = 0;
  int Part = -1;  // node index of the GPU engine the Pack ran on (-1: a pinned Device)
};
class PackWriteCloser : public WriteCloser {
 public:
  virtual const PackStats &Stats() const = 0;  // valid after a nil Close()
  // io.ReaderFrom (what io.Copy(tw, tr) picks, convert_unix.go:881): src
  // reads straight into the engine's pinned staging.  A source error ends the
  // Pack (no Close will come for it) and is returned.
  virtual Error ReadFrom(Reader &src, uint64_t *n) = 0;
  // ctx.Done(): the running Write / ReadFrom / Close fails ("signal: killed",
  // code NGPU_ECANCELED) at its next staging slot, and the Pack is released
  // -- also when no Write or Close ever comes again (the reference's error
  // paths skip tw.Close(), convert_unix.go:885-907).  Safe from any thread.
  // Destroying the writer without Close releases the Pack too.
  virtual void Cancel() = 0;
};

Error Pack(Writer &dest, const PackOption &opt, std::unique_ptr<PackWriteCloser> *out);
Error Merge(const std::vector<Layer> &layers, Writer &dest, const MergeOption &opt,
            std::vector<std::string> *blobDigests);
Error UnpackEntry(ReaderAt &ra, const std::string &targetName, Writer &target, TOCEntry *entry);
// Unpack (convert_unix.go:669-719): a nydus layer stream back to the OCI tar.
Error Unpack(ReaderAt &ra, Writer &dest, const UnpackOption &opt);

// ErrNotFound (types.go:33-35) is code NGPU_ENOTFOUND.
bool IsNotFound(const Error &e);

// Leak check of the Pack paths (not in the Go API): what each GPU engine of
// the option set's node (or its pinned engine) holds now.
struct EngineCounters {
  uint64_t OpenPacks, StagingPoolBufs, StagingPoolBytes, PackPool, LandPool;
  bool operator==(const EngineCounters &o) const {
    return OpenPacks == o.OpenPacks && StagingPoolBufs == o.StagingPoolBufs &&
           StagingPoolBytes == o.StagingPoolBytes && PackPool == o.PackPool && LandPool == o.LandPool;
  }
};
Error GpuCounters(const PackOption &opt, std::vector<EngineCounters> *out);

}  // namespace converter
}  // namespace nydus
