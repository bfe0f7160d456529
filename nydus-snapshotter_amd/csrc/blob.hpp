// blob.hpp — host side of converter.Pack's output stream (SURVEY.md §8(f)
// next-3, §8(a) a9): per-chunk compression of the layer's NEW chunks, the
// nydus tar-like stream `data | tar_header | ... | toc | tar_header`
// (pkg/converter/convert_unix.go:296-300, 314-321) and the image.boot
// bootstrap.  Shared by blob.cpp (C ABI) and pack.hip (streaming Pack finish).
// Not installed.
#pragma once

#include <stddef.h>

#include <stdint.h>

#include <memory>
#include <new>
#include <string>
#include <vector>

#include <openssl/evp.h>

#include "nydus_gpu.h"
#include "tarstream.hpp"

namespace ngpu {

// RAFS v6 on-disk records (decoded from the reference fixture
// pkg/filesystem/testdata/v6-bootstrap-chunk-pos-438272.tar.gz).
#pragma pack(push, 1)
struct RafsV6ChunkInfo {  // 80 B
  uint8_t block_id[32];
  uint32_t blob_index;
  uint32_t flags;  // bit 0: chunk data compressed
  uint32_t compressed_size;
  uint32_t uncompressed_size;
  uint64_t compressed_offset;
  uint64_t uncompressed_offset;
  uint64_t file_offset;
  uint32_t index;
  uint32_t reserved;
};
struct RafsV6BlobInfo {  // 256 B
  char blob_id[64];      // 64 ASCII hex chars
  uint32_t blob_index;
  uint32_t chunk_size;
  uint32_t chunk_count;
  uint32_t compression_algo;  // nydus compress::Algorithm (fixture: lz4_block = 1)
  uint32_t digest_algo;       // 0 blake3, 1 sha256
  uint32_t features;          // fixture: 1 (4K-aligned uncompressed chunks)
  uint64_t compressed_size;   // end of the chunk data
  uint64_t uncompressed_size; // 4K-aligned end of the uncompressed chunks
  uint8_t meta[152];          // blob.meta location fields (zero: not emitted)
};
struct TocEntry {  // 128 B, pkg/converter/types.go:147-163
  uint32_t flags;  // compressor of the entry data (types.go:22-31)
  uint32_t reserved1;
  char name[16];
  uint8_t uncompressed_digest[32];  // sha256 of the uncompressed entry data
  uint64_t compressed_offset;
  uint64_t compressed_size;
  uint64_t uncompressed_size;
  uint8_t reserved2[48];  // Go reads the first 124 B of each 128-B entry (types.go:147-163, convert_unix.go:220)
};
// RafsV6BlobInfo::meta, field by field ([nydus v2.3.0] RafsV6Blob,
// rafs/src/metadata/layout/v6.rs, restated).  Bytes 104..135 are pinned by the
// reference v6 fixture's blob record (blob_toc_size 0, ci_compressor 1,
// ci_offset = the blob's compressed size, 35,949 / 40,240 ci bytes); the
// toc / meta digests and blob_meta_size that follow (a merged targz-ref
// bootstrap's --blob-toc-digests / --blob-digests / --blob-sizes) are
// restated only: parity unpinned.
struct RafsV6BlobMeta {
  uint32_t blob_toc_size;
  uint32_t ci_compressor;
  uint64_t ci_offset;
  uint64_t ci_compressed_size;
  uint64_t ci_uncompressed_size;
  uint8_t blob_toc_digest[32];
  uint8_t blob_meta_digest[32];
  uint64_t blob_meta_size;
  uint8_t reserved[48];
};
#pragma pack(pop)
static_assert(sizeof(RafsV6BlobMeta) == sizeof(((RafsV6BlobInfo *)0)->meta), "RafsV6Blob tail is 152 B");
static_assert(offsetof(RafsV6BlobInfo, meta) == 104, "RafsV6Blob: ci fields start at 104");
static_assert(offsetof(RafsV6BlobInfo, meta) + offsetof(RafsV6BlobMeta, ci_offset) == 112, "ci_offset @112");
static_assert(offsetof(RafsV6BlobInfo, meta) + offsetof(RafsV6BlobMeta, blob_toc_digest) == 136,
              "blob_toc_digest @136");
static_assert(offsetof(RafsV6BlobInfo, meta) + offsetof(RafsV6BlobMeta, blob_meta_digest) == 168,
              "blob_meta_digest @168");
static_assert(offsetof(RafsV6BlobInfo, meta) + offsetof(RafsV6BlobMeta, blob_meta_size) == 200,
              "blob_meta_size @200");
static_assert(sizeof(RafsV6ChunkInfo) == 80, "RAFS v6 chunk info is 80 bytes");
static_assert(sizeof(RafsV6BlobInfo) == 256, "RAFS v6 blob info is 256 bytes");
static_assert(sizeof(TocEntry) == 128, "TOC entry is 128 bytes");

// Compressed placement of a chunk-dict entry: what a DICT chunk record of a
// layer bootstrap copies from the dict's record (nydus chunk.copy_from).
struct DictPlace {
  uint64_t compressed_offset;
  uint32_t compressed_size;
  uint32_t flags;
};

constexpr uint32_t kRafsV6Magic = 0xE0F5E1E2u;        // pkg/layout/layout.go:24
constexpr uint64_t kRafsV6SuperBlockOffset = 1024;     // layout.go:26
constexpr uint64_t kRafsV6ExtSuperBlockOffset = 1152;  // 1024 + 128
constexpr uint64_t kBlobTableOffset = 4096;            // as in the reference fixture

// C ABI entry points run their body through guarded(): no C++ exception
// (bad_alloc from a hostile size, length_error, ...) crosses the boundary.
template <class F>
int guarded(F &&f) noexcept {
  try {
    return f();
  } catch (const std::bad_alloc &) {
    return NGPU_ENOMEM;
  } catch (...) {
    return NGPU_EINVAL;
  }
}

// Incremental SHA-256 (OpenSSL EVP).
struct Sha {
  EVP_MD_CTX *c = EVP_MD_CTX_new();
  Sha() { EVP_DigestInit_ex(c, EVP_sha256(), nullptr); }
  ~Sha() { EVP_MD_CTX_free(c); }
  Sha(const Sha &) = delete;
  Sha &operator=(const Sha &) = delete;
  void update(const void *p, uint64_t n) { EVP_DigestUpdate(c, p, n); }
  void final(uint8_t out[32]) {
    unsigned int l = 32;
    EVP_DigestFinal_ex(c, out, &l);
  }
  void copy_from(const Sha &o) { EVP_MD_CTX_copy_ex(c, o.c); }
};

// Host helpers (blob.cpp): the thread's last host error (ngpu_host_error),
// OpenSSL SHA-256, lower-case hex, the dlopen'ed compressors.
int host_fail(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
const char *host_error();
void sha256(const void *p, uint64_t n, uint8_t out[32]);
std::string hex(const uint8_t *d, int n);
struct ZInBuf;
struct ZOutBuf;
struct Codecs;
const Codecs &codecs();
// Decompress one chunk stored with blob compression_algo `algo` (nydus
// compress::Algorithm: 1 lz4_block, 3 zstd) into exactly `usize` bytes.
int decompress_chunk(uint32_t algo, const uint8_t *src, uint64_t csize, uint8_t *dst,
                     uint64_t usize);

// Parsed (minimal) RAFS v6 bootstrap: blob table + chunk table.
struct Bootstrap {
  uint64_t flags = 0;
  uint32_t chunk_size = 0;
  std::vector<RafsV6BlobInfo> blobs;
  std::vector<RafsV6ChunkInfo> chunks;
};
constexpr uint32_t kRafsV5Magic = 0x52414653u;  // "RAFS"
constexpr uint32_t kRafsV5Version = 0x500;
// A RAFS v5 bootstrap as a chunk dict: every regular file's 80-B chunk infos
// in inode-table order (recs) and its blobs as 256-B v6 blob records (blobs);
// *digester / *chunk_size from its flags / block size.  Untrusted input:
// every offset is bounds-checked (NGPU_EFORMAT + ngpu_host_error()).
int parse_v5_bootstrap(const uint8_t *p, uint64_t n, uint32_t *digester, uint32_t *chunk_size,
                       std::vector<uint8_t> *recs, std::vector<uint8_t> *blobs);
// with_chunks = false: the blob table only (the chunk table is still bounds-checked)
int parse_bootstrap(const uint8_t *p, uint64_t n, Bootstrap *out, bool with_chunks = true);
std::vector<uint8_t> write_bootstrap(const Bootstrap &b);
std::string blob_id_of(const RafsV6BlobInfo &b);

// An OCIRef layer's own blob is the ORIGINAL gzip blob (targz-ref): its
// chunks are addressed through gzip checkpoints (zran.hpp) instead of image.blob
// data.  Per NEW chunk (index order): the checkpoint it starts after, its
// offset in that checkpoint's output, and the compressed range that produces
// it; the checkpoint table and dictionaries go into blob.meta.
struct ZranRef {
  uint8_t digest[32];        // sha256 of the gzip blob: the own blob's id
  uint64_t gz_size = 0, tar_size = 0;
  std::vector<uint64_t> coff, csize;   // per NEW chunk: compressed range in the gzip blob
  std::vector<uint32_t> ctx, ctx_off;  // per NEW chunk: checkpoint index, offset in its output
  // checkpoint table (40-B records) and dictionary area, as written to blob.meta
  std::vector<uint8_t> table, dicts;
  uint64_t n_points = 0;
};

// Sequential writer of the nydus formatted stream for one layer.
class BlobWriter {
 public:
  // dict_blobs: the chunk dict's blob table (its inner-index order);
  // dict_place: compressed placement per dict entry (DICT results' `ref`),
  // n_place entries (0: unknown, csize = usize and offset 0).
  BlobWriter(const ngpu_blob_options &opt, ngpu_write_fn w, void *ctx,
             std::vector<RafsV6BlobInfo> dict_blobs, const DictPlace *dict_place = nullptr,
             uint64_t n_place = 0);
  ~BlobWriter();
  int init();  // loads the compressor; NGPU_EUNSUPP if unavailable
  // NEW chunks in index order (src[k] = host bytes of chunk with index
  // base+k).  The bytes may be reused as soon as the call returns.
  // src_stable: the k chunks' bytes stay valid and unchanged until finish()
  // returns (then raw pieces are written from there, not copied)
  int add(const uint8_t *const *src, const uint32_t *len, uint64_t k, bool src_stable = false);
  // Writes image.blob's header, blob.meta (v6), image.boot -- the inode tree
  // of `entries`, the layer tar's entries (tarstream.hpp) -- and the TOC (v6).
  int finish(const ngpu_chunk *chunks, const ngpu_result *res, uint64_t n,
             const ngpu_layer_stats &st, const std::vector<TarEntry> &entries,
             ngpu_blob_info *info);
  const std::string &error() const { return err_; }
  // Cancellation: checked before each compression batch (NGPU_ECANCELED).
  void set_cancel(const volatile int32_t *flag);
  // OCIRef (targz-ref): finish() writes no image.blob; the own blob is the
  // gzip blob of `z` (set before finish; add() is not called).
  void set_zran(const ZranRef *z);

 private:
  struct Impl;
  std::unique_ptr<Impl> im_;
  std::string err_;
};

}  // namespace ngpu
