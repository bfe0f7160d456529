// host.cpp — host side of libnydusgpu.so around the GPU stage:
//   * tar-rafs chunk enumeration,
//   * RAFS v6 chunk-table reader for PackOption.ChunkDictPath and writer for
//     the layer's chunk records (§8(a) a7, §8(f) next-2),
//   * ngpu_pack_tar: tar in host memory -> chunks -> GPU digest/dedup.
//
// Tar rules follow what `nydus-image create --type tar-rafs` consumes
// (pkg/converter/tool/builder.go:97-110, fed by packFromTar,
// pkg/converter/convert_unix.go:443-539): POSIX ustar headers, GNU base-256
// sizes, GNU long name/link ('L'/'K'), PAX extended headers ('x' may override
// the next entry's size; 'g' skipped); regular files ('0', '\0', '7') of
// non-zero size are cut into fixed-size chunks that never span files;
// hardlinks, symlinks, directories, devices and fifos carry no chunks;
// whiteouts are plain entries (`--whiteout-spec none`, builder.go:91-92);
// GNU sparse ('S') is unsupported.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "blob.hpp"
#include "nydus_gpu.h"
#include "tarstream.hpp"

using ngpu::RafsV6ChunkInfo;
using ngpu::kRafsV6ExtSuperBlockOffset;
using ngpu::kRafsV6Magic;
using ngpu::kRafsV6SuperBlockOffset;

extern "C" {

uint32_t ngpu_engine_chunk_size(const ngpu_engine *);  // engine.hip (internal)

int ngpu_tar_chunks(const void *tar_v, uint64_t len, uint32_t chunk_size, ngpu_chunk *out,
                    uint64_t cap, uint64_t *n_chunks, uint64_t *n_files) {
  return ngpu::guarded([&]() -> int {
    if ((!tar_v && len) || chunk_size == 0) return NGPU_EINVAL;
    struct Rec : ngpu::TarSink {
      ngpu_chunk *out;
      uint64_t cap, n = 0;
      int chunk(uint64_t off, uint32_t l, uint32_t fi, uint64_t fo) override {
        if (n < cap && out) out[n] = ngpu_chunk{off, l, fi, fo};
        ++n;
        return 0;
      }
      int data(const uint8_t *, uint64_t) override { return 0; }
    } rec;
    rec.out = out;
    rec.cap = cap;
    ngpu::TarScanner sc(chunk_size);
    int rc = sc.feed((const uint8_t *)tar_v, len, rec);
    if (!rc) rc = sc.finish();
    if (rc) return rc;
    if (n_chunks) *n_chunks = rec.n;
    if (n_files) *n_files = sc.files();
    return NGPU_OK;
  });
}

void ngpu_free_host(void *p) { free(p); }

int ngpu_chunk_table(const ngpu_chunk *chunks, const ngpu_result *results, uint64_t n,
                     uint8_t *out, uint64_t cap, uint64_t *n_records) {
  return ngpu::guarded([&]() -> int {
    if ((n && (!chunks || !results)) || !n_records) return NGPU_EINVAL;
    // NEW chunks in index order; compressor "none": csize = usize, compressed
    // offsets packed back to back (the fixture's coff rule with csize = usize).
    std::vector<uint64_t> order;
    for (uint64_t i = 0; i < n; ++i)
      if (results[i].kind == NGPU_NEW) order.push_back(i);
    // NEW indices are assigned in stream order, so order is already sorted by
    // index; verify rather than assume.
    for (uint64_t k = 0; k < order.size(); ++k)
      if (results[order[k]].index != k) return NGPU_EINVAL;
    uint64_t coff = 0;
    for (uint64_t k = 0; k < order.size() && k < cap && out; ++k) {
      const uint64_t i = order[k];
      RafsV6ChunkInfo r;
      memset(&r, 0, sizeof r);
      memcpy(r.block_id, results[i].digest, 32);
      r.blob_index = results[i].blob_index;
      r.flags = 0;  // not compressed
      r.compressed_size = chunks[i].length;
      r.uncompressed_size = chunks[i].length;
      r.compressed_offset = coff;
      r.uncompressed_offset = results[i].uncompressed_offset;
      r.file_offset = chunks[i].file_offset;
      r.index = results[i].index;
      memcpy(out + 80 * k, &r, 80);
      coff += chunks[i].length;
    }
    *n_records = order.size();
    return NGPU_OK;
  });
}

}  // extern "C"
