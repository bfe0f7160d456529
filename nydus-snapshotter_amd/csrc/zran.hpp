// zran.hpp — gzip random-access index for PackOption.OCIRef (`nydus-image
// create --type targz-ref`, pkg/converter/tool/builder.go:180-218,
// convert_unix.go:346-351, 500-509).  Not installed.
//
// An OCIRef Pack keeps the layer's chunks in the ORIGINAL gzip blob: the
// conversion inflates the blob (the tar stream then takes the same path as a
// tar-rafs Pack: tar walk, GPU digests, dedup) and records checkpoints of the
// deflate stream, so that a reader can start inflating at any checkpoint
// instead of at the beginning.  A checkpoint sits on a deflate block boundary
// every `span` bytes of output and holds the compressed byte offset, the bit
// offset inside that byte, the output offset and the last 32 KiB of output
// (the inflate dictionary).  This is zlib's zran technique (examples/zran.c);
// nydus' ZranContext stores the same fields ([nydus v2.3.0] utils/src/
// compress/zlib_random.rs, external, VERIFY).  Host code, zlib.
#pragma once

#include <stdint.h>

#include <functional>
#include <memory>
#include <vector>

#include "blob.hpp"

namespace ngpu {

struct ZranPoint {
  uint64_t in_offset;   // compressed bytes consumed at the block boundary
  uint64_t out_offset;  // decompressed bytes produced there
  uint32_t bits;        // bits of byte in_offset - 1 still unread (0..7)
  uint32_t byte;        // that byte (when bits != 0): a reader primes inflate with it
  uint32_t dict_size;   // bytes of dictionary (<= 32 KiB; less near the start)
  uint64_t dict_offset; // into GzipIndexer::dicts()
};

class GzipIndexer {
 public:
  static constexpr uint64_t kWindow = 32768;
  // span: output bytes between checkpoints (>= kWindow).
  explicit GzipIndexer(uint64_t span);
  ~GzipIndexer();
  int init();  // NGPU_EUNSUPP without zlib
  // Inflate n more bytes of the gzip blob; each piece of the tar stream goes
  // to out(p, len) (non-zero return aborts with that code).  Also hashes the
  // compressed bytes (the blob id: the layer's gzip digest).
  int feed(const uint8_t *in, uint64_t n, const std::function<int(const uint8_t *, uint64_t)> &out);
  // The gzip stream ended exactly at the end of the input (one member).
  int finish();
  const std::vector<ZranPoint> &points() const;
  const std::vector<uint8_t> &dicts() const;
  uint64_t in_bytes() const;
  uint64_t out_bytes() const;
  void blob_digest(uint8_t out[32]);  // sha256 of the gzip bytes (after finish)
  // Index of the last checkpoint at or before output offset `off`.
  uint64_t point_of(uint64_t off) const;
  // Compressed end of the deflate data that produces output [0, end_out): the
  // input offset of the first checkpoint past it, or the whole input.
  uint64_t in_end_of(uint64_t end_out) const;

 private:
  struct Impl;
  std::unique_ptr<Impl> im_;
};

// Random access: `len` bytes of the decompressed stream starting `skip` bytes
// after checkpoint `pt`, from the gzip bytes `gz` (the whole blob).
int zran_extract(const uint8_t *gz, uint64_t gz_len, const ZranPoint &pt, const uint8_t *dict,
                 uint64_t skip, uint8_t *out, uint64_t len);

}  // namespace ngpu
