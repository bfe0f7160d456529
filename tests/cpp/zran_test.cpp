// zran_test.cpp — the gzip checkpoint index (csrc/zran.cpp) on the CPU, under
// ASan + UBSan: inflate a gzip file through GzipIndexer in random-sized
// pieces, check the inflated bytes against zlib's one-shot output, then read
// random ranges back through zran_extract from the checkpoint each starts
// after, and check every checkpoint (increasing offsets, <= 32 KiB
// dictionaries, bit offsets 0..7, at most `span` + one block apart).
// usage: zran_test GZIP_FILE SPAN SEED  -> prints "points=<n> reads=<n> ok"
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

#include <random>
#include <vector>

#include "zran.hpp"

using namespace ngpu;

static std::vector<uint8_t> read_file(const char *p) {
  std::vector<uint8_t> v;
  FILE *f = fopen(p, "rb");
  if (!f) return v;
  uint8_t b[1 << 16];
  size_t r;
  while ((r = fread(b, 1, sizeof b, f)) > 0) v.insert(v.end(), b, b + r);
  fclose(f);
  return v;
}

int main(int argc, char **argv) {
  if (argc < 4) return 2;
  const std::vector<uint8_t> gz = read_file(argv[1]);
  const uint64_t span = strtoull(argv[2], nullptr, 0);
  std::mt19937_64 rng(strtoull(argv[3], nullptr, 0));
  GzipIndexer ix(span);
  if (ix.init()) return 3;
  std::vector<uint8_t> out;
  for (size_t a = 0; a < gz.size();) {
    const size_t n = std::min<size_t>(gz.size() - a, 1 + rng() % 200000);
    const int rc = ix.feed(gz.data() + a, n, [&](const uint8_t *p, uint64_t k) {
      out.insert(out.end(), p, p + k);
      return 0;
    });
    if (rc) {
      printf("feed failed: %s\n", host_error());
      return 4;
    }
    a += n;
  }
  if (ix.finish()) {
    printf("finish failed: %s\n", host_error());
    return 5;
  }
  // zlib one-shot
  std::vector<uint8_t> ref(out.size() + 1);
  z_stream zs{};
  inflateInit2(&zs, 15 + 16);
  zs.next_in = const_cast<Bytef *>(gz.data());
  zs.avail_in = (uInt)gz.size();
  zs.next_out = ref.data();
  zs.avail_out = (uInt)ref.size();
  const int zr = inflate(&zs, Z_FINISH);
  inflateEnd(&zs);
  if (zr != Z_STREAM_END || zs.total_out != out.size() || memcmp(ref.data(), out.data(), out.size())) {
    printf("inflated stream differs from zlib's\n");
    return 6;
  }
  const auto &pts = ix.points();
  if (pts.empty() || pts[0].out_offset != 0) return 7;
  for (size_t i = 0; i < pts.size(); ++i) {
    const ZranPoint &p = pts[i];
    if (p.bits > 7 || p.dict_size > GzipIndexer::kWindow || p.in_offset > gz.size() ||
        (i && (p.out_offset <= pts[i - 1].out_offset || p.in_offset < pts[i - 1].in_offset))) {
      printf("bad checkpoint %zu\n", i);
      return 8;
    }
  }
  int reads = 0;
  for (int t = 0; t < 300 && !out.empty(); ++t) {
    const uint64_t off = rng() % out.size();
    const uint64_t len = std::min<uint64_t>(out.size() - off, 1 + rng() % (3 * span));
    const ZranPoint &p = pts[ix.point_of(off)];
    std::vector<uint8_t> got(len);
    if (zran_extract(gz.data(), gz.size(), p, ix.dicts().data() + p.dict_offset, off - p.out_offset,
                     got.data(), len)) {
      printf("extract failed at %llu: %s\n", (unsigned long long)off, host_error());
      return 9;
    }
    if (memcmp(got.data(), out.data() + off, len)) {
      printf("extract differs at %llu\n", (unsigned long long)off);
      return 10;
    }
    // the compressed range the pack records for it covers the deflate data
    const uint64_t end = ix.in_end_of(off + len);
    if (end < p.in_offset || end > gz.size()) return 11;
    ++reads;
  }
  printf("points=%zu reads=%d ok\n", pts.size(), reads);
  return 0;
}
