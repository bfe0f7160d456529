// blob_fuzz.cpp — mutation fuzzing of the host blob-stream reader and merge
// (csrc/blob.cpp: ngpu_unpack_entry, ngpu_merge) under AddressSanitizer +
// UBSan.  Reads a valid Pack output stream, applies random mutations (byte
// flips concentrated on the tail: tar headers, TOC, bootstrap; truncations;
// size-digit rewrites) and prints one line per case:
//   "<new size> <pos:val,...>|<rc>,<len>,<fnv>;<rc>,<len>,<fnv>"
// (UnpackEntry of image.boot, then image.blob).  tests/test_blob.py replays
// the edits and compares each case with the reference reader restated in
// oracle/blob_ref.py.
// usage: blob_fuzz STREAM CASES SEED
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <string>
#include <utility>
#include <vector>

#include "nydus_gpu.h"

struct Out {
  std::vector<uint8_t> v;
};
static int wr(void *ctx, const void *p, uint64_t n) {
  Out *o = static_cast<Out *>(ctx);
  const uint8_t *b = static_cast<const uint8_t *>(p);
  o->v.insert(o->v.end(), b, b + n);
  return 0;
}
struct Src {
  const std::vector<uint8_t> *v;
};
static int64_t ra(void *ctx, void *p, uint64_t n, uint64_t off) {
  const std::vector<uint8_t> &v = *static_cast<Src *>(ctx)->v;
  if (off >= v.size()) return -1;
  if (n > v.size() - off) n = v.size() - off;
  memcpy(p, v.data() + off, n);
  return (int64_t)n;
}
static uint64_t fnv(const std::vector<uint8_t> &v) {
  uint64_t h = 1469598103934665603ull;
  for (uint8_t c : v) h = (h ^ c) * 1099511628211ull;
  return h;
}

int main(int argc, char **argv) {
  if (argc < 4) return 2;
  FILE *f = fopen(argv[1], "rb");
  if (!f) return 2;
  std::vector<uint8_t> base;
  uint8_t buf[1 << 16];
  size_t r;
  while ((r = fread(buf, 1, sizeof buf, f)) > 0) base.insert(base.end(), buf, buf + r);
  fclose(f);
  const int cases = atoi(argv[2]);
  std::mt19937_64 rng(strtoull(argv[3], nullptr, 0));
  for (int c = 0; c < cases; ++c) {
    std::vector<uint8_t> s = base;
    std::vector<std::pair<uint64_t, uint8_t>> edits;
    auto set = [&](uint64_t pos, uint8_t val) {
      s[pos] = val;
      edits.emplace_back(pos, val);
    };
    const int kind = (int)(rng() % 5);
    const uint64_t tail = s.size() < 20000 ? s.size() : 20000;  // headers, TOC, bootstrap
    if (kind == 0) {  // flip a few bytes in the tail
      const int k = 1 + (int)(rng() % 4);
      for (int i = 0; i < k; ++i) {
        const uint64_t p = s.size() - 1 - rng() % tail;
        set(p, s[p] ^ (uint8_t)(1u << (rng() % 8)));
      }
    } else if (kind == 1) {  // truncate
      s.resize(s.size() - 1 - rng() % tail);
    } else if (kind == 2) {  // rewrite an octal size digit of one of the last headers
      const uint64_t h = s.size() - 512 * (1 + rng() % 3);
      set(h + 124 + rng() % 11, (uint8_t)('0' + rng() % 8));
    } else if (kind == 3) {  // random byte over the TOC entries
      set(s.size() - 512 - 1 - rng() % 256, (uint8_t)rng());
    } else {  // one field of one TOC entry: flags -> zstd, or a huge size / offset
      const uint64_t toc_len = strtoull(std::string((const char *)&s[s.size() - 512 + 124], 11).c_str(),
                                        nullptr, 8);
      const uint64_t n = toc_len / 128;
      if (n && toc_len <= s.size() - 512) {
        const uint64_t e = s.size() - 512 - toc_len + 128 * (rng() % n);
        const int field = (int)(rng() % 4);
        if (field == 0) {
          set(e, 0x2);  // compressor zstd on whatever the entry holds
        } else {      // 1 compressed_offset, 2 compressed_size, 3 uncompressed_size
          const uint64_t at = e + 56 + 8 * (field - 1);
          const uint64_t v = field == 3 ? rng() : rng() >> (rng() % 64);
          for (int b = 0; b < 8; ++b) set(at + b, (uint8_t)(v >> (8 * b)));
        }
      }
    }
    printf("%zu ", s.size());
    for (size_t i = 0; i < edits.size(); ++i)
      printf("%s%llu:%u", i ? "," : "", (unsigned long long)edits[i].first, edits[i].second);
    printf("|");
    Src src{&s};
    for (const char *name : {"image.boot", "image.blob", "blob.meta"}) {
      Out o;
      uint8_t toc[128];
      const int rc = ngpu_unpack_entry(ra, &src, s.size(), name, wr, &o, toc);
      printf("%s%d,%zu,%llu", strcmp(name, "image.boot") ? ";" : "", rc, o.v.size(),
             (unsigned long long)(rc ? 0 : fnv(o.v)));
      if (rc == 0 && !strcmp(name, "image.boot")) {  // merge must not crash on it either
        const void *bp = o.v.data();
        const uint64_t bs = o.v.size();
        const char *dg = "00";
        char *ids = nullptr;
        Out m;
        if (ngpu_merge(&bp, &bs, &dg, 1, nullptr, 0, wr, &m, &ids) == 0) free(ids);
      }
    }
    printf("\n");
  }
  return 0;
}
