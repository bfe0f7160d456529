// ASan/UBSan fuzz of the RAFS v5 chunk-dict parser (parse_v5_bootstrap,
// nydus-snapshotter_amd/csrc/blob.cpp) on mutations of a real v5 bootstrap.
// Host only.  usage: v5dict_fuzz BOOT N SEED
// Prints one line per case: "<rc> <records> <blobs>"; the unmutated input
// first.  Any memory error aborts (the test sees a non-zero exit).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <vector>

#include "blob.hpp"

int main(int argc, char **argv) {
  if (argc < 4) return 2;
  FILE *f = fopen(argv[1], "rb");
  if (!f) return 2;
  std::vector<uint8_t> boot;
  uint8_t buf[65536];
  size_t r;
  while ((r = fread(buf, 1, sizeof buf, f)) > 0) boot.insert(boot.end(), buf, buf + r);
  fclose(f);
  const int n = atoi(argv[2]);
  std::mt19937_64 rng(strtoull(argv[3], nullptr, 0));
  for (int k = 0; k <= n; ++k) {
    std::vector<uint8_t> b = boot;
    if (k > 0) {
      const int mode = k % 4;
      if (mode == 0) {
        b.resize(rng() % b.size());
      } else {
        // super block (mode 1), anywhere (mode 2), or 8-B words set to
        // extremes (mode 3: 0, ~0, large offsets)
        const int edits = 1 + (int)(rng() % 8);
        for (int e = 0; e < edits; ++e) {
          const size_t p = mode == 1 ? rng() % 96 : rng() % (b.size() - 8);
          if (mode == 3) {
            const uint64_t vals[4] = {0, ~0ull, 1ull << 40, b.size() - 1};
            const uint64_t v = vals[rng() % 4];
            memcpy(&b[p & ~size_t(3)], &v, b.size() - (p & ~size_t(3)) >= 8 ? 8 : 4);
          } else {
            b[p] = (uint8_t)rng();
          }
        }
      }
    }
    uint32_t dg = 0, cs = 0;
    std::vector<uint8_t> recs, blobs;
    const int rc = ngpu::parse_v5_bootstrap(b.data(), b.size(), &dg, &cs, &recs, &blobs);
    printf("%d %zu %zu\n", rc, recs.size() / 80, blobs.size() / 256);
  }
  return 0;
}
