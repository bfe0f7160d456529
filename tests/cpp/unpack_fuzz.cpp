// unpack_fuzz.cpp — mutation fuzzing of the RAFS v5 / v6 bootstrap reader
// (csrc/rafs.cpp read_rafs) and of Unpack (csrc/blob.cpp ngpu_unpack) under
// AddressSanitizer + UBSan, host only.  Reads a valid Pack output stream,
// finds its image.boot, and per case mutates the bootstrap in place (byte
// flips, 16/32/64-bit fields set to 0 / all-ones / huge / small values at
// aligned offsets, concentrated on the superblocks, inode and dirent areas)
// and sometimes the blob data, then runs read_rafs on the mutated bootstrap
// ngpu_unpack on the whole mutated stream and ngpu_merge of the layer with
// its mutated copy.  Every outcome must be a
// return code (0 or NGPU_E*): no memory error, no crash, no unbounded output.
// Prints "cases=<n> read_ok=<n> unpack_ok=<n> rc:<code>=<n> ...".
// usage: unpack_fuzz STREAM CASES SEED
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <map>
#include <random>
#include <vector>

#include "nydus_gpu.h"
#include "rafs.hpp"

struct Out {
  std::vector<uint8_t> v;
  uint64_t total = 0;
};
static int wr(void *ctx, const void *p, uint64_t n) {
  Out *o = static_cast<Out *>(ctx);
  o->total += n;
  if (o->total > (1ull << 30)) return -1;  // runaway output: the writer refuses
  const uint8_t *b = static_cast<const uint8_t *>(p);
  if (o->v.size() < (64u << 20)) o->v.insert(o->v.end(), b, b + n);
  return 0;
}
static int64_t ra(void *ctx, void *p, uint64_t n, uint64_t off) {
  const std::vector<uint8_t> &v = *static_cast<const std::vector<uint8_t> *>(ctx);
  if (off >= v.size()) return -1;
  if (n > v.size() - off) n = v.size() - off;
  memcpy(p, v.data() + off, n);
  return (int64_t)n;
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
  Out boot;
  if (ngpu_unpack_entry(ra, &base, base.size(), "image.boot", wr, &boot, nullptr) != 0) return 3;
  const uint8_t *at = (const uint8_t *)memmem(base.data(), base.size(), boot.v.data(), boot.v.size());
  if (!at) return 3;
  const uint64_t boff = (uint64_t)(at - base.data()), blen = boot.v.size();
  {  // the unmutated stream unpacks
    Out o;
    if (ngpu_unpack(ra, &base, base.size(), wr, &o) != 0) return 4;
  }
  const int cases = atoi(argv[2]);
  std::mt19937_64 rng(strtoull(argv[3], nullptr, 0));
  std::map<int, int> rcs;
  int read_ok = 0, unpack_ok = 0, merge_ok = 0;
  for (int c = 0; c < cases; ++c) {
    std::vector<uint8_t> s = base;
    uint8_t *b = s.data() + boff;
    const int nedit = 1 + (int)(rng() % 4);
    for (int k = 0; k < nedit; ++k) {
      // half the edits land in the first 8 KiB (superblocks, device / blob
      // tables, the first inodes), the rest anywhere in the bootstrap
      const uint64_t span = (rng() & 1) ? std::min<uint64_t>(blen, 8192) : blen;
      uint64_t pos = rng() % span;
      switch (rng() % 6) {
        case 0: b[pos] ^= (uint8_t)(1u << (rng() % 8)); break;
        case 1: b[pos] = (uint8_t)rng(); break;
        default: {  // a whole field
          const int w = 2 << (rng() % 3);  // 2, 4, 8 bytes
          pos &= ~(uint64_t)(w - 1);
          if (pos + w > blen) break;
          uint64_t v;
          switch (rng() % 5) {
            case 0: v = 0; break;
            case 1: v = ~0ull; break;
            case 2: v = 1ull << (rng() % 64); break;
            case 3: v = rng() % 64; break;
            default: v = rng(); break;
          }
          memcpy(b + pos, &v, w);
        }
      }
    }
    if (rng() % 8 == 0 && boff > 1024) s[rng() % boff] ^= 0x5a;  // the blob data too
    std::vector<ngpu::RafsNode> nodes;
    std::vector<ngpu::RafsV6BlobInfo> blobs;
    uint32_t fsv = 0;
    if (ngpu::read_rafs(b, blen, &nodes, &blobs, &fsv) == 0) ++read_ok;
    Out o;
    const int rc = ngpu_unpack(ra, &s, s.size(), wr, &o);
    ++rcs[rc];
    if (rc == 0) ++unpack_ok;
    // Merge reads the same tree (overlaid over the unmutated layer)
    const void *boots[2] = {boot.v.data(), b};
    const uint64_t sizes[2] = {blen, blen};
    const char *names[2] = {"", ""};
    Out mo;
    char *ids = nullptr;
    if (ngpu_merge(boots, sizes, names, 2, nullptr, 0, wr, &mo, &ids) == 0) ++merge_ok;
    free(ids);  // malloc'd (ngpu_free_host lives in the GPU library)
  }
  printf("cases=%d read_ok=%d unpack_ok=%d merge_ok=%d", cases, read_ok, unpack_ok, merge_ok);
  for (auto &kv : rcs) printf(" rc:%d=%d", kv.first, kv.second);
  printf("\n");
  return 0;
}
