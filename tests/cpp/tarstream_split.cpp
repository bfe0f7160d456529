// Feeds a tar file to ngpu::TarScanner in random-size pieces and prints the
// chunk list (offset,length,file_index,file_offset) plus a checksum of the
// data bytes each chunk received.  Used by tests/test_tarstream.py.
#include <stdio.h>
#include <stdlib.h>

#include <random>
#include <vector>

#include "tarstream.hpp"

struct Print : ngpu::TarSink {
  uint64_t sum = 0, got = 0, want = 0;
  bool open = false;
  int bad = 0;
  void close_chunk() {
    if (open) {
      if (got != want) bad = 1;
      printf(",%llu\n", (unsigned long long)sum);
    }
    open = false;
  }
  int chunk(uint64_t off, uint32_t len, uint32_t fi, uint64_t fo) override {
    close_chunk();
    printf("%llu,%u,%u,%llu", (unsigned long long)off, len, fi, (unsigned long long)fo);
    sum = 1469598103934665603ull;
    got = 0;
    want = len;
    open = true;
    return 0;
  }
  int data(const uint8_t *p, uint64_t len) override {
    for (uint64_t i = 0; i < len; ++i) sum = (sum ^ p[i]) * 1099511628211ull;
    got += len;
    return 0;
  }
};

int main(int argc, char **argv) {
  if (argc < 4) return 2;
  FILE *f = fopen(argv[1], "rb");
  if (!f) return 2;
  std::vector<uint8_t> buf;
  uint8_t tmp[65536];
  size_t r;
  while ((r = fread(tmp, 1, sizeof tmp, f)) > 0) buf.insert(buf.end(), tmp, tmp + r);
  fclose(f);
  const uint32_t cs = (uint32_t)strtoul(argv[2], nullptr, 0);
  std::mt19937_64 rng(strtoull(argv[3], nullptr, 0));
  ngpu::TarScanner sc(cs);
  Print pr;
  size_t pos = 0;
  while (pos < buf.size()) {
    size_t piece = 1 + rng() % (rng() % 3 == 0 ? 7 : 9000);
    if (piece > buf.size() - pos) piece = buf.size() - pos;
    int rc = sc.feed(buf.data() + pos, piece, pr);
    if (rc) { printf("ERR %d\n", rc); return 0; }
    pos += piece;
  }
  int rc = sc.finish();
  pr.close_chunk();
  if (rc) printf("ERR %d\n", rc);
  printf("FILES %llu BAD %d\n", (unsigned long long)sc.files(), pr.bad);
  return 0;
}
