// blob_tsan.cpp — the host blob writer's thread pool + sink (csrc/blob.cpp,
// ngpu_blob_write with threads > 1) built under ThreadSanitizer.  Reads the
// layer bytes and its chunks / results / stats (and optionally the chunk
// dict's blob table and chunk table) as raw little-endian files, writes the
// stream to OUT; tests/test_blob.py compares OUT with the regular build's
// stream byte for byte.  BLOB_TSAN_WRITERS=W (env) runs W writers at once,
// all on the process-wide shared compression pool (concurrent Packs closing
// together), and checks their streams are identical.  Host only.
// usage: blob_tsan DATA CHUNKS RESULTS STATS OUT COMPRESSOR THREADS CHUNK_SIZE
//                  DIGESTER [DICT_BLOBS DICT_CHUNKS]
#include <stdio.h>
#include <stdlib.h>

#include <string.h>

#include <thread>
#include <vector>

#include "nydus_gpu.h"

static std::vector<uint8_t> slurp(const char *path) {
  std::vector<uint8_t> v;
  FILE *f = fopen(path, "rb");
  if (!f) {
    perror(path);
    exit(2);
  }
  uint8_t buf[1 << 16];
  size_t r;
  while ((r = fread(buf, 1, sizeof buf, f)) > 0) v.insert(v.end(), buf, buf + r);
  fclose(f);
  return v;
}

static int wr(void *ctx, const void *p, uint64_t n) {
  return fwrite(p, 1, n, static_cast<FILE *>(ctx)) == n ? 0 : -1;
}

static int wr_mem(void *ctx, const void *p, uint64_t n) {
  auto *v = static_cast<std::vector<uint8_t> *>(ctx);
  v->insert(v->end(), (const uint8_t *)p, (const uint8_t *)p + n);
  return 0;
}

int main(int argc, char **argv) {
  if (argc != 10 && argc != 12) return 2;
  const std::vector<uint8_t> data = slurp(argv[1]), ch = slurp(argv[2]), res = slurp(argv[3]),
                             st = slurp(argv[4]);
  std::vector<uint8_t> dblobs, dchunks;
  ngpu_blob_options opt = {};
  opt.compressor = (uint32_t)atoi(argv[6]);
  opt.threads = (uint32_t)atoi(argv[7]);
  opt.chunk_size = (uint32_t)strtoul(argv[8], nullptr, 0);
  opt.digester = (uint32_t)atoi(argv[9]);
  if (argc == 12) {
    dblobs = slurp(argv[10]);
    dchunks = slurp(argv[11]);
    opt.dict_blobs = dblobs.data();
    opt.n_dict_blobs = (uint32_t)(dblobs.size() / 256);
    opt.dict_chunks = dchunks.data();
    opt.n_dict_chunks = dchunks.size() / 80;
  }
  const uint64_t n = ch.size() / sizeof(ngpu_chunk);
  if (res.size() != n * sizeof(ngpu_result) || st.size() != sizeof(ngpu_layer_stats)) return 2;
  const char *wv = getenv("BLOB_TSAN_WRITERS");
  const int W = wv ? atoi(wv) : 1;
  if (W > 1) {  // W concurrent writers into memory, then the first to OUT
    std::vector<std::vector<uint8_t>> outs(W);
    std::vector<int> rcs(W, 0);
    std::vector<std::thread> th;
    for (int w = 0; w < W; ++w)
      th.emplace_back([&, w] {
        ngpu_blob_info inf;
        rcs[w] = ngpu_blob_write(data.data(), data.size(), (const ngpu_chunk *)ch.data(),
                                 (const ngpu_result *)res.data(), n,
                                 (const ngpu_layer_stats *)st.data(), &opt, wr_mem, &outs[w], &inf);
      });
    for (auto &t : th) t.join();
    for (int w = 0; w < W; ++w) {
      if (rcs[w]) {
        fprintf(stderr, "writer %d: ngpu_blob_write %d\n", w, rcs[w]);
        return 1;
      }
      if (outs[w] != outs[0]) {
        fprintf(stderr, "writer %d: stream differs from writer 0\n", w);
        return 1;
      }
    }
    FILE *o = fopen(argv[5], "wb");
    if (!o || fwrite(outs[0].data(), 1, outs[0].size(), o) != outs[0].size()) return 2;
    fclose(o);
    return 0;
  }
  FILE *out = fopen(argv[5], "wb");
  if (!out) return 2;
  ngpu_blob_info info;
  const int rc = ngpu_blob_write(data.data(), data.size(), (const ngpu_chunk *)ch.data(),
                                 (const ngpu_result *)res.data(), n,
                                 (const ngpu_layer_stats *)st.data(), &opt, wr, out, &info);
  fclose(out);
  if (rc) fprintf(stderr, "ngpu_blob_write: %d %s\n", rc, ngpu_host_error());
  return rc ? 1 : 0;
}
