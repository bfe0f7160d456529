/* Plain-C client of libnydusgpu.so — what the cgo pkg/gpu binding does
 * (INTEGRATION.md): create an engine from PackOption-like settings, stream a
 * tar through the Pack writer, print one line per chunk, destroy.
 * usage: abi_client TAR [CHUNK_SIZE] [DIGESTER 0|1]  (needs a gfx950 GPU) */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "nydus_gpu.h"

int main(int argc, char **argv) {
  if (argc < 2) return 2;
  FILE *f = fopen(argv[1], "rb");
  if (!f) return 2;
  ngpu_config cfg;
  memset(&cfg, 0, sizeof cfg);
  cfg.chunk_size = argc > 2 ? (uint32_t)strtoul(argv[2], NULL, 0) : 0;
  cfg.digester = argc > 3 ? (uint32_t)atoi(argv[3]) : NGPU_DIGEST_BLAKE3;
  ngpu_engine *eng = NULL;
  int rc = ngpu_create(&cfg, &eng);
  if (rc) {
    printf("create failed %d\n", rc);
    return 1;
  }
  ngpu_pack *p = NULL;
  if ((rc = ngpu_pack_open(eng, &p))) {
    printf("open failed %d: %s\n", rc, ngpu_last_error(eng));
    return 1;
  }
  char buf[300000];
  size_t r;
  while ((r = fread(buf, 1, sizeof buf, f)) > 0) {
    if ((rc = ngpu_pack_write(p, buf, r))) {
      printf("write failed %d: %s\n", rc, ngpu_last_error(eng));
      ngpu_pack_abort(p);
      return 1;
    }
  }
  fclose(f);
  ngpu_chunk *ch = NULL;
  ngpu_result *res = NULL;
  uint64_t n = 0;
  ngpu_layer_stats st;
  if ((rc = ngpu_pack_close(p, &ch, &res, &n, &st))) {
    printf("close failed %d: %s\n", rc, ngpu_last_error(eng));
    return 1;
  }
  for (uint64_t i = 0; i < n; ++i) {
    printf("%llu,%u,", (unsigned long long)ch[i].offset, ch[i].length);
    for (int k = 0; k < 32; ++k) printf("%02x", res[i].digest[k]);
    printf(",%u,%u\n", res[i].kind, res[i].index);
  }
  printf("STATS %llu %llu %llu %llu\n", (unsigned long long)st.chunks,
         (unsigned long long)st.new_chunks, (unsigned long long)st.intra_chunks,
         (unsigned long long)st.dict_chunks);
  ngpu_free_host(ch);
  ngpu_free_host(res);
  ngpu_destroy(eng);
  return 0;
}
