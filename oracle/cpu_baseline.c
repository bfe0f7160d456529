/*
 * cpu_baseline.c — the timed CPU baseline (bench.py cpu_baseline leg).
 *
 * TEST / MEASUREMENT INFRASTRUCTURE ONLY (see oracle.h).
 *
 * The reference's CPU path is nydus-image (Rust; `blake3` and `sha2`
 * crates with SIMD / SHA-NI), which cannot run offline.  To time a CPU
 * digest+dedup stage of the same speed class (BASELINE.md "CPU-baseline
 * plan"), this file hashes chunks with:
 *   - BLAKE3: the official BLAKE3 C implementation (AVX-512/AVX2 dispatch)
 *     that ROCm LLVM vendors as llvm_blake3_* in libclang-cpp.so, via dlopen;
 *     falls back to the scalar oracle_blake3 if absent;
 *   - SHA-256: OpenSSL's SHA256() (SHA-NI) via dlopen of libcrypto; falls back
 *     to the scalar oracle_sha256;
 * spread over T pthreads (each takes the next chunk from a shared counter,
 * so ragged layers balance), followed by the single-stream oracle_dedup pass
 * (what nydus-image does in stream order).
 */
#include <dlfcn.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

typedef void (*b3_init_t)(void *);
typedef void (*b3_update_t)(void *, const void *, size_t);
typedef void (*b3_final_t)(const void *, uint8_t *, size_t);
typedef unsigned char *(*sha_t)(const unsigned char *, size_t, unsigned char *);

typedef size_t (*zstd_c_t)(void *, size_t, const void *, size_t, int);
typedef size_t (*zstd_bound_t)(size_t);
typedef unsigned (*zstd_err_t)(size_t);
typedef int (*sha_init_t)(void *);
typedef int (*sha_update_t)(void *, const void *, size_t);
typedef int (*sha_final_t)(unsigned char *, void *);

static b3_init_t b3_init;
static zstd_c_t zstd_c;
static zstd_bound_t zstd_bound;
static zstd_err_t zstd_err;
static sha_init_t sha_init;
static sha_update_t sha_update;
static sha_final_t sha_final;
static b3_update_t b3_update;
static b3_final_t b3_final;
static sha_t sha_fn;
static int resolved;

static void resolve(void) {
  if (resolved) return;
  resolved = 1;
  const char *libs[] = {"/opt/rocm/lib/llvm/lib/libclang-cpp.so",
                        "libclang-cpp.so", "libLLVM-15.so.1", NULL};
  for (int i = 0; libs[i]; i++) {
    void *h = dlopen(libs[i], RTLD_NOW | RTLD_LOCAL);
    if (!h) continue;
    b3_init = (b3_init_t)dlsym(h, "llvm_blake3_hasher_init");
    b3_update = (b3_update_t)dlsym(h, "llvm_blake3_hasher_update");
    b3_final = (b3_final_t)dlsym(h, "llvm_blake3_hasher_finalize");
    if (b3_init && b3_update && b3_final) break;
    b3_init = NULL;
  }
  const char *cl[] = {"libcrypto.so.3", "libcrypto.so", NULL};
  for (int i = 0; cl[i]; i++) {
    void *h = dlopen(cl[i], RTLD_NOW | RTLD_LOCAL);
    if (h && (sha_fn = (sha_t)dlsym(h, "SHA256"))) {
      sha_init = (sha_init_t)dlsym(h, "SHA256_Init");
      sha_update = (sha_update_t)dlsym(h, "SHA256_Update");
      sha_final = (sha_final_t)dlsym(h, "SHA256_Final");
      break;
    }
  }
  void *z = dlopen("libzstd.so.1", RTLD_NOW | RTLD_LOCAL);
  if (z) {
    zstd_c = (zstd_c_t)dlsym(z, "ZSTD_compress");
    zstd_bound = (zstd_bound_t)dlsym(z, "ZSTD_compressBound");
    zstd_err = (zstd_err_t)dlsym(z, "ZSTD_isError");
  }
}

/* The CPU converter pipeline for one layer, single-threaded (a goroutine +
 * its nydus-image in the reference, convert_unix.go:467-538, 870-914): chunk
 * digests, stream-order dedup, zstd (level 1, per NEW chunk in index order,
 * as the blob writer compresses) and the SHA-256 of the compressed stream
 * (the layer digest LayerConvertFunc computes).  Returns the compressed
 * bytes, or 0 with *ok = 0 when zstd / OpenSSL are absent. */
uint64_t oracle_cpu_pack_pipeline(const uint8_t *data, const oracle_chunk *chunks, uint64_t n,
                                  int digester, uint8_t *digests, const uint32_t *sizes,
                                  oracle_decision *decisions, uint8_t stream_digest[32], int *ok) {
  resolve();
  *ok = zstd_c && zstd_bound && zstd_err && sha_init && sha_update && sha_final;
  if (!*ok) return 0;
  _Alignas(64) uint8_t state[8192];
  for (uint64_t i = 0; i < n; i++) {
    const uint8_t *p = data + chunks[i].offset;
    size_t l = chunks[i].length;
    uint8_t *o = digests + 32 * i;
    if (digester == 1) {
      if (sha_fn) sha_fn(p, l, o); else oracle_sha256(p, l, o);
    } else if (b3_init) {
      b3_init(state);
      b3_update(state, p, l);
      b3_final(state, o, 32);
    } else {
      oracle_blake3(p, l, o);
    }
  }
  uint32_t own;
  oracle_dedup(digests, sizes, n, NULL, NULL, NULL, NULL, NULL, 0, 4096, decisions, &own);
  size_t cap = 0;
  for (uint64_t i = 0; i < n; i++) {
    const size_t b = zstd_bound(chunks[i].length);
    if (b > cap) cap = b;
  }
  uint8_t *buf = (uint8_t *)malloc(cap ? cap : 1);
  _Alignas(64) uint8_t ctx[512];
  sha_init(ctx);
  uint64_t total = 0;
  /* NEW chunks in index order (the blob's order) */
  uint64_t *order = (uint64_t *)malloc(sizeof(uint64_t) * (n ? n : 1));
  uint64_t k = 0;
  for (uint64_t i = 0; i < n; i++)
    if (decisions[i].kind == 0) order[decisions[i].index] = i, k++;
  for (uint64_t x = 0; x < k; x++) {
    const uint64_t i = order[x];
    size_t z = zstd_c(buf, cap, data + chunks[i].offset, chunks[i].length, 1);
    if (zstd_err(z)) z = 0;
    const uint8_t *src = buf;
    if (z == 0 || z >= chunks[i].length) {  /* stored raw, as the writer does */
      src = data + chunks[i].offset;
      z = chunks[i].length;
    }
    sha_update(ctx, src, z);
    total += z;
  }
  sha_final(stream_digest, ctx);
  free(order);
  free(buf);
  return total;
}

/* Which implementations will be used: bit0 = SIMD blake3, bit1 = OpenSSL sha. */
int oracle_cpu_impl(void) {
  resolve();
  return (b3_init ? 1 : 0) | (sha_fn ? 2 : 0);
}

typedef struct {
  const uint8_t *data;
  const oracle_chunk *chunks;
  uint64_t n;
  int digester, tid, nthreads;
  uint8_t *out;
  uint64_t *next;  /* shared chunk counter */
} job_t;

static void *worker(void *arg) {
  job_t *j = (job_t *)arg;
  _Alignas(64) uint8_t state[8192];
  for (uint64_t i; (i = __atomic_fetch_add(j->next, 1, __ATOMIC_RELAXED)) < j->n;) {
    const uint8_t *p = j->data + j->chunks[i].offset;
    size_t l = j->chunks[i].length;
    uint8_t *o = j->out + 32 * i;
    if (j->digester == 1) {
      if (sha_fn) sha_fn(p, l, o); else oracle_sha256(p, l, o);
    } else if (b3_init) {
      b3_init(state);
      b3_update(state, p, l);
      b3_final(state, o, 32);
    } else {
      oracle_blake3(p, l, o);
    }
  }
  return NULL;
}

/* Digest all chunks with `threads` threads, then run the stream-order dedup.
 * Returns the number of NEW chunks. */
uint64_t oracle_cpu_digest_dedup(const uint8_t *data, const oracle_chunk *chunks,
                                 uint64_t n, int digester, int threads,
                                 uint8_t *digests, const uint32_t *sizes,
                                 oracle_decision *decisions) {
  resolve();
  if (threads < 1) threads = 1;
  pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)threads);
  job_t *jobs = (job_t *)malloc(sizeof(job_t) * (size_t)threads);
  uint64_t next = 0;
  for (int t = 0; t < threads; t++) {
    jobs[t] = (job_t){data, chunks, n, digester, t, threads, digests, &next};
    pthread_create(&th[t], NULL, worker, &jobs[t]);
  }
  for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
  free(th);
  free(jobs);
  uint32_t own;
  return oracle_dedup(digests, sizes, n, NULL, NULL, NULL, NULL, NULL, 0, 4096,
                      decisions, &own);
}
