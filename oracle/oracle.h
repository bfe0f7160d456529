/*
 * oracle.h — CPU restatement of the nydus chunk digest + dedup path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing under oracle/ is part of the product:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load liboracle.so, and only as the checker (or the timed CPU baseline).
 * The product path (libnydusgpu.so) never links or calls it.
 *
 * What this restates:
 *   a3  tar-rafs chunking: each regular file with size>0 is split into
 *       fixed-size chunks [k*S, min((k+1)*S, size)); chunks never span files
 *       ([nydus v2.3.0] builder/src/tarball.rs, called from
 *       pkg/converter/tool/builder.go:97-110 "--type tar-rafs").
 *   a4  RafsDigest::from_buf: BLAKE3-256 (default digester, see
 *       pkg/converter/tool/feature_test.go:228-229) or SHA-256 of the raw
 *       uncompressed chunk bytes ([nydus v2.3.0] utils/src/digest.rs).
 *   a5  Node::deduplicate_chunk: global chunk dict first, then the layered
 *       (intra-build) dict; NEW chunks get sequential indices
 *       ([nydus v2.3.0] builder/src/core/node.rs).
 *   a6  HashChunkDict: hit iff digest present and (dict usize==0 || ==size);
 *       first insertion wins ([nydus v2.3.0] builder/src/core/chunk_dict.rs).
 *   a7  RAFS v6 chunk table record, 80 B (pkg/layout/layout.go:25-27, decoded
 *       from pkg/filesystem/testdata/v6-bootstrap-chunk-pos-438272.tar.gz).
 *
 * Parity pinning: digests are pinned by golden vectors produced in the build
 * container by independent implementations (ROCm LLVM's vendored official
 * BLAKE3 C v1.8.2 and OpenSSL SHA-256) — tests/golden/make_golden.py.  Dedup
 * decisions are pinned by a second, independent Python restatement in the
 * same script and by the TestPack outcome (tests/converter_test.go:513-527).
 * nydus-image itself (Rust, external) is unavailable offline, so the dedup
 * semantics are "restated, VERIFY" — see DESIGN.md §Oracle.
 */
#ifndef NYDUS_ORACLE_H
#define NYDUS_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- digests ------------------------------------------------------------ */
void oracle_blake3(const uint8_t *data, size_t len, uint8_t out[32]);
void oracle_sha256(const uint8_t *data, size_t len, uint8_t out[32]);

/* ---- tar chunking ------------------------------------------------------- */
typedef struct {
  uint64_t offset;     /* byte offset of chunk data in the tar buffer */
  uint32_t length;     /* bytes in this chunk (<= chunk_size) */
  uint32_t file_index; /* index of the owning file in stream order */
  uint64_t file_offset;/* offset of the chunk inside its file */
} oracle_chunk;

/* Returns number of chunks written (may exceed cap: call again with a bigger
 * array), or a negative error: -1 malformed header, -2 truncated data,
 * -3 unsupported entry (GNU sparse). n_files receives the count of regular
 * files with data. */
int64_t oracle_tar_chunks(const uint8_t *tar, uint64_t len, uint32_t chunk_size,
                          oracle_chunk *out, uint64_t cap, uint64_t *n_files);

/* ---- dedup -------------------------------------------------------------- */
enum { ORACLE_NEW = 0, ORACLE_INTRA = 1, ORACLE_DICT = 2 };

typedef struct {
  uint32_t kind;   /* ORACLE_NEW / ORACLE_INTRA / ORACLE_DICT */
  uint32_t index;  /* NEW: sequential chunk index in the layer blob;
                      INTRA: index of the referenced NEW chunk;
                      DICT: dict entry's own chunk index field */
  uint64_t ref;    /* NEW: own chunk id; INTRA: chunk id of the first
                      occurrence; DICT: dict entry id (table order) */
  uint32_t blob_index; /* real blob index (first-hit allocation order) */
  uint32_t pad;
  uint64_t uncompressed_offset; /* NEW: 4K-aligned running offset (v6) */
} oracle_decision;

/* digests: n x 32 B; sizes: n uncompressed sizes.
 * dict_*: m dict entries in chunk-table order (may be NULL / m=0).
 * dict_blob: inner blob index of each dict entry.
 * align: uncompressed-offset alignment for NEW chunks (4096 for v6, 1 for
 * unaligned v5).  Returns the number of NEW chunks; *own_blob receives the
 * real blob index of the layer's own blob (or UINT32_MAX if none). */
uint64_t oracle_dedup(const uint8_t *digests, const uint32_t *sizes, uint64_t n,
                      const uint8_t *dict_digests, const uint32_t *dict_sizes,
                      const uint32_t *dict_blob, const uint32_t *dict_index,
                      const uint64_t *dict_uoff, uint64_t m, uint32_t align,
                      oracle_decision *out, uint32_t *own_blob);

/* Digest every chunk of `data` (one call per chunk) into out (n x 32 B). */
void oracle_digest_chunks(const uint8_t *data, const oracle_chunk *chunks,
                          uint64_t n, int digester, uint8_t *out);

/* ---- timed CPU baseline (cpu_baseline.c; bench.py's cpu_baseline leg) ---- */
int oracle_cpu_impl(void);
uint64_t oracle_cpu_digest_dedup(const uint8_t *data, const oracle_chunk *chunks, uint64_t n,
                                 int digester, int threads, uint8_t *digests,
                                 const uint32_t *sizes, oracle_decision *decisions);
uint64_t oracle_cpu_pack_pipeline(const uint8_t *data, const oracle_chunk *chunks, uint64_t n,
                                  int digester, uint8_t *digests, const uint32_t *sizes,
                                  oracle_decision *decisions, uint8_t stream_digest[32], int *ok);

#ifdef __cplusplus
}
#endif
#endif
