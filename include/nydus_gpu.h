/*
 * nydus_gpu.h — C ABI of the MI355X chunk digest + dedup engine
 * (libnydusgpu.so).  Plain pointers and sizes only; no C++ or torch types.
 *
 * What this boundary replaces:
 *   The reference hands the digest/dedup stage to an external process:
 *   pkg/converter/tool/builder.go:148-178 (tool.Pack) execs
 *   `nydus-image create --type tar-rafs [--chunk-dict bootstrap=P]
 *    [--chunk-size S] ...` (argv built at builder.go:78-146) over FIFOs set up
 *   by packFromTar (pkg/converter/convert_unix.go:443-539).  Inside that
 *   process, per chunk: RafsDigest::from_buf + Node::deduplicate_chunk
 *   ([nydus v2.3.0] utils/src/digest.rs, builder/src/core/node.rs).
 *   This library performs exactly that stage in-process on the GPU; the Go
 *   side binds it from a new pkg/gpu cgo package.
 *
 * Errors: every function returns 0 on success or a negative NGPU_E* code;
 * ngpu_last_error() gives the per-engine message (Go wraps both into an
 * `error`, as builder.go:169-175 wraps the process exit status).  No
 * exceptions cross the ABI.  A missing or unusable GPU is an error
 * (NGPU_ENODEV): there is no CPU fallback in this library.
 *
 * Threading: one engine per device serves any number of goroutines.  Calls
 * take the engine's lock only while they enqueue work.  Calls on distinct
 * streams use distinct HBM workspaces (NGPU_WS_SLOTS, default 4) and run side
 * by side on the GPU; calls on one stream are ordered by it.  Every pack has
 * its own compute stream and waits for it, and writes its blob stream,
 * outside the lock, so Packs of an image's layers proceed concurrently.  A
 * split-stage caller (ngpu_digest_device, then ngpu_dedup_device) keeps both
 * stages of a layer on one stream: the dedup stage reports the bad-descriptor
 * count of the digest stage that ran last on its workspace.
 *
 * Lifetimes: engines, chunk dicts and packs are reference counted.  A pack
 * holds its engine and the dict it was opened with until it ends (close,
 * finish or abort), so ngpu_destroy / ngpu_dict_release with packs still open
 * only drop the caller's reference; the memory goes when the last pack ends.
 */
#ifndef NYDUS_GPU_H
#define NYDUS_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NGPU_ABI_VERSION 7

/* PackOption.Digester (API extension; maps to nydus-image --digester). */
enum ngpu_digester { NGPU_DIGEST_BLAKE3 = 0, NGPU_DIGEST_SHA256 = 1 };

/* Per-chunk dedup outcome ([nydus v2.3.0] Node::deduplicate_chunk), and the
 * two states a record has around it. */
enum ngpu_kind {
  NGPU_NEW = 0,   /* first occurrence: new data in this layer's blob */
  NGPU_INTRA = 1, /* duplicate of an earlier NEW chunk of this layer */
  NGPU_DICT = 2,  /* found in the chunk dict (PackOption.ChunkDictPath) */
  /* Written by the digest stage next to each digest (ngpu_digest_device).  The
   * dedup stage takes only records marked so: a caller that supplies its own
   * digests to ngpu_dedup_* sets kind = NGPU_DIGESTED. */
  NGPU_DIGESTED = 3,
  /* Set by the dedup stage on a record that reached it without a digest (kind
   * not NGPU_DIGESTED, or an all-zero digest): the record takes no part in
   * dedup, and the call fails with NGPU_EDEVICE when its stats are read
   * (ngpu_device_status for calls that read none). */
  NGPU_UNHASHED = 4
};

enum ngpu_error {
  NGPU_OK = 0,
  NGPU_EINVAL = -1,    /* bad argument (e.g. ChunkSize not a power of two) */
  NGPU_EHIP = -2,      /* HIP runtime error */
  NGPU_ENOMEM = -3,    /* device or pinned allocation failed */
  NGPU_ETAR = -4,      /* malformed / truncated tar stream */
  NGPU_EUNSUPP = -5,   /* unsupported input (GNU sparse tar entry) */
  NGPU_ENODEV = -6,    /* no usable gfx950 device */
  NGPU_EIO = -7,       /* file I/O (chunk-dict bootstrap) */
  NGPU_EFORMAT = -8,   /* not a RAFS v6 bootstrap / bad chunk table */
  NGPU_ENOTFOUND = -9, /* entry not found in a nydus blob (ErrNotFound,
                          pkg/converter/types.go:33-35) */
  NGPU_ECANCELED = -10, /* cancelled through the pack's cancel flag (the
                          reference's ctx.Done() / PackOption.Timeout kill of
                          the builder, builder.go:153-174) */
  NGPU_EDEVICE = -11   /* a device-side check failed: a chunk reached the
                          dedup stage without its digest (NGPU_UNHASHED) */
};

typedef struct ngpu_engine ngpu_engine;

/* Mirrors the PackOption fields this stage consumes
 * (pkg/converter/types.go:58-90). */
typedef struct {
  int32_t device;         /* HIP device ordinal */
  uint32_t digester;      /* enum ngpu_digester (default blake3) */
  uint32_t chunk_size;    /* PackOption.ChunkSize: power of two in
                             [0x1000, 0x1000000] (types.go:76); 0 -> 0x100000 */
  uint32_t fs_version;    /* PackOption.FsVersion 5 or 6; 0 -> 6
                             (builder.go:79-81).  v6 aligns uncompressed
                             offsets of NEW chunks to 4 KiB (v5 with
                             NGPU_FLAG_ALIGNED_CHUNK). */
  uint64_t staging_bytes; /* pinned staging slot size for host-buffer calls;
                             0 -> 256 MiB (two slots are allocated) */
  uint32_t leaves_per_lane; /* BLAKE3 tuning: 1 KiB leaves hashed per lane
                               (1, 2, 4, 8 or 16); 0 -> auto */
  uint32_t flags;         /* NGPU_FLAG_* */
} ngpu_config;

/* ngpu_config.flags */
#define NGPU_FLAG_TIMING 0x1u /* record HIP events around each stage */
/* PackOption.AlignedChunk (types.go:73-74, `--aligned-chunk`, builder.go:131-133):
 * 4 KiB-align the uncompressed offsets of NEW chunks for RAFS v5 too (v6
 * always aligns). */
#define NGPU_FLAG_ALIGNED_CHUNK 0x2u
/* Tuning / tests: never take the small-call paths.  By default chunk planning
 * and the dedup stage of calls with <= 4096 chunks run in one fused workgroup
 * each, and BLAKE3 layers of <= 32K leaves (one leaf per lane) hash each
 * compression on a quad of lanes; this flag keeps the multi-kernel grid path
 * and one lane per leaf (same results). */
#define NGPU_FLAG_GRID_STAGES 0x4u
/* Packs whose whole layer fit one staging slot and that close at about the
 * same time on one engine share ONE digest + multi-layer dedup launch set
 * (round 5: containerd converting an image's small layers concurrently).
 * The first to close waits for the other packs that may still join -- open,
 * not OCIRef, and with no more than one staging slot of tar so far -- to
 * close too: BLAKE3 at most 250 us; SHA-256 2 ms, restarted by every pack
 * that joins, at most 12 ms after the first (a SHA-256 batch holds the GPU
 * for one 1 MiB chunk's chain, ~21 ms, whatever its size).  A pack that cannot
 * join (its layer outgrew one slot, an OCIRef pack, a pack closing without
 * chunks) stops being waited for at that moment.  This flag gives every pack
 * its own launches (A/B, or a caller whose packs must never wait for each
 * other).  Same results. */
#define NGPU_FLAG_NO_BATCH 0x8u
/* Tuning (benchmarks only): bits 8..10 = 1 + BLAKE3 load mode (0 plain loads
 * with the whole-leaf fast path, 1 non-temporal loads, 2 next-block prefetch,
 * 3 both, 5 plain loads without the fast path); 0 = library default.  Every
 * mode computes the same digests; other values (5, 7) are rejected with
 * NGPU_EINVAL. */
#define NGPU_FLAG_LOAD_MODE_SHIFT 8
/* Tuning (benchmarks only): bits 11..13 = 1 + SHA-256 kernel (0: one lane per
 * chunk with schedule/round waves, 1: two lanes per chunk, 2: one lane per
 * chunk, each wave schedules its own blocks, 4: two lanes, one chunk group per
 * workgroup, 5: two lanes, four groups per workgroup); 0 = library default
 * (by chunk count); other values are rejected (NGPU_EINVAL). */
#define NGPU_FLAG_SHA_MODE_SHIFT 11

/* The builder's exit status (builder.go:169-175) for work enqueued on a
 * caller's stream: errors of device-pointer calls that read no stats (stats == NULL,
 * ngpu_digest_device, the *_layers_device calls): synchronises every stream
 * the engine's workspaces were last used on, returns the first error any
 * stage recorded since the previous ngpu_device_status (NGPU_EINVAL for bad or
 * overlapping descriptors, NGPU_EDEVICE for unhashed chunks; message in
 * ngpu_last_error) and clears them.  0: no stage recorded an error. */
int ngpu_device_status(ngpu_engine *eng);

/* Per-stage device time of the last process call (NGPU_FLAG_TIMING). */
typedef struct {
  float digest_ms;   /* leaf/group digest kernel (b3_groups / b3_quad_leaves /
                        sha256_*); BLAKE3: from the end of chunk planning, i.e.
                        the kernel plus its dispatch */
  float tree_ms;     /* BLAKE3 upper-tree kernel (0 for sha256) */
  float dedup_ms;    /* dict probe + intra-layer dedup + scans + finalize */
  float total_ms;    /* whole enqueue, first to last kernel */
  uint32_t group_log2; /* leaves-per-lane log2 used (BLAKE3) */
  uint32_t reserved;
} ngpu_timing;

/* One chunk of layer file data. 24 bytes.  Chunks lie
 * inside the data buffer and do not overlap (a tar's file extents never do):
 * a descriptor past the buffer, or overlaps adding up to more BLAKE3 leaves
 * than the buffer holds, fail the call with NGPU_EINVAL once its stats are
 * read. */
typedef struct {
  uint64_t offset;      /* byte offset of the chunk in the data buffer */
  uint32_t length;      /* 1 .. chunk_size bytes */
  uint32_t file_index;  /* ordinal of the owning regular file in the tar */
  uint64_t file_offset; /* offset of the chunk inside its file */
} ngpu_chunk;

/* Per-chunk result. 64 bytes. */
typedef struct {
  uint8_t digest[32];   /* BLAKE3-256 or SHA-256 of the raw chunk bytes
                           (RafsV5/V6 ChunkInfo block_id) */
  uint32_t kind;        /* enum ngpu_kind */
  uint32_t index;       /* NEW: sequential chunk index in this layer's blob;
                           INTRA: index of the referenced NEW chunk;
                           DICT: the dict entry's chunk index */
  uint64_t ref;         /* NEW: own chunk id; INTRA: chunk id of the first
                           occurrence; DICT: dict entry id (table order) */
  uint32_t blob_index;  /* real blob index, allocated in first-hit order */
  uint32_t dict_blob;   /* DICT: the entry's inner blob index in the chunk
                           dict (its blob table); otherwise 0 */
  uint64_t uncompressed_offset; /* NEW/INTRA: offset in the layer blob;
                           DICT: the dict chunk's offset in ITS blob (nydus
                           copies the cached chunk, chunk.copy_from) */
} ngpu_result;

/* Summary of one layer. */
typedef struct {
  uint64_t chunks, new_chunks, intra_chunks, dict_chunks;
  uint64_t new_bytes;        /* uncompressed bytes of NEW chunks */
  uint32_t own_blob_index;   /* UINT32_MAX if the layer has no NEW chunk */
  uint32_t blobs;            /* blob-table entries this layer references */
  uint64_t uncompressed_size;/* end of the last NEW chunk (v6: 4K aligned) */
} ngpu_layer_stats;

int ngpu_abi_version(void);

/* Engine lifetime.  Replaces the per-Pack builder process spawn
 * (builder.go:163 exec.CommandContext). */
int ngpu_create(const ngpu_config *cfg, ngpu_engine **out);
void ngpu_destroy(ngpu_engine *eng);
const char *ngpu_last_error(const ngpu_engine *eng);
int ngpu_device_count(void);

/* Pinned host memory owned by the engine (cgo must not hand Go-heap memory
 * to async DMA). */
int ngpu_alloc_pinned(ngpu_engine *eng, uint64_t bytes, void **out);
int ngpu_free_pinned(ngpu_engine *eng, void *ptr);

/* ---- chunk dict handles (PackOption.ChunkDictPath; builder.go:122-124) ----
 * The reference runs one nydus-image process per Pack, each loading its own
 * `--chunk-dict bootstrap=P` ([nydus v2.3.0] HashChunkDict).  Here a dict is
 * an HBM-resident, read-only, reference-counted object: a Pack captures the
 * dict it is opened with, so packs with different dicts (or none) can be open
 * on one engine at once, and 1000 Packs against one ChunkDictPath share one
 * loaded table.  First table entry wins for duplicate digests; usize == 0
 * matches any chunk size.
 *
 * ngpu_dict_open: load the chunk table (80-B records at the extended
 * superblock's chunk_table_offset, pkg/layout/layout.go:25-27) and the blob
 * table of a RAFS v6 bootstrap on the engine's device.  Rejected with
 * NGPU_EINVAL, as nydus-image rejects an incompatible chunk-dict bootstrap
 * ([nydus v2.3.0] RafsSuperConfig::check_compatibility, VERIFY): a digester
 * flag (RafsSuperFlags HASH_BLAKE3 0x4 / HASH_SHA256 0x8) or chunk_size that
 * differs from the engine's, or an engine with FsVersion 5.  The engine
 * caches the dicts it opened by (path, device, inode, size, mtime): opening an
 * unchanged file again returns the same dict with one more reference. */
typedef struct ngpu_dict ngpu_dict;
int ngpu_dict_open(ngpu_engine *eng, const char *path, ngpu_dict **out);
/* From a chunk table in memory: n 80-B RAFS v6 chunk-info records (table
 * order) and n_blobs 256-B RAFS v6 blob records (inner-index order; may be
 * NULL / 0, the blob count is then max(blob_index) + 1). */
int ngpu_dict_create(ngpu_engine *eng, const void *records, uint64_t n,
                     const void *blob_table, uint32_t n_blobs, ngpu_dict **out);
/* From device-resident arrays (entry order = table order), e.g. a 200M-entry
 * dict built on the GPU.  d_uoff (u64 uncompressed offsets) may be NULL.
 * The build runs on a stream of the library's own and returns when it is
 * done; it does not wait for the caller's streams, so the arrays must be
 * complete when the call is made (synchronise the stream that wrote them). */
int ngpu_dict_create_device(ngpu_engine *eng, const uint8_t *d_digests, const uint32_t *d_usize,
                            const uint32_t *d_blob_index, const uint32_t *d_chunk_index,
                            const uint64_t *d_uoff, uint64_t n, uint32_t n_blobs,
                            ngpu_dict **out);
/* The same with each entry's GLOBAL id (d_gid, device u32; NULL = its
 * position): a rank's digest-prefix share of a dict partitioned across
 * processes (nydus_gpu/dist.py) then answers probes with global entry ids.
 * The rows must be in global table order.  (ABI 4) */
int ngpu_dict_create_device_gid(ngpu_engine *eng, const uint8_t *d_digests,
                                const uint32_t *d_usize, const uint32_t *d_blob_index,
                                const uint32_t *d_chunk_index, const uint64_t *d_uoff,
                                const uint32_t *d_gid, uint64_t n, uint32_t n_blobs,
                                ngpu_dict **out);
void ngpu_dict_retain(ngpu_dict *d);
void ngpu_dict_release(ngpu_dict *d);
uint64_t ngpu_dict_entries(const ngpu_dict *d);
/* The engine's default dict, used by the calls without a dict argument
 * (ngpu_process*, ngpu_pack_open*, ngpu_dict_probe_device) and captured by a
 * pack when it opens.  NULL = no dict.  Takes a reference. */
int ngpu_set_dict(ngpu_engine *eng, ngpu_dict *d);

/* Legacy default-dict loaders (each = create + ngpu_set_dict + release).
 * Replacing the default never changes the dict of a pack already open.
 * ngpu_dict_load: n entries in chunk-table order; blob_index: inner blob index
 * per entry; chunk_index: the entry's RAFS chunk index (copied into DICT
 * results); compressed placement unknown (csize = usize, offsets 0). */
int ngpu_dict_load(ngpu_engine *eng, const uint8_t *digests /* n x 32 */,
                   const uint32_t *usize, const uint32_t *blob_index,
                   const uint32_t *chunk_index, uint64_t n);
int ngpu_dict_load_bootstrap(ngpu_engine *eng, const char *path);
int ngpu_dict_clear(ngpu_engine *eng);
uint64_t ngpu_dict_size(const ngpu_engine *eng);

/* ---- tar front end (host) ------------------------------------------------ */
/* Enumerate the chunks of a tar-rafs layer.  Writes at
 * most cap chunks; *n_chunks receives the full count (call again with a
 * larger array if it exceeds cap).  *n_files: regular files seen. */
int ngpu_tar_chunks(const void *tar, uint64_t len, uint32_t chunk_size,
                    ngpu_chunk *out, uint64_t cap, uint64_t *n_chunks,
                    uint64_t *n_files);

/* ---- digest + dedup ------------------------------------------------------- */
/* Host buffers in, host results out (synchronous).  `data` is the layer's
 * bytes (e.g. the uncompressed tar), `chunks` index into it.  Data moves to
 * HBM through the engine's pinned staging slots with hipMemcpyAsync. */
int ngpu_process(ngpu_engine *eng, const void *data, uint64_t len,
                 const ngpu_chunk *chunks, uint64_t n, ngpu_result *out,
                 ngpu_layer_stats *stats);

/* Device-resident variant: data, chunks and out are device pointers; work is
 * enqueued on `stream` (a hipStream_t; NULL = the null/default stream, as in
 * HIP itself) and the call returns without synchronising, so it is stream-
 * ordered after whatever the caller enqueued on the same stream to produce
 * d_data / d_chunks.  stats may be NULL; if not NULL the call synchronises
 * the stream to fill it.  The same holds for every *_device entry point
 * below except ngpu_dict_load_device (synchronous: its inputs must be
 * complete when it is called). */
int ngpu_process_device(ngpu_engine *eng, const void *d_data, uint64_t len,
                        const ngpu_chunk *d_chunks, uint64_t n,
                        ngpu_result *d_out, void *stream,
                        ngpu_layer_stats *stats);

/* ---- split stages (device pointers, async on `stream`) -------------------
 * For callers that route dict probes themselves, e.g. a chunk dict
 * partitioned across GPUs by digest prefix:
 *   ngpu_digest_device     -> digests only (d_out[i].digest);
 *   ngpu_dict_probe_device -> look digests up in THIS engine's dict;
 *   ngpu_dedup_device      -> dedup decisions from digests + given dict hits.
 * ngpu_process_device == digest + dedup against the engine's own dict. */
typedef struct {
  uint32_t entry;  /* dict entry id (chunk-table order) or 0xFFFFFFFF: miss */
  uint32_t index;  /* the entry's RAFS chunk index */
  uint32_t blob;   /* the entry's inner blob index */
  uint32_t usize;  /* the entry's uncompressed size (0 = any) */
  uint64_t uncompressed_offset; /* the entry's offset in its blob */
} ngpu_dict_hit;   /* 24 bytes */

int ngpu_digest_device(ngpu_engine *eng, const void *d_data, uint64_t len,
                       const ngpu_chunk *d_chunks, uint64_t n,
                       ngpu_result *d_out, void *stream);
/* d_digests: n digests at byte stride `stride` (32 for packed, 64 to read
 * ngpu_result.digest in place).  No size rule is applied here: the hit
 * carries usize and the requester's dedup applies it. */
int ngpu_dict_probe_device(ngpu_engine *eng, const uint8_t *d_digests,
                           uint64_t stride, uint64_t n,
                           ngpu_dict_hit *d_hits, void *stream);
/* d_hits: per-chunk dict hits (NULL: probe this engine's dict).
 * n_dict_blobs: number of inner blobs of the (global) chunk dict; 0 = use
 * this engine's dict.  stats as in ngpu_process_device. */
int ngpu_dedup_device(ngpu_engine *eng, const ngpu_chunk *d_chunks, uint64_t n,
                      ngpu_result *d_out, const ngpu_dict_hit *d_hits,
                      uint32_t n_dict_blobs, void *stream,
                      ngpu_layer_stats *stats);
/* Many layers per call (e.g. 1000 small layers against one chunk dict):
 * layer l owns chunks [d_layer_first[l], d_layer_first[l+1]) (device u64
 * array of n_layers+1, d_layer_first[n_layers] == n).  Each layer is deduped
 * exactly as if it were packed alone (its own layered dict, NEW indices,
 * offsets and blob order); the chunk dict is shared.  d_stats: device
 * ngpu_layer_stats[n_layers] (written asynchronously), or NULL. */
int ngpu_dedup_layers_device(ngpu_engine *eng, const ngpu_chunk *d_chunks, uint64_t n,
                             ngpu_result *d_out, const ngpu_dict_hit *d_hits,
                             uint32_t n_dict_blobs, const uint64_t *d_layer_first,
                             uint64_t n_layers, ngpu_layer_stats *d_stats, void *stream);
int ngpu_process_layers_device(ngpu_engine *eng, const void *d_data, uint64_t len,
                               const ngpu_chunk *d_chunks, uint64_t n, ngpu_result *d_out,
                               const uint64_t *d_layer_first, uint64_t n_layers,
                               ngpu_layer_stats *d_stats, void *stream);
/* Build the default dict from device-resident arrays (entry order = table
 * order); = ngpu_dict_create_device + ngpu_set_dict. */
int ngpu_dict_load_device(ngpu_engine *eng, const uint8_t *d_digests,
                          const uint32_t *d_usize, const uint32_t *d_blob_index,
                          const uint32_t *d_chunk_index, uint64_t n,
                          uint32_t n_blobs);

/* The same against an explicit dict (NULL = no chunk dict) instead of the
 * engine's default.  ngpu_process_dict_device: d_layer_first NULL = one layer
 * of n chunks (n_layers ignored); d_stats: device ngpu_layer_stats[n_layers]
 * or NULL; stats: host, as in ngpu_process_device (synchronises), one-layer
 * calls only. */
int ngpu_dict_probe(const ngpu_dict *dict, const uint8_t *d_digests, uint64_t stride,
                    uint64_t n, ngpu_dict_hit *d_hits, void *stream);

/* Digest-prefix routing for a dict partitioned over `world` owners (<= 64;
 * owner(d) = ((d[0] << 8 | d[1]) * world) >> 16), device pointers, async on
 * `stream` (ABI 4).  Each of the n digests (byte stride `stride`, 16-B
 * aligned) goes to its owner's segment of d_out (32 B per row) with its row id
 * in d_rows.  d_counts: 128 device u32, written by the call: [0, world) =
 * rows per owner.  seg_cap == 0: owners back to back in owner order (owner o
 * at the sum of the counts before it), d_out / d_rows hold n rows.  seg_cap >
 * 0 (equal splits): row k of owner o goes to slot [k / seg_cap][o][k %
 * seg_cap] of rounds x world x seg_cap slots; the call zeroes d_out and sets
 * every d_rows slot to 0xFFFFFFFF first (padding), and rounds * seg_cap must
 * cover n.  Order inside a segment is unspecified: hits return by row id. */
int ngpu_route_digests(const uint8_t *d_digests, uint64_t stride, uint64_t n, uint32_t world,
                       uint64_t seg_cap, uint32_t rounds, uint8_t *d_out, uint32_t *d_rows,
                       uint32_t *d_counts, void *stream);
/* d_hits[d_rows[i]] = d_routed[i] for the m routed rows (rows of 0xFFFFFFFF,
 * padding, are skipped): an owner's hits back in the requester's row order. */
int ngpu_route_hits(const ngpu_dict_hit *d_routed, const uint32_t *d_rows, uint64_t m,
                    ngpu_dict_hit *d_hits, void *stream);
int ngpu_process_dict(ngpu_engine *eng, ngpu_dict *dict, const void *data, uint64_t len,
                      const ngpu_chunk *chunks, uint64_t n, ngpu_result *out,
                      ngpu_layer_stats *stats);
int ngpu_process_dict_device(ngpu_engine *eng, ngpu_dict *dict, const void *d_data,
                             uint64_t len, const ngpu_chunk *d_chunks, uint64_t n,
                             ngpu_result *d_out, const uint64_t *d_layer_first,
                             uint64_t n_layers, ngpu_layer_stats *d_stats, void *stream,
                             ngpu_layer_stats *stats);

/* Whole tar layer in host memory -> chunk list + results (tar parse on the
 * host, digest/dedup on the GPU).  *chunks_out / *results_out are allocated
 * with malloc and must be released with ngpu_free_host. */
int ngpu_pack_tar(ngpu_engine *eng, const void *tar, uint64_t len,
                  ngpu_chunk **chunks_out, ngpu_result **results_out,
                  uint64_t *n_out, ngpu_layer_stats *stats);
void ngpu_free_host(void *p);

/* Batched Pack closes so far (NGPU_FLAG_NO_BATCH): out[0] launch sets,
 * out[1] packs closed in them, out[2] the most packs in one. */
int ngpu_batch_stats(ngpu_engine *eng, uint64_t out[3]);
/* Stage timings of the last ngpu_process / ngpu_process_device call on this
 * engine (synchronises on the recorded events).  NGPU_EINVAL unless the
 * engine was created with NGPU_FLAG_TIMING. */
int ngpu_last_timing(ngpu_engine *eng, ngpu_timing *out);
/* The same for the call `back` calls before the last one (0 = the last).
 * The engine keeps the events of its last 64 calls, so a caller can time a
 * run of back-to-back calls without synchronising between them. */
int ngpu_timing_at(ngpu_engine *eng, uint32_t back, ngpu_timing *out);

/* ---- streaming Pack (converter.Pack, pkg/converter/convert_unix.go:325) ----
 * The reference returns an io.WriteCloser fed with the uncompressed layer tar
 * (packFromTar :443-539 pipes it to nydus-image through a FIFO).  Here:
 * open -> write (copying) or reserve/commit (zero-copy into engine-pinned
 * staging) in any split -> close.  Full staging slots are copied to HBM and
 * digested while the caller keeps writing; dedup runs at close in stream
 * order.  close (success or not) and abort release the pack; *chunks_out /
 * *results_out are malloc'd (ngpu_free_host).  A malformed or truncated tar
 * fails with NGPU_ETAR / NGPU_EUNSUPP at write/commit or close.
 * A pack dedups against the dict it was opened with: ngpu_pack_open* take the
 * engine's default dict at open time, ngpu_pack_open_dict an explicit one
 * (NULL = none; its digester and chunk size must be the engine's). */
typedef struct ngpu_pack ngpu_pack;
int ngpu_pack_open(ngpu_engine *eng, ngpu_pack **out);
int ngpu_pack_open_dict(ngpu_engine *eng, ngpu_dict *dict, uint32_t flags, ngpu_pack **out);
/* Cancellation (ctx.Done() / PackOption.Timeout): `flag` is caller-owned
 * memory that must outlive the pack; once another thread stores a non-zero
 * value there, the pack's next write / commit / reserve, or the running
 * close / finish at its next slot, blob window or compression batch, fails
 * with NGPU_ECANCELED (the reference kills the builder process,
 * builder.go:153-174, convert_unix.go:530-535).  close / finish release the
 * pack on every outcome; after a failed write / commit / reserve the pack
 * stays open until the caller aborts it (ngpu_pack_abort).  NULL removes the
 * flag. */
int ngpu_pack_set_cancel(ngpu_pack *p, const volatile int32_t *flag);
int ngpu_pack_write(ngpu_pack *p, const void *buf, uint64_t len);
int ngpu_pack_reserve(ngpu_pack *p, void **ptr, uint64_t *avail);
int ngpu_pack_commit(ngpu_pack *p, uint64_t n);
int ngpu_pack_close(ngpu_pack *p, ngpu_chunk **chunks_out, ngpu_result **results_out,
                    uint64_t *n_out, ngpu_layer_stats *stats);
/* Ends a pack without output: its staging, HBM and emitter thread are
 * released.  A binding calls it on every path that will never reach close --
 * a failed write, a source read error, ctx.Done() with no Close to follow
 * (convert_unix.go:885-907 skips tw.Close() on those paths).  Not concurrently
 * with another call on the same pack. */
void ngpu_pack_abort(ngpu_pack *p);
/* The engine a pack runs on (borrowed; e.g. to see where ngpu_node_pack_open
 * placed it: compare with ngpu_node_engine).  (ABI 7) */
ngpu_engine *ngpu_pack_engine(const ngpu_pack *p);

/* What an engine holds right now (ABI 7): a leak check for the bindings'
 * error paths (every aborted or finished pack gives all of it back). */
typedef struct {
  uint64_t open_packs;          /* packs opened and not yet ended */
  uint64_t staging_pool_bufs;   /* pinned staging slots kept for the next packs */
  uint64_t staging_pool_bytes;  /* their pinned bytes */
  uint64_t pack_pool;           /* per-pack stream + buffer sets kept */
  uint64_t land_pool;           /* early-emission landing buffers kept */
  uint64_t batch_waitable;      /* open packs a batch leader would still wait for */
  uint64_t reserved[2];
} ngpu_engine_counters;
int ngpu_engine_counters_get(ngpu_engine *eng, ngpu_engine_counters *out);

/* ---- multi-GPU node ------------------------------------
 * One process drives the GPUs of a node: one engine per listed device (a
 * device may be listed twice, e.g. to rehearse a 2-GPU node on one GPU).
 * Layers are independent units (north star: "the chunk stream is sharded by
 * layer"): ngpu_node_pack_open places each streaming Pack on the engine with
 * the fewest open packs (ties round robin) -- containerd's per-layer
 * goroutines (convert_unix.go:467-538) then spread over every GPU and every
 * GPU's own PCIe link -- and ngpu_node_process_device runs device-resident
 * layers on a chosen engine.  A node chunk dict is either partitioned by
 * digest prefix -- entry with digest d lives on device
 * ((d[0] << 8 | d[1]) * n) >> 16, keeping table order, so "first entry wins"
 * holds per digest -- or replicated on every device.  Probing a partitioned
 * dict is the node's exchange step: the requester's digests go to every
 * owner, each owner probes the entries it owns and the hits come back with
 * GLOBAL entry ids, ordered by cross-device events -- the in-process form of
 * the north star's digest-prefix all-to-all (nydus_gpu/dist.py keeps the
 * one-process-per-GPU RCCL form).  Default exchange (ABI 7, "copy"): every
 * digest to every owner and every owner's n hits back by hipMemcpyPeerAsync
 * (DMA engines; W x n x 56 bytes per call), merged by owner on the
 * requester.  NGPU_NODE_EXCHANGE_ROUTED in `mode` (opt-in, the ABI 4-6
 * default) runs the routed exchange instead when every pair of listed devices
 * has peer access: the requester buckets its digests by owner in its own HBM;
 * each owner's probe kernel reads only its own rows (peer loads over xGMI)
 * and writes each hit into the requester's hit array at the row's id (peer
 * stores), so a call moves n x (32 + 4) bytes out and n x 24 back in total.
 * Peer access between the listed devices is enabled at creation.
 * UNVERIFIED ON DISTINCT GPUs: every test so far lists one GPU several times
 * (the copies and peer stores then stay inside one HBM); the routed
 * exchange's peer stores, the copy exchange and the RCCL node step first
 * meet separate GPUs in the driver's multi-GPU bench, whose `node_cabi` entry
 * runs all three against a replicated dict, prints them in its
 * `multi_gpu_checks` summary and fails the run if any disagrees.  Until that
 * has passed, a caller that needs certainty uses NGPU_NODE_DICT_REPLICATE (no
 * exchange), as the converter mirrors do for ChunkDictPath. */
typedef struct ngpu_node ngpu_node;
int ngpu_node_create(const int32_t *devices, uint32_t n, const ngpu_config *cfg, ngpu_node **out);
void ngpu_node_destroy(ngpu_node *node);
uint32_t ngpu_node_size(const ngpu_node *node);
/* The node's engine i (borrowed: valid until ngpu_node_destroy). */
ngpu_engine *ngpu_node_engine(ngpu_node *node, uint32_t i);
#define NGPU_NODE_DICT_PARTITION 0u /* shard by digest prefix (default) */
#define NGPU_NODE_DICT_REPLICATE 1u /* a full copy on every device */
#define NGPU_NODE_EXCHANGE_COPY 0x100u   /* | PARTITION: broadcast + DMA exchange (default) */
#define NGPU_NODE_EXCHANGE_ROUTED 0x200u /* | PARTITION: peer-kernel exchange (opt-in) */
/* Node chunk dicts, usable by any engine of the node (ngpu_pack_open_dict,
 * ngpu_process_dict*, ngpu_node_*); checks as ngpu_dict_open.
 * ngpu_node_dict_open caches what it opened, as ngpu_dict_open does per
 * engine: opening an unchanged file (path, device, inode, size, mtime) with
 * the same mode again returns the same dict with one more reference, so 1000
 * Packs naming one ChunkDictPath load it once per node. */
int ngpu_node_dict_open(ngpu_node *node, const char *path, uint32_t mode, ngpu_dict **out);
int ngpu_node_dict_create(ngpu_node *node, const void *records, uint64_t n,
                          const void *blob_table, uint32_t n_blobs, uint32_t mode,
                          ngpu_dict **out);
/* Device index of the node device that owns digests[32] (partitioned dicts). */
uint32_t ngpu_node_owner(const ngpu_node *node, const uint8_t *digest);
/* A Pack on the node's least-loaded engine (fewest open packs, ties round
 * robin); flags as ngpu_pack_open_dict.  ngpu_pack_engine tells which. */
int ngpu_node_pack_open(ngpu_node *node, ngpu_dict *dict, uint32_t flags, ngpu_pack **out);
int ngpu_node_process_device(ngpu_node *node, uint32_t i, ngpu_dict *dict, const void *d_data,
                             uint64_t len, const ngpu_chunk *d_chunks, uint64_t n,
                             ngpu_result *d_out, const uint64_t *d_layer_first,
                             uint64_t n_layers, ngpu_layer_stats *d_stats, void *stream);

/* ---- node step: every device at once, one all-to-all each way (ABI 5) ----
 * The bulk-synchronous form of the exchange, for a caller that converts one
 * batch of layers per device per step (C4: layers round robin over the
 * node's GPUs; convert_unix.go:467-538 runs a layer per goroutine): part i
 * (device-resident layers on node device i, its own stream there; n = 0
 * takes part with nothing) is digested, its digests are bucketed by owner
 * (ngpu_route_digests), every part's segments cross the node in ONE
 * all-to-all-v, each owner probes what it received against its partition,
 * the hits return in one all-to-all-v the other way, go back to their rows
 * and each part dedups its own layers.  Nothing in the step waits for the
 * device (ABI 5, round 5): each part's digests are bucketed into padded
 * per-owner segments of n rows, so every transfer size is known when the
 * step is enqueued, and the per-owner counts cross in band (one u32 per
 * pair) for the owners' probes to read on the device.  A caller can enqueue
 * step k+1 behind step k; the cost is W x n x 32 B out per part instead of
 * n x 32 B (csrc/a2a_plan.hpp).
 * flags NGPU_NODE_STEP_RCCL: the two all-to-alls are RCCL ncclAllToAllv
 * calls over a communicator of the node's devices (ncclCommInitAll, created on
 * the first such step; RCCL takes one rank per GPU, so a node listing a
 * device twice returns NGPU_EUNSUPP).  Without it the same segments move
 * by hipMemcpyPeerAsync (any node, also one GPU listed several times).
 * dict: a partitioned node dict (replicated or NULL: no exchange, each part
 * is processed on its own).  Returns once everything is enqueued; each
 * part's results are ready when its stream is. */
typedef struct {
  const void *d_data;             /* part's layer bytes on its device */
  uint64_t len;
  const ngpu_chunk *d_chunks;     /* n descriptors (device) */
  uint64_t n;
  ngpu_result *d_out;             /* n results (device) */
  const uint64_t *d_layer_first;  /* n_layers + 1 (device), or NULL: one layer */
  uint64_t n_layers;
  ngpu_layer_stats *d_stats;      /* device, n_layers, or NULL */
  void *stream;                   /* on the part's device (NULL: its null stream) */
} ngpu_node_part;
#define NGPU_NODE_STEP_RCCL 1u
int ngpu_node_process_step(ngpu_node *node, ngpu_dict *dict, const ngpu_node_part *parts,
                           uint32_t n_parts, uint32_t flags);

/* ---- RAFS v6 chunk table ---------------------------- */
/* Serialise the layer's unique chunk records (NEW chunks in index order) as
 * 80-byte RAFS v6 chunk-info entries.  compressor "none": compressed size =
 * uncompressed size, compressed offsets packed back to back.  `blob_index`
 * of each record is the result's real blob index.  Writes at most cap
 * records; *n_records receives the count. */
int ngpu_chunk_table(const ngpu_chunk *chunks, const ngpu_result *results,
                     uint64_t n, uint8_t *out /* cap x 80 */, uint64_t cap,
                     uint64_t *n_records);

/* ---- nydus blob stream: converter.Pack's output --
 * The stream nydus-image writes for `--type tar-rafs --blob-inline-meta
 * --features blob-toc` (builder.go:97-110) and packFromTar copies to `dest`
 * (convert_unix.go:486-495): `data | tar_header | ... | toc | tar_header`
 * (convert_unix.go:296-300).  Entries: image.blob (the layer's NEW chunks in
 * index order, each compressed on its own, raw when compression does not
 * shrink it), image.boot (the RAFS v6 -- or, FsVersion 5, v5 -- bootstrap of
 * the layer: the tar's whole inode tree, every regular file's chunks, blob
 * table, prefetch table, and the chunk table: one record per distinct chunk
 * the layer references -- its NEW chunks and the chunk-dict chunks it reuses,
 * copied with their dict blob placement),
 * blob.meta + blob.meta.header (convert_unix.go:47-48: the chunk-info array
 * of the layer's blob and its 4 KiB header) and blob.digest (the chunks'
 * digests, index order) when the blob has chunks, and
 * rafs.blob.toc (128-B TOCEntry records, types.go:147-163).  Compression and
 * SHA-256 run on the host (north star: compression stays on the host path). */

/* PackOption.Compressor / TOCEntry.Flags values (types.go:22-31). */
enum ngpu_compressor {
  NGPU_COMPRESSOR_NONE = 0x1,
  NGPU_COMPRESSOR_ZSTD = 0x2,
  NGPU_COMPRESSOR_LZ4_BLOCK = 0x4
};

/* io.Writer: return 0 after consuming all len bytes, non-zero on error. */
typedef int (*ngpu_write_fn)(void *ctx, const void *buf, uint64_t len);
/* content.ReaderAt: bytes read (> 0) or a negative error. */
typedef int64_t (*ngpu_read_at_fn)(void *ctx, void *buf, uint64_t len, uint64_t off);

typedef struct {
  uint32_t compressor;   /* enum ngpu_compressor; 0 -> zstd */
  int32_t level;         /* compressor level; 0 -> library default (zstd: 1) */
  uint32_t threads;      /* host compression threads; 0 -> min(16, cores) */
  uint32_t digester;     /* ngpu_blob_write only: bootstrap digest flag */
  uint32_t chunk_size;   /* ngpu_blob_write only: bootstrap chunk size */
  uint32_t n_dict_blobs; /* records in dict_blobs */
  const uint8_t *dict_blobs; /* the chunk dict's blob table (n x 256-B RAFS v6
                                blob records, inner-index order), or NULL;
                                ngpu_pack_finish defaults to the blob table of
                                the pack's dict */
  const void *dict_chunks;   /* ngpu_blob_write: the chunk dict's chunk table
                                (80-B RAFS v6 records, entry order) the DICT
                                results' `ref` index, for the compressed
                                placement their records copy; NULL: csize =
                                usize, offset 0.  ngpu_pack_finish uses the
                                pack's dict */
  uint64_t n_dict_chunks;
  uint32_t fs_version;       /* ngpu_blob_write only: PackOption.FsVersion 5 or 6
                                (0 -> 6); ngpu_pack_finish uses the engine's.  v6:
                                RAFS v6 image.boot + blob.meta + TOC (`--features
                                blob-toc`, builder.go:104-110); v5: RAFS v5
                                image.boot, no TOC */
  uint32_t reserved;
  const char *prefetch_patterns; /* PackOption.PrefetchPatterns: newline-separated
                                paths (the builder's stdin, builder.go:125-127,
                                166); NULL or "" -> "/" */
} ngpu_blob_options;

typedef struct {
  uint64_t stream_bytes;      /* bytes written to dest */
  uint64_t blob_bytes;        /* image.blob: compressed chunk data */
  uint64_t bootstrap_bytes;   /* image.boot */
  uint64_t blob_chunks;       /* chunk records of the layer's own blob (NEW) */
  uint64_t compressed_chunks; /* of which stored compressed */
  uint8_t stream_digest[32];  /* sha256 of the whole stream: the layer blob
                                 digest (LayerConvertFunc, convert_unix.go:870-914) */
  uint8_t blob_digest[32];    /* sha256 of image.blob (the own blob's id) */
  uint8_t toc_digest[32];     /* sha256 of the TOC (calcBlobTOCDigest :541-555) */
  uint64_t dict_records;      /* chunk records copied from the chunk dict */
  uint64_t meta_entries;      /* entries of the blob.meta chunk-info array (0: none) */
} ngpu_blob_info;

/* Thread-local message of the last failing engine-less call below. */
const char *ngpu_host_error(void);
/* A ready-made ngpu_write_fn: ctx is a file descriptor ((void *)(intptr_t)fd). */
int ngpu_write_fd(void *ctx, const void *buf, uint64_t len);

/* Host: write the stream of one packed layer whose bytes are in host memory
 * (chunks/results/stats as returned by ngpu_pack_tar).  `data` must be the
 * layer tar the chunks were cut from: its entries are the bootstrap's inode
 * tree (NGPU_EINVAL when walking it does not give `chunks`). */
int ngpu_blob_write(const void *data, uint64_t len, const ngpu_chunk *chunks,
                    const ngpu_result *results, uint64_t n, const ngpu_layer_stats *stats,
                    const ngpu_blob_options *opt, ngpu_write_fn w, void *ctx,
                    ngpu_blob_info *info);

/* Streaming Pack that writes the stream at the end: NGPU_PACK_RETAIN keeps the
 * layer bytes in HBM (288 GB) instead of recycling the device slots, so that
 * ngpu_pack_finish can gather the NEW chunks on the GPU, copy only those to
 * the host and compress them.  ngpu_pack_finish = ngpu_pack_close + stream
 * (releases the pack in every case). */
#define NGPU_PACK_RETAIN 0x1u
/* PackOption.OCIRef (ABI 4; `nydus-image create --type targz-ref`,
 * builder.go:180-218): ngpu_pack_write takes the ORIGINAL gzip layer blob.  The
 * library inflates it on the host (one gzip member), the tar stream takes the
 * tar-rafs path (tar walk, GPU digests, layered dedup; no chunk dict, as
 * packRef passes none), and a checkpoint of the deflate stream is kept every
 * max(chunk size, 1 MiB) of output.  The output stream holds no image.blob:
 * blob.meta (chunk-info array with each chunk's checkpoint, the checkpoint
 * table and the 32 KiB dictionaries), blob.digest, image.boot and the TOC; the
 * bootstrap's own blob is the gzip blob (id = its sha256, the digest Merge
 * returns for the layer, converter_test.go TestPackRef), each chunk record
 * carrying the deflate range that produces it.
 * EXPERIMENTAL: the blob.meta zran layout (ZranInflateContext records, the
 * zran header words, super flag 0x40, the chunk entry's data word) is
 * restated from nydus v2.3.0 and NOT pinned by any reference fixture; this
 * library's own reader (ngpu_ref_chunk_read) round-trips it, nydusd has not
 * read it.  A chunk whose deflate range or checkpoint offset does not fit its
 * field (24-bit size, 40-bit offset, 32-bit offsets) fails with NGPU_EFORMAT,
 * never truncated.  ngpu_pack_reserve / ngpu_pack_commit are not available
 * (EINVAL). */
#define NGPU_PACK_OCIREF 0x2u
/* The reader side of an OCIRef layer (host; what nydusd does with a targz-ref
 * blob): chunk `index` of the layer's own blob, located through `blob_meta`
 * (the layer stream's blob.meta tar entry: chunk-info array, checkpoint table,
 * dictionaries, then the 4 KiB header -- through the TOC, the "blob.meta"
 * entry followed by "blob.meta.header") and inflated out of the original gzip blob `gz` from
 * its checkpoint.  *len_out = the chunk's size (<= cap).  (ABI 4) */
int ngpu_ref_chunk_read(const void *gz, uint64_t gz_len, const void *blob_meta, uint64_t meta_len,
                        uint32_t index, void *out, uint32_t cap, uint32_t *len_out);
int ngpu_pack_open_ex(ngpu_engine *eng, uint32_t flags, ngpu_pack **out);
int ngpu_pack_finish(ngpu_pack *p, const ngpu_blob_options *opt, ngpu_write_fn w, void *ctx,
                     ngpu_chunk **chunks_out, ngpu_result **results_out, uint64_t *n_out,
                     ngpu_layer_stats *stats, ngpu_blob_info *info);
/* Early emission (ABI 4): give a NGPU_PACK_RETAIN pack its output before the
 * first write (converter.Pack knows `dest` when it opens, convert_unix.go:325).
 * An emitter thread then writes the blob stream while the tar is still
 * arriving: after each staging slot is digested it dedups the prefix so far
 * (a chunk's decision depends only on the chunks before it) and compresses,
 * hashes and writes the NEW chunks that became final, so the sequential host
 * SHA-256 of the stream overlaps the copies and digests of the rest of the
 * layer.  Finish with ngpu_pack_finish(p, NULL, NULL, NULL, ...): it writes the
 * rest, image.boot and the TOC.  The bytes are the same as with a writer given
 * to ngpu_pack_finish.  `opt` is copied (prefetch_patterns too); dict_blobs /
 * dict_chunks must stay valid until finish.  w is called from the library's
 * threads.  An emitter error fails the next write and the finish. */
int ngpu_pack_set_output(ngpu_pack *p, const ngpu_blob_options *opt, ngpu_write_fn w, void *ctx);

/* UnpackEntry (convert_unix.go:284-320): find `name` through the TOC
 * (seekFileByTOC :219-276; entry compressor none or zstd), else by walking
 * the tar headers from the tail (seekFileByTarHeader :162-213), and copy its
 * data to w.  toc_entry_out (128 B, may be NULL) receives the TOC entry, or
 * zeros when found by tar header.  NGPU_ENOTFOUND = ErrNotFound. */
int ngpu_unpack_entry(ngpu_read_at_fn ra, void *ctx, uint64_t size, const char *name,
                      ngpu_write_fn w, void *wctx, uint8_t *toc_entry_out);

/* Unpack (convert_unix.go:669-719, `nydus-image unpack`): the nydus stream of
 * a packed layer (read through ra, `size` bytes) back to an OCI tar written to
 * w: image.boot's inode tree depth first in name order, each regular file's
 * chunks read from image.blob and decompressed.  Headers use the Go
 * archive/tar USTAR encoding (PAX records where USTAR cannot hold a value),
 * user / group names from the host's passwd / group; a hardlinked inode is a
 * file at its first path and a hardlink ('1') at the others.  A chunk in
 * another blob (a chunk-dict blob) is NGPU_ENOTFOUND: only the layer's own
 * blob travels in its stream. */
int ngpu_unpack(ngpu_read_at_fn ra, void *ctx, uint64_t size, ngpu_write_fn w, void *wctx);

/* converter.Merge (convert_unix.go:560-666) -> tool.Merge (builder.go:220-294,
 * `nydus-image merge --prefetch-policy fs [--chunk-dict] [--parent-bootstrap]`):
 * per-layer bootstraps (the image.boot entries, lowest layer first) into the
 * image's bootstrap, written to w in the layers' RAFS version (v5 or v6; all
 * layers must share it and the chunk size).  The inode trees are overlaid
 * with the OCI layer rules: an upper entry replaces the lower one of its path,
 * directories merge, `.wh.<name>` removes <name> and its subtree from the
 * layers below, `.wh..wh..opq` hides everything below its directory, and the
 * whiteouts themselves are dropped.  Chunk records keep their placement; their
 * blob indices point into the merged blob table.  A layer's own blob (any
 * blob not in the chunk dict bootstrap's blob table) is named
 * layer_digests[l] (hex of Layer.Digest, the bootstrap file name the
 * reference passes to nydus-image merge); at most one per layer.
 * *blob_ids_out (malloc'd, ngpu_free_host) = comma-separated blob ids in
 * first-appearance order (the output JSON's "Blobs"). */
int ngpu_merge(const void *const *bootstraps, const uint64_t *sizes,
               const char *const *layer_digests, uint64_t n, const void *dict_bootstrap,
               uint64_t dict_size, ngpu_write_fn w, void *ctx, char **blob_ids_out);

/* `nydus-image inspect`, restated (north_star: bootstraps "compared via
 * nydus-image inspect"): one JSON object for a RAFS
 * v5 or v6 bootstrap, written to w --
 *   {"fs_version", "chunk_size", "flags", "blobs": [{"id", "chunk_count",
 *    "compressed_size", "uncompressed_size"}], "inodes": [{"path" ("/" first,
 *    then depth first in name order), "mode", "uid", "gid", "size", "nlink",
 *    "ino", "rdev", "mtime", "mtime_ns", "link" (symlinks), "xattrs" (name ->
 *    hex value), "chunks": [[digest hex, blob index, flags, compressed
 *    offset, compressed size, uncompressed offset, uncompressed size, file
 *    offset, chunk index], ...]}]}
 * Bytes outside printable ASCII in names are \u00XX escapes (latin-1).
 * Untrusted input: bounds-checked (NGPU_EFORMAT). */
int ngpu_rafs_dump(const void *bootstrap, uint64_t size, ngpu_write_fn w, void *ctx);

/* MergeOption fields beyond the chunk dict (types.go:92-133). */
typedef struct ngpu_merge_options {
  /* ParentBootstrapPath's contents (--parent-bootstrap): the lowest layer,
   * its blobs keep their ids (any number of them); NULL = none */
  const void *parent_bootstrap;
  uint64_t parent_size;
  /* PrefetchPatterns (the builder's stdin, builder.go:238-240, 269):
   * newline-separated paths; NULL or "" = "/" */
  const char *prefetch_patterns;
  /* (ABI 6 appended the targz-ref arrays here; ABI 7 takes them as arguments
   * of ngpu_merge_ex2 instead, so a caller built against either header passes
   * a struct this library reads no further than its end.) */
} ngpu_merge_options;

/* ngpu_merge with MergeOption's parent bootstrap and prefetch patterns
 * (opt may be NULL: ngpu_merge). */
int ngpu_merge_ex(const void *const *bootstraps, const uint64_t *sizes,
                  const char *const *layer_digests, uint64_t n, const void *dict_bootstrap,
                  uint64_t dict_size, const ngpu_merge_options *opt, ngpu_write_fn w, void *ctx,
                  char **blob_ids_out);
/* ngpu_merge_ex with targz-ref layers (ABI 7; Layer.OriginalDigest:
 * convert_unix.go:577-590 hands nydus-image --blob-digests / --blob-sizes /
 * --blob-toc-digests, builder.go:242-253).  The three arrays are NULL (no
 * targz-ref layer) or n entries each, entry l NULL / ignored for a layer
 * without OriginalDigest: 64 hex chars of the layer's RAFS blob (its nydus
 * stream) digest, its size, and 64 hex chars of the sha256 of its TOC entry
 * data (calcBlobTOCDigest, convert_unix.go:541-554).  Recorded in the layer's
 * own blob record of the merged bootstrap (RafsV6Blob blob_toc_digest /
 * blob_meta_digest / blob_meta_size; offsets restated from nydus v2.3.0,
 * parity unpinned). */
int ngpu_merge_ex2(const void *const *bootstraps, const uint64_t *sizes,
                   const char *const *layer_digests, uint64_t n, const void *dict_bootstrap,
                   uint64_t dict_size, const ngpu_merge_options *opt,
                   const char *const *rafs_blob_digests, const uint64_t *rafs_blob_sizes,
                   const char *const *rafs_blob_toc_digests, ngpu_write_fn w, void *ctx,
                   char **blob_ids_out);

#ifdef __cplusplus
}
#endif
#endif /* NYDUS_GPU_H */
