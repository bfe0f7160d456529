/*
 * dedup_ref.c — restated chunk dedup decisions.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Restates, in stream order per chunk ([nydus v2.3.0]
 * builder/src/core/node.rs Node::deduplicate_chunk and
 * builder/src/core/chunk_dict.rs HashChunkDict, external, VERIFY):
 *   1. global dict lookup get_chunk(d, size): hit iff the digest is present
 *      and (dict.uncompressed_size == 0 || == size).  The dict keeps the FIRST
 *      entry of the chunk-dict bootstrap's chunk table for a digest.  A hit
 *      copies the dict chunk; its inner blob index is mapped to a real blob
 *      index allocated at the first hit of that dict blob.
 *   2. else layered (intra-build) dict lookup, same size rule; the layered
 *      dict holds only NEW chunks and keeps the first insertion.
 *   3. else NEW: the layer's own blob is allocated (get_or_create_current_
 *      blob) at its first NEW chunk; index = sequential; the uncompressed
 *      offset is the running offset, and the running offset advances to
 *      round_up(off + size, align) — align 4096 for RAFS v6, which the v6
 *      fixture's chunk table confirms (tests/test_rafs.py).
 * Reference callers: pkg/converter/tool/builder.go:122-124 passes
 * `--chunk-dict bootstrap=P` for PackOption.ChunkDictPath.
 */
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

typedef struct {
  const uint8_t *keys; /* digest array the ids index into */
  uint64_t *slot;      /* id + 1, 0 = empty */
  uint64_t mask;
} map_t;

static uint64_t h64(const uint8_t *d) {
  uint64_t x;
  memcpy(&x, d + 8, 8);
  return x * 0x9E3779B97F4A7C15ull;
}

static int map_init(map_t *m, const uint8_t *keys, uint64_t n) {
  uint64_t cap = 16;
  while (cap < 2 * n + 16) cap *= 2;
  m->slot = (uint64_t *)calloc(cap, sizeof(uint64_t));
  m->mask = cap - 1;
  m->keys = keys;
  return m->slot ? 0 : -1;
}

/* Returns the id stored for digest d, or UINT64_MAX. */
static uint64_t map_get(const map_t *m, const uint8_t *d) {
  for (uint64_t i = h64(d) & m->mask;; i = (i + 1) & m->mask) {
    uint64_t s = m->slot[i];
    if (!s) return UINT64_MAX;
    if (memcmp(m->keys + 32 * (s - 1), d, 32) == 0) return s - 1;
  }
}

/* Insert id if its digest is absent (first insertion wins). */
static void map_add(map_t *m, uint64_t id) {
  const uint8_t *d = m->keys + 32 * id;
  for (uint64_t i = h64(d) & m->mask;; i = (i + 1) & m->mask) {
    uint64_t s = m->slot[i];
    if (!s) { m->slot[i] = id + 1; return; }
    if (memcmp(m->keys + 32 * (s - 1), d, 32) == 0) return;
  }
}

uint64_t oracle_dedup(const uint8_t *digests, const uint32_t *sizes, uint64_t n,
                      const uint8_t *dict_digests, const uint32_t *dict_sizes,
                      const uint32_t *dict_blob, const uint32_t *dict_index,
                      const uint64_t *dict_uoff, uint64_t m, uint32_t align,
                      oracle_decision *out, uint32_t *own_blob) {
  map_t gdict = {0}, layered = {0};
  uint32_t max_inner = 0;
  for (uint64_t j = 0; j < m; j++)
    if (dict_blob[j] + 1 > max_inner) max_inner = dict_blob[j] + 1;
  uint32_t *real = (uint32_t *)malloc(sizeof(uint32_t) * (max_inner + 1));
  for (uint32_t b = 0; b <= max_inner; b++) real[b] = UINT32_MAX;
  if (m) {
    map_init(&gdict, dict_digests, m);
    for (uint64_t j = 0; j < m; j++) map_add(&gdict, j);
  }
  map_init(&layered, digests, n);
  uint32_t next_blob = 0, own = UINT32_MAX;
  uint64_t new_count = 0, cur = 0;
  if (align == 0) align = 1;
  for (uint64_t i = 0; i < n; i++) {
    const uint8_t *d = digests + 32 * i;
    oracle_decision *o = &out[i];
    memset(o, 0, sizeof *o);
    uint64_t e = m ? map_get(&gdict, d) : UINT64_MAX;
    if (e != UINT64_MAX && (dict_sizes[e] == 0 || dict_sizes[e] == sizes[i])) {
      uint32_t inner = dict_blob[e];
      if (real[inner] == UINT32_MAX) real[inner] = next_blob++;
      /* chunk.copy_from(cached_chunk): index and uncompressed offset are the
       * dict chunk's (its place in the dict's blob) */
      o->kind = ORACLE_DICT;
      o->ref = e;
      o->index = dict_index ? dict_index[e] : 0;
      o->blob_index = real[inner];
      o->uncompressed_offset = dict_uoff ? dict_uoff[e] : 0;
      continue;
    }
    uint64_t l = map_get(&layered, d);
    if (l != UINT64_MAX && (sizes[l] == 0 || sizes[l] == sizes[i])) {
      o->kind = ORACLE_INTRA;
      o->ref = l;
      o->index = out[l].index;
      o->blob_index = out[l].blob_index;
      o->uncompressed_offset = out[l].uncompressed_offset;
      continue;
    }
    if (own == UINT32_MAX) own = next_blob++;
    o->kind = ORACLE_NEW;
    o->ref = i;
    o->index = (uint32_t)new_count++;
    o->blob_index = own;
    o->uncompressed_offset = cur;
    cur = (cur + sizes[i] + align - 1) / align * align;
    map_add(&layered, i);
  }
  free(gdict.slot);
  free(layered.slot);
  free(real);
  if (own_blob) *own_blob = own;
  return new_count;
}
