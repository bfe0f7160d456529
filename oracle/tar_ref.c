/*
 * tar_ref.c — restated tar-rafs chunk enumeration.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Semantics restated from [nydus v2.3.0] builder/src/tarball.rs (external,
 * VERIFY), which the reference drives via `nydus-image create --type tar-rafs`
 * (pkg/converter/tool/builder.go:97-110) over a FIFO fed by packFromTar
 * (pkg/converter/convert_unix.go:443-539):
 *   - entries are read sequentially in stream order;
 *   - each regular file ('0', '\0', '7') of size S_f > 0 contributes chunks
 *     [k*S, min((k+1)*S, S_f)) of its data; chunks never span files;
 *   - directories, symlinks, hardlinks ('1' reuses its target's chunks),
 *     devices, fifos and zero-size files contribute no chunks; whiteouts are
 *     plain entries under `--whiteout-spec none` (builder.go:91-92);
 *   - GNU long name/link ('L'/'K') and PAX ('x', 'g') headers are metadata;
 *     a PAX "size" record overrides the next entry's size;
 *   - GNU sparse ('S') is rejected (nydus does not support it).
 * Header parsing follows POSIX.1-1988 ustar + the GNU base-256 size
 * extension (what Go's archive/tar writes for tests/converter_test.go:139-175).
 * The entry's data region is skipped by its header size for every type (the
 * Rust `tar` crate's rule).
 */
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

static int all_zero(const uint8_t *p, size_t n) {
  for (size_t i = 0; i < n; i++)
    if (p[i]) return 0;
  return 1;
}

static int parse_num(const uint8_t *f, size_t n, uint64_t *v) {
  if (f[0] & 0x80) { /* GNU base-256 */
    uint64_t x = f[0] & 0x7f;
    for (size_t i = 1; i < n; i++) {
      if (x >> 56) return -1;
      x = (x << 8) | f[i];
    }
    *v = x;
    return 0;
  }
  uint64_t x = 0;
  size_t i = 0;
  while (i < n && (f[i] == ' ' || f[i] == 0)) i++; /* leading pad */
  if (i == n) { *v = 0; return 0; }
  for (; i < n && f[i] >= '0' && f[i] <= '7'; i++) x = x * 8 + (uint64_t)(f[i] - '0');
  for (; i < n; i++)
    if (f[i] != ' ' && f[i] != 0) return -1;
  *v = x;
  return 0;
}

static int checksum_ok(const uint8_t *h) {
  uint64_t want;
  if (parse_num(h + 148, 8, &want)) return 0;
  uint64_t u = 0;
  int64_t s = 0;
  for (int i = 0; i < 512; i++) {
    uint8_t c = (i >= 148 && i < 156) ? ' ' : h[i];
    u += c;
    s += (int8_t)c;
  }
  return u == want || (uint64_t)s == want;
}

/* Parse the PAX "size" record out of an extended header body, if present. */
static int pax_size(const uint8_t *p, uint64_t n, uint64_t *size) {
  uint64_t i = 0;
  int found = 0;
  while (i < n) {
    uint64_t reclen = 0, j = i;
    while (j < n && p[j] >= '0' && p[j] <= '9') reclen = reclen * 10 + (p[j++] - '0');
    if (j >= n || p[j] != ' ' || reclen == 0 || i + reclen > n) break;
    const uint8_t *kv = p + j + 1, *end = p + i + reclen - 1; /* end at '\n' */
    if (end - kv > 5 && memcmp(kv, "size=", 5) == 0) {
      uint64_t v = 0;
      for (const uint8_t *q = kv + 5; q < end; q++) {
        if (*q < '0' || *q > '9') return -1;
        v = v * 10 + (uint64_t)(*q - '0');
      }
      *size = v;
      found = 1;
    }
    i += reclen;
  }
  return found;
}

int64_t oracle_tar_chunks(const uint8_t *tar, uint64_t len, uint32_t chunk_size,
                          oracle_chunk *out, uint64_t cap, uint64_t *n_files) {
  uint64_t pos = 0, n = 0, files = 0;
  int have_pax_size = 0;
  uint64_t pax_sz = 0;
  if (chunk_size == 0) return -1;
  while (pos + 512 <= len) {
    const uint8_t *h = tar + pos;
    if (all_zero(h, 512)) break; /* end-of-archive marker */
    if (!checksum_ok(h)) return -1;
    uint64_t size;
    if (parse_num(h + 124, 12, &size)) return -1;
    char type = (char)h[156];
    uint64_t data = pos + 512;
    if (type == 'x' || type == 'g') {
      if (data + size > len) return -2;
      if (type == 'x') {
        int r = pax_size(tar + data, size, &pax_sz);
        if (r < 0) return -1;
        if (r > 0) have_pax_size = 1;
      }
    } else if (type == 'L' || type == 'K') {
      if (data + size > len) return -2;
    } else if (type == 'S') {
      return -3;
    } else {
      if (have_pax_size) size = pax_sz;
      have_pax_size = 0;
      if (type == '0' || type == 0 || type == '7') {
        if (data + size > len) return -2;
        for (uint64_t off = 0; off < size; off += chunk_size) {
          uint64_t l = size - off < chunk_size ? size - off : chunk_size;
          if (n < cap) {
            out[n].offset = data + off;
            out[n].length = (uint32_t)l;
            out[n].file_index = (uint32_t)files;
            out[n].file_offset = off;
          }
          n++;
        }
        files++;
      }
    }
    uint64_t adv = (size + 511) / 512 * 512;
    if (data + adv < data) return -1;
    pos = data + adv;
  }
  if (n_files) *n_files = files;
  return (int64_t)n;
}

/* ---- helpers ------------------------------------------------------------ */
void oracle_digest_chunks(const uint8_t *data, const oracle_chunk *chunks,
                          uint64_t n, int digester, uint8_t *out) {
  for (uint64_t i = 0; i < n; i++) {
    if (digester == 1)
      oracle_sha256(data + chunks[i].offset, chunks[i].length, out + 32 * i);
    else
      oracle_blake3(data + chunks[i].offset, chunks[i].length, out + 32 * i);
  }
}
