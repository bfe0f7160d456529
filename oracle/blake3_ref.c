/*
 * blake3_ref.c — scalar BLAKE3-256 restated from the BLAKE3 specification
 * (Aumasson, Neves, O'Connor, Wilcox-O'Hearn, 2020, §2.1-2.6).
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Written for clarity, not speed:
 * the tree is built by the spec's recursive left-complete rule (left subtree
 * = largest power-of-two number of 1 KiB chunks strictly below the total).
 *
 * Reference call site: nydus-image's RafsDigest::from_buf(buf, Blake3)
 * ([nydus v2.3.0] utils/src/digest.rs, external) — blake3 is the default
 * digester because pkg/converter/tool/builder.go:78-146 never passes
 * --digester.  Pinned against ROCm LLVM's vendored official BLAKE3 v1.8.2 in
 * tests/golden/make_golden.py.
 */
#include <string.h>

#include "oracle.h"

static const uint32_t IV[8] = {0x6A09E667u, 0xBB67AE85u, 0x3C6EF372u,
                               0xA54FF53Au, 0x510E527Fu, 0x9B05688Cu,
                               0x1F83D9ABu, 0x5BE0CD19u};
static const unsigned PERM[16] = {2, 6,  3,  10, 7,  0,  4,  13,
                                  1, 11, 12, 5,  9, 14, 15, 8};
enum { CHUNK_START = 1, CHUNK_END = 2, PARENT = 4, ROOT = 8 };

static uint32_t rotr(uint32_t x, unsigned n) { return (x >> n) | (x << (32 - n)); }

static void g(uint32_t *s, int a, int b, int c, int d, uint32_t mx, uint32_t my) {
  s[a] = s[a] + s[b] + mx;
  s[d] = rotr(s[d] ^ s[a], 16);
  s[c] = s[c] + s[d];
  s[b] = rotr(s[b] ^ s[c], 12);
  s[a] = s[a] + s[b] + my;
  s[d] = rotr(s[d] ^ s[a], 8);
  s[c] = s[c] + s[d];
  s[b] = rotr(s[b] ^ s[c], 7);
}

/* compress -> first 8 output words (what a CV or a 32-byte root needs). */
static void compress(const uint32_t cv[8], const uint32_t m_in[16],
                     uint64_t counter, uint32_t block_len, uint32_t flags,
                     uint32_t out[8]) {
  uint32_t s[16], m[16], t[16];
  memcpy(m, m_in, sizeof m);
  for (int i = 0; i < 8; i++) s[i] = cv[i];
  for (int i = 0; i < 4; i++) s[8 + i] = IV[i];
  s[12] = (uint32_t)counter;
  s[13] = (uint32_t)(counter >> 32);
  s[14] = block_len;
  s[15] = flags;
  for (int r = 0; r < 7; r++) {
    g(s, 0, 4, 8, 12, m[0], m[1]);
    g(s, 1, 5, 9, 13, m[2], m[3]);
    g(s, 2, 6, 10, 14, m[4], m[5]);
    g(s, 3, 7, 11, 15, m[6], m[7]);
    g(s, 0, 5, 10, 15, m[8], m[9]);
    g(s, 1, 6, 11, 12, m[10], m[11]);
    g(s, 2, 7, 8, 13, m[12], m[13]);
    g(s, 3, 4, 9, 14, m[14], m[15]);
    for (int i = 0; i < 16; i++) t[i] = m[PERM[i]];
    memcpy(m, t, sizeof m);
  }
  for (int i = 0; i < 8; i++) out[i] = s[i] ^ s[i + 8];
}

static void load_block(const uint8_t *p, size_t len, uint32_t m[16]) {
  uint8_t buf[64];
  memset(buf, 0, sizeof buf);
  memcpy(buf, p, len);
  for (int i = 0; i < 16; i++)
    m[i] = (uint32_t)buf[4 * i] | ((uint32_t)buf[4 * i + 1] << 8) |
           ((uint32_t)buf[4 * i + 2] << 16) | ((uint32_t)buf[4 * i + 3] << 24);
}

/* One 1 KiB BLAKE3 chunk (called a "leaf" here to avoid clashing with nydus
 * chunks).  len in [0, 1024]; root marks the final block ROOT. */
static void leaf_cv(const uint8_t *p, size_t len, uint64_t counter, int root,
                    uint32_t out[8]) {
  uint32_t cv[8], m[16];
  memcpy(cv, IV, sizeof cv);
  size_t nblocks = len == 0 ? 1 : (len + 63) / 64;
  for (size_t b = 0; b < nblocks; b++) {
    size_t bl = (b + 1 < nblocks) ? 64 : len - 64 * b;
    uint32_t flags = 0;
    if (b == 0) flags |= CHUNK_START;
    if (b + 1 == nblocks) {
      flags |= CHUNK_END;
      if (root) flags |= ROOT;
    }
    load_block(p + 64 * b, bl, m);
    compress(cv, m, counter, (uint32_t)bl, flags, cv);
  }
  memcpy(out, cv, sizeof cv);
}

static void parent_cv(const uint32_t l[8], const uint32_t r[8], int root,
                      uint32_t out[8]) {
  uint32_t m[16];
  memcpy(m, l, 32);
  memcpy(m + 8, r, 32);
  compress(IV, m, 0, 64, PARENT | (root ? ROOT : 0), out);
}

/* Subtree over leaves [first, first+n) of the input. */
static void subtree(const uint8_t *data, size_t len, uint64_t first, uint64_t n,
                    int root, uint32_t out[8]) {
  if (n == 1) {
    size_t off = (size_t)first * 1024;
    size_t l = len - off < 1024 ? len - off : 1024;
    leaf_cv(data + off, l, first, root, out);
    return;
  }
  uint64_t left = 1;
  while (left * 2 < n) left *= 2; /* largest power of two < n */
  uint32_t lc[8], rc[8];
  subtree(data, len, first, left, 0, lc);
  subtree(data, len, first + left, n - left, 0, rc);
  parent_cv(lc, rc, root, out);
}

void oracle_blake3(const uint8_t *data, size_t len, uint8_t out[32]) {
  uint64_t n = len == 0 ? 1 : (len + 1023) / 1024;
  uint32_t h[8];
  subtree(data, len, 0, n, 1, h);
  for (int i = 0; i < 8; i++) {
    out[4 * i] = (uint8_t)h[i];
    out[4 * i + 1] = (uint8_t)(h[i] >> 8);
    out[4 * i + 2] = (uint8_t)(h[i] >> 16);
    out[4 * i + 3] = (uint8_t)(h[i] >> 24);
  }
}
