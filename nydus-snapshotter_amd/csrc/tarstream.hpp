// tarstream.hpp — incremental tar-rafs chunk scanner (SURVEY.md §8(a) a3,
// §8(f) next-1).  Bytes may arrive in any split (the reference streams the
// layer tar through a FIFO in 1 MiB buffers: pkg/converter/convert_unix.go:
// 56-61, 478-486); the scanner reports every chunk when it starts (its full
// length is known from the file size) and hands file-data bytes to a sink.
//
// Rules (what `nydus-image create --type tar-rafs` consumes,
// pkg/converter/tool/builder.go:97-110): POSIX ustar headers with checksum,
// GNU base-256 sizes, GNU long name/link ('L'/'K') and PAX global ('g')
// headers skipped, PAX extended ('x') "size" overrides the next entry's size,
// GNU sparse ('S') unsupported; regular files ('0', '\0', '7') of size > 0
// are cut into [k*S, min((k+1)*S, size)); other entry types carry no chunks
// (hardlinks reuse their target's chunks; `--whiteout-spec none` makes
// whiteouts plain entries, builder.go:91-92); a zero block ends the archive.
#pragma once

#include <stdint.h>
#include <string.h>

#include <string>

#include "nydus_gpu.h"

namespace ngpu {

struct TarSink {
  virtual ~TarSink() = default;
  // A chunk starts at stream offset `off` (its `len` bytes follow as data()).
  virtual int chunk(uint64_t off, uint32_t len, uint32_t file_index, uint64_t file_offset) = 0;
  // File-data bytes of the current chunk, in order.
  virtual int data(const uint8_t *p, uint64_t len) = 0;
};

class TarScanner {
 public:
  explicit TarScanner(uint32_t chunk_size) : S_(chunk_size) {}

  uint64_t files() const { return files_; }
  uint64_t chunks() const { return chunks_; }
  uint64_t offset() const { return pos_; }

  // Feed the next bytes of the stream.  Returns 0 or a negative NGPU_E*.
  int feed(const uint8_t *p, uint64_t len, TarSink &sink) {
    if (err_) return err_;
    while (len) {
      switch (st_) {
        case HDR: {
          const uint64_t take = min64(512 - hdr_fill_, len);
          memcpy(hdr_ + hdr_fill_, p, take);
          hdr_fill_ += (uint32_t)take;
          adv(p, len, take);
          if (hdr_fill_ == 512) {
            hdr_fill_ = 0;
            const int rc = header();
            if (rc) return err_ = rc;
          }
          break;
        }
        case DATA: {
          if (file_off_ % S_ == 0) {
            const uint64_t cl = min64(S_, file_size_ - file_off_);
            const int rc = sink.chunk(pos_, (uint32_t)cl, (uint32_t)files_, file_off_);
            if (rc) return err_ = rc;
            ++chunks_;
          }
          const uint64_t to_chunk_end = S_ - file_off_ % S_;
          const uint64_t take = min64(min64(remain_, len), to_chunk_end);
          const int rc = sink.data(p, take);
          if (rc) return err_ = rc;
          adv(p, len, take);
          remain_ -= take;
          file_off_ += take;
          if (remain_ == 0) {
            ++files_;
            enter_skip(pad_, false);
          }
          break;
        }
        case PAX: {
          const uint64_t take = min64(remain_, len);
          pax_.append(reinterpret_cast<const char *>(p), take);
          adv(p, len, take);
          remain_ -= take;
          if (remain_ == 0) {
            const int r = pax_size();
            if (r < 0) return err_ = NGPU_ETAR;
            enter_skip(pad_, false);
          }
          break;
        }
        case SKIP: {
          const uint64_t take = min64(remain_, len);
          adv(p, len, take);
          remain_ -= take;
          if (remain_ == 0) st_ = HDR;
          break;
        }
        case END:
          adv(p, len, len);
          break;
      }
    }
    return 0;
  }

  // End of stream: truncated file data / metadata is an error.
  int finish() {
    if (err_) return err_;
    if (st_ == DATA || st_ == PAX || (st_ == SKIP && skip_meta_)) return err_ = NGPU_ETAR;
    return 0;
  }

 private:
  enum State { HDR, DATA, PAX, SKIP, END };

  static uint64_t min64(uint64_t a, uint64_t b) { return a < b ? a : b; }
  void adv(const uint8_t *&p, uint64_t &len, uint64_t n) {
    p += n;
    len -= n;
    pos_ += n;
  }
  void enter_skip(uint64_t n, bool meta) {
    remain_ = n;
    skip_meta_ = meta;
    st_ = n ? SKIP : HDR;
  }

  static bool number(const uint8_t *f, size_t n, uint64_t *v) {
    if (f[0] & 0x80) {  // GNU base-256
      uint64_t x = f[0] & 0x7f;
      for (size_t i = 1; i < n; ++i) {
        if (x >> 56) return false;
        x = (x << 8) | f[i];
      }
      *v = x;
      return true;
    }
    size_t i = 0;
    while (i < n && (f[i] == ' ' || f[i] == 0)) ++i;
    uint64_t x = 0;
    for (; i < n && f[i] >= '0' && f[i] <= '7'; ++i) x = (x << 3) | (uint64_t)(f[i] - '0');
    for (; i < n; ++i)
      if (f[i] != ' ' && f[i] != 0) return false;
    *v = x;
    return true;
  }

  // ustar checksum: the unsigned (or, for old tars, signed) byte sum of the
  // header with the checksum field read as 8 spaces.  SWAR over 64-bit words
  // (the per-byte loop cost ~0.75 us per header: 0.27 ms of a 10 MB layer's
  // walk); the field's bytes are taken out again at the end.
  bool checksum_ok() const {
    uint64_t want;
    if (!number(hdr_ + 148, 8, &want)) return false;
    uint64_t w[64];
    memcpy(w, hdr_, 512);
    uint64_t s16 = 0, hi8 = 0;  // 4 x 16-bit pair sums; 8 x 8-bit high-bit counts
    for (int i = 0; i < 64; ++i) {
      s16 += (w[i] & 0x00FF00FF00FF00FFull) + ((w[i] >> 8) & 0x00FF00FF00FF00FFull);
      hi8 += (w[i] >> 7) & 0x0101010101010101ull;
    }
    const uint64_t hi16 = (hi8 & 0x00FF00FF00FF00FFull) + ((hi8 >> 8) & 0x00FF00FF00FF00FFull);
    uint64_t u = (s16 & 0xFFFF) + ((s16 >> 16) & 0xFFFF) + ((s16 >> 32) & 0xFFFF) + (s16 >> 48);
    uint64_t hi = (hi16 & 0xFFFF) + ((hi16 >> 16) & 0xFFFF) + ((hi16 >> 32) & 0xFFFF) + (hi16 >> 48);
    for (int i = 148; i < 156; ++i) {
      u -= hdr_[i];
      hi -= hdr_[i] >> 7;
    }
    u += 8 * ' ';
    const int64_t sgn = (int64_t)u - 256 * (int64_t)hi;  // bytes >= 0x80 counted negative
    return u == want || (uint64_t)sgn == want;
  }

  int header() {
    bool zero = true;
    for (int i = 0; i < 512 && zero; ++i) zero = hdr_[i] == 0;
    if (zero) {
      st_ = END;
      return 0;
    }
    if (!checksum_ok()) return NGPU_ETAR;
    uint64_t size;
    if (!number(hdr_ + 124, 12, &size)) return NGPU_ETAR;
    const char type = (char)hdr_[156];
    const uint64_t padded = (size + 511) & ~511ull;
    if (padded < size) return NGPU_ETAR;
    switch (type) {
      case 'x':
        pax_.clear();
        remain_ = size;
        pad_ = padded - size;
        st_ = size ? PAX : HDR;
        if (!size) enter_skip(0, false);
        return 0;
      case 'g':
      case 'L':
      case 'K':
        enter_skip(padded, true);
        return 0;
      case 'S':
        return NGPU_EUNSUPP;
      default:
        break;
    }
    if (have_pax_) size = pax_sz_;
    have_pax_ = false;
    const uint64_t pad = ((size + 511) & ~511ull) - size;
    if (type == '0' || type == '\0' || type == '7') {
      if (size == 0) {
        ++files_;
        enter_skip(0, false);
        return 0;
      }
      file_size_ = size;
      file_off_ = 0;
      remain_ = size;
      pad_ = pad;
      st_ = DATA;
      return 0;
    }
    enter_skip(size + pad, false);
    return 0;
  }

  // PAX records "len key=value\n"; a "size" record overrides the next entry.
  int pax_size() {
    const uint8_t *p = reinterpret_cast<const uint8_t *>(pax_.data());
    const uint64_t n = pax_.size();
    uint64_t i = 0;
    while (i < n) {
      uint64_t rl = 0, j = i;
      while (j < n && p[j] >= '0' && p[j] <= '9') rl = rl * 10 + (p[j++] - '0');
      if (j >= n || p[j] != ' ' || rl == 0 || i + rl > n) break;
      const uint8_t *kv = p + j + 1, *end = p + i + rl - 1;
      if (end - kv > 5 && memcmp(kv, "size=", 5) == 0) {
        uint64_t v = 0;
        for (const uint8_t *q = kv + 5; q < end; ++q) {
          if (*q < '0' || *q > '9') return -1;
          v = v * 10 + (uint64_t)(*q - '0');
        }
        pax_sz_ = v;
        have_pax_ = true;
      }
      i += rl;
    }
    return 0;
  }

  const uint32_t S_;
  State st_ = HDR;
  uint8_t hdr_[512];
  uint32_t hdr_fill_ = 0;
  uint64_t pos_ = 0, remain_ = 0, pad_ = 0;
  uint64_t file_size_ = 0, file_off_ = 0;
  uint64_t files_ = 0, chunks_ = 0;
  bool skip_meta_ = false, have_pax_ = false;
  uint64_t pax_sz_ = 0;
  std::string pax_;
  int err_ = 0;
};

}  // namespace ngpu
