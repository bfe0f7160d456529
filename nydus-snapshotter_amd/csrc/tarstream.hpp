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
#include <stdlib.h>
#include <string.h>

#include <string>
#include <utility>
#include <vector>

#include "nydus_gpu.h"

namespace ngpu {

// One tar entry's metadata, for the RAFS inode tree (TarScanner::record).
// GNU long names / links and PAX path, linkpath, size, mtime, uid, gid and
// SCHILY.xattr.* records are applied.  type: '0' regular (also '\0', '7'),
// '1' hardlink, '2' symlink, '3' char, '4' block, '5' dir, '6' fifo.
struct TarEntry {
  std::string path;   // normalised: no leading "./" or "/", no trailing "/"; "" = root
  std::string link;   // symlink target (as written), or hardlink target (normalised)
  char type = '0';
  uint32_t mode = 0, uid = 0, gid = 0, devmajor = 0, devminor = 0;
  int64_t mtime = 0;
  uint32_t mtime_ns = 0;
  uint64_t size = 0;
  int64_t file_index = -1;  // regular files: ordinal among regular files (ngpu_chunk.file_index)
  std::vector<std::pair<std::string, std::string>> xattrs;
};

inline std::string tar_normalize(std::string p) {
  for (;;) {
    if (p.compare(0, 2, "./") == 0) p.erase(0, 2);
    else if (!p.empty() && p[0] == '/') p.erase(0, 1);
    else break;
  }
  while (!p.empty() && p.back() == '/') p.pop_back();
  if (p == ".") p.clear();
  return p;
}

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
  // Also collect every entry's metadata (the RAFS inode tree); off by default:
  // the digest path needs only the chunks.
  void record(std::vector<TarEntry> *entries) { rec_ = entries; }

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
            if (meta_kind_ == 'L' || meta_kind_ == 'K') {  // GNU long name / link (recording)
              std::string &dst = meta_kind_ == 'L' ? long_name_ : long_link_;
              dst.assign(pax_.c_str());  // NUL-terminated in the archive
              have_long_ |= meta_kind_ == 'L' ? 1 : 2;
            } else {
              const int r = pax_size();
              if (r < 0) return err_ = NGPU_ETAR;
            }
            enter_skip(pad_, meta_kind_ != 'x');
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
        meta_kind_ = 'x';
        st_ = size ? PAX : HDR;
        if (!size) enter_skip(0, false);
        return 0;
      case 'L':
      case 'K':
        // a long name / link the tree needs but will not capture would leave
        // the next entry under its truncated ustar name: fail like Go's
        // archive/tar (ErrFieldTooLong)
        if (rec_ && size > (1u << 20)) return NGPU_ETAR;
        if (rec_) {  // captured: the next entry's long name / link
          pax_.clear();
          remain_ = size;
          pad_ = padded - size;
          meta_kind_ = type;
          st_ = size ? PAX : HDR;
          if (!size) enter_skip(0, true);
          return 0;
        }
        enter_skip(padded, true);
        return 0;
      case 'g':
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
    if (rec_) record_entry(type, size);
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
  // When recording, path / linkpath / mtime / uid / gid / SCHILY.xattr.* are
  // kept for the next entry too.
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
      } else if (rec_) {
        const uint8_t *eq = (const uint8_t *)memchr(kv, '=', end - kv);
        if (eq) pax_kv_.emplace_back(std::string((const char *)kv, eq - kv),
                                     std::string((const char *)eq + 1, end - eq - 1));
      }
      i += rl;
    }
    return 0;
  }

  static std::string field(const uint8_t *f, size_t n) {
    return std::string(reinterpret_cast<const char *>(f), strnlen(reinterpret_cast<const char *>(f), n));
  }

  // The entry of the header in hdr_ (type, size already PAX-resolved).
  void record_entry(char type, uint64_t size) {
    TarEntry e;
    const bool posix = memcmp(hdr_ + 257, "ustar\0", 6) == 0;
    std::string name = field(hdr_, 100);
    if (posix && hdr_[345]) name = field(hdr_ + 345, 155) + "/" + name;
    std::string link = field(hdr_ + 157, 100);
    if (have_long_ & 1) name = long_name_;
    if (have_long_ & 2) link = long_link_;
    uint64_t v = 0;
    e.mode = number(hdr_ + 100, 8, &v) ? (uint32_t)(v & 07777) : 0;
    e.uid = number(hdr_ + 108, 8, &v) ? (uint32_t)v : 0;
    e.gid = number(hdr_ + 116, 8, &v) ? (uint32_t)v : 0;
    e.mtime = number(hdr_ + 136, 12, &v) ? (int64_t)v : 0;
    if (posix || memcmp(hdr_ + 257, "ustar ", 6) == 0) {
      e.devmajor = number(hdr_ + 329, 8, &v) ? (uint32_t)v : 0;
      e.devminor = number(hdr_ + 337, 8, &v) ? (uint32_t)v : 0;
    }
    for (auto &kv : pax_kv_) {
      if (kv.first == "path") name = kv.second;
      else if (kv.first == "linkpath") link = kv.second;
      else if (kv.first == "uid") e.uid = (uint32_t)strtoull(kv.second.c_str(), nullptr, 10);
      else if (kv.first == "gid") e.gid = (uint32_t)strtoull(kv.second.c_str(), nullptr, 10);
      else if (kv.first == "mtime") {
        const char *s = kv.second.c_str();
        char *dot = nullptr;
        e.mtime = strtoll(s, &dot, 10);
        if (dot && *dot == '.') {  // fraction: nanoseconds, 9 digits
          uint32_t ns = 0;
          int d = 0;
          for (const char *q = dot + 1; *q >= '0' && *q <= '9' && d < 9; ++q, ++d) ns = ns * 10 + (*q - '0');
          for (; d < 9; ++d) ns *= 10;
          e.mtime_ns = ns;
        }
      } else if (kv.first.compare(0, 13, "SCHILY.xattr.") == 0) {
        e.xattrs.emplace_back(kv.first.substr(13), kv.second);
      }
    }
    pax_kv_.clear();
    have_long_ = 0;
    e.size = size;
    switch (type) {
      case '\0': case '7': case '0': e.type = '0'; e.file_index = (int64_t)files_; break;
      case '1': e.type = '1'; e.size = 0; link = tar_normalize(link); break;
      case '2': case '3': case '4': case '5': case '6': e.type = type; break;
      default: return;  // other types carry no inode (as they carry no chunks)
    }
    if (e.type != '0') e.size = e.type == '2' ? link.size() : 0;
    e.path = tar_normalize(name);
    e.link = std::move(link);
    rec_->push_back(std::move(e));
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
  // entry recording (record())
  std::vector<TarEntry> *rec_ = nullptr;
  char meta_kind_ = 'x';
  int have_long_ = 0;  // bit 0: long_name_, bit 1: long_link_ pending
  std::string long_name_, long_link_;
  std::vector<std::pair<std::string, std::string>> pax_kv_;
};

}  // namespace ngpu
