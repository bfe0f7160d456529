// zran.cpp — gzip random-access index (zran.hpp) for OCIRef Packs.
#include "zran.hpp"

#include <string.h>
#include <zlib.h>

#include <algorithm>

namespace ngpu {

struct GzipIndexer::Impl {
  uint64_t span;
  z_stream zs{};
  bool live = false, ended = false;
  std::vector<ZranPoint> pts;
  std::vector<uint8_t> dict;   // every checkpoint's dictionary, back to back
  uint8_t ring[kWindow];       // the last kWindow bytes of output (circular)
  uint64_t out_total = 0, in_total = 0, last = 0;
  bool have_point = false;
  std::vector<uint8_t> obuf;
  Sha sha;
  uint8_t digest[32] = {};

  void remember(const uint8_t *p, uint64_t n) {  // output -> ring (out_total: before these bytes)
    uint64_t pos = out_total;  // stream offset of p[0]
    if (n >= kWindow) {
      pos += n - kWindow;
      p += n - kWindow;
      n = kWindow;
    }
    const uint64_t at = pos % kWindow;
    const uint64_t first = std::min(n, kWindow - at);
    memcpy(ring + at, p, first);
    memcpy(ring, p + first, n - first);
  }
  void add_point(uint32_t bits, uint32_t byte) {
    ZranPoint pt;
    pt.in_offset = in_total;
    pt.out_offset = out_total;
    pt.bits = bits;
    pt.byte = bits ? byte : 0;
    pt.dict_size = (uint32_t)std::min<uint64_t>(out_total, kWindow);
    pt.dict_offset = dict.size();
    dict.resize(dict.size() + pt.dict_size);
    // the dictionary is the window in output order, oldest byte first
    const uint64_t at = out_total % kWindow;
    if (pt.dict_size) {
      uint8_t *d = dict.data() + pt.dict_offset;
      if (pt.dict_size == kWindow) {
        memcpy(d, ring + at, kWindow - at);
        memcpy(d + (kWindow - at), ring, at);
      } else {
        memcpy(d, ring, pt.dict_size);  // the stream has not wrapped yet
      }
    }
    pts.push_back(pt);
    last = out_total;
    have_point = true;
  }
};

GzipIndexer::GzipIndexer(uint64_t span) : im_(new Impl) {
  im_->span = std::max<uint64_t>(span, kWindow);
}

GzipIndexer::~GzipIndexer() {
  if (im_->live) inflateEnd(&im_->zs);
}

int GzipIndexer::init() {
  // 15 + 16: gzip wrapper only (an OCI layer is a gzip stream)
  if (inflateInit2(&im_->zs, 15 + 16) != Z_OK) return host_fail(NGPU_EUNSUPP, "zlib inflateInit2 failed");
  im_->live = true;
  im_->obuf.resize(1 << 20);
  return 0;
}

int GzipIndexer::feed(const uint8_t *in, uint64_t n,
                      const std::function<int(const uint8_t *, uint64_t)> &out) {
  Impl &m = *im_;
  if (!m.live) return host_fail(NGPU_EINVAL, "gzip index: not initialised");
  m.sha.update(in, n);
  while (n) {
    if (m.ended)
      return host_fail(NGPU_EUNSUPP, "OCIRef: data after the end of the gzip stream "
                       "(multi-member gzip layers are not supported)");
    const uInt take = (uInt)std::min<uint64_t>(n, 1u << 30);
    m.zs.next_in = const_cast<Bytef *>(in);
    m.zs.avail_in = take;
    while (m.zs.avail_in && !m.ended) {
      m.zs.next_out = m.obuf.data();
      m.zs.avail_out = (uInt)m.obuf.size();
      const uInt before_in = m.zs.avail_in;
      // Z_BLOCK: stop at every deflate block boundary so a checkpoint can be
      // taken there (zran.c)
      const int ret = inflate(&m.zs, Z_BLOCK);
      const uint64_t produced = m.obuf.size() - m.zs.avail_out;
      if (ret != Z_OK && ret != Z_STREAM_END && !(ret == Z_BUF_ERROR && produced))
        return host_fail(NGPU_ETAR, "OCIRef: gzip stream error %d (%s)", ret,
                         m.zs.msg ? m.zs.msg : "corrupt deflate data");
      m.in_total += before_in - m.zs.avail_in;
      if (produced) {
        if (int rc = out(m.obuf.data(), produced)) return rc;
        m.remember(m.obuf.data(), produced);
        m.out_total += produced;
      }
      if (ret == Z_STREAM_END) {
        m.ended = true;
        break;
      }
      // data_type bit 7: at the end of a block header or block; bit 6: last
      // block -- a checkpoint at the first boundary and every `span` bytes
      if ((m.zs.data_type & 128) && !(m.zs.data_type & 64) &&
          (!m.have_point || m.out_total - m.last >= m.span))
        m.add_point((uint32_t)(m.zs.data_type & 7), m.zs.next_in[-1]);
    }
    const uint64_t used = take - m.zs.avail_in;
    if (m.ended && m.zs.avail_in)
      return host_fail(NGPU_EUNSUPP, "OCIRef: data after the end of the gzip stream "
                       "(multi-member gzip layers are not supported)");
    in += used;
    n -= used;
    if (!used && !m.ended) return host_fail(NGPU_ETAR, "OCIRef: gzip inflate made no progress");
  }
  return 0;
}

int GzipIndexer::finish() {
  Impl &m = *im_;
  if (!m.ended) return host_fail(NGPU_ETAR, "OCIRef: truncated gzip stream");
  m.sha.final(m.digest);
  return 0;
}

const std::vector<ZranPoint> &GzipIndexer::points() const { return im_->pts; }
const std::vector<uint8_t> &GzipIndexer::dicts() const { return im_->dict; }
uint64_t GzipIndexer::in_bytes() const { return im_->in_total; }
uint64_t GzipIndexer::out_bytes() const { return im_->out_total; }
void GzipIndexer::blob_digest(uint8_t out[32]) { memcpy(out, im_->digest, 32); }

uint64_t GzipIndexer::point_of(uint64_t off) const {
  const auto &p = im_->pts;
  auto it = std::upper_bound(p.begin(), p.end(), off,
                             [](uint64_t o, const ZranPoint &x) { return o < x.out_offset; });
  return it == p.begin() ? 0 : (uint64_t)(it - p.begin()) - 1;
}

uint64_t GzipIndexer::in_end_of(uint64_t end_out) const {
  // the block boundary of checkpoint x lies inside byte in_offset - 1 (or at
  // its end): bytes [.., in_offset) hold everything that produces output
  // before x.out_offset
  for (const ZranPoint &x : im_->pts)
    if (x.out_offset >= end_out) return x.in_offset;
  return im_->in_total;
}

int zran_extract(const uint8_t *gz, uint64_t gz_len, const ZranPoint &pt, const uint8_t *dict,
                 uint64_t skip, uint8_t *out, uint64_t len) {
  if (pt.in_offset > gz_len || (pt.bits && pt.in_offset == 0) || pt.bits > 7)
    return host_fail(NGPU_EFORMAT, "zran: checkpoint outside the blob");
  z_stream zs{};
  if (inflateInit2(&zs, -15) != Z_OK) return host_fail(NGPU_EUNSUPP, "zlib inflateInit2 failed");
  int rc = 0;
  uint64_t pos = pt.in_offset;
  if (pt.bits) {  // the boundary is inside byte in_offset - 1
    const int byte = gz[pt.in_offset - 1];
    if (inflatePrime(&zs, (int)pt.bits, byte >> (8 - pt.bits)) != Z_OK)
      rc = host_fail(NGPU_EFORMAT, "zran: inflatePrime failed");
  }
  if (!rc && pt.dict_size && inflateSetDictionary(&zs, dict, pt.dict_size) != Z_OK)
    rc = host_fail(NGPU_EFORMAT, "zran: inflateSetDictionary failed");
  std::vector<uint8_t> junk(skip ? std::min<uint64_t>(skip, 1 << 20) : 0);
  uint64_t got = 0;
  while (!rc && got < len) {
    uint8_t *dst;
    uint64_t room;
    if (skip) {
      dst = junk.data();
      room = std::min<uint64_t>(skip, junk.size());
    } else {
      dst = out + got;
      room = len - got;
    }
    zs.next_out = dst;
    zs.avail_out = (uInt)std::min<uint64_t>(room, 1u << 30);
    const uInt want = zs.avail_out;
    if (!zs.avail_in) {
      const uint64_t chunk = std::min<uint64_t>(gz_len - pos, 1u << 20);
      zs.next_in = const_cast<Bytef *>(gz + pos);
      zs.avail_in = (uInt)chunk;
      pos += chunk;
    }
    const int r = inflate(&zs, Z_NO_FLUSH);
    const uint64_t made = want - zs.avail_out;
    if (skip) skip -= made;
    else got += made;
    if (r == Z_STREAM_END && (skip || got < len)) rc = host_fail(NGPU_EFORMAT, "zran: stream ended early");
    else if (r != Z_OK && r != Z_STREAM_END && !(r == Z_BUF_ERROR && made))
      rc = host_fail(NGPU_EFORMAT, "zran: inflate error %d", r);
    else if (!made && pos >= gz_len && !zs.avail_in)
      rc = host_fail(NGPU_EFORMAT, "zran: ran out of compressed data");
  }
  inflateEnd(&zs);
  return rc;
}

}  // namespace ngpu

// ngpu_ref_chunk_read: the reader side of an OCIRef layer -- what nydusd does
// with a targz-ref blob: find chunk `index` of the layer's own blob in its
// blob.meta (chunk-info entry -> checkpoint), then inflate it out of the
// original gzip blob from that checkpoint (zran_extract).
extern "C" int ngpu_ref_chunk_read(const void *gz, uint64_t gz_len, const void *blob_meta,
                                   uint64_t meta_len, uint32_t index, void *out, uint32_t cap,
                                   uint32_t *len_out) {
  using namespace ngpu;
  if (!gz || !blob_meta || !out || !len_out) return NGPU_EINVAL;
  return guarded([&]() -> int {
    const uint8_t *m = (const uint8_t *)blob_meta;
    if (meta_len < 4096) return host_fail(NGPU_EFORMAT, "blob.meta too short");
    const uint8_t *h = m + meta_len - 4096;  // BlobCompressionContextHeader (last 4 KiB)
    uint32_t magic, feat, algo, entries;
    uint64_t zt_off, zt_size, zt_cnt, zd_off, zd_size;
    memcpy(&magic, h, 4);
    memcpy(&feat, h + 4, 4);
    memcpy(&algo, h + 8, 4);
    memcpy(&entries, h + 12, 4);
    memcpy(&zt_off, h + 40, 8);
    memcpy(&zt_size, h + 48, 8);
    memcpy(&zt_cnt, h + 56, 8);
    memcpy(&zd_off, h + 64, 8);
    memcpy(&zd_size, h + 72, 8);
    const uint64_t body = meta_len - 4096;
    if (magic != 0xB10BB10Bu || !(feat & 0x8) || algo != 0)
      return host_fail(NGPU_EFORMAT, "blob.meta: not an uncompressed zran chunk-info array");
    if (index >= entries || (uint64_t)entries * 24 > body || zt_off > body || zt_size > body - zt_off ||
        zt_size % 40 || zt_cnt != zt_size / 40 || zd_off > body || zd_size > body - zd_off)
      return host_fail(NGPU_EFORMAT, "blob.meta: bad zran table bounds");
    uint64_t w[3];
    memcpy(w, m + 24ull * index, 24);
    if (!((w[0] >> 56) & 0x2)) return host_fail(NGPU_EFORMAT, "chunk %u is not a zran chunk", index);
    const uint32_t usize = (uint32_t)((w[0] >> 32) & 0xFFFFFF) + 1;
    const uint64_t ctx = w[2] >> 32, ctx_off = w[2] & 0xFFFFFFFFull;
    if (ctx >= zt_cnt) return host_fail(NGPU_EFORMAT, "chunk %u: checkpoint %llu of %llu", index,
                                        (unsigned long long)ctx, (unsigned long long)zt_cnt);
    if (usize > cap) return host_fail(NGPU_EINVAL, "chunk %u: %u bytes, buffer %u", index, usize, cap);
    const uint8_t *r = m + zt_off + 40 * ctx;
    ZranPoint pt{};
    memcpy(&pt.in_offset, r, 8);
    memcpy(&pt.out_offset, r + 8, 8);
    pt.byte = r[24];
    pt.bits = r[25];
    memcpy(&pt.dict_size, r + 28, 4);
    memcpy(&pt.dict_offset, r + 32, 8);
    if (pt.dict_size > GzipIndexer::kWindow || pt.dict_offset > zd_size ||
        pt.dict_size > zd_size - pt.dict_offset)
      return host_fail(NGPU_EFORMAT, "chunk %u: dictionary outside blob.meta", index);
    if (int rc = zran_extract((const uint8_t *)gz, gz_len, pt, m + zd_off + pt.dict_offset, ctx_off,
                              (uint8_t *)out, usize))
      return rc;
    *len_out = usize;
    return 0;
  });
}
