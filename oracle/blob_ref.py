"""TEST INFRASTRUCTURE ONLY — CPU restatement of the reference's nydus blob
reader and of the on-disk rules the blob writer must satisfy.  Only tests/
may import this module; the product (libnydusgpu.so) never does.

Restates (pkg/converter/convert_unix.go):
* seekFileByTarHeader  :162-213 — walk `data | tar_header` pairs from the tail;
* seekFileByTOC        :219-276 — the last entry is `rafs.blob.toc`, 128-B
                                  TOCEntry records (types.go:147-163, the Go
                                  struct reads the first 124 B of each);
* seekFile / UnpackEntry :284-320 — TOC first, tar-header walk as fallback;
* calcBlobTOCDigest    :541-555 — sha256 of the TOC entry data.
Compressors: zstd (the only compressed entry kind the Go reader accepts) and,
for chunk data, lz4_block — decoded with the system libzstd.so.1 /
liblz4.so.1 through ctypes.

Pinning: the reader logic is the reference's own Go code restated line by
line; the chunk-record rules (raw storage when compression does not shrink a
chunk, compressed offsets back to back, blob compressed size = end of chunk
data, uncompressed size 4K-rounded) are the ones the reference v6 fixture
pkg/filesystem/testdata/v6-bootstrap-chunk-pos-438272.tar.gz obeys
(tests/test_blob.py checks them on the fixture itself).
"""
from __future__ import annotations

import ctypes
import hashlib
import struct
import tarfile

import numpy as np

ENTRY_BLOB = "image.blob"        # convert_unix.go:45
ENTRY_BOOTSTRAP = "image.boot"   # :46
ENTRY_TOC = "rafs.blob.toc"      # :49
COMPRESSOR_NONE, COMPRESSOR_ZSTD, COMPRESSOR_LZ4_BLOCK = 0x1, 0x2, 0x4  # types.go:27-30
COMPRESSOR_MASK = 0xF

TOC_ENTRY = struct.Struct("<II16s32sQQQ44s")  # the Go TOCEntry (124 B)
TOC_ENTRY_SIZE = 128                          # entrySize, convert_unix.go:220


class NotFound(Exception):
    """ErrNotFound (types.go:33-35)."""


def _hdr(block: bytes):
    try:
        ti = tarfile.TarInfo.frombuf(block, "utf-8", "surrogateescape")
    except tarfile.TarError as e:
        raise ValueError(f"parse nydus tar header: {e}") from e
    return ti.name, ti.size


def seek_file_by_tar_header(ra: bytes, target: str, max_size=None):
    """convert_unix.go:162-213 -> (offset, size) of the entry data."""
    header_size = 512
    if header_size > len(ra):
        raise ValueError(f"invalid nydus tar size {len(ra)}")
    cur = len(ra) - header_size
    while True:
        name, size = _hdr(ra[cur:cur + header_size])
        if cur < size:
            raise ValueError(f"invalid nydus tar data, name {name}, size {size}")
        if name == target:
            if max_size is not None and size > max_size:
                raise ValueError(f"invalid nydus tar size {len(ra)}")
            return cur - size, size
        cur = cur - size - header_size
        if cur < 0:
            break
    raise NotFound(f"can't find target {target} by seeking tar")


def parse_toc(data: bytes):
    if len(data) % TOC_ENTRY_SIZE:
        raise ValueError(f"invalid entries length {len(data)}")
    out = []
    for i in range(len(data) // TOC_ENTRY_SIZE):
        f = TOC_ENTRY.unpack_from(data, i * TOC_ENTRY_SIZE)
        # TOCEntry.GetName (types.go:181-191): bytes up to the first NUL, one rune each
        name = "".join(chr(c) for c in f[2].split(b"\0", 1)[0])
        out.append({"flags": f[0], "name": name, "uncompressed_digest": f[3].hex(),
                    "compressed_offset": f[4], "compressed_size": f[5], "uncompressed_size": f[6]})
    return out


def seek_file_by_toc(ra: bytes, target: str):
    """convert_unix.go:219-276 -> (entry data, toc entry)."""
    off, size = seek_file_by_tar_header(ra, ENTRY_TOC, max_size=1 << 20)
    for e in parse_toc(ra[off:off + size]):
        if e["name"] != target:
            continue
        comp = e["flags"] & COMPRESSOR_MASK
        if comp not in (COMPRESSOR_NONE, COMPRESSOR_ZSTD, COMPRESSOR_LZ4_BLOCK):
            raise ValueError(f"unsupported compressor, entry flags {e['flags']:x}")
        # io.NewSectionReader + io.Copy: a range past the end yields the bytes
        # that exist (EOF ends the copy without an error)
        raw = ra[e["compressed_offset"]:e["compressed_offset"] + e["compressed_size"]]
        if comp == COMPRESSOR_ZSTD:
            # zstd.NewReader(sr) + io.Copy: the frame(s) decide the length;
            # the entry's uncompressed_size is never read
            data = zstd_stream_decompress(raw)
        elif comp == COMPRESSOR_NONE:
            data = raw
        else:
            raise ValueError(f"unsupported compressor {comp:x}")
        return data, e
    raise NotFound(f"can't find target {target} by seeking TOC")


def unpack_entry(ra: bytes, target: str):
    """seekFile / UnpackEntry (convert_unix.go:284-320) -> (data, toc entry|None)."""
    try:
        return seek_file_by_toc(ra, target)
    except NotFound:
        pass
    off, size = seek_file_by_tar_header(ra, target)
    return ra[off:off + size], None


def calc_blob_toc_digest(ra: bytes) -> str:
    """convert_unix.go:541-555."""
    off, size = seek_file_by_tar_header(ra, ENTRY_TOC, max_size=1 << 20)
    return hashlib.sha256(ra[off:off + size]).hexdigest()


# ---- decompressors (system libraries, ctypes) --------------------------------
_zstd = _lz4 = None


def _load_zstd():
    global _zstd
    if _zstd is None:
        z = ctypes.CDLL("libzstd.so.1")
        z.ZSTD_decompress.restype = ctypes.c_size_t
        z.ZSTD_decompress.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                      ctypes.c_size_t]
        z.ZSTD_isError.argtypes = [ctypes.c_size_t]
        z.ZSTD_createDStream.restype = ctypes.c_void_p
        z.ZSTD_freeDStream.argtypes = [ctypes.c_void_p]
        z.ZSTD_decompressStream.restype = ctypes.c_size_t
        z.ZSTD_decompressStream.argtypes = [ctypes.c_void_p, ctypes.POINTER(_ZBuf),
                                            ctypes.POINTER(_ZBuf)]
        _zstd = z
    return _zstd


class _ZBuf(ctypes.Structure):
    _fields_ = [("ptr", ctypes.c_void_p), ("size", ctypes.c_size_t), ("pos", ctypes.c_size_t)]


def zstd_decompress(src: bytes, usize: int) -> bytes:
    """One frame of exactly usize bytes (chunk data: the record's size)."""
    _load_zstd()
    dst = ctypes.create_string_buffer(max(1, usize))
    r = _zstd.ZSTD_decompress(dst, usize, src, len(src))
    if _zstd.ZSTD_isError(r) or r != usize:
        raise ValueError("zstd decompression failed")
    return dst.raw[:usize]


def zstd_stream_decompress(src: bytes) -> bytes:
    """What klauspost/compress v1.17.11 zstd.Decoder yields through io.Copy
    (the reader at convert_unix.go:252-265): back-to-back frames decoded
    until the input ends; empty input is a clean EOF (no bytes, no error);
    input that ends inside a frame, or a bad frame, is an error."""
    z = _load_zstd()
    ds = z.ZSTD_createDStream()
    out, chunk = [], ctypes.create_string_buffer(1 << 20)
    src_buf = ctypes.create_string_buffer(src, max(1, len(src)))
    ib = _ZBuf(ctypes.cast(src_buf, ctypes.c_void_p), len(src), 0)
    last = 0  # 0: between frames
    try:
        while True:
            ob = _ZBuf(ctypes.cast(chunk, ctypes.c_void_p), len(chunk), 0)
            if ib.pos == ib.size and last == 0:
                break
            before = ib.pos
            last = z.ZSTD_decompressStream(ds, ctypes.byref(ob), ctypes.byref(ib))
            if z.ZSTD_isError(last):
                raise ValueError("zstd: bad frame")
            out.append(chunk.raw[:ob.pos])
            if ib.pos == ib.size and ob.pos == 0 and before == ib.pos and last != 0:
                raise ValueError("zstd: unexpected EOF")
    finally:
        z.ZSTD_freeDStream(ds)
    return b"".join(out)


def lz4_block_decompress(src: bytes, usize: int) -> bytes:
    global _lz4
    if _lz4 is None:
        _lz4 = ctypes.CDLL("liblz4.so.1")
        _lz4.LZ4_decompress_safe.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int,
                                             ctypes.c_int]
    dst = ctypes.create_string_buffer(max(1, usize))
    r = _lz4.LZ4_decompress_safe(src, dst, len(src), usize)
    if r != usize:
        raise ValueError("lz4 decompression failed")
    return dst.raw[:usize]


def chunk_bytes(blob: bytes, rec, compressor: int) -> bytes:
    """Bytes of one chunk record (80-B RAFS v6 chunk info) from image.blob."""
    off, cs, us = int(rec["compressed_offset"]), int(rec["compressed_size"]), int(rec["uncompressed_size"])
    raw = blob[off:off + cs]
    if not int(rec["flags"]) & 1:
        if cs != us:
            raise ValueError("raw chunk with csize != usize")
        return raw
    if compressor == COMPRESSOR_ZSTD:
        return zstd_decompress(raw, us)
    if compressor == COMPRESSOR_LZ4_BLOCK:
        return lz4_block_decompress(raw, us)
    raise ValueError("compressed chunk in an uncompressed blob")


def check_record_rules(recs: np.ndarray, blob_compressed_size=None, blob_uncompressed_size=None):
    """The fixture's chunk-record rules (see module doc)."""
    r = recs[np.argsort(recs["index"], kind="stable")]
    flags = r["flags"].astype(np.int64)
    cs, us = r["compressed_size"].astype(np.int64), r["uncompressed_size"].astype(np.int64)
    ok = bool(((flags & 1) | (cs == us)).all()) and bool((cs[(flags & 1) == 1] < us[(flags & 1) == 1]).all())
    co = r["compressed_offset"].astype(np.int64)
    if len(r):
        ok = ok and bool((co[1:] == co[:-1] + cs[:-1]).all()) and int(co[0]) == 0
        if blob_compressed_size is not None:
            ok = ok and int(co[-1] + cs[-1]) == int(blob_compressed_size)
        if blob_uncompressed_size is not None:
            end = int(r["uncompressed_offset"][-1]) + int(us[-1])
            ok = ok and (end + 4095) // 4096 * 4096 == int(blob_uncompressed_size)
    return ok
